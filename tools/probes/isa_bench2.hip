// Second ISA micro-benchmark: the ops considered for the tie-in-LSB ACS redesign (gfx950).
// Per instruction: clocks per instruction for one wave (s_memtime around an unrolled
// block), and whole-chip wall clocks per wave-instruction per SIMD at 2 and 4 waves/SIMD
// (computed at a nominal 2.4 GHz, so absolute values read high if the chip clocks lower;
// compare ratios).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REP8(X) X X X X X X X X
#define REP64(X) REP8(REP8(X))
#define OUTS "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
#define ROW8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define STR_(x) #x
#define STR(x) STR_(x)

// 8 independent destinations: "<op> %k, <args>" for k = 0..7; args reference %8 / %9.
#define BODY(op, args)                                                                     \
  REP8(op " %0, " args "\n\t" op " %1, " args "\n\t" op " %2, " args "\n\t" op " %3, " args \
       "\n\t" op " %4, " args "\n\t" op " %5, " args "\n\t" op " %6, " args "\n\t" op " %7, " args "\n\t")
#define INDEP(op, args) asm volatile(BODY(op, args) : OUTS : "v"(a), "v"(b));

template <int K>
__global__ void bench(uint64_t* out, int iters) {
  uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5, r6 = r0 + 6, r7 = r0 + 7;
  uint32_t a = threadIdx.x * 3 + 1, b = threadIdx.x ^ 5;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    if constexpr (K == 0) INDEP("v_and_b32", "%8, %9")
    if constexpr (K == 1) INDEP("v_or_b32", "%8, %9")
    if constexpr (K == 2) INDEP("v_max_u32", "%8, %9")
    if constexpr (K == 3) INDEP("v_mov_b32", "%8")
    if constexpr (K == 4) INDEP("v_lshrrev_b32", "%8, %9")
    if constexpr (K == 5) INDEP("v_xad_u32", "%8, %9, %8")
    if constexpr (K == 6) INDEP("v_add3_u32", "%8, %9, %8")
    if constexpr (K == 7) INDEP("v_lshl_or_b32", "%8, 2, %9")
    if constexpr (K == 8) INDEP("v_and_or_b32", "%8, %9, %8")
    if constexpr (K == 9) INDEP("v_lshl_add_u32", "%8, 2, %9")
    if constexpr (K == 10) INDEP("v_or3_b32", "%8, %9, %8")
    if constexpr (K == 11) INDEP("v_bitop3_b32", "%8, %9, %8 bitop3:0xca")
    if constexpr (K == 12) INDEP("v_add_u16", "%8, %9")
    if constexpr (K == 13) INDEP("v_min_u16", "%8, %9")
    if constexpr (K == 14) INDEP("v_pk_sub_u16", "%8, %9")
    if constexpr (K == 15) INDEP("v_pk_sub_i16", "%8, %9")
    if constexpr (K == 16) INDEP("v_sub_u32_dpp", "%8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
    if constexpr (K == 17) INDEP("v_add_u32_dpp", "%8, %9 row_half_mirror row_mask:0xf bank_mask:0xf")
    if constexpr (K == 18) INDEP("v_add_co_u32", "vcc, %8, %9")
    if constexpr (K == 19) INDEP("v_min_i32", "%8, %9")
    if constexpr (K == 20) INDEP("v_mul_u32_u24", "%8, %9")
    if constexpr (K == 21) INDEP("v_alignbit_b32", "%8, %9, 3")
    if constexpr (K == 22) INDEP("v_bfe_u32", "%8, 3, 2")
    if constexpr (K == 23) asm volatile(REP64("v_readlane_b32 s20, %0, 0\n\t") :: "v"(r0) : "s20");
    if constexpr (K == 24) INDEP("v_add_u32_e64", "%8, %9")
    if constexpr (K == 25) INDEP("v_pk_max_u16", "%8, %9")
    if constexpr (K == 26) INDEP("v_pk_add_u16", "%8, %9 op_sel:[1,0] op_sel_hi:[0,1]")
    if constexpr (K == 27) asm volatile(REP8(REP8("v_add_u32 %1, %0, %8\n\tv_add_u32 %2, %1, %9\n\tv_add_u32_dpp %3, %0, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_pk_min_u16 %0, %1, %3\n\tv_pk_sub_i16 %4, %2, %3\n\t")) : OUTS : "v"(a), "v"(b));
    if constexpr (K == 28) asm volatile(REP8(REP8("v_add_u32 %1, %0, %8\n\tv_add_u32_dpp %3, %0, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_pk_min_u16 %0, %1, %3\n\t")) : OUTS : "v"(a), "v"(b));
    if constexpr (K == 29) asm volatile(REP8(REP8("v_add_u32 %1, %0, %8\n\tv_add_u32_dpp %3, %0, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_add_u32 %5, %4, %8\n\tv_add_u32_dpp %6, %4, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_pk_min_u16 %0, %1, %3\n\tv_pk_min_u16 %4, %5, %6\n\t")) : OUTS : "v"(a), "v"(b));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7 == 0x12345) out[1 << 20] = 1;
}

template <int K>
void run(const char* name, uint64_t* d, int ninstr_per_iter) {
  const int iters = 200;
  uint64_t h[1];
  hipLaunchKernelGGL(bench<K>, dim3(1), dim3(64), 0, 0, d, iters);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
  double c1 = double(h[0]) / (iters * ninstr_per_iter);
  double r[2];
  int wps[2] = {2, 4};
  for (int i = 0; i < 2; i++) {
    int waves = 256 * 4 * wps[i];
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(bench<K>, dim3(waves), dim3(64), 0, 0, d, iters);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(bench<K>, dim3(waves), dim3(64), 0, 0, d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    r[i] = ms * 1e-3 * 2.4e9 / (double(iters) * ninstr_per_iter * wps[i]);
  }
  printf("%-34s 1 wave: %6.2f   2 w/SIMD: %6.2f   4 w/SIMD: %6.2f\n", name, c1, r[0], r[1]);
}

int main() {
  uint64_t* d;
  if (hipMalloc(&d, (1 << 20) * 8 + 64) != hipSuccess) return 1;
  run<0>("v_and_b32", d, 64);
  run<1>("v_or_b32", d, 64);
  run<2>("v_max_u32", d, 64);
  run<3>("v_mov_b32", d, 64);
  run<4>("v_lshrrev_b32", d, 64);
  run<5>("v_xad_u32", d, 64);
  run<6>("v_add3_u32", d, 64);
  run<7>("v_lshl_or_b32", d, 64);
  run<8>("v_and_or_b32", d, 64);
  run<9>("v_lshl_add_u32", d, 64);
  run<10>("v_or3_b32", d, 64);
  run<11>("v_bitop3_b32", d, 64);
  run<12>("v_add_u16", d, 64);
  run<13>("v_min_u16", d, 64);
  run<14>("v_pk_sub_u16", d, 64);
  run<15>("v_pk_sub_i16", d, 64);
  run<16>("v_sub_u32_dpp", d, 64);
  run<17>("v_add_u32_dpp", d, 64);
  run<18>("v_add_co_u32", d, 64);
  run<19>("v_min_i32", d, 64);
  run<20>("v_mul_u32_u24", d, 64);
  run<21>("v_alignbit_b32", d, 64);
  run<22>("v_bfe_u32", d, 64);
  run<23>("v_readlane_b32_x", d, 64);
  run<24>("v_add_u32_e64", d, 64);
  run<25>("v_pk_max_u16", d, 64);
  run<26>("v_pk_add_u16 op_sel", d, 64);
  run<27>("ACS old step (add,add,adddpp,pkmin,pksub) /instr", d, 320);
  run<28>("ACS new step (add,adddpp,pkmin) /instr", d, 192);
  run<29>("2 chains new step /instr", d, 384);
  return 0;
}
