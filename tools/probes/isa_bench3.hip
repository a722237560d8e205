// Third ISA micro-benchmark: which VALU ops issue at the fast (two-pass) rate on gfx950.
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
    if constexpr (K == 0) INDEP("v_min_f32", "%8, %9")
    if constexpr (K == 1) INDEP("v_max_f32", "%8, %9")
    if constexpr (K == 2) INDEP("v_add_f32", "%8, %9")
    if constexpr (K == 3) INDEP("v_pk_min_f16", "%8, %9")
    if constexpr (K == 4) INDEP("v_pk_add_f16", "%8, %9")
    if constexpr (K == 5) INDEP("v_min_f16", "%8, %9")
    if constexpr (K == 6) INDEP("v_min3_u32", "%8, %9, %8")
    if constexpr (K == 7) INDEP("v_med3_u32", "%8, %9, %8")
    if constexpr (K == 8) INDEP("v_and_b32_dpp", "%8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
    if constexpr (K == 9) INDEP("v_xor_b32_dpp", "%8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
    if constexpr (K == 10) INDEP("v_min_u32_dpp", "%8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
    if constexpr (K == 11) INDEP("v_add_f32_dpp", "%8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
    if constexpr (K == 12) INDEP("v_sub_u16", "%8, %9")
    if constexpr (K == 13) INDEP("v_cndmask_b32_e64", "%8, %9, s[0:1]")
    if constexpr (K == 14) INDEP("v_mul_lo_u32", "%8, %9")
    if constexpr (K == 15) INDEP("v_subrev_u32", "%8, %9")
    if constexpr (K == 16) INDEP("v_lshlrev_b16", "%8, %9")
    if constexpr (K == 17) INDEP("v_sub_u32_e64", "%8, %9")
    if constexpr (K == 18) INDEP("v_not_b32", "%8")
    if constexpr (K == 19) INDEP("v_bfrev_b32", "%8")
    if constexpr (K == 20) INDEP("v_add_u32_sdwa", "%8, %9 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0")
    if constexpr (K == 21) INDEP("v_and_b32_e64", "%8, %9")
    if constexpr (K == 22) INDEP("v_pk_min_i16", "%8, %9")
    if constexpr (K == 23) INDEP("v_maximum3_f32", "%8, %9, %8")
    if constexpr (K == 24) INDEP("v_pk_minimum3_f16", "%8, %9, %8")
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
  run<0>("v_min_f32", d, 64);
  run<1>("v_max_f32", d, 64);
  run<2>("v_add_f32", d, 64);
  run<3>("v_pk_min_f16", d, 64);
  run<4>("v_pk_add_f16", d, 64);
  run<5>("v_min_f16", d, 64);
  run<6>("v_min3_u32", d, 64);
  run<7>("v_med3_u32", d, 64);
  run<8>("v_and_b32_dpp", d, 64);
  run<9>("v_xor_b32_dpp", d, 64);
  run<10>("v_min_u32_dpp", d, 64);
  run<11>("v_add_f32_dpp", d, 64);
  run<12>("v_sub_u16", d, 64);
  run<13>("v_cndmask_b32_e64", d, 64);
  run<14>("v_mul_lo_u32", d, 64);
  run<15>("v_subrev_u32", d, 64);
  run<16>("v_lshlrev_b16", d, 64);
  run<17>("v_sub_u32_e64", d, 64);
  run<18>("v_not_b32", d, 64);
  run<19>("v_bfrev_b32", d, 64);
  run<20>("v_add_u32_sdwa", d, 64);
  run<21>("v_and_b32_e64", d, 64);
  run<22>("v_pk_min_i16", d, 64);
  run<23>("v_maximum3_f32", d, 64);
  run<24>("v_pk_minimum3_f16", d, 64);
  return 0;
}
