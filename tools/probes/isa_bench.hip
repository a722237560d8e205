// Micro-benchmark of the instruction types the ACS / traceback loops use (gfx950).
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
    if constexpr (K == 0) INDEP("v_add_u32", "%8, %9")
    if constexpr (K == 1) asm volatile(REP64("v_add_u32 %0, %0, %1\n\t") : "+v"(r0) : "v"(a));
    if constexpr (K == 2) INDEP("v_pk_add_u16", "%8, %9")
    if constexpr (K == 3) asm volatile(REP64("v_pk_add_u16 %0, %0, %1\n\t") : "+v"(r0) : "v"(a));
    if constexpr (K == 4) INDEP("v_pk_min_u16", "%8, %9")
    if constexpr (K == 5) INDEP("v_pk_mad_u16", "%8, %9, %8")
    if constexpr (K == 6) INDEP("v_mov_b32_dpp", "%8 row_ror:8 row_mask:0xf bank_mask:0xf")
    if constexpr (K == 7) INDEP("v_add_u32_dpp", "%8, %9 row_ror:8 row_mask:0xf bank_mask:0xf")
    if constexpr (K == 8) INDEP("v_add_u32_dpp", "%8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
    if constexpr (K == 9) asm volatile(REP64("v_mov_b32_dpp %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\ts_nop 1\n\t") : "+v"(r0));
    if constexpr (K == 10) asm volatile(REP8("v_permlane32_swap_b32 %0, %1\n\tv_permlane32_swap_b32 %2, %3\n\tv_permlane32_swap_b32 %4, %5\n\tv_permlane32_swap_b32 %6, %7\n\t") : OUTS);
    if constexpr (K == 11) asm volatile(REP8("v_permlane16_swap_b32 %0, %1\n\tv_permlane16_swap_b32 %2, %3\n\tv_permlane16_swap_b32 %4, %5\n\tv_permlane16_swap_b32 %6, %7\n\t") : OUTS);
    if constexpr (K == 12) asm volatile(REP64("v_cmp_lt_i16_sdwa s[20:21], %0, %1 src0_sel:WORD_1 src1_sel:WORD_1\n\t") :: "v"(r0), "v"(a) : "s20", "s21");
    if constexpr (K == 13) asm volatile(REP64("v_cmp_ne_u16_e32 vcc, %0, %1\n\t") :: "v"(r0), "v"(a) : "vcc");
    if constexpr (K == 14) asm volatile("s_mov_b32 s22, 0xffff\n\t" REP64("v_cmp_lt_u32_e64 s[20:21], s22, %0\n\t") :: "v"(r0) : "s20", "s21", "s22");
    if constexpr (K == 15) asm volatile("s_mov_b64 s[20:21], 0x5555\n\t" BODY("v_cndmask_b32_e64", "%8, %9, s[20:21]") : OUTS : "v"(a), "v"(b) : "s20", "s21");
    if constexpr (K == 16) asm volatile("s_mov_b64 vcc, 0x5555\n\t" BODY("v_cndmask_b32_e32", "%8, %9, vcc") : OUTS : "v"(a), "v"(b) : "vcc");
    if constexpr (K == 17) INDEP("v_sub_u32", "%8, %9")
    if constexpr (K == 18) INDEP("v_min_u32", "%8, %9")
    if constexpr (K == 19) INDEP("v_bfi_b32", "%8, %9, %8")
    if constexpr (K == 20) INDEP("v_lshlrev_b32", "%8, %9")
    if constexpr (K == 21) INDEP("v_perm_b32", "%8, %9, %8")
    if constexpr (K == 22) asm volatile(REP8("v_writelane_b32 %0, s20, 1\n\tv_writelane_b32 %1, s21, 2\n\tv_writelane_b32 %2, s20, 3\n\tv_writelane_b32 %3, s21, 4\n\tv_writelane_b32 %4, s20, 5\n\tv_writelane_b32 %5, s21, 6\n\tv_writelane_b32 %6, s20, 7\n\tv_writelane_b32 %7, s21, 8\n\t") : OUTS :: "s20", "s21");
    if constexpr (K == 23) asm volatile(REP8("ds_swizzle_b32 %0, %8 offset:swizzle(SWAP,16)\n\tds_swizzle_b32 %1, %8 offset:swizzle(SWAP,16)\n\tds_swizzle_b32 %2, %8 offset:swizzle(SWAP,16)\n\tds_swizzle_b32 %3, %8 offset:swizzle(SWAP,16)\n\tds_swizzle_b32 %4, %8 offset:swizzle(SWAP,16)\n\tds_swizzle_b32 %5, %8 offset:swizzle(SWAP,16)\n\tds_swizzle_b32 %6, %8 offset:swizzle(SWAP,16)\n\tds_swizzle_b32 %7, %8 offset:swizzle(SWAP,16)\n\ts_waitcnt lgkmcnt(0)\n\t") : OUTS : "v"(a));
    if constexpr (K == 24) asm volatile(REP64("ds_swizzle_b32 %0, %0 offset:swizzle(SWAP,16)\n\ts_waitcnt lgkmcnt(0)\n\t") : "+v"(r0));
    if constexpr (K == 25) INDEP("v_max3_u32", "%8, %9, %8")
    if constexpr (K == 26) INDEP("v_dot2_i32_i16", "%8, %9, %8")
    if constexpr (K == 27) INDEP("v_xor_b32", "%8, %9")
    if constexpr (K == 28) asm volatile(REP64("v_add_u32 %0, %0, %1\n\tv_pk_min_u16 %0, %0, %1\n\t") : "+v"(r0) : "v"(a));
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
  run<0>("v_add_u32 indep", d, 64);
  run<1>("v_add_u32 dep", d, 64);
  run<2>("v_pk_add_u16 indep", d, 64);
  run<3>("v_pk_add_u16 dep", d, 64);
  run<4>("v_pk_min_u16 indep", d, 64);
  run<5>("v_pk_mad_u16 indep", d, 64);
  run<6>("v_mov_b32_dpp row_ror indep", d, 64);
  run<7>("v_add_u32_dpp row_ror indep", d, 64);
  run<8>("v_add_u32_dpp quad_perm indep", d, 64);
  run<9>("v_mov_dpp dep (+s_nop 1)", d, 64);
  run<10>("v_permlane32_swap indep", d, 32);
  run<11>("v_permlane16_swap indep", d, 32);
  run<12>("v_cmp_lt_i16_sdwa -> sgpr", d, 64);
  run<13>("v_cmp_ne_u16_e32 -> vcc", d, 64);
  run<14>("v_cmp_lt_u32_e64 -> sgpr", d, 64);
  run<15>("v_cndmask_b32_e64 (sgpr mask)", d, 64);
  run<16>("v_cndmask_b32_e32 (vcc)", d, 64);
  run<17>("v_sub_u32 indep", d, 64);
  run<18>("v_min_u32 indep", d, 64);
  run<19>("v_bfi_b32 indep", d, 64);
  run<20>("v_lshlrev_b32 indep", d, 64);
  run<21>("v_perm_b32 indep", d, 64);
  run<22>("v_writelane_b32 indep", d, 64);
  run<23>("ds_swizzle SWAP16 (batch 8)", d, 64);
  run<24>("ds_swizzle dep (latency)", d, 64);
  run<25>("v_max3_u32 indep", d, 64);
  run<26>("v_dot2_i32_i16 indep", d, 64);
  run<27>("v_xor_b32 indep", d, 64);
  run<28>("v_add_u32 -> v_pk_min dep", d, 128);
  return 0;
}
