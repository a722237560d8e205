// Probe: latency of s_store_dwordx2 (issue -> lgkmcnt(0)), for a fresh line per store, for
// the same line, and for a 12-store burst; plus ds_read_b64 latency.  Cycles from s_memtime,
// one wave, and with 2048 waves resident (2 per SIMD) all doing the same.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int MODE>
__global__ void k(uint64_t* ws, uint64_t* out, int iters) {
  __shared__ uint64_t lds[512];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  uint64_t base = (uint64_t)(ws + (size_t)blockIdx.x * iters * 16);
  base = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)base) | ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(base >> 32)) << 32);
  uint64_t v = 0x1234;
  uint64_t total = 0;
  uint32_t acc = 0;
  for (int i = 0; i < iters; i++) {
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 0) {  // one store, new 64-B line each iteration
      asm volatile("s_store_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" ::"s"(v), "s"(base + (uint64_t)i * 128) : "memory");
    } else if (MODE == 1) {  // one store, same line every iteration
      asm volatile("s_store_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" ::"s"(v), "s"(base) : "memory");
    } else if (MODE == 2) {  // 12 stores over 96 B (two frames x 6 steps), then wait
      uint64_t b = base + (uint64_t)i * 96;
      asm volatile(
          "s_store_dwordx2 %0, %1, 0x0\n\ts_store_dwordx2 %0, %1, 0x8\n\ts_store_dwordx2 %0, %1, 0x10\n\t"
          "s_store_dwordx2 %0, %1, 0x18\n\ts_store_dwordx2 %0, %1, 0x20\n\ts_store_dwordx2 %0, %1, 0x28\n\t"
          "s_store_dwordx2 %0, %1, 0x30\n\ts_store_dwordx2 %0, %1, 0x38\n\ts_store_dwordx2 %0, %1, 0x40\n\t"
          "s_store_dwordx2 %0, %1, 0x48\n\ts_store_dwordx2 %0, %1, 0x50\n\ts_store_dwordx2 %0, %1, 0x58\n\t"
          "s_waitcnt lgkmcnt(0)" ::"s"(v), "s"(b) : "memory");
    } else if (MODE == 3) {  // ds_read_b64 latency
      uint64_t x;
      asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"((uint32_t)(threadIdx.x * 8)) : "memory");
      acc += (uint32_t)x;
    } else if (MODE == 4) {  // 12 stores to a fresh region, wait deferred by 300 cycles of VALU
      uint64_t b = base + (uint64_t)i * 96;
      asm volatile(
          "s_store_dwordx2 %0, %1, 0x0\n\ts_store_dwordx2 %0, %1, 0x8\n\ts_store_dwordx2 %0, %1, 0x10\n\t"
          "s_store_dwordx2 %0, %1, 0x18\n\ts_store_dwordx2 %0, %1, 0x20\n\ts_store_dwordx2 %0, %1, 0x28\n\t"
          "s_store_dwordx2 %0, %1, 0x30\n\ts_store_dwordx2 %0, %1, 0x38\n\ts_store_dwordx2 %0, %1, 0x40\n\t"
          "s_store_dwordx2 %0, %1, 0x48\n\ts_store_dwordx2 %0, %1, 0x50\n\ts_store_dwordx2 %0, %1, 0x58\n\t"
          ::"s"(v), "s"(b) : "memory");
      uint64_t t1 = __builtin_amdgcn_s_memtime();
      asm volatile(".rept 64\n\tv_add_u32 %0, %0, 1\n\t.endr" : "+v"(acc));
      uint64_t t2 = __builtin_amdgcn_s_memtime();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      t0 += t2 - t1;  // report only the time spent waiting after the VALU block + issue
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    total += t1 - t0;
  }
  asm volatile("s_dcache_wb\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) out[blockIdx.x] = total;
  if (acc == 0x12345) out[1 << 20] = acc;
}

template <int MODE>
void run(const char* name, uint64_t* ws, uint64_t* out, int blocks) {
  const int iters = 200;
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, ws, out, iters);
  (void)hipDeviceSynchronize();
  static uint64_t h[4096];
  (void)hipMemcpy(h, out, blocks * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (int b = 0; b < blocks; b++) s += h[b];
  printf("%-44s blocks %5d: %8.1f cycles per iteration\n", name, blocks, s / blocks / iters);
}

int main() {
  uint64_t *ws, *out;
  (void)hipMalloc(&ws, (size_t)2048 * 200 * 16 * 8 + 4096);
  (void)hipMalloc(&out, ((1 << 20) + 8) * 8);
  for (int blocks : {1, 2048}) {
    run<0>("s_store new line + wait", ws, out, blocks);
    run<1>("s_store same line + wait", ws, out, blocks);
    run<2>("12 s_store (96 B) + wait", ws, out, blocks);
    run<3>("ds_read_b64 + wait", ws, out, blocks);
    run<4>("12 s_store, 64 v_add, then wait (incl.)", ws, out, blocks);
  }
  return 0;
}
