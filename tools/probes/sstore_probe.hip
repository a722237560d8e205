// Probe: does s_store_dwordx2 (scalar store through the scalar data cache) work on gfx950,
// and is the data visible to the host after s_dcache_wb + kernel end?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int MODE>
__global__ void k(uint64_t* out, const int* in, int steps) {
  int lane = threadIdx.x;
  uint64_t* base = out + (size_t)blockIdx.x * steps * 2;
  for (int t = 0; t < steps; t++) {
    int v = __builtin_amdgcn_readfirstlane(0) + (int)(((unsigned)(t * 64 + lane + blockIdx.x) * 2654435761u) >> 7) - (1 << 24);
    uint64_t m1, m2;
    asm("v_cmp_lt_i32_e64 %0, %1, 0" : "=s"(m1) : "v"(v));
    asm("v_cmp_gt_i32_e64 %0, %1, 0" : "=s"(m2) : "v"(v));
    uint64_t addr = (uint64_t)(base + 2 * t);
    if (MODE == 0) asm volatile("s_store_dwordx2 %0, %1, 0x0\n\ts_store_dwordx2 %2, %1, 0x8" :: "s"(m1), "s"(addr), "s"(m2) : "memory");
    if (MODE == 1) { if (t == steps - 1) asm volatile("s_store_dwordx2 %0, %1, 0x0\n\ts_store_dwordx2 %2, %1, 0x8" :: "s"(m1), "s"(addr), "s"(m2) : "memory"); else asm volatile("" :: "s"(m1), "s"(m2)); }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_dcache_wb\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
}

int main() {
  const int blocks = 2048, steps = 1030;
  std::vector<int> h(4096);
  for (int i = 0; i < 4096; i++) h[i] = (int)((i * 2654435761u) >> 7) - (1 << 24);
  int* din; uint64_t* dout;
  hipMalloc(&din, 4096 * 4); hipMalloc(&dout, (size_t)blocks * steps * 16);
  hipMemcpy(din, h.data(), 4096 * 4, hipMemcpyHostToDevice);
  hipMemset(dout, 0xAB, (size_t)blocks * steps * 16);
  hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, dout, din, steps);
  hipError_t e = hipDeviceSynchronize();
  std::vector<uint64_t> o((size_t)blocks * steps * 2);
  hipMemcpy(o.data(), dout, o.size() * 8, hipMemcpyDeviceToHost);
  long bad = 0;
  for (int b = 0; b < blocks; b++)
    for (int t = 0; t < steps; t++) {
      uint64_t m1 = 0, m2 = 0;
      for (int l = 0; l < 64; l++) {
        int v = (int)(((unsigned)(t * 64 + l + b) * 2654435761u) >> 7) - (1 << 24);
        if (v < 0) m1 |= 1ull << l;
        if (v > 0) m2 |= 1ull << l;
      }
      bad += (o[((size_t)b * steps + t) * 2] != m1) + (o[((size_t)b * steps + t) * 2 + 1] != m2);
    }
  // timing
  hipEvent_t a, z; hipEventCreate(&a); hipEventCreate(&z);
  hipEventRecord(a);
  for (int i = 0; i < 20; i++) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, dout, din, steps);
  hipEventRecord(z); hipEventSynchronize(z);
  float ms; hipEventElapsedTime(&ms, a, z);
  hipEventRecord(a);
  for (int i = 0; i < 20; i++) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, dout, din, steps);
  hipEventRecord(z); hipEventSynchronize(z);
  float ms1; hipEventElapsedTime(&ms1, a, z);
  printf("no-store variant: %.2f us/launch\n", ms1 * 1000 / 20);
  printf("sstore probe: err=%d mismatches=%ld of %zu, %.2f us/launch\n", (int)e, bad, o.size(), ms * 1000 / 20);
  return bad != 0;
}
