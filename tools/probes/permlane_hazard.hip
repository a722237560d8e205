// Probe: wait states needed between a VALU write of a VGPR and v_permlane{16,32}_swap
// reading it in place (vdst == src0).  Each variant writes the source with v_add_u32 right
// before the swap, separated by s_nop N.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define VARIANT(NOPS, OP)                                                              \
  {                                                                                    \
    uint32_t a;                                                                        \
    asm volatile("v_add_u32 %0, %1, %2\n\t" NOPS OP " %0, %0" : "=&v"(a) : "v"(l), "v"(base)); \
    out[idx++ * 64 + l] = a;                                                           \
  }

__global__ void k(uint32_t* out, uint32_t base) {
  uint32_t l = threadIdx.x;
  int idx = 0;
  VARIANT("", "v_permlane32_swap_b32")
  VARIANT("s_nop 0\n\t", "v_permlane32_swap_b32")
  VARIANT("s_nop 1\n\t", "v_permlane32_swap_b32")
  VARIANT("s_nop 2\n\t", "v_permlane32_swap_b32")
  VARIANT("s_nop 3\n\t", "v_permlane32_swap_b32")
  VARIANT("", "v_permlane16_swap_b32")
  VARIANT("s_nop 0\n\t", "v_permlane16_swap_b32")
  VARIANT("s_nop 1\n\t", "v_permlane16_swap_b32")
  VARIANT("s_nop 2\n\t", "v_permlane16_swap_b32")
  VARIANT("s_nop 3\n\t", "v_permlane16_swap_b32")
}

int main() {
  uint32_t* d;
  uint32_t h[640];
  (void)hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 1000u);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[10] = {"p32 nop-", "p32 nop0", "p32 nop1", "p32 nop2", "p32 nop3",
                           "p16 nop-", "p16 nop0", "p16 nop1", "p16 nop2", "p16 nop3"};
  for (int v = 0; v < 10; v++) {
    int x = v < 5 ? 32 : 16, bad = 0;
    for (int l = 0; l < 64; l++) bad += h[v * 64 + l] != (uint32_t)((l ^ x) + 1000);
    printf("%s mismatches %d\n", names[v], bad);
  }
  return 0;
}
