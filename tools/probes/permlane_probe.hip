// Probe: v_permlane{16,32}_swap_b32 with vdst == src0 -- does it exchange the two halves of
// one register in place (lane l <- lane l ^ 16 / l ^ 32)?  Also checks v_add_u32_dpp with
// row_ror:8 / quad_perm / row_half_mirror chained, as used by the ACS exchange.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__global__ void k(uint32_t* out) {
  uint32_t l = threadIdx.x;
  uint32_t a = l * 7 + 100, b = a;
  asm volatile("s_nop 4\n\tv_permlane32_swap_b32 %0, %0" : "+v"(a));
  asm volatile("v_permlane16_swap_b32 %0, %0" : "+v"(b));
  uint32_t w = 1000;
  uint32_t c = l * 3 + 5, d;
  asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %1, %2 row_ror:8 row_mask:0xf bank_mask:0xf" : "=v"(d) : "v"(c), "v"(w));
  out[l] = a;
  out[64 + l] = b;
  out[128 + l] = d;
}

int main() {
  uint32_t* d;
  uint32_t h[192];
  (void)hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad32 = 0, bad16 = 0, badror = 0;
  for (int l = 0; l < 64; l++) {
    bad32 += h[l] != (uint32_t)((l ^ 32) * 7 + 100);
    bad16 += h[64 + l] != (uint32_t)((l ^ 16) * 7 + 100);
    int src = (l & ~15) | ((l + 8) & 15);  // row_ror:8 within a 16-lane row
    badror += h[128 + l] != (uint32_t)(src * 3 + 5 + 1000);
  }
  printf("permlane32 in-place mismatches %d, permlane16 in-place mismatches %d, add_dpp ror8 mismatches %d\n", bad32,
         bad16, badror);
  for (int l = 0; l < 4; l++) printf("lane %d: p32 %u p16 %u ror %u\n", l, h[l], h[64 + l], h[128 + l]);
  return 0;
}
