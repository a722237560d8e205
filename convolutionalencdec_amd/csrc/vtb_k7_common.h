// Device helpers of the K=7 register-resident kernel (vtb_k7_lds.hip; survivor words in LDS
// or in a global workspace).  See the header of vtb_k7_lds.hip for the layout these helpers
// assume.
#pragma once

#include "vtb_internal.h"

namespace vtb {
namespace k7 {

constexpr int kChunk = 48;          // ACS steps per unrolled body = lcm(6 phases, 16-step words)

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_h2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) {
    return as_u(__builtin_elementwise_min(as_h2(a), as_h2(b)));
}
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) { return as_u(as_h2(a) + as_h2(b)); }

// Wave-uniform value in SGPRs (base addresses of saddr-form global loads and stores).
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(x));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(x >> 32));
    return uint64_t(lo) | (uint64_t(hi) << 32);
}

__device__ __forceinline__ int rotl6(int x, int r) { return ((x << r) | (x >> (6 - r))) & 63; }

// Partner metric across lane bit P (XOR 1 << P) plus w.  For P = 4, 5 the swap happens in
// place on a copy (one wait state is required between the VALU write of the source and
// the swap: tools/probes/permlane_hazard.hip).
template <int P>
__device__ __forceinline__ uint32_t partner_plus(uint32_t m, uint32_t w) {
    if constexpr (P == 0) {
        return __builtin_amdgcn_update_dpp(0u, m, 0xB1, 0xF, 0xF, true) + w;  // quad_perm [1,0,3,2]
    } else if constexpr (P == 1) {
        return __builtin_amdgcn_update_dpp(0u, m, 0x4E, 0xF, 0xF, true) + w;  // quad_perm [2,3,0,1]
    } else if constexpr (P == 2) {
        uint32_t h = __builtin_amdgcn_mov_dpp(m, 0x141, 0xF, 0xF, false);   // row_half_mirror: i <- 7-i
        return __builtin_amdgcn_update_dpp(0u, h, 0x1B, 0xF, 0xF, true) + w;  // quad_perm [3,2,1,0]
    } else if constexpr (P == 3) {
        return __builtin_amdgcn_update_dpp(0u, m, 0x128, 0xF, 0xF, true) + w;  // row_ror:8
    } else if constexpr (P == 4) {
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %0" : "+v"(m));
        return m + w;
    } else {
        asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %0" : "+v"(m));
        return m + w;
    }
}

}  // namespace k7
}  // namespace vtb
