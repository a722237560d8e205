// Device helpers shared by the two K=7 register-resident kernels (vtb_k7_lds.hip: survivor
// words in LDS; vtb_reg_path.hip: survivor words in a global workspace).  See the header of
// vtb_k7_lds.hip for the layout these helpers assume.
#pragma once

#include "vtb_internal.h"

namespace vtb {
namespace k7 {

constexpr int kChunk = 48;          // ACS steps per unrolled body = lcm(6 phases, 16-step words)
constexpr int kTabBytes = 64;       // branch-metric table, per step: 8 (V, W) u32 pairs
constexpr uint32_t kBias = 8192;    // renormalised doubled metrics stay within kBias +- 6120

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_h2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) {
    return as_u(__builtin_elementwise_min(as_h2(a), as_h2(b)));
}
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) { return as_u(as_h2(a) + as_h2(b)); }
__device__ __forceinline__ uint32_t pk_sub(uint32_t a, uint32_t b) { return as_u(as_h2(a) - as_h2(b)); }

// Wave-uniform value in SGPRs (scalar-store base addresses).
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(x));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(x >> 32));
    return uint64_t(lo) | (uint64_t(hi) << 32);
}

__device__ __forceinline__ int rotl6(int x, int r) { return ((x << r) | (x >> (6 - r))) & 63; }

// Location-bit masks: bit l set iff bit p of l is set.
__host__ __device__ constexpr uint64_t loc_mask(int p) {
    return p == 0 ? 0xAAAAAAAAAAAAAAAAull : p == 1 ? 0xCCCCCCCCCCCCCCCCull : p == 2 ? 0xF0F0F0F0F0F0F0F0ull
         : p == 3 ? 0xFF00FF00FF00FF00ull : p == 4 ? 0xFFFF0000FFFF0000ull : 0xFFFFFFFF00000000ull;
}

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

// Byte offset of lane's (V, W) pair inside a step's table row, per phase ph = t mod 6.  At
// phase ph the pairing bit is p = 5 - ph; the butterfly's upper-half state is
// j = rotl6(lane with bit p cleared, ph); the lane's own edge has label c = symm[j] (the
// partner's has ~c) and R = bit p of the lane.
__device__ __forceinline__ void table_offsets(const Launch& table, int lane, uint32_t off[6]) {
#pragma unroll
    for (int ph = 0; ph < 6; ph++) {
        const int p = 5 - ph;
        const int j = rotl6(lane & ~(1 << p), ph);
        const int c = table.symm[j];
        const int R = (lane >> p) & 1;
        off[ph] = uint32_t(8 * (c + 4 * R));
    }
}

// Received pair of step t of one frame as (q0 | q1 << 16); hard input is one byte per
// segment (bit i = coded bit i, reference convEncode.c layout), soft is two bytes.
template <bool SOFT>
__device__ __forceinline__ uint32_t load_q(const uint8_t* frame, int t) {
    if constexpr (SOFT) {
        const uint8_t* p = frame + 2 * (size_t)t;
        return uint32_t(p[0]) | (uint32_t(p[1]) << 16);
    } else {
        const uint32_t c = frame[t];
        return (c & 1u) | (((c >> 1) & 1u) << 16);
    }
}

// One table row from the packed pairs of frames A and B: entries (c, R) for labels
// c = 0..3 (bit 0 of the label <-> coded bit 0) and R = 0/1 hold V = 2e(c) + R and
// W = 2e(~c), both frames packed [A, B].
template <uint32_t Q>
__device__ __forceinline__ void write_row(uint8_t* row_ptr, uint32_t qa, uint32_t qb) {
    const uint32_t q0 = (qa & 0xffffu) | (qb << 16);      // [q0_A, q0_B]
    const uint32_t q1 = (qa >> 16) | (qb & 0xffff0000u);  // [q1_A, q1_B]
    const uint32_t n0 = Q * 0x10001u - q0, n1 = Q * 0x10001u - q1;
    const uint32_t e0 = 2 * (q0 + q1), e1 = 2 * (n0 + q1), e2 = 2 * (q0 + n1), e3 = 2 * (n0 + n1);
    constexpr uint32_t R1 = 0x10001u;
    uint4* row = reinterpret_cast<uint4*>(row_ptr);
    row[0] = make_uint4(e0, e3, e1, e2);            // (c=0,R=0) (c=1,R=0)
    row[1] = make_uint4(e2, e1, e3, e0);            // (c=2,R=0) (c=3,R=0)
    row[2] = make_uint4(e0 + R1, e3, e1 + R1, e2);  // (c=0,R=1) (c=1,R=1)
    row[3] = make_uint4(e2 + R1, e1, e3 + R1, e0);  // (c=2,R=1) (c=3,R=1)
}

}  // namespace k7
}  // namespace vtb
