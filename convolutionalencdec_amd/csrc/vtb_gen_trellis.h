// The generic register-resident trellis (every K = 3..9), shared by the batch and single-frame
// kernels (vtb_lds_path.hip) and the generic stream kernel (vtb_stream_gen.hip).
//
// N = 2^S states over G = min(N, 64) lanes, R = N / G registers per lane, F = 64 / G frames per
// wave.  The states move with the step (vtb_k7_lds.hip's in-place butterfly, generalised): at
// step t, phase ph = t mod S, location l holds state rotl_S(l, ph).  The two predecessors of a
// butterfly, j and j + N/2 (reference viterbiDecoderButterflyk1.c:101-152), are a location and its
// partner across location bit p = S-1-ph; the butterfly's destinations 2j and 2j+1 land back in
// those two locations (location l receives state rotl_S(l, ph+1)).  The gather is one DPP (p = 0..3:
// lane XOR 1, 2, 7, 8 under the lane <-> location involution lane_of), a v_permlane16/32_swap
// (p = 4, 5) or the lane's other register (p >= 6).  Decision bit of the state a location
// receives = bit (lane) of the wave's word: 1 = the upper predecessor won (strict compare, ties
// keep the lower: reference :129-130).  State 0 is location 0 at every phase.
//
// Traceback in locations: with k = (t+1) mod S the state after step t is d = rotl_S(loc, k), so
// its information bit (bit 0 of d) is location bit b = (S - k) mod S, and the predecessor's
// location after step t-1 is loc with bit b replaced by the decision bit (no rotation in the walk).
#pragma once

#include <utility>

#include "vtb_internal.h"

// v_writelane_b32 (no clang builtin in this toolchain: the LLVM intrinsic by name)
__device__ int vtb_writelane(int value, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

namespace vtb {
namespace gen {

template <int S>
struct Geometry {
    static constexpr int N = 1 << S;
    static constexpr int G = N < 64 ? N : 64;  // lanes per frame
    static constexpr int R = N / G;            // states per lane
    static constexpr int F = 64 / G;           // frames per wave
    // the recursion's loop body: U phase cycles, P = U S steps (>= 6: the body outlasts the LDS
    // latency of the next body's input reads)
    static constexpr int U = S <= 2 ? 4 : S <= 4 ? 2 : 1;
    static constexpr int P = U * S;
    static constexpr int C = P * (64 / P);  // steps per keep/store round: whole loop bodies
};

// host side: steps of one loop body (Geometry<S>::P)
constexpr int body_steps(int S) { return S <= 2 ? 4 * S : S <= 4 ? 2 * S : S; }

template <int... Is, class Fn>
__device__ __forceinline__ void gen_static_for(std::integer_sequence<int, Is...>, Fn&& fn) {
    (fn(std::integral_constant<int, Is>{}), ...);
}

// lane <-> location involution (location bit 2 set: bits 0, 1 flipped), so that location
// XOR 4 is lane XOR 7 (DPP row_half_mirror); XOR 1, 2, 8, 16, 32 are unchanged
template <int S>
__host__ __device__ constexpr unsigned lane_of(unsigned l) {
    return S >= 3 ? l ^ (((l >> 2) & 1u) * 3u) : l;
}

template <int S>
__device__ __forceinline__ unsigned rotl_s(unsigned x, int k) {
    return ((x << k) | (x >> (S - k))) & ((1u << S) - 1u);
}

// The partner's metric across location bit P < 6.  For the permlane swaps (in place on a copy)
// one wait state each way (tools/probes/permlane_hazard.hip).
template <int P>
__device__ __forceinline__ int partner(int m) {
    if constexpr (P == 0) {
        return __builtin_amdgcn_update_dpp(0, m, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]: XOR 1
    } else if constexpr (P == 1) {
        return __builtin_amdgcn_update_dpp(0, m, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]: XOR 2
    } else if constexpr (P == 2) {
        return __builtin_amdgcn_update_dpp(0, m, 0x141, 0xF, 0xF, true);  // row_half_mirror: XOR 7
    } else if constexpr (P == 3) {
        return __builtin_amdgcn_update_dpp(0, m, 0x128, 0xF, 0xF, true);  // row_ror:8: XOR 8
    } else if constexpr (P == 4) {
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %0\n\ts_nop 0" : "+v"(m));
        return m;
    } else {
        asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %0\n\ts_nop 0" : "+v"(m));
        return m;
    }
}

typedef short short2_t __attribute__((ext_vector_type(2)));

// Hard input as staged into LDS: the symbol byte's two low bits times 8 (a byte of offsets), and
// the same for the four bytes of a word.
__host__ __device__ constexpr uint32_t hard_offset(uint32_t byte) { return (byte & 3u) << 3; }
__host__ __device__ constexpr uint32_t hard_offset4(uint32_t word) { return (word & 0x03030303u) << 3; }

// Received pair of one step: the staged bytes (hard: one byte, soft: two bytes), then the
// branch-metric operand: soft, the packed bytes for v_dot2; hard, the symbol's bit offset 8 c into
// the location's table of the four branch metrics, which the kernels store in place of the symbol
// byte when they stage the input (hard_offset: the symbol's bits above its two are dropped, as the
// reference's `coded & 3` drops them).  The recursion converts a cycle's bytes only after the
// previous cycle's steps, so that their LDS reads are waited for there and not where they are
// issued.
template <bool SOFT>
__device__ __forceinline__ int rx_raw(const uint8_t* p) {
    if constexpr (SOFT) {
        return int(p[0]) | (int(p[1]) << 16);
    } else {
        return int(p[0]);
    }
}
template <bool SOFT>
__device__ __forceinline__ int rx_pair(int raw) {
    if constexpr (SOFT) {
        return raw;
    } else {
        return raw;  // (staged as hard_offset)
    }
}

// Branch-metric coefficients of location l at phase ph: the centred metric of the lower
// predecessor's edge into the state l receives is v_dot2(sig, rx) + kap, as signed for the
// location's own candidate (own + mu, partner - mu: the sign of the destination parity cancels
// against which of the pair the location holds).
template <int S, int Q>
__device__ __forceinline__ void coefficients(const Launch& table, unsigned l, int ph, int& sig, int& kap) {
    const unsigned s = rotl_s<S>(l, ph);
    const int c = table.symm[s & ((1u << (S - 1)) - 1u)];
    const int s0 = (c & 1) ? -1 : 1, s1 = (c & 2) ? -1 : 1;
    sig = (s0 & 0xffff) | (s1 << 16);
    kap = (((c & 1) + ((c >> 1) & 1)) - 1) * Q;
}

// The per-lane constants of the recursion, by register and phase: branch-metric coefficients (soft:
// v_dot2 operands sig, kap; hard: sig holds the four metrics mu(c) = sig . (c & 1, c >> 1) + kap,
// c = 0..3, as signed bytes -- one v_bfe_i32 per step instead of a v_dot2 and the copy of its
// accumulator) and up = -1 where the location holds the upper predecessor (location bit
// p = S-1-ph set), else 0.
template <int S, int R, bool SOFT>
struct Coef {
    int sig[R][S], kap[R][S], up[R][S];
};
template <int S, int R, bool SOFT>
__device__ __forceinline__ void setup_coef(const Launch& table, unsigned l0, Coef<S, R, SOFT>& k) {
#pragma unroll
    for (int r = 0; r < R; r++) {
        const unsigned l = unsigned(r) * 64u + l0;
#pragma unroll
        for (int ph = 0; ph < S; ph++) {
            int sig, kap;
            coefficients<S, SOFT ? 255 : 1>(table, l, ph, sig, kap);
            if constexpr (SOFT) {
                k.sig[r][ph] = sig, k.kap[r][ph] = kap;
            } else {
                const int s0 = int(short(sig & 0xffff)), s1 = sig >> 16;
                unsigned tab = 0;
                for (int c = 0; c < 4; c++) tab |= unsigned((s0 * (c & 1) + s1 * (c >> 1) + kap) & 0xff) << (8 * c);
                k.sig[r][ph] = int(tab), k.kap[r][ph] = 0;
            }
            k.up[r][ph] = ((l >> (S - 1 - ph)) & 1u) ? -1 : 0;
        }
    }
}

// One trellis step at phase PH (compile time): metrics m[R] in place, the R decision words out.
// The decision (lower's candidate > upper's, strict) is one compare on the VALU:
// ((own - partner's) ^ up) > up, i.e. own > partner's where the location holds the lower
// predecessor and partner's > own where it holds the upper (tools/probes/genstep_probe.hip: 12 %
// fewer cycles per step than two compares combined with the upper-lane mask on the SALU).
template <int S, int PH, int R, bool SOFT>
__device__ __forceinline__ void rot_step(int (&m)[R], int qp, const Coef<S, R, SOFT>& k, uint64_t (&bal)[R]) {
    constexpr int P = S - 1 - PH;
    int nm[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        int mu;
        if constexpr (SOFT) {
            mu = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, k.sig[r][PH]), __builtin_bit_cast(short2_t, qp),
                                        k.kap[r][PH], false);
        } else {
            mu = __builtin_amdgcn_sbfe(k.sig[r][PH], unsigned(qp), 8u);
        }
        int pm;
        if constexpr (P >= 6) {
            pm = m[r ^ (1 << (P - 6))];
        } else {
            pm = partner<P>(m[r]);
        }
        const int a = m[r] + mu, b = pm - mu;  // own candidate, partner's candidate
        int up;
        if constexpr (P >= 6) {
            up = ((r >> (P - 6)) & 1) ? -1 : 0;  // (the register is the location bit: a constant)
        } else {
            up = k.up[r][PH];
        }
        bal[r] = __ballot(((a - b) ^ up) > up);
        nm[r] = a < b ? a : b;
    }
#pragma unroll
    for (int r = 0; r < R; r++) m[r] = nm[r];
}

// One phase cycle (S steps) from the prepared received pairs q, the decision words kept by lanes
// i .. i + S - 1 of klo / khi (v_writelane).
template <int S, int R, bool SOFT>
__device__ __forceinline__ void acs_cycle(int (&m)[R], const int* q, const Coef<S, R, SOFT>& k, uint32_t (&klo)[R],
                                          uint32_t (&khi)[R], int i) {
    gen_static_for(std::make_integer_sequence<int, S>{}, [&](auto pc) {
        constexpr int PH = decltype(pc)::value;
        uint64_t bal[R];
        rot_step<S, PH, R, SOFT>(m, q[PH], k, bal);
#pragma unroll
        for (int r = 0; r < R; r++) {
            klo[r] = uint32_t(vtb_writelane(int(uint32_t(bal[r])), i + PH, int(klo[r])));
            khi[r] = uint32_t(vtb_writelane(int(uint32_t(bal[r] >> 32)), i + PH, int(khi[r])));
        }
    });
}

// Traceback helpers (locations).  Bit of step t's information bit: b = (S - (t+1) mod S) mod S;
// b of step t - 1 is b + 1 mod S.
template <int S>
__device__ __forceinline__ int info_bit_pos(int t) {
    const int k = (t + 1) % S;
    return k == 0 ? 0 : S - k;
}
template <int S>
__device__ __forceinline__ int next_pos(int b) {
    return b + 1 == S ? 0 : b + 1;
}
// The location after step t - 1 from the location after step t, step t's R words and b;
// `base` = the frame's first lane in the words.
template <int S, int R>
__device__ __forceinline__ unsigned tb_step(unsigned loc, const uint64_t (&w)[R], int b, unsigned base) {
    constexpr unsigned G = unsigned(Geometry<S>::G);
    const unsigned sh = base + lane_of<S>(loc & (G - 1u));
    unsigned x[R];
#pragma unroll
    for (int r = 0; r < R; r++) x[r] = unsigned(w[r] >> sh) & 1u;  // (bits first: no word select)
    unsigned d = x[0];
    if constexpr (R == 2) d = (loc & 64u) ? x[1] : x[0];
    if constexpr (R == 4) {
        const unsigned lo2 = (loc & 64u) ? x[1] : x[0], hi2 = (loc & 64u) ? x[3] : x[2];
        d = (loc & 128u) ? hi2 : lo2;
    }
    return (loc & ~(1u << b)) | (d << b);
}


// Traceback warm-up of a block walk (steps walked from a guessed state past the block's end):
// survivor paths merge within a few constraint lengths, and a walk that entered on the wrong
// state is caught by the chain verification and re-walked, so this only trades walk length
// against re-walk rounds.
template <int S>
constexpr int kTbWarm = 4 * S + 24;

// Terminated traceback from state 0 (reference viterbiDecoderButterflyk1.c:200-256) of one frame
// per chain of GC lanes, block-parallel and verified: chain ci = lane / GC,
// block bi = lane % GC of tbb steps (a multiple of 8: every block owns whole output bytes).  A
// block walks back to itself from kTbWarm steps past its end starting in location 0 there (exact
// when that is T, the terminated end), writing its bytes (MSB-first, reference :243-249) as it
// walks; it is right once it entered on its successor's exit location and that successor is
// proven, and failed blocks re-walk (rewriting their bytes) from a proven successor until all are.
// Chains of GC blocks need at most GC - 1 re-walk rounds.  Completeness guard: a chain with a
// block still unproven after the cap (VTB_DEBUG bit 17: every chain with a walked block) is
// walked again serially from location 0 at T by its block 0 (the reference's walk), whose bytes
// overwrite the others' later in program order.  row(t, w) loads step t's R survivor words;
// `base` is the frame's first bit in them; o the frame's output bytes (L bits); every lane of the
// wave calls this (the chain checks are wave-wide).
// traceback_span: the same over steps [t0, T) (t0 a multiple of 8) ending in location locT after
// step T - 1, the bytes of steps t at o[(t - t0) >> 3] (the streaming decoder's emitted range,
// vtb_stream_gen.hip); T = t0: nothing to walk.
template <int S, int R, class Row>
__device__ __forceinline__ void traceback_span(int t0, int T, int L, unsigned locT, int GC, unsigned base, uint8_t* o,
                                               bool tbforce, uint32_t* guard_hits, Row&& row) {
    constexpr int kWarm = kTbWarm<S>;
    // A step's R survivor words do not depend on the walk's location (only the bit taken from them
    // does), so the walks load kTb steps' words at once and then take the kTb dependent steps
    // (kTb loads in flight instead of one: L2 / HBM or LDS latency).
    constexpr int kTb = R == 1 ? 16 : R == 2 ? 8 : 4;
    const int lane = int(threadIdx.x & 63), ci = lane / GC, bi = lane % GC;
    // the location before steps [lo, hi) given the location after step hi - 1
    auto walk = [&](unsigned loc, int hi, int lo) -> unsigned {
        int t = hi, b = info_bit_pos<S>(hi - 1);
        for (; t - kTb >= lo; t -= kTb) {
            uint64_t w[kTb][R];
#pragma unroll
            for (int j = 0; j < kTb; j++) row(t - 1 - j, w[j]);
#pragma unroll
            for (int j = 0; j < kTb; j++) {
                loc = tb_step<S, R>(loc, w[j], b, base);
                b = next_pos<S>(b);
            }
        }
        for (; t > lo; t--) {
            uint64_t w[R];
            row(t - 1, w);
            loc = tb_step<S, R>(loc, w, b, base);
            b = next_pos<S>(b);
        }
        return loc;
    };
    // the same walk, writing the bytes of [lo, hi) (lo a multiple of 8): the steps above the last
    // whole octet one by one, then octets with their 8 rows loaded at once
    auto walk_emit = [&](unsigned loc, int hi, int lo) -> unsigned {
        unsigned byte = 0;
        auto put = [&](int t) {
            if (t < L) o[(t - t0) >> 3] = uint8_t(t + 8 > L ? byte & (0xffu << (t + 8 - L)) : byte);
        };
        int t = hi - 1, b = info_bit_pos<S>(hi - 1);
        for (; t >= lo && ((t + 1) & 7) != 0; t--) {
            byte = ((byte >> 1) | (((loc >> b) & 1u) << 7)) & 0xffu;
            if ((t & 7) == 0) put(t);
            uint64_t w[R];
            row(t, w);
            loc = tb_step<S, R>(loc, w, b, base);
            b = next_pos<S>(b);
        }
        for (; t >= lo; t -= 8) {  // t = 7 mod 8: steps t .. t - 7
            uint64_t w[8][R];
#pragma unroll
            for (int j = 0; j < 8; j++) row(t - j, w[j]);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                byte = ((byte >> 1) | (((loc >> b) & 1u) << 7)) & 0xffu;
                loc = tb_step<S, R>(loc, w[j], b, base);
                b = next_pos<S>(b);
            }
            put(t - 7);
        }
        return loc;
    };
    const int tbb = ((T - t0 + GC - 1) / GC + 7) / 8 * 8;
    const int lo = t0 + bi * tbb, top = lo + tbb < T ? lo + tbb : T;
    const bool active = lo < T;
    const int start = top + kWarm < T ? top + kWarm : T;
    unsigned st = active ? walk(start == T ? locT : 0u, start, top) : 0u;
    unsigned s_top = st;
    if (active) st = walk_emit(st, top, lo);
    unsigned fin = st;
    bool fixed = !active || start == T;
    const uint64_t cmask = (GC == 64 ? ~uint64_t(0) : ((uint64_t(1) << (GC & 63)) - 1)) << (ci * GC);
    const int rounds = tbforce ? 0 : GC + 1;
    const uint64_t live = __ballot(true);  // (lanes of frames past the batch have returned)
    uint64_t unproven = 0;
    for (int round = 0;; round++) {
        const unsigned sf = unsigned(__shfl_down(int(fin), 1));  // successor block's entry location
        const bool ok = fixed || (s_top == sf && !tbforce);
        const uint64_t bad = ~__ballot(ok) & live;
        if (bad == 0) break;
        if (round == rounds) {
            unproven = bad;
            break;
        }
        const uint64_t badc = (bad & cmask) >> (ci * GC);  // this chain's failed blocks
        if (!ok && (badc >> (bi + 1)) == 0) {
            s_top = sf;
            fin = walk_emit(sf, top, lo);
            fixed = true;
        }
    }
    if ((unproven & cmask) && bi == 0) {
        note_guard(guard_hits);
        walk_emit(locT, T, t0);
    }
}
template <int S, int R, class Row>
__device__ __forceinline__ void traceback_chains(int T, int L, int GC, unsigned base, uint8_t* o, bool force,
                                                 uint32_t* guard_hits, Row&& row) {
    traceback_span<S, R>(0, T, L, 0u, GC, base, o, force, guard_hits, row);
}

// rotate right within S bits (k in [0, S)): the location of state x after a step of phase k - 1
template <int S>
__device__ __forceinline__ unsigned rotr_s(unsigned x, int k) {
    return ((x >> k) | (x << (S - k))) & ((1u << S) - 1u);
}

}  // namespace gen
}  // namespace vtb
