// Register-resident fast path, K=7 (64 states).
//
// Layout.  One wave64 decodes two frames, A and B.  Lane l holds the path metric of the
// trellis state living at "location" l for both frames as one packed i16 pair
// [m_A, m_B] (v_pk_* arithmetic does both frames per instruction).
//
// In-place state relabelling (no data movement between steps).  Instead of moving state
// s to lane s every step (the reference's destination-indexed butterfly,
// viterbiDecoderButterflyk1.c:101-152), each butterfly writes its two destinations back
// into the two locations its sources came from.  Then location l holds state
// rotl6(l, t mod 6) at step t, and the two sources of a butterfly (states j and j+32)
// always sit in lanes that differ in exactly one bit, p = 5 - (t mod 6).  So every step
// is: fetch the partner lane's metric with ONE cross-lane op (DPP quad_perm for XOR 1/2,
// half_mirror+quad_perm for XOR 4, row_ror:8 for XOR 8, v_permlane16/32_swap for XOR
// 16/32), then add-compare-select in registers.
//
// Metrics are centred (candidate = m +/- mu, mu = e - Q, Q = 1 hard / 255 soft; see
// vtb_lds_path.hip) so both frames share the lane's per-phase code coefficients, and a
// renormalisation every 16 steps (subtract location 0's metric) keeps them in i16.  Ties
// keep the lower predecessor exactly as the reference's strict '>' (:129-130).
//
// Decisions.  Two SDWA compares per step give, for each frame, the 64-bit word
// D_t[l] = "survivor of the state at location l came from the upper predecessor".  The
// words are collected with v_writelane into a 48-step register ring and flushed to LDS.
//
// Traceback (reference :200-256) runs in location space: going back from step t+1 to t
// emits bit p_t of the current location (= the LSB of the state, the decoded bit) and
// replaces that bit with D_t[location].  It is made parallel and still exact: each lane
// owns a block of TBB steps and walks back from a point kWarm steps past the block's end
// carrying the SET of locations the survivor could be in (a 64-bit mask; the image of a
// set under one step is a few shifts and bit-selects).  If the set has collapsed to one
// location by the time the walk enters the block, the block's bits are exactly the
// reference's.  A block whose set did not collapse is re-walked from the location its
// successor block proved for that boundary (the last block starts from the known state
// 0 at t = T), so the result is exact for every input; only the time depends on how fast
// survivor paths merge.

#include "vtb_internal.h"

namespace vtb {
namespace {

constexpr int kChunk = 48;  // ACS steps per unrolled body = lcm(6 phases, 16-step renorm)
#ifndef VTB_WARM
#define VTB_WARM 48
#endif
constexpr int kWarm = VTB_WARM;  // traceback warm-up steps past a block's end (multiple of 6)

typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s16x2 as_s2(uint32_t x) { return __builtin_bit_cast(s16x2, x); }
__device__ __forceinline__ uint32_t as_u(s16x2 x) { return __builtin_bit_cast(uint32_t, x); }

__device__ __forceinline__ int rotl6(int x, int r) { return ((x << r) | (x >> (6 - r))) & 63; }

// Decision word index of (step t, frame f): 16 B per step, plus one spare 16-B slot per
// 48 steps so that traceback lanes reading the same offset of different blocks do not
// all hit one LDS bank.
__device__ __forceinline__ size_t dec_index(int t, int f) { return 2 * (size_t)(t + t / kChunk) + f; }

// Partner metric across lane bit p (XOR 1 << p).
template <int P>
__device__ __forceinline__ uint32_t exchange(uint32_t m, int lane) {
    if constexpr (P == 0) {
        return __builtin_amdgcn_mov_dpp(m, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    } else if constexpr (P == 1) {
        return __builtin_amdgcn_mov_dpp(m, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    } else if constexpr (P == 2) {
        uint32_t h = __builtin_amdgcn_mov_dpp(m, 0x141, 0xF, 0xF, false);  // row_half_mirror: i <- 7-i
        return __builtin_amdgcn_mov_dpp(h, 0x1B, 0xF, 0xF, false);         // quad_perm [3,2,1,0]: i <- i^3
    } else if constexpr (P == 3) {
        return __builtin_amdgcn_mov_dpp(m, 0x128, 0xF, 0xF, false);  // row_ror:8
    } else if constexpr (P == 4) {
        auto r = __builtin_amdgcn_permlane16_swap(m, m, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else {
        auto r = __builtin_amdgcn_permlane32_swap(m, m, false, false);
        return (lane & 32) ? r[0] : r[1];
    }
}

// Decisions for the two packed frames: lane bit = (nw.half < x.half), signed 16-bit.
__device__ __forceinline__ void decide(uint32_t nw, uint32_t x, uint64_t& da, uint64_t& db) {
    asm("v_cmp_lt_i16_sdwa %0, %1, %2 src0_sel:WORD_0 src1_sel:WORD_0" : "=s"(da) : "v"(nw), "v"(x));
    asm("v_cmp_lt_i16_sdwa %0, %1, %2 src0_sel:WORD_1 src1_sel:WORD_1" : "=s"(db) : "v"(nw), "v"(x));
}

template <int LANE>
__device__ __forceinline__ void ring_put(uint32_t& ring, uint32_t v) {
    asm("v_writelane_b32 %0, %1, %2" : "+v"(ring) : "s"(v), "i"(LANE));
}

// Measurement-only variants (built into separate libraries by tools/build_variants.sh,
// never the shipped library): drop the decision store, the compares, or the exchange.
#if defined(VTB_EXP_NO_STORE) || defined(VTB_EXP_NO_DECIDE)
#define VTB_EXP_STORE(I, da, db) (void)(da), (void)(db)
#else
#define VTB_EXP_STORE(I, da, db)                  \
    ring_put<I>(r_alo, uint32_t(da));             \
    ring_put<I>(r_ahi, uint32_t((da) >> 32));     \
    ring_put<I>(r_blo, uint32_t(db));             \
    ring_put<I>(r_bhi, uint32_t((db) >> 32))
#endif
#ifdef VTB_EXP_NO_DECIDE
#define VTB_EXP_DECIDE(nw, x, da, db) (da = (nw), db = (x))
#else
#define VTB_EXP_DECIDE(nw, x, da, db) decide(nw, x, da, db)
#endif
#ifdef VTB_EXP_NO_EXCHANGE
#define VTB_EXP_EXCHANGE(PH) (M ^ 0x10001u)
#else
#define VTB_EXP_EXCHANGE(PH) exchange<5 - PH>(M, lane)
#endif

struct PhaseCoef {
    uint32_t s0, s1, k;  // packed [x, x] multipliers of q0, q1 and the constant
};

// One backward traceback step on a location set S (bit l = "survivor may be at l"),
// pairing bit P: locations with D_t = 0 get bit P cleared, D_t = 1 get it set.
template <int P>
__device__ __forceinline__ void set_step(uint32_t& lo, uint32_t& hi, uint64_t w) {
    const uint32_t wlo = uint32_t(w), whi = uint32_t(w >> 32);
    const uint32_t z0 = lo & ~wlo, z1 = hi & ~whi;  // d = 0
    const uint32_t o0 = lo & wlo, o1 = hi & whi;    // d = 1
    if constexpr (P == 5) {
        lo = z0 | z1;
        hi = o0 | o1;
    } else {
        constexpr uint32_t MP = P == 0 ? 0xAAAAAAAAu : P == 1 ? 0xCCCCCCCCu : P == 2 ? 0xF0F0F0F0u
                                : P == 3 ? 0xFF00FF00u : 0xFFFF0000u;
        constexpr int SH = 1 << P;
        lo = ((o0 & MP) | (z0 & ~MP)) | (((o0 << SH) & MP) | ((z0 >> SH) & ~MP));
        hi = ((o1 & MP) | (z1 & ~MP)) | (((o1 << SH) & MP) | ((z1 >> SH) & ~MP));
    }
}

template <int P>
__device__ __forceinline__ uint32_t set_bit_p(uint32_t lo, uint32_t hi) {
    if constexpr (P == 5) {
        return hi != 0;
    } else {
        constexpr uint32_t MP = P == 0 ? 0xAAAAAAAAu : P == 1 ? 0xCCCCCCCCu : P == 2 ? 0xF0F0F0F0u
                                : P == 3 ? 0xFF00FF00u : 0xFFFF0000u;
        return ((lo | hi) & MP) != 0;
    }
}

// Emits decoded bits of one traceback lane, most recent step first, and writes them in
// 48-bit pieces aligned to 48-step boundaries measured from the block start.
struct BitSink {
    uint64_t acc = 0;
    __device__ __forceinline__ void put(uint32_t bit) { acc = (acc << 1) | bit; }
    // flush the bits for steps [t, t_top) (t_top - t <= 48, t a multiple of 8)
    __device__ __forceinline__ void flush(uint8_t* o, int t, int t_top) {
        // bit for step t' sits at position t'-t; bytes are MSB-first
        uint64_t w = __builtin_bswap64(__builtin_bitreverse64(acc));
        int nbytes = (t_top - t + 7) >> 3;
        for (int k = 0; k < nbytes; k++) o[(t >> 3) + k] = uint8_t(w >> (8 * k));
        acc = 0;
    }
};

template <bool SOFT>
__global__ __launch_bounds__(64) void reg_k7_kernel(const uint8_t* __restrict__ in, size_t in_stride,
                                                     uint8_t* __restrict__ out, size_t out_stride, int T, int L,
                                                     int Tpad, int tbb, size_t frames, int dbg, Launch table) {
    constexpr int Q = SOFT ? 255 : 1;
    constexpr int INIT = 65 * Q;  // (uint8_t)(NUM_STATES+1) for N=64, reference :62
    extern __shared__ uint64_t smem[];
    uint64_t* dec = smem;                                           // decision words, dec_index()
    uint64_t* qbuf = smem + 2 * (size_t)(Tpad + Tpad / kChunk);     // [2][kChunk] packed (Q0, Q1)
    const int lane = threadIdx.x;
    const size_t fa = (size_t)blockIdx.x * 2, fb = fa + 1;
    const bool has_b = fb < frames;

    // Per-lane, per-phase code coefficients.  At phase ph the pairing bit is p = 5 - ph;
    // the butterfly's upper-half state is j = rotl6(lane with bit p cleared, ph).
    PhaseCoef coef[6];
#pragma unroll
    for (int ph = 0; ph < 6; ph++) {
        int p = 5 - ph;
        int j = rotl6(lane & ~(1 << p), ph);
        int c = table.symm[j];
        int s0 = (c & 1) ? -1 : 1, s1 = (c & 2) ? -1 : 1;
        int kk = ((c & 1) + ((c >> 1) & 1) - 1) * Q;
        coef[ph].s0 = (uint32_t)(s0 & 0xffff) * 0x10001u;
        coef[ph].s1 = (uint32_t)(s1 & 0xffff) * 0x10001u;
        coef[ph].k = (uint32_t)(kk & 0xffff) * 0x10001u;
    }

    auto load_chunk = [&](int t0, uint32_t& qa, uint32_t& qb) {
        // lane i < kChunk fetches step t0+i of both frames as (q0 | q1 << 16)
        int t = t0 + lane;
        qa = qb = 0;
        if (lane < kChunk && t < T) {
            if (SOFT) {
                const uint8_t* pa = in + fa * in_stride + 2 * (size_t)t;
                qa = uint32_t(pa[0]) | (uint32_t(pa[1]) << 16);
                if (has_b) {
                    const uint8_t* pb = in + fb * in_stride + 2 * (size_t)t;
                    qb = uint32_t(pb[0]) | (uint32_t(pb[1]) << 16);
                }
            } else {
                uint32_t ca = in[fa * in_stride + t];
                qa = (ca & 1u) | (((ca >> 1) & 1u) << 16);
                if (has_b) {
                    uint32_t cb = in[fb * in_stride + t];
                    qb = (cb & 1u) | (((cb >> 1) & 1u) << 16);
                }
            }
        }
    };
    auto stage_chunk = [&](int buf, uint32_t qa, uint32_t qb) {
        if (lane < kChunk) {
            // (Q0, Q1) = ([q0_A, q0_B], [q1_A, q1_B])
            uint32_t q0 = (qa & 0xffffu) | (qb << 16);
            uint32_t q1 = (qa >> 16) | (qb & 0xffff0000u);
            qbuf[buf * kChunk + lane] = uint64_t(q0) | (uint64_t(q1) << 32);
        }
    };

    uint32_t M = (lane == 0) ? 0u : (uint32_t)INIT * 0x10001u;
    {
        uint32_t qa, qb;
        load_chunk(0, qa, qb);
        stage_chunk(0, qa, qb);
    }
    __syncthreads();

    uint32_t r_alo = 0, r_ahi = 0, r_blo = 0, r_bhi = 0;
    for (int t0 = 0; t0 < ((dbg & 2) ? 0 : Tpad); t0 += kChunk) {
        const int buf = (t0 / kChunk) & 1;
        uint32_t nqa, nqb;
        load_chunk(t0 + kChunk, nqa, nqb);  // prefetch next chunk (consumed after this body)
        const uint64_t* qc = qbuf + buf * kChunk;
        uint64_t qg[6], qn[6];
#pragma unroll
        for (int k = 0; k < 6; k++) qg[k] = qc[k];

#define VTB_STEP(I, PH)                                                                           \
    {                                                                                             \
        if (PH == 0 && I + 6 < kChunk) {                                                          \
            _Pragma("unroll") for (int k = 0; k < 6; k++) qn[k] = qc[I + 6 + k];                  \
        }                                                                                         \
        uint64_t qq = qg[PH];                                                                     \
        s16x2 q0 = as_s2(uint32_t(qq)), q1 = as_s2(uint32_t(qq >> 32));                           \
        s16x2 mu = as_s2(coef[PH].s0) * q0 + (as_s2(coef[PH].s1) * q1 + as_s2(coef[PH].k));      \
        uint32_t P = VTB_EXP_EXCHANGE(PH);                                                        \
        s16x2 A = as_s2(M) + mu, B = as_s2(P) - mu;                                               \
        s16x2 nw = __builtin_elementwise_min(A, B);                                               \
        uint32_t X = ((lane >> (5 - PH)) & 1) ? as_u(B) : as_u(A);                                \
        uint64_t da, db;                                                                          \
        VTB_EXP_DECIDE(as_u(nw), X, da, db);                                                      \
        VTB_EXP_STORE(I, da, db);                                                                 \
        M = as_u(nw);                                                                             \
        if (PH == 5) {                                                                            \
            _Pragma("unroll") for (int k = 0; k < 6; k++) qg[k] = qn[k];                          \
        }                                                                                         \
        if ((I & 15) == 15) {                                                                     \
            uint32_t ref = __builtin_amdgcn_readlane(M, 0);                                       \
            M = as_u(as_s2(M) - as_s2(ref));                                                      \
        }                                                                                         \
    }
#define VTB_GROUP(G) VTB_STEP(6 * G + 0, 0) VTB_STEP(6 * G + 1, 1) VTB_STEP(6 * G + 2, 2) \
                     VTB_STEP(6 * G + 3, 3) VTB_STEP(6 * G + 4, 4) VTB_STEP(6 * G + 5, 5)
        VTB_GROUP(0) VTB_GROUP(1) VTB_GROUP(2) VTB_GROUP(3) VTB_GROUP(4) VTB_GROUP(5) VTB_GROUP(6) VTB_GROUP(7)
#undef VTB_GROUP
#undef VTB_STEP

        if (lane < kChunk) {
            uint64_t* d = dec + dec_index(t0 + lane, 0);
            d[0] = uint64_t(r_alo) | (uint64_t(r_ahi) << 32);
            d[1] = uint64_t(r_blo) | (uint64_t(r_bhi) << 32);
        }
        stage_chunk(buf ^ 1, nqa, nqb);
        __syncthreads();
    }
    if (dbg & 1) return;

    // ---------------- block-parallel exact traceback ----------------
    // lanes 0-31: frame A, lanes 32-63: frame B; lane (f, b) owns steps [b*tbb, (b+1)*tbb).
    const int f = lane >> 5, blk = lane & 31;
    const size_t frame = fa + f;
    const int nb = (T + tbb - 1) / tbb;
    const bool active = frame < frames && blk < nb;
    const int s0 = blk * tbb;
    const int s1 = min(s0 + tbb, T);
    const int e_top = min(s1, L);  // first (highest) step whose bit is emitted, exclusive
    int E = min(s1 + kWarm, T);
    bool known = (E == T);
    // Lanes starting at T (known location 0) idle `delta` iterations so that every live
    // lane sits on the same phase (t = E-1-(k-delta) == 5-k (mod 6)); tbb, kWarm are
    // multiples of 6.
    int delta = known ? (6 - T % 6) % 6 : 0;
    uint32_t slo = known ? 1u : 0xFFFFFFFFu, shi = known ? 0u : 0xFFFFFFFFu;
    bool ok = true;
    BitSink sink;
    uint8_t* o = out + frame * out_stride;

    const int nit = tbb + kWarm + 6;
    for (int k0 = 0; k0 < nit; k0 += 6) {
        uint64_t w6[6];
#pragma unroll
        for (int ph = 0; ph < 6; ph++) {
            int t = E - 1 - (k0 + ph - delta);
            w6[ph] = dec[dec_index(t < 0 ? 0 : (t >= T ? T - 1 : t), f)];
        }
#define VTB_TB(PH)                                                                        \
        {                                                                                 \
            const int t = E - 1 - (k0 + PH - delta);                                      \
            if (active && k0 + PH >= delta && t >= s0) {                                  \
                if (t == s1 - 1) ok = (__builtin_popcount(slo) + __builtin_popcount(shi)) == 1; \
                if (t < e_top) {                                                          \
                    sink.put(set_bit_p<PH>(slo, shi));                                    \
                    if (((t - s0) % 48) == 0) sink.flush(o, t, min(t + 48, e_top));       \
                }                                                                         \
                set_step<PH>(slo, shi, w6[PH]);                                           \
            }                                                                             \
        }
        VTB_TB(0) VTB_TB(1) VTB_TB(2) VTB_TB(3) VTB_TB(4) VTB_TB(5)
#undef VTB_TB
    }

    // Blocks whose set did not collapse: re-walk from the successor's proven entry.
    int entry = (slo != 0) ? __builtin_ctz(slo) : 32 + __builtin_ctz(shi);
    for (int round = 0; round < 32; round++) {
        const bool bad = active && !ok;
        if (!__any(bad)) break;
        const int succ_entry = __shfl_down(entry, 1);
        const int succ_ok = __shfl_down(ok ? 1 : 0, 1);
        const bool redo = bad && succ_ok;  // a failing block is never the last one
        uint32_t rlo = 0, rhi = 0;
        if (redo) {
            rlo = succ_entry < 32 ? (1u << succ_entry) : 0u;
            rhi = succ_entry < 32 ? 0u : (1u << (succ_entry - 32));
            sink.acc = 0;
        }
        for (int k0 = 0; k0 < tbb; k0 += 6) {
#define VTB_RE(PH)                                                                        \
            {                                                                             \
                const int t = s1 - 1 - (k0 + PH);                                         \
                if (redo) {                                                               \
                    uint64_t w = dec[dec_index(t, f)];                                    \
                    if (t < e_top) {                                                      \
                        sink.put(set_bit_p<PH>(rlo, rhi));                                \
                        if (((t - s0) % 48) == 0) sink.flush(o, t, min(t + 48, e_top));   \
                    }                                                                     \
                    set_step<PH>(rlo, rhi, w);                                            \
                }                                                                         \
            }
            VTB_RE(0) VTB_RE(1) VTB_RE(2) VTB_RE(3) VTB_RE(4) VTB_RE(5)
#undef VTB_RE
        }
        if (redo) {
            ok = true;
            entry = (rlo != 0) ? __builtin_ctz(rlo) : 32 + __builtin_ctz(rhi);
        }
    }
}

int tb_block(int T) {
    // multiple of 24 (6 phases x byte alignment), at most 32 blocks per frame
    int per = (T + 31) / 32;
    return (per + 23) / 24 * 24;
}

size_t lds_bytes(int T) {
    int Tpad = (T + kChunk - 1) / kChunk * kChunk;
    return 16 * (size_t)(Tpad + Tpad / kChunk) + 2 * kChunk * 8;
}

}  // namespace

bool reg_path_supported(const Launch& a) {
    return a.S == 6 && a.T > a.S && lds_bytes(a.T) <= 160 * 1024;
}

hipError_t launch_reg_path(const Launch& a) {
    if (a.frames == 0) return hipSuccess;
    const int Tpad = (a.T + kChunk - 1) / kChunk * kChunk;
    const size_t lds = lds_bytes(a.T);
    const size_t blocks = (a.frames + 1) / 2;
    auto kern = a.soft ? reg_k7_kernel<true> : reg_k7_kernel<false>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(unsigned(blocks)), dim3(64), lds, a.stream, a.in, a.in_stride, a.out, a.out_stride,
                       a.T, a.L, Tpad, tb_block(a.T), a.frames, debug_flags(), a);
    return hipGetLastError();
}

}  // namespace vtb
