// Register-resident fast path, K=7 (64 states), hard and 8-bit soft input.
//
// Layout.  One wave64 decodes two frames, A and B.  Lane l holds the path metric of the
// trellis state living at "location" l for both frames as one packed u16 pair
// [m_A, m_B]: every packed instruction advances both frames.
//
// In-place state relabelling (no data movement between steps).  Instead of moving state
// s to lane s every step (the reference's destination-indexed butterfly,
// viterbiDecoderButterflyk1.c:101-152), each butterfly writes its two destinations back
// into the two locations its sources came from.  Then location l holds state
// rotl6(l, t mod 6) at step t, and the two sources of a butterfly (states j and j+32)
// always sit in lanes that differ in exactly one bit, p = 5 - (t mod 6).  A step fetches
// the partner lane's metric with one cross-lane op (DPP quad_perm for XOR 1/2,
// half_mirror+quad_perm for XOR 4, row_ror:8 for XOR 8, in-place v_permlane16/32_swap
// for XOR 16/32) and add-compare-selects in registers.
//
// Branch metrics come from a per-step table in LDS.  For each step the staging code
// (once per 48 steps, all lanes in parallel) computes e(c) for the four trellis labels c
// of both frames and stores eight (V, W) pairs: V = 2e(c) + R, W = 2e(~c), for c = 0..3
// and R = 0/1.  Lane l reads its pair with one ds_read_b64 at a per-phase offset (its
// label c and R = bit p of l), so the ACS itself is
//     A = M + V;  B = partner(M) + W;  M' = min(A, B) & ~1;  C = [A > B]
// with one full-rate add, one DPP add (or swap + add), one packed min, one full-rate and
// and two SDWA compares.  Metrics are kept doubled so that the +R bit in the own-path
// candidate A turns "strictly greater" into "greater or equal" for lanes whose own state
// is the upper predecessor j+32: the compare always reads [A > B] while the decision
// D = C xor R is exactly the reference's strict '>' toward the lower predecessor j
// (viterbiDecoderButterflyk1.c:129-130); the and clears the bit again.  D itself is never
// formed: the traceback works directly with C (see below).
//
// Metrics are unsigned u16 with a bias; every 16 steps the wave subtracts location 0's
// metric and adds the bias back (the spread of exact metrics is bounded,
// so this is the reference's renormalisation in another form).
//
// Decisions.  The two compares leave C for each frame as a 64-bit SGPR pair; two scalar
// stores (s_store_dwordx2 through the scalar cache, no VALU) write them to a global
// workspace, 8 bytes per frame per step.
//
// Traceback (reference :200-256) runs in location space: going back from step t+1 to t
// emits bit p_t of the current location (= the decoded bit) and replaces that bit with
// D_t[location].  Within a group of six steps p runs 0..5, so the six decoded bits of a
// sextet are exactly the location at its start, read MSB first.  It is parallel and
// still exact: lanes 0-31 own blocks of frame A, lanes 32-63 of frame B; each walks back
// from kWarm steps past its block carrying the SET of locations the survivor could be in
// (64-bit mask; with C, one step is  move = S & C;  S' = (S & ~C) | flip_p(move)).  If the
// set is a single location when the walk enters the block, the block's bits are exact.
// Blocks that did not collapse are re-walked from the location their successor proved
// (steps past T carry D = 0, so every walk that starts beyond T collapses to the known
// state 0 at T), so the result is exact for every input; only the time depends on how
// fast survivor paths merge.

#include "vtb_k7_common.h"

namespace vtb {
namespace {

using namespace k7;

constexpr int kWarm = 48;  // traceback warm-up steps past a block's end (multiple of 12)
constexpr size_t kMaxWsBytes = size_t(1) << 30;  // workspace per launch slab

// ---------------------------------------------------------------- traceback helpers

// Move the bits of m across location bit P (l <-> l ^ (1 << P)), P < 5, within 32 bits.
template <int P>
__device__ __forceinline__ uint32_t flip32(uint32_t m) {
    if constexpr (P == 3) {
        return __builtin_amdgcn_perm(m, m, 0x02030001u);  // swap the bytes of each 16-bit half
    } else if constexpr (P == 4) {
        return __builtin_amdgcn_alignbit(m, m, 16);
    } else {
        constexpr uint32_t MP = uint32_t(loc_mask(P));
        constexpr int SH = 1 << P;
        return ((m & MP) >> SH) | ((m << SH) & MP);
    }
}

// One backward step of a location set S = (lo, hi) with the step's compare word C.
template <int P>
__device__ __forceinline__ void set_step(uint32_t& lo, uint32_t& hi, uint32_t clo, uint32_t chi) {
    const uint32_t mlo = lo & clo, mhi = hi & chi;
    if constexpr (P == 5) {
        lo = (lo & ~clo) | mhi;
        hi = (hi & ~chi) | mlo;
    } else {
        lo = (lo & ~clo) | flip32<P>(mlo);
        hi = (hi & ~chi) | flip32<P>(mhi);
    }
}

// Index of the lowest location in the set (the location, when the set is a singleton).
__device__ __forceinline__ uint32_t set_first(uint32_t lo, uint32_t hi) {
    return lo ? uint32_t(__builtin_ctz(lo)) : 32u + uint32_t(__builtin_ctz(hi | 0x80000000u));
}

__device__ __forceinline__ bool set_single(uint32_t lo, uint32_t hi) {
    return __builtin_popcount(lo) + __builtin_popcount(hi) == 1;
}

// OR nbits (<= 48, in the low bits of acc, MSB = earliest step) into the big-endian bit
// string ob at bit offset tg.
__device__ __forceinline__ void flush_bits(uint32_t* ob, int tg, uint64_t acc, int nbits) {
    const uint64_t U = acc << (64 - nbits);
    const int w = tg >> 5, sh = tg & 31;
    const uint32_t w0 = uint32_t(U >> (32 + sh));
    const uint32_t w1 = uint32_t(U >> sh);
    const uint32_t w2 = sh ? uint32_t(U << (32 - sh)) : 0u;
    atomicOr(ob + w, __builtin_bswap32(w0));
    atomicOr(ob + w + 1, __builtin_bswap32(w1));
    if (w2) atomicOr(ob + w + 2, __builtin_bswap32(w2));
}

struct Words12 {
    uint4 v[6];
};

__device__ __forceinline__ void load12(Words12& d, const uint64_t* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int k = 0; k < 6; k++) d.v[k] = q[k];
}

// compare word of step (t_lo + k), k in [0, 12)
__device__ __forceinline__ uint32_t wlo(const Words12& d, int k) {
    const uint4& u = d.v[k >> 1];
    return (k & 1) ? u.z : u.x;
}
__device__ __forceinline__ uint32_t whi(const Words12& d, int k) {
    const uint4& u = d.v[k >> 1];
    return (k & 1) ? u.w : u.y;
}

// Walk back from step `top` through nwarm + nout batches of 12 steps (all lanes in
// lockstep; top is a multiple of 12, so step j of every sextet has pairing bit j).  The
// first nwarm batches only move the set; `ok` records whether it is a singleton when the
// output part starts; the output part emits the decoded bits into ob when ok.
__device__ __forceinline__ void tb_walk(const uint64_t* D, int top, int nwarm, int nout, uint32_t& lo, uint32_t& hi,
                                        bool& ok, uint32_t* ob) {
    const int nb = nwarm + nout;
    Words12 cur, nxt;
    load12(cur, D + max(top - 12, 0));
    uint64_t acc = 0;
    int nsx = 0;                   // sextets in acc
    int gtop = top - 12 * nwarm;   // step just above the bits in acc
    for (int i = 0; i < nb; i++) {
        load12(nxt, D + max(top - 12 * (i + 2), 0));
        const bool emit = i >= nwarm;  // wave-uniform
        if (i == nwarm) ok = set_single(lo, hi);
#pragma unroll
        for (int h = 0; h < 2; h++) {
            if (emit) {
                acc |= uint64_t(set_first(lo, hi)) << (6 * nsx);
                nsx++;
            }
            const int k0 = 11 - 6 * h;  // word index of the sextet's first (latest) step
            set_step<0>(lo, hi, wlo(cur, k0 - 0), whi(cur, k0 - 0));
            set_step<1>(lo, hi, wlo(cur, k0 - 1), whi(cur, k0 - 1));
            set_step<2>(lo, hi, wlo(cur, k0 - 2), whi(cur, k0 - 2));
            set_step<3>(lo, hi, wlo(cur, k0 - 3), whi(cur, k0 - 3));
            set_step<4>(lo, hi, wlo(cur, k0 - 4), whi(cur, k0 - 4));
            set_step<5>(lo, hi, wlo(cur, k0 - 5), whi(cur, k0 - 5));
        }
        if (emit && (nsx == 8 || i == nb - 1)) {
            if (ok) flush_bits(ob, gtop - 6 * nsx, acc, 6 * nsx);
            gtop -= 6 * nsx;
            acc = 0;
            nsx = 0;
        }
        cur = nxt;
    }
}

// Measurement-only variants (tools/build_variants.sh builds them into separate libraries,
// never the shipped one; their outputs are wrong): drop the compares, the table reads or
// the decision stores of the ACS loop.
#ifdef VTB_EXP_NO_CMP
#define VTB_EXP_CMP(PH, A, B) ca[PH] = pA + (PH); cb[PH] = pB;
#else
#define VTB_EXP_CMP(PH, A, B)                                                                             \
    asm("v_cmp_gt_u16_sdwa %0, %1, %2 src0_sel:WORD_0 src1_sel:WORD_0" : "=s"(ca[PH]) : "v"(A), "v"(B)); \
    asm("v_cmp_gt_u16_sdwa %0, %1, %2 src0_sel:WORD_1 src1_sel:WORD_1" : "=s"(cb[PH]) : "v"(A), "v"(B));
#endif
#ifdef VTB_EXP_NO_LDS
#define VTB_EXP_LDS(x) cur[k]
#else
#define VTB_EXP_LDS(x) (x)
#endif

// ---------------------------------------------------------------- the kernel

template <bool SOFT>
__global__ __launch_bounds__(64) void reg_k7_kernel(const uint8_t* __restrict__ in, size_t in_stride,
                                                     uint8_t* __restrict__ out, size_t out_stride,
                                                     uint64_t* __restrict__ ws, int T, int L, int Tpad, int Tdec,
                                                     int tbb, size_t frames, int dbg, Launch table) {
    constexpr uint32_t Q = SOFT ? 255 : 1;
    constexpr uint32_t INIT2 = 2 * 65 * Q;  // doubled (uint8_t)(NUM_STATES+1) for N=64, reference :62
    extern __shared__ uint4 smem4[];
    uint8_t* smem = reinterpret_cast<uint8_t*>(smem4);
    uint8_t* tab = smem;                                                 // [2][kChunk][64 B]
    uint32_t* obuf = reinterpret_cast<uint32_t*>(smem + 2 * kChunk * kTabBytes);  // [2][tbb + 4] words
    const int obw = tbb + 4;
    const int lane = threadIdx.x;
    const size_t fa = (size_t)blockIdx.x * 2, fb = fa + 1;
    const bool has_b = fb < frames;
    uint64_t* wsA = ws + (size_t)blockIdx.x * 2 * Tdec;
    uint64_t* wsB = wsA + Tdec;

    for (int i = lane; i < 2 * obw; i += 64) obuf[i] = 0;

    // Per-lane, per-phase table offsets.  At phase ph the pairing bit is p = 5 - ph; the
    // butterfly's upper-half state is j = rotl6(lane with bit p cleared, ph); lane's own
    // edge has label c = symm[j] (the partner's has ~c), R = bit p of the lane.
    uint32_t off[6];
#pragma unroll
    for (int ph = 0; ph < 6; ph++) {
        const int p = 5 - ph;
        const int j = rotl6(lane & ~(1 << p), ph);
        const int c = table.symm[j];
        const int R = (lane >> p) & 1;
        off[ph] = uint32_t(8 * (c + 4 * R));
    }

    auto load_chunk = [&](int t0, uint32_t& qa, uint32_t& qb) {
        // lane i < kChunk fetches step t0+i of both frames as (q0 | q1 << 16)
        const int t = t0 + lane;
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
                const uint32_t ca = in[fa * in_stride + t];
                qa = (ca & 1u) | (((ca >> 1) & 1u) << 16);
                if (has_b) {
                    const uint32_t cb = in[fb * in_stride + t];
                    qb = (cb & 1u) | (((cb >> 1) & 1u) << 16);
                }
            }
        }
    };
    auto stage_chunk = [&](int buf, uint32_t qa, uint32_t qb) {
        if (lane < kChunk) {
            const uint32_t q0 = (qa & 0xffffu) | (qb << 16);        // [q0_A, q0_B]
            const uint32_t q1 = (qa >> 16) | (qb & 0xffff0000u);    // [q1_A, q1_B]
            const uint32_t n0 = Q * 0x10001u - q0, n1 = Q * 0x10001u - q1;
            // doubled branch metrics of labels 0..3 (bit 0 of the label <-> coded bit 0)
            const uint32_t e0 = 2 * (q0 + q1), e1 = 2 * (n0 + q1), e2 = 2 * (q0 + n1), e3 = 2 * (n0 + n1);
            constexpr uint32_t R1 = 0x10001u;
            uint4* row = reinterpret_cast<uint4*>(tab + (buf * kChunk + lane) * kTabBytes);
            row[0] = make_uint4(e0, e3, e1, e2);                  // (c=0,R=0) (c=1,R=0)
            row[1] = make_uint4(e2, e1, e3, e0);                  // (c=2,R=0) (c=3,R=0)
            row[2] = make_uint4(e0 + R1, e3, e1 + R1, e2);        // (c=0,R=1) (c=1,R=1)
            row[3] = make_uint4(e2 + R1, e1, e3 + R1, e0);        // (c=2,R=1) (c=3,R=1)
        }
    };

    uint32_t M = (lane == 0) ? kBias * 0x10001u : (kBias + INIT2) * 0x10001u;
    {
        uint32_t qa, qb;
        load_chunk(0, qa, qb);
        stage_chunk(0, qa, qb);
    }
    // Software pipeline: the table pairs of the next group of six steps are read while the
    // current group computes, and the group's compare words are stored (scalar stores)
    // only after the compiler's wait for those reads.  LDS reads and scalar stores share
    // lgkmcnt and scalar stores complete out of order, so every LDS wait also waits for
    // all earlier stores: this way that wait covers stores issued a whole group earlier.
    uint2 cur[6];
#pragma unroll
    for (int k = 0; k < 6; k++) cur[k] = *reinterpret_cast<const uint2*>(tab + k * kTabBytes + off[k]);

    const int tacs = (dbg & 2) ? 0 : Tpad;
    for (int t0 = 0; t0 < tacs; t0 += kChunk) {
        const int buf = (t0 / kChunk) & 1;
        uint32_t nqa, nqb;
        load_chunk(t0 + kChunk, nqa, nqb);  // prefetch next chunk (staged in group 3)
        const uint2* ap[6];
        const uint2* an[6];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            ap[k] = reinterpret_cast<const uint2*>(tab + buf * kChunk * kTabBytes + off[k]);
            an[k] = reinterpret_cast<const uint2*>(tab + (buf ^ 1) * kChunk * kTabBytes + off[k]);
        }
        const uint64_t pA = uniform64(reinterpret_cast<uint64_t>(wsA + t0));
        const uint64_t pB = uniform64(reinterpret_cast<uint64_t>(wsB + t0));

#define VTB_STEP(I, PH)                                                                              \
    {                                                                                                \
        const uint32_t A = M + cur[PH].x;                                                            \
        const uint32_t B = partner_plus<5 - (PH)>(M, cur[PH].y);                                     \
        const uint32_t nw = pk_min(A, B);                                                            \
        VTB_EXP_CMP(PH, A, B)                                                                        \
        M = nw & 0xFFFEFFFEu;                                                                        \
        if (((I) & 15) == 15) {                                                                      \
            const uint32_t ref = __builtin_amdgcn_readlane(M, 0);                                    \
            const uint32_t d = ((kBias - (ref & 0xffffu)) & 0xffffu) | ((kBias - (ref >> 16)) << 16); \
            M = pk_add(M, d);                                                                        \
        }                                                                                            \
    }
#ifdef VTB_EXP_NO_STORE
#define VTB_STORE(I, PH) asm volatile("" ::"s"(ca[PH]), "s"(cb[PH]));
#else
#define VTB_STORE(I, PH)                                                                   \
    asm volatile("s_store_dwordx2 %0, %1, %2" ::"s"(ca[PH]), "s"(pA), "i"((I) * 8));       \
    asm volatile("s_store_dwordx2 %0, %1, %2" ::"s"(cb[PH]), "s"(pB), "i"((I) * 8));
#endif
#define VTB_GROUP(G)                                                                              \
    {                                                                                             \
        uint2 nxt[6];                                                                             \
        _Pragma("unroll") for (int k = 0; k < 6; k++) nxt[k] =                                    \
            VTB_EXP_LDS((G) < 7 ? ap[k][(6 * ((G) + 1) + k) * (kTabBytes / 8)] : an[k][k * (kTabBytes / 8)]); \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        uint64_t ca[6], cb[6];                                                                    \
        VTB_STEP(6 * (G) + 0, 0) VTB_STEP(6 * (G) + 1, 1) VTB_STEP(6 * (G) + 2, 2)                \
        VTB_STEP(6 * (G) + 3, 3) VTB_STEP(6 * (G) + 4, 4) VTB_STEP(6 * (G) + 5, 5)                \
        if ((G) == 3) stage_chunk(buf ^ 1, nqa, nqb);                                             \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        _Pragma("unroll") for (int k = 0; k < 6; k++) asm volatile("" ::"v"(nxt[k].x), "v"(nxt[k].y)); \
        VTB_STORE(6 * (G) + 0, 0) VTB_STORE(6 * (G) + 1, 1) VTB_STORE(6 * (G) + 2, 2)             \
        VTB_STORE(6 * (G) + 3, 3) VTB_STORE(6 * (G) + 4, 4) VTB_STORE(6 * (G) + 5, 5)             \
        __builtin_amdgcn_sched_barrier(0);                                                        \
        _Pragma("unroll") for (int k = 0; k < 6; k++) cur[k] = nxt[k];                            \
    }
        VTB_GROUP(0) VTB_GROUP(1) VTB_GROUP(2) VTB_GROUP(3) VTB_GROUP(4) VTB_GROUP(5) VTB_GROUP(6) VTB_GROUP(7)
#undef VTB_GROUP
#undef VTB_STORE
#undef VTB_STEP
    }
    // Scalar-cache write-back of the compare words, then vector stores of the steps past T:
    // C = R there, i.e. D = 0 (every location keeps its bit p, the set collapses to state 0).
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_dcache_wb\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    {
        const int nv = Tdec - T;
        for (int i = lane; i < 2 * nv; i += 64) {
            const int f = i >= nv;
            const int t = T + i - f * nv;
            (f ? wsB : wsA)[t] = loc_mask(5 - t % 6);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (dbg & 1) return;

    // ---------------- block-parallel exact traceback ----------------
    const int f = lane >> 5, blk = lane & 31;
    const uint64_t* D = f ? wsB : wsA;
    uint32_t* ob = obuf + f * obw;
    uint32_t lo = 0xFFFFFFFFu, hi = 0xFFFFFFFFu;
    bool ok = false;
    const int top = (blk + 1) * tbb;
    tb_walk(D, top + kWarm, kWarm / 12, tbb / 12, lo, hi, ok, ob);

    // Blocks whose set did not collapse: re-walk from the successor's proven entry.  The
    // last block of each frame starts beyond T and never fails.
    for (int round = 0; round < 32; round++) {
        const bool bad = !ok;
        if (!__any(bad)) break;
        const uint32_t slo = __shfl_down(lo, 1), shi = __shfl_down(hi, 1);
        const int sok = __shfl_down(ok ? 1 : 0, 1);
        if (bad && sok) {
            lo = slo;
            hi = shi;
            tb_walk(D, top, 0, tbb / 12, lo, hi, ok, ob);
        }
    }
    __syncthreads();

    // copy the decoded bytes out (bits past L are zero: the survivor ends in state 0)
    const int nbytes = (L + 7) >> 3;
    const uint8_t* obb = reinterpret_cast<const uint8_t*>(obuf);
    uint8_t* oa = out + fa * out_stride;
    for (int i = lane; i < nbytes; i += 64) oa[i] = obb[i];
    if (has_b) {
        uint8_t* o2 = out + fb * out_stride;
        for (int i = lane; i < nbytes; i += 64) o2[i] = obb[4 * obw + i];
    }
}

int tb_block(int T) {
    int per = (T + 31) / 32;  // 32 blocks per frame, multiple of 12 steps
    return (per + 11) / 12 * 12;
}

int dec_steps(int T) { return (32 * tb_block(T) + kWarm + 7) / 8 * 8; }

size_t lds_bytes(int T) { return 2 * kChunk * kTabBytes + 2 * 4 * (size_t)(tb_block(T) + 4); }

}  // namespace

bool reg_path_supported(const Launch& a) {
    return a.S == 6 && a.T > a.S && lds_bytes(a.T) <= 64 * 1024;
}

// Waves (frame pairs) per launch: the whole batch, unless its workspace would exceed
// kMaxWsBytes; then the batch runs as several launches over one workspace.
static size_t slab_waves(const Launch& a) {
    const size_t wave_bytes = 2 * (size_t)dec_steps(a.T) * 8;
    const size_t waves = (a.frames + 1) / 2;
    size_t slab = kMaxWsBytes / wave_bytes;
    if (slab < 1) slab = 1;
    return slab < waves ? slab : waves;
}

size_t reg_path_workspace_bytes(const Launch& a) { return slab_waves(a) * 2 * (size_t)dec_steps(a.T) * 8; }

hipError_t launch_reg_path(const Launch& a) {
    if (a.frames == 0) return hipSuccess;
    if (!a.ws) return hipErrorInvalidValue;
    const int Tpad = (a.T + kChunk - 1) / kChunk * kChunk;
    const int Tdec = dec_steps(a.T);
    const int tbb = tb_block(a.T);
    const size_t lds = lds_bytes(a.T);
    const size_t waves = (a.frames + 1) / 2;
    const size_t slab = slab_waves(a);
    auto kern = a.soft ? reg_k7_kernel<true> : reg_k7_kernel<false>;
    const int dbg = debug_flags();
    for (size_t w0 = 0; w0 < waves; w0 += slab) {
        const size_t nw = waves - w0 < slab ? waves - w0 : slab;
        const size_t f0 = 2 * w0;
        const size_t nf = a.frames - f0 < 2 * nw ? a.frames - f0 : 2 * nw;
        hipLaunchKernelGGL(kern, dim3(unsigned(nw)), dim3(64), lds, a.stream, a.in + f0 * a.in_stride, a.in_stride,
                           a.out + f0 * a.out_stride, a.out_stride, static_cast<uint64_t*>(a.ws), a.T, a.L, Tpad,
                           Tdec, tbb, nf, dbg, a);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace vtb
