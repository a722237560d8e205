// K=7 (64 states) decoder with LDS-resident survivors: the fast path for frames whose
// survivor words fit in LDS at two waves per SIMD (L up to ~1000 at 8 waves/CU; longer
// frames run at lower occupancy).  Hard and 8-bit soft input.
//
// Layout.  One wave64 decodes two frames, A and B.  Lane l holds the path metric of the
// trellis state living at "location" l for both frames as one packed u16 pair
// [m_A, m_B]: every packed instruction advances both frames.
//
// In-place state relabelling.  Instead of moving state s to lane s every step (the
// reference's destination-indexed butterfly, viterbiDecoderButterflyk1.c:101-152), each
// butterfly writes its two destinations back into the two locations its sources came
// from.  Location l then holds state rotl6(l, t mod 6) at step t, and the two sources of
// a butterfly (states j and j+32) sit in lanes that differ in one bit, p = 5 - (t mod 6).
// Location l is kept in lane L(l) = l ^ (3 if bit 2 of l else 0), a linear involution
// chosen so that every pairing bit maps to an XOR of the lane index that one cross-lane op
// performs: location bits 0..5 -> lane XOR 1, 2, 7, 8, 16, 32 = DPP quad_perm,
// quad_perm, row_half_mirror, row_ror:8 (folded into the add), in-place
// v_permlane16_swap, v_permlane32_swap.
//
// Branch metrics: a ring of 48 table rows in LDS, staged 24 steps at a time by 24 lanes
// (vtb_k7_common.h write_row): per step eight (V, W) pairs, V = 2e(c) + R, W = 2e(~c).
// Lane l reads its pair with one ds_read_b64 at a per-phase offset (its label c, and
// R = bit p of l), one group of six steps ahead.  The ACS step is
//     A = M + V;  B = partner(M) + W;  M' = min(A, B) & ~1;  d = B - A
// Metrics are doubled so that the R bit added to the own-path candidate of lanes whose
// own state is the upper predecessor j+32 turns "A > B" into "A >= B" for exactly those
// lanes: the sign of d (per 16-bit half) is C = [A > B], and the reference's decision
// (strict '>' toward the lower predecessor j, viterbiDecoderButterflyk1.c:129-130) is
// D = C xor R.  The and clears the R bit again.
//
// Initial metrics: the reference starts state 0 at 0 and every other state at
// (uint8)(N+1) = 65 (x255 soft).  For K=7 any start value above 12Q (six steps of the
// largest branch metric) yields the same decisions -- during the first six steps a path
// from state 0 always beats one from another state, paths from other states compare
// with equal offsets, and from step 6 on every state descends from state 0 -- so this
// kernel uses 12Q + 1, which keeps all candidate differences far inside int16.
//
// Renormalisation every 16 steps (subtract location 0's metric, add a bias) replaces the
// reference's uint8 renorm (exact metrics have a bounded spread).
//
// Survivors.  The sign bits of d accumulate in one VGPR per lane, frame A in bits 0..15
// and frame B in bits 16..31 (bit j = step 16k + j), and every 16 steps the wave writes
// its 64 words (256 B, one ds_write_b32) to LDS.  No scalar stores, no VALU lane writes.
//
// Traceback (reference :200-256), in location space: going back from step t+1 to t the
// decoded bit is bit p_t of the location and the location's bit p_t becomes D_t[loc],
// i.e. loc ^= C_t[loc] << p_t.  Within a sextet p runs 0..5, so a sextet's six decoded
// bits are the location at its start, MSB first.  Lanes 0-31 trace blocks of frame A,
// lanes 32-63 of frame B, each block of TBB steps (a multiple of 48) walking back from
// 48 steps past its end as a chain of dependent LDS reads.  A block whose walk starts at
// or beyond T starts at the known location 0 (the terminated path ends in state 0; the
// survivor words of steps past T are cleared so location 0 stays put).  Every other
// block starts at a guess and is verified: its location on entering the block must equal
// the location its successor ended on; a block that disagrees is re-walked from its
// successor's proven location.  So the output is exactly the reference's for every
// input; only the time depends on how fast survivor paths merge.

#include "vtb_k7_common.h"

namespace vtb {
namespace {

using namespace k7;

constexpr int kHalf = 24;     // table rows staged at a time (ring of 2 halves = kChunk rows)
constexpr int kRowBytes = 32; // branch-metric table row: (V, W) of the four edge labels
constexpr int kTbWarm = 48;   // traceback warm-up steps past a block's end
constexpr uint32_t kBias1 = 4096;  // renormalised metrics: kBias1 +- 3060 (soft)

int tb_block(int T) {
    const int per = (T + 31) / 32;  // 32 blocks per frame, multiple of 48 steps
    return (per + 47) / 48 * 48;
}
int t_pad(int T) { return (T + kChunk - 1) / kChunk * kChunk; }
// LDS: [0, r0) table ring, later the decoded bytes of both frames; [r0, r0 + 16*Tpad)
// survivor words.
int region0(int T) { return 8 * tb_block(T) > kChunk * kRowBytes ? 8 * tb_block(T) : kChunk * kRowBytes; }
size_t lds_bytes(int T) { return (size_t)region0(T) + 16 * (size_t)t_pad(T); }

// lane <-> location map (an involution)
__device__ __forceinline__ uint32_t lane_of(uint32_t l) { return l ^ (((l >> 2) & 1u) * 3u); }

// Partner metric across location bit P, plus w (lane XOR 1, 2, 7, 8, 16, 32).
template <int P>
__device__ __forceinline__ uint32_t exch_plus(uint32_t m, uint32_t w) {
    if constexpr (P == 2) {
        return __builtin_amdgcn_update_dpp(0u, m, 0x141, 0xF, 0xF, true) + w;  // row_half_mirror: XOR 7
    } else {
        return partner_plus<P>(m, w);
    }
}

__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) { return (a & mask) | (b & ~mask); }

// The candidates of a step: A = own metric + V, B = partner's metric + W, and A1 = A + R
// (R = 1 in both halves for lanes whose own state is the upper predecessor), so that
// [A1 > B] is the reference's decision rule for either lane of a butterfly.  For the
// permlane phases the add of A separates the last write of M from the swap and the add of
// A1 separates the swap from the read of its result, inside one asm block (the swap needs
// one wait state after a VALU write of its operand: permlane_hazard probe).
template <int P>
__device__ __forceinline__ void acs_pair(uint32_t m, uint2 vw, uint32_t r, uint32_t& A, uint32_t& A1, uint32_t& B) {
    if constexpr (P == 4 || P == 5) {
        if constexpr (P == 4) {
            asm volatile("v_add_u32 %0, %2, %3\n\tv_permlane16_swap_b32 %2, %2\n\tv_add_u32 %1, %0, %4"
                         : "=&v"(A), "=&v"(A1), "+v"(m) : "v"(vw.x), "v"(r));
        } else {
            asm volatile("v_add_u32 %0, %2, %3\n\tv_permlane32_swap_b32 %2, %2\n\tv_add_u32 %1, %0, %4"
                         : "=&v"(A), "=&v"(A1), "+v"(m) : "v"(vw.x), "v"(r));
        }
        B = m + vw.y;
    } else {
        A = m + vw.x;
        A1 = A + r;
        B = exch_plus<P>(m, vw.y);
    }
}

// Bit of step s (0..15) of a frame in its 16-bit half of a decision word (see the ACS).
constexpr int word_bit(int s) {
    return 8 * ((s >> 1) & 1) + 7 - (s & 1) - 2 * ((s >> 2) & 1) - 4 * ((s >> 3) & 1);
}

// 48 traceback steps over steps [tlo, tlo + 48) (tlo a multiple of 48), newest first, on
// the lane index lam of the survivor's location.  Returns the 48 decoded bits (MSB = step
// tlo): each sextet's bits are its starting location.
__device__ __forceinline__ uint64_t tb_body(const uint8_t* decf, int tlo, uint32_t& lam) {
    const uint8_t* base = decf + (tlo >> 4) * 256;
    uint64_t bits = 0;
#pragma unroll
    for (int j = 0; j < 48; j++) {
        const int s = word_bit((47 - j) & 15);  // bit of step t = tlo + 47 - j in its half-word
        const int p = j % 6;          // pairing bit of that step
        if (p == 0) bits |= uint64_t(lane_of(lam)) << (6 * (j / 6));
        const uint32_t w = *reinterpret_cast<const unsigned short*>(base + ((47 - j) >> 4) * 256 + lam * 4);
        if (p == 2) {
            lam ^= uint32_t(int32_t(w << (31 - s)) >> 31) & 7u;  // C ? XOR 7
        } else {
            const uint32_t x = s >= p ? (w >> (s - p)) : (w << (p - s));
            lam ^= x & (1u << p);
        }
    }
    return bits;
}

__device__ __forceinline__ void put_bits48(uint8_t* ob, int tlo, uint64_t bits) {
    unsigned short* o = reinterpret_cast<unsigned short*>(ob + (tlo >> 3));
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t hi = uint32_t(bits >> (40 - 16 * k)) & 0xffu, lo = uint32_t(bits >> (32 - 16 * k)) & 0xffu;
        o[k] = (unsigned short)(hi | (lo << 8));
    }
}

// Measurement-only variants (tools/build_variants.sh builds them into separate libraries,
// never the shipped one; their outputs are wrong): no table staging inside the ACS loop /
// no survivor-word stores.
#ifdef VTB_EXP_K15
#define VTB_EXP_ODD(d) ((d) >> 1)
#else
#define VTB_EXP_ODD(d) (d)
#endif
#ifdef VTB_EXP_NO_STAGE
#define VTB_EXP_STAGE false
#else
#define VTB_EXP_STAGE true
#endif
#ifdef VTB_EXP_NO_WORD
#define VTB_EXP_WORD(x) asm volatile("" ::"v"(r), "v"(r_p))
#else
#define VTB_EXP_WORD(x) x
#endif

template <bool SOFT>
__global__ __launch_bounds__(64) void k7_lds_kernel(const uint8_t* __restrict__ in, size_t in_stride,
                                                    uint8_t* __restrict__ out, size_t out_stride, int T, int L,
                                                    int Tpad, int tbb, int r0, size_t frames, int dbg, Launch table) {
    constexpr uint32_t Q = SOFT ? 255 : 1;
    constexpr uint32_t INIT = 12 * Q + 1;  // start metric of states != 0 (see header)
    extern __shared__ uint4 smem4[];
    uint8_t* smem = reinterpret_cast<uint8_t*>(smem4);
    uint8_t* tab = smem;
    uint32_t* dec = reinterpret_cast<uint32_t*>(smem + r0);
    const int lane = threadIdx.x;
    const size_t fa = (size_t)blockIdx.x * 2, fb = fa + 1;
    const bool has_b = fb < frames;
    const uint8_t* inA = in + fa * in_stride;
    const uint8_t* inB = in + (has_b ? fb : fa) * in_stride;

    // Per phase: byte offset of the lane's (V, W) pair in a table row (its edge label c) and
    // the tie bit R (bit p of the lane's location), packed for both frames.
    uint32_t off[6], rr[6];
    {
        const int loc = int(lane_of(lane));
#pragma unroll
        for (int ph = 0; ph < 6; ph++) {
            const int p = 5 - ph;
            off[ph] = 8u * table.symm[rotl6(loc & ~(1 << p), ph)];
            // A1 = A + R - 1 + 2^k: bit k of A1 - B is [A + R > B] (k = 15 on even, 14 on
            // odd steps; |A + R - B| < 2^14 and A1 < 65536 keep both halves apart)
#ifdef VTB_EXP_K15
            rr[ph] = (uint32_t((loc >> p) & 1) + (1u << 15) - 1u) * 0x10001u;
#else
            rr[ph] = (uint32_t((loc >> p) & 1) + (1u << (15 - (ph & 1))) - 1u) * 0x10001u;
#endif
        }
    }

    // Table staging.  Lane r < 24 builds the rows of steps 24k + r.  The raw input bytes of
    // a chunk (48 steps: both halves, both frames) are loaded a whole chunk ahead into one of
    // two register sets and first touched (behind an empty asm, so the compiler cannot
    // hoist the byte unpacking next to the load) when a half is staged, 48-72 steps later.
    const int lrow = lane % kHalf;
    struct Raw {
        uint32_t a[2], b[2];  // [half]: frame A / B bytes of step t (soft q0 | q1 << 8, hard the byte)
    };
    auto load_chunk = [&](int c, Raw& r) {
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int t = c * kChunk + k * kHalf + lrow;
            const int tc = t < T ? t : T - 1;
            if constexpr (SOFT) {
                unsigned short x, y;
                __builtin_memcpy(&x, inA + 2 * (size_t)tc, 2);
                __builtin_memcpy(&y, inB + 2 * (size_t)tc, 2);
                r.a[k] = x;
                r.b[k] = y;
            } else {
                r.a[k] = inA[tc];
                r.b[k] = inB[tc];
            }
        }
    };
    auto stage_half = [&](int h, uint32_t ra, uint32_t rb) {
        asm volatile("" : "+v"(ra), "+v"(rb));
        const int t = h * kHalf + lrow;
        // packed [frame A, frame B] received values of coded bits 0 and 1
        uint32_t q0 = __builtin_amdgcn_perm(rb, ra, 0x0C040C00u);
        uint32_t q1 = __builtin_amdgcn_perm(rb, ra, 0x0C050C01u);
        if constexpr (!SOFT) {
            q1 = (q0 >> 1) & 0x00010001u;
            q0 &= 0x00010001u;
        }
        const uint32_t keep = (t < T ? 0x0000FFFFu : 0u) | ((t < T && has_b) ? 0xFFFF0000u : 0u);
        q0 &= keep;
        q1 &= keep;
        // doubled branch metrics of labels 0..3 (bit 0 of a label <-> coded bit 0):
        // e0 = q0+q1, e3 = 2Q - e0, e1 = Q - q0 + q1, e2 = Q + q0 - q1
        constexpr uint32_t R1 = 0x10001u;
        const uint32_t e0 = q0 + q1;
        const uint32_t e3 = 2 * Q * R1 - e0;
        const uint32_t dq = pk_sub(q1, q0);
        const uint32_t e1 = pk_add(Q * R1, dq);
        const uint32_t e2 = pk_sub(Q * R1, dq);
        if (lane < kHalf) {
            uint4* row = reinterpret_cast<uint4*>(tab + ((h & 1) * kHalf + lrow) * kRowBytes);
            row[0] = make_uint4(e0, e3, e1, e2);  // (V, W) of labels c = 0, 1
            row[1] = make_uint4(e2, e1, e3, e0);  // (V, W) of labels c = 2, 3
        }
    };

    uint32_t M = (lane == 0) ? kBias1 * 0x10001u : (kBias1 + INIT) * 0x10001u;
    Raw sa, sb;  // raw input of chunks c and c+1
    load_chunk(0, sa);
    stage_half(0, sa.a[0], sa.b[0]);
    load_chunk(1, sb);
    // software pipeline: the table pairs of group G+2 are read while group G computes
    uint2 cur[6], nx1[6];
#pragma unroll
    for (int k = 0; k < 6; k++) {
        cur[k] = *reinterpret_cast<const uint2*>(tab + k * kRowBytes + off[k]);
        nx1[k] = *reinterpret_cast<const uint2*>(tab + (6 + k) * kRowBytes + off[k]);
    }

    // Decision words: the decision of an even step lands on bits 15/31 of d, of an odd step
    // on bits 14/30 (rr); a tree -- bit-field insert of two steps, v_perm of the decision
    // bytes of two pairs, two levels of shift + insert -- gathers the 32 bits of 16 steps
    // into one word per lane (bit positions: word_bit()).
    uint32_t d_even = 0, u_p = 0, p_p = 0, r_p = 0;
    const int tacs = (dbg & 2) ? 0 : Tpad;
    for (int t0 = 0; t0 < tacs; t0 += kChunk) {
        const int h0 = t0 / kHalf;  // half index of this chunk's first half
        const uint2* ap[6];
#pragma unroll
        for (int k = 0; k < 6; k++) ap[k] = reinterpret_cast<const uint2*>(tab + off[k]);
        uint32_t* dchunk = dec + (t0 >> 4) * 64 + lane;

#define VTB_STEP(I, PH)                                                                              \
    {                                                                                                \
        uint32_t A, A1, B;                                                                           \
        acs_pair<5 - (PH)>(M, cur[PH], rr[PH], A, A1, B);                                            \
        M = pk_min(A, B);                                                                            \
        const uint32_t d = pk_sub(A1, B); /* bit k, 16 + k: C = [A + R > B] of frames A, B */       \
        if (((I) & 1) == 0) {                                                                        \
            d_even = d;                                                                              \
        } else {                                                                                     \
            const uint32_t u = bfi(0x80008000u, d_even, VTB_EXP_ODD(d)); /* bits 15, 14 of each half */ \
            if (((I) & 3) == 1) {                                                                    \
                u_p = u;                                                                             \
            } else {                                                                                 \
                const uint32_t pq = __builtin_amdgcn_perm(u, u_p, 0x07030501u);                      \
                if (((I) & 7) == 3) {                                                                \
                    p_p = pq;                                                                        \
                } else {                                                                             \
                    const uint32_t r = bfi(0xC0C0C0C0u, p_p, pq >> 2);                               \
                    if (((I) & 15) == 7) {                                                           \
                        r_p = r;                                                                     \
                    } else {                                                                         \
                        VTB_EXP_WORD(dchunk[((I) >> 4) * 64] = bfi(0xF0F0F0F0u, r_p, r >> 4));       \
                    }                                                                                \
                }                                                                                    \
            }                                                                                        \
        }                                                                                            \
    }
#define VTB_GROUP(G)                                                                              \
    {                                                                                             \
        uint2 nx2[6];                                                                             \
        _Pragma("unroll") for (int k = 0; k < 6; k++) nx2[k] =                                    \
            ap[k][((6 * ((G) + 2) + k) % kChunk) * (kRowBytes / 8)];                              \
        if ((G) == 1 && VTB_EXP_STAGE) {                                                          \
            stage_half(h0 + 1, sa.a[1], sa.b[1]);                                                 \
            load_chunk(h0 / 2 + 2, sa);                                                           \
        }                                                                                         \
        if ((G) == 5 && VTB_EXP_STAGE) stage_half(h0 + 2, sb.a[0], sb.b[0]);                      \
        VTB_STEP(6 * (G) + 0, 0) VTB_STEP(6 * (G) + 1, 1) VTB_STEP(6 * (G) + 2, 2)                \
        VTB_STEP(6 * (G) + 3, 3) VTB_STEP(6 * (G) + 4, 4) VTB_STEP(6 * (G) + 5, 5)                \
        _Pragma("unroll") for (int k = 0; k < 6; k++) {                                           \
            cur[k] = nx1[k];                                                                      \
            nx1[k] = nx2[k];                                                                      \
        }                                                                                         \
    }
        VTB_GROUP(0) VTB_GROUP(1) VTB_GROUP(2) VTB_GROUP(3) VTB_GROUP(4) VTB_GROUP(5) VTB_GROUP(6) VTB_GROUP(7)
#undef VTB_GROUP
#undef VTB_STEP
        // renormalise once per chunk: 48 steps add at most 48 * 510 to a metric, so values
        // stay below kBias1 + 3061 + 3060 + 24480 (+ 2^15 in A1) < 65536
        {
            const uint32_t ref = __builtin_amdgcn_readlane(M, 0);
            const uint32_t dd = ((kBias1 - (ref & 0xffffu)) & 0xffffu) | ((kBias1 - (ref >> 16)) << 16);
            M = pk_add(M, dd);
        }
        const Raw t = sa;
        sa = sb;
        sb = t;
    }
    // Steps past T: clear their survivor bits so that location 0 keeps its place there.
    for (int k = T >> 4; k < (Tpad >> 4); k++) {
        uint32_t keep = 0;
        if (k == (T >> 4)) {
            for (int st = 0; st < (T & 15); st++) keep |= 0x00010001u << word_bit(st);
        }
        dec[k * 64 + lane] &= keep;
    }
    __syncthreads();
    if (dbg & 1) return;

    // ---------------- traceback: verified block-parallel chains ----------------
    const int f = lane >> 5, blk = lane & 31;
    const uint8_t* decf = reinterpret_cast<const uint8_t*>(dec) + 2 * f;  // this frame's 16-bit half
    uint8_t* ob = tab + f * 4 * tbb;                                      // decoded bytes, index t/8
    const int top = (blk + 1) * tbb;
    const int start_full = top + kTbWarm;
    const int start = min(start_full, Tpad);
    const bool known = start >= T;  // walk starts on the known path (location 0 at and past T)
    const int nbody = (kTbWarm + tbb) / 48;
    uint32_t lam = 0, lam_top = 0;
    for (int g = 0; g < nbody; g++) {
        const int tlo = start_full - 48 * (g + 1);
        if (g == kTbWarm / 48) lam_top = lam;
        if (tlo < start) {  // lane's walk has begun (start is a multiple of 48)
            const uint64_t bits = tb_body(decf, tlo, lam);
            if (g >= kTbWarm / 48) put_bits48(ob, tlo, bits);
        }
    }
    uint32_t fin = lam;  // survivor's lane index at step blk * tbb
    bool ok = known;
    for (int round = 0; round < 32; round++) {
        if (!__any(!ok)) break;
        const uint32_t sf = __shfl_down(fin, 1);
        const int sok = __shfl_down(ok ? 1 : 0, 1);
        const bool cand = !ok && sok;
        if (cand && lam_top == sf) ok = true;  // entered the block on the proven path
        if (cand && !ok) {
            lam = sf;
            for (int g = kTbWarm / 48; g < nbody; g++) {
                const int tlo = start_full - 48 * (g + 1);
                put_bits48(ob, tlo, tb_body(decf, tlo, lam));
            }
            fin = lam;
            ok = true;
        }
    }
    __syncthreads();

    // copy the decoded bytes out (bits past L are zero: the survivor ends in state 0)
    const int nbytes = (L + 7) >> 3;
    uint8_t* oa = out + fa * out_stride;
    for (int i = lane; i < nbytes; i += 64) oa[i] = tab[i];
    if (has_b) {
        uint8_t* o2 = out + fb * out_stride;
        for (int i = lane; i < nbytes; i += 64) o2[i] = tab[4 * tbb + i];
    }
}

}  // namespace

bool k7_lds_supported(const Launch& a) { return a.S == 6 && a.T > a.S && lds_bytes(a.T) <= 160 * 1024; }

size_t k7_lds_bytes(const Launch& a) { return lds_bytes(a.T); }

hipError_t launch_k7_lds(const Launch& a) {
    if (a.frames == 0) return hipSuccess;
    const size_t lds = lds_bytes(a.T);
    auto kern = a.soft ? k7_lds_kernel<true> : k7_lds_kernel<false>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
    }
    const size_t waves = (a.frames + 1) / 2;
    hipLaunchKernelGGL(kern, dim3(unsigned(waves)), dim3(64), lds, a.stream, a.in, a.in_stride, a.out, a.out_stride,
                       a.T, a.L, t_pad(a.T), tb_block(a.T), region0(a.T), a.frames, debug_flags(), a);
    return hipGetLastError();
}

}  // namespace vtb
