// Baseline gfx950 decoder: "LDS path".
//
// One wave64 decodes F = 64/G frames; each frame's N = 2^S trellis states are spread over
// G = min(N, 64) lanes with R = N/G states per lane in registers (state s lives in lane
// s % G, register s / G).  Per trellis step every lane gathers the two predecessor
// metrics of each of its states with ds_bpermute (predecessors of s are s>>1 and
// (s>>1) + N/2, reference viterbiDecoderButterflyk1.c:101-152), does the add-compare-
// select, and the wave's __ballot of the decisions (one 64-bit word per register per
// step) is written to LDS.  After the last step the traceback (reference :200-256) walks
// the LDS survivor words from state 0.
//
// This is the simple, obviously-correct kernel: the register-resident kernel
// (vtb_k7_lds.hip) is the fast path; this one also covers every K in 3..9.
//
// Two variants of the one kernel (template parameter GS; lds_path_global picks one):
//   * LDS: every survivor word and the wave's whole input in LDS, 8 R T + F T B bytes per wave
//     (B = 1 hard, 2 soft) -- K = 3, 4 frames of 2,048+ steps while that LDS leaves the CU
//     the batch's waves;
//   * GS (global survivors): the survivor words in a global workspace (8 R T bytes per wave,
//     the lane that owns step t mod 64 keeps its ballot words in registers and the wave stores
//     64 steps' words at once, coalesced), the input staged through LDS kStage steps at a time
//     (F kStage B bytes), the traceback reading the words back from L2/HBM.  Every frame up to
//     VTB_MAX_FRAME_BITS (the reference's MAX_PKT_LEN_UNCODED_BITS, viterbiDecoder.h:18), at
//     any K, hard or soft (VERDICT r5 missing #1).
// Decisions, metrics and traceback are the same code in both: the outputs are identical.
//
#include "vtb_internal.h"

namespace vtb {
namespace {

constexpr int kWavesPerBlock = 4;

__device__ __forceinline__ int shfl_idx(int v, int src_lane) {
    return __builtin_amdgcn_ds_bpermute(src_lane << 2, v);
}

// Decisions for state s at step t:  bit (fi*G + s%G) of word [t][s/G].
template <int S>
struct Geometry {
    static constexpr int N = 1 << S;
    static constexpr int G = N < 64 ? N : 64;  // lanes per frame
    static constexpr int R = N / G;            // states per lane
    static constexpr int F = 64 / G;           // frames per wave
};

constexpr int kStage = 64;  // GS: steps of input staged into LDS per round (= lanes: one keeper per step)

template <int S, bool SOFT, bool GS>
__global__ __launch_bounds__(64 * kWavesPerBlock) void lds_path_kernel(const uint8_t* __restrict__ in, size_t in_stride,
                                                                        uint8_t* __restrict__ out, size_t out_stride,
                                                                        int T, int L, size_t frames, int waves_per_block,
                                                                        Launch table) {
    using Gm = Geometry<S>;
    constexpr int N = Gm::N, G = Gm::G, R = Gm::R, F = Gm::F;
    constexpr int Q = SOFT ? 255 : 1;
    constexpr int INIT = int(uint8_t(N + 1)) * Q;  // (uint8_t)(NUM_STATES+1), reference :62
    constexpr int BYTES_PER_SEG = SOFT ? 2 : 1;

    extern __shared__ uint64_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int fi = lane / G;
    const int lam = lane % G;

    const size_t dec_words = (size_t)T * R;
    uint64_t* dec;
    uint8_t* inbuf;
    if constexpr (GS) {
        // one wave per block: the block's slot of the launch's workspace, the staging buffer in LDS
        dec = static_cast<uint64_t*>(table.ws) + (size_t)blockIdx.x * dec_words;
        inbuf = reinterpret_cast<uint8_t*>(smem);
    } else {
        const size_t in_bytes = ((size_t)F * T * BYTES_PER_SEG + 7) & ~size_t(7);
        dec = smem + (size_t)wave * (dec_words + in_bytes / 8);
        inbuf = reinterpret_cast<uint8_t*>(dec + dec_words);
    }

    const size_t frame0 = ((size_t)blockIdx.x * waves_per_block + wave) * F;
    const size_t myframe = frame0 + fi;
    const bool valid = myframe < frames;

    // Per-register branch-metric coefficients.  Destination d = r*G + lam has
    // predecessors j = d>>1 and j + N/2; with b = d&1 the candidate from j is m[j] + mu_b
    // and from j + N/2 is m[j+N/2] - mu_b, where mu_0 = mu(c) and mu_1 = -mu(c).
    int sig[R], kap[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        int d = r * G + lam;
        int c = table.symm[d >> 1];
        int sb = (d & 1) ? -1 : 1;
        int s0 = ((c & 1) ? -1 : 1) * sb, s1 = ((c & 2) ? -1 : 1) * sb;
        sig[r] = (s0 & 0xffff) | (s1 << 16);
        kap[r] = (((c & 1) + ((c >> 1) & 1)) - 1) * Q * sb;
    }

    int m[R];
#pragma unroll
    for (int r = 0; r < R; r++) m[r] = (r * G + lam == 0) ? 0 : INIT;

    const int src_base = fi * G;
    // One trellis step from the frame's received pair at `seg`: the R ballot words out.
    auto acs_step = [&](const uint8_t* seg, uint64_t* ballots) {
        int qp;
        if (SOFT) {
            qp = int(seg[0]) | (int(seg[1]) << 16);
        } else {
            int c = seg[0];
            qp = (c & 1) | (((c >> 1) & 1) << 16);
        }
        int nm[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int lane0 = src_base + (r & 1) * (G / 2) + (lam >> 1);
            int a0, a1;
            if (R == 1) {
                a0 = shfl_idx(m[0], lane0);
                a1 = shfl_idx(m[0], lane0 + G / 2);
            } else {
                a0 = shfl_idx(m[r >> 1], lane0);
                a1 = shfl_idx(m[(r >> 1) + R / 2], lane0);
            }
            typedef short short2_t __attribute__((ext_vector_type(2)));
            int mu = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, sig[r]), __builtin_bit_cast(short2_t, qp),
                                            kap[r], false);
            int c0 = a0 + mu, c1 = a1 - mu;
            bool d = c0 > c1;  // strict: ties keep the lower predecessor (reference :129-130)
            nm[r] = d ? c1 : c0;
            ballots[r] = __ballot(d);
        }
#pragma unroll
        for (int r = 0; r < R; r++) m[r] = nm[r];
    };

    if constexpr (GS) {
        constexpr int kRow = kStage * BYTES_PER_SEG;  // staged bytes per frame
        const uint8_t* myin = inbuf + fi * kRow;
        for (int c0 = 0; c0 < T; c0 += kStage) {
            const int n = T - c0 < kStage ? T - c0 : kStage;
            const int nb = n * BYTES_PER_SEG;
            __syncthreads();  // (one wave: the previous round's reads of the buffer are done)
            for (int idx = lane; idx < F * nb; idx += 64) {
                const int f = idx / nb, off = idx - f * nb;
                inbuf[f * kRow + off] =
                    frame0 + f < frames ? in[(frame0 + f) * in_stride + (size_t)c0 * BYTES_PER_SEG + off] : 0;
            }
            __syncthreads();
            uint64_t keep[R];  // lane i keeps the words of step c0 + i
#pragma unroll
            for (int r = 0; r < R; r++) keep[r] = 0;
            for (int i = 0; i < n; i++) {
                uint64_t ballots[R];
                acs_step(myin + i * BYTES_PER_SEG, ballots);
#pragma unroll
                for (int r = 0; r < R; r++) keep[r] = lane == i ? ballots[r] : keep[r];
            }
            if (lane < n) {
#pragma unroll
                for (int r = 0; r < R; r++) dec[(size_t)(c0 + lane) * R + r] = keep[r];
            }
        }
        __threadfence_block();  // the survivor words before any lane's traceback reads them
    } else {
        // Stage this wave's input frames into LDS (coalesced byte loads).
        const int seg_bytes = T * BYTES_PER_SEG;
        for (int idx = lane; idx < F * seg_bytes; idx += 64) {
            int f = idx / seg_bytes, off = idx - f * seg_bytes;
            uint8_t v = 0;
            if (frame0 + f < frames) v = in[(frame0 + f) * in_stride + off];
            inbuf[idx] = v;
        }
        __syncthreads();
        const uint8_t* myin = inbuf + fi * seg_bytes;
        for (int t = 0; t < T; t++) {
            uint64_t ballots[R];
            acs_step(myin + t * BYTES_PER_SEG, ballots);
            if (lane == 0) {
#pragma unroll
                for (int r = 0; r < R; r++) dec[(size_t)t * R + r] = ballots[r];
            }
        }
    }

    __syncthreads();
    if (!valid) return;

    // Terminated traceback from state 0 (reference :200-256), block-parallel and verified
    // (the K=7 kernel's scheme, vtb_k7_lds.hip): the frame's G lanes each take a block of tbb
    // steps (a multiple of 8: every block owns whole output bytes), walk back to it from
    // kWarm steps past its end starting in state 0 there (exact when that is T, the
    // terminated end), and a block is right once it entered on its successor's exit state and
    // that successor is proven; failed blocks re-walk from a proven successor until all are.
    // The state after step t is s; its bit 0 is the information bit of step t, and the
    // predecessor is (s >> 1) | (decision << (S - 1)).
    constexpr int kWarm = 8 * S + 48;
    // A step's R survivor words do not depend on the walk's state (only the bit taken from them
    // does), so the walks load kTb steps' words at once and then take the kTb dependent steps:
    // kTb loads in flight instead of one (GS: L2 / HBM latency; LDS: ds_read latency).
    constexpr int kTb = R == 4 ? 4 : 8;
    auto row = [&](int t, uint64_t (&w)[R]) {
#pragma unroll
        for (int r = 0; r < R; r++) w[r] = dec[(size_t)t * R + r];
    };
    // (each word's bit is taken before the select: a select between the 64-bit words is
    // compiled as a dynamically indexed array in scratch memory)
    auto step = [&](unsigned st, const uint64_t (&w)[R]) -> unsigned {
        const unsigned sh = unsigned(fi * G) + (st % G);
        unsigned b[R];
#pragma unroll
        for (int r = 0; r < R; r++) b[r] = unsigned(w[r] >> sh) & 1u;
        unsigned x = b[0];
        if constexpr (R == 2) x = (st & unsigned(G)) ? b[1] : b[0];
        if constexpr (R == 4) {
            const unsigned lo2 = (st & unsigned(G)) ? b[1] : b[0], hi2 = (st & unsigned(G)) ? b[3] : b[2];
            x = (st & unsigned(2 * G)) ? hi2 : lo2;
        }
        return (st >> 1) | (x << (S - 1));
    };
    // the state before steps [lo, hi) given the state after step hi - 1
    auto walk = [&](unsigned st, int hi, int lo) -> unsigned {
        int t = hi;
        for (; t - kTb >= lo; t -= kTb) {
            uint64_t w[kTb][R];
#pragma unroll
            for (int j = 0; j < kTb; j++) row(t - 1 - j, w[j]);
#pragma unroll
            for (int j = 0; j < kTb; j++) st = step(st, w[j]);
        }
        for (; t > lo; t--) {
            uint64_t w[R];
            row(t - 1, w);
            st = step(st, w);
        }
        return st;
    };
    const int tbb = ((T + G - 1) / G + 7) / 8 * 8;
    const int lo = lam * tbb, top = lo + tbb < T ? lo + tbb : T;
    const bool active = lo < T;
    const int start = top + kWarm < T ? top + kWarm : T;
    unsigned st = active ? walk(0u, start, top) : 0u;
    unsigned s_top = st;
    if (active) st = walk(st, top, lo);
    unsigned fin = st;
    bool fixed = !active || start == T;
    const uint64_t fmask = (G == 64 ? ~uint64_t(0) : ((uint64_t(1) << (G & 63)) - 1)) << (fi * G);
    // (chains of G blocks: at most G - 1 re-walk rounds.)  Completeness guard: a frame with a
    // block still unproven after the cap (VTB_DEBUG bit 17: every chain with a walked block) is emitted by its lane 0
    // alone, walking serially from state 0 at T (the reference's walk, :200-256)
    const bool tbforce = (table.dbg & kDbgTbCap) != 0;
    const int rounds = tbforce ? 0 : G + 1;
    uint64_t unproven = 0;
    for (int round = 0;; round++) {
        const unsigned sf = unsigned(__shfl_down(int(fin), 1));  // successor block's entry state
        const bool ok = fixed || (s_top == sf && !tbforce);
        const uint64_t bad = ~__ballot(ok);
        if (bad == 0) break;
        if (round == rounds) {
            unproven = bad;
            break;
        }
        const uint64_t badf = (bad & fmask) >> (fi * G);  // this frame's failed blocks
        if (!ok && (badf >> (lam + 1)) == 0) {
            s_top = sf;
            fin = walk(sf, top, lo);
            fixed = true;
        }
    }
    int elo = lo, etop = top;  // emitted steps [elo, etop), from s_top after step etop - 1
    bool emit = active;
    if (unproven & fmask) {
        emit = lam == 0, elo = 0, etop = T, s_top = 0;
        if (lam == 0 && valid) note_guard(table.guard_hits);
    }
    if (!valid || !emit) return;
    // Emission, MSB-first bytes (reference :243-249): bit t of the frame is bit 0 of the state
    // after step t; byte t / 8 is complete at step t = 0 mod 8 (elo is a multiple of 8).  The
    // steps above the last whole octet of [elo, etop) one by one, then octets with their 8 rows
    // loaded at once.
    uint8_t* o = out + myframe * out_stride;
    unsigned byte = 0;
    st = s_top;
    auto put = [&](int t) {
        if (t < L) o[t >> 3] = uint8_t(t + 8 > L ? byte & (0xffu << (t + 8 - L)) : byte);
    };
    int t = etop - 1;
    for (; t >= elo && ((t + 1) & 7) != 0; t--) {
        byte = ((byte >> 1) | ((st & 1u) << 7)) & 0xffu;
        if ((t & 7) == 0) put(t);
        uint64_t w[R];
        row(t, w);
        st = step(st, w);
    }
    for (; t >= elo; t -= 8) {  // t = 7 mod 8: steps t .. t - 7
        uint64_t w[8][R];
#pragma unroll
        for (int j = 0; j < 8; j++) row(t - j, w[j]);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            byte = ((byte >> 1) | ((st & 1u) << 7)) & 0xffu;
            st = step(st, w[j]);
        }
        put(t - 7);
    }
}

template <int S>
size_t lds_bytes_per_wave(int soft, int T) {
    using Gm = Geometry<S>;
    size_t dec = (size_t)T * Gm::R * 8;
    size_t inb = ((size_t)Gm::F * T * (soft ? 2 : 1) + 7) & ~size_t(7);
    return dec + inb;
}

size_t bytes_per_wave(int S, int soft, int T) {
    switch (S) {
        case 2: return lds_bytes_per_wave<2>(soft, T);
        case 3: return lds_bytes_per_wave<3>(soft, T);
        case 4: return lds_bytes_per_wave<4>(soft, T);
        case 5: return lds_bytes_per_wave<5>(soft, T);
        case 6: return lds_bytes_per_wave<6>(soft, T);
        case 7: return lds_bytes_per_wave<7>(soft, T);
        case 8: return lds_bytes_per_wave<8>(soft, T);
        default: return 0;
    }
}

constexpr size_t kLdsLimit = 160 * 1024;
// GS: the workspace holds at most this many bytes of survivor words; a batch with more waves
// runs as several launches over the one workspace (stream-ordered)
constexpr size_t kGsWorkspaceCap = size_t(1) << 30;

int states_per_lane(int S) { return S <= 6 ? 1 : (1 << S) / 64; }
int frames_per_wave(int S) { return S >= 6 ? 1 : 64 >> S; }
size_t gs_bytes_per_wave(const Launch& a) { return (size_t)a.T * states_per_lane(a.S) * 8; }
size_t gs_waves(const Launch& a) { return (a.frames + frames_per_wave(a.S) - 1) / frames_per_wave(a.S); }
// Waves per launch: at most 1 GiB of survivor words, but never fewer than the CUs hold at once
// (32 per CU), and the launches of one batch balanced -- a remainder launch of a few waves runs a
// whole frame's dependent steps at low occupancy (K = 8, 4,096 x 16,384 bits: 4,094 + 2 waves
// took 5.5 ms against one launch's ~3.6)
size_t gs_waves_per_launch(const Launch& a) {
    const size_t floor_w = (size_t)(a.cus > 0 ? a.cus : 256) * 32;
    size_t cap = kGsWorkspaceCap / gs_bytes_per_wave(a);
    if (cap < floor_w) cap = floor_w;
    const size_t w = gs_waves(a);
    if (w <= cap) return w;
    const size_t launches = (w + cap - 1) / cap;
    return (w + launches - 1) / launches;
}

template <int S, bool SOFT>
hipError_t launch_typed(const Launch& a) {
    using Gm = Geometry<S>;
    if (lds_path_global(a)) {
        // one wave per block; launches of at most gs_waves_per_launch waves over the workspace
        const size_t per = gs_waves_per_launch(a), waves = gs_waves(a);
        const size_t lds = (size_t)Gm::F * kStage * (SOFT ? 2 : 1);
        for (size_t w0 = 0; w0 < waves; w0 += per) {
            const size_t nw = waves - w0 < per ? waves - w0 : per;
            const size_t f0 = w0 * Gm::F;
            const size_t nf = a.frames - f0 < nw * Gm::F ? a.frames - f0 : nw * Gm::F;
            hipLaunchKernelGGL((lds_path_kernel<S, SOFT, true>), dim3(unsigned(nw)), dim3(64), lds, a.stream,
                               a.in + f0 * a.in_stride, a.in_stride, a.out + f0 * a.out_stride, a.out_stride, a.T, a.L,
                               nf, 1, a);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    size_t per_wave = lds_bytes_per_wave<S>(SOFT, a.T);
    int wpb = int(kLdsLimit / per_wave);
    if (wpb > kWavesPerBlock) wpb = kWavesPerBlock;
    if (wpb < 1) return hipErrorInvalidValue;
    size_t frames_per_block = (size_t)wpb * Gm::F;
    size_t blocks = (a.frames + frames_per_block - 1) / frames_per_block;
    size_t lds = per_wave * wpb;
    auto kern = lds_path_kernel<S, SOFT, false>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(unsigned(blocks)), dim3(64 * wpb), lds, a.stream, a.in, a.in_stride, a.out,
                       a.out_stride, a.T, a.L, a.frames, wpb, a);
    return hipGetLastError();
}

template <bool SOFT>
hipError_t launch_soft(const Launch& a) {
    switch (a.S) {
        case 2: return launch_typed<2, SOFT>(a);
        case 3: return launch_typed<3, SOFT>(a);
        case 4: return launch_typed<4, SOFT>(a);
        case 5: return launch_typed<5, SOFT>(a);
        case 6: return launch_typed<6, SOFT>(a);
        case 7: return launch_typed<7, SOFT>(a);
        case 8: return launch_typed<8, SOFT>(a);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

bool lds_path_supported(const Launch& a) {
    // the GS variant takes every frame the LDS variant cannot hold
    return a.S >= 2 && a.S <= kMaxS && a.T > a.S && a.T <= VTB_MAX_FRAME_BITS + a.S;
}

// Which variant runs (measured on MI355X, 4,096-frame batches, K = 3..8 x L = 1,024..16,384,
// tools/generic_sweep.py, profiles/r06/generic/sweep_r06c_batched_walk_noscratch.jsonl): GS, whose
// waves need a few KB of LDS each (the CU holds every wave the batch gives it) and whose walks
// load kTb steps' words at once, ran at or above the LDS variant everywhere (K = 4, L = 4,096
// hard: 35.4 against 34.1 Gbit/s; K = 8, L = 4,096: 18.6 against 3.7, the LDS survivors cutting
// the CU to one wave) except for K = 3 frames of 2,048+ steps, where a lane's walk covers T / 4
// steps and the LDS variant fits the one wave per CU a 4,096-frame batch gives (L = 4,096 hard:
// 27.6 against 26.1).  So: the LDS variant for K <= 4 frames of T >= 2,048 steps while it leaves
// the CU the waves the batch needs, GS for everything else.
bool lds_path_global(const Launch& a) {
    if (a.dbg & kDbgGenericGs) return true;
    if (a.S >= 4 || a.T < 2048) return true;
    const size_t w = bytes_per_wave(a.S, a.soft, a.T);
    if (w == 0 || w > kLdsLimit) return true;
    const size_t cus = a.cus > 0 ? (size_t)a.cus : 256;
    size_t need = (gs_waves(a) + cus - 1) / cus;  // waves per CU the batch gives
    if (need > 8) need = 8;
    return kLdsLimit / w < need;
}

size_t lds_path_workspace_bytes(const Launch& a) {
    if (!lds_path_supported(a) || !lds_path_global(a) || a.frames == 0) return 0;
    return gs_waves_per_launch(a) * gs_bytes_per_wave(a);
}

hipError_t launch_lds_path(const Launch& a) {
    if (a.frames == 0) return hipSuccess;
    if (!lds_path_supported(a)) return hipErrorInvalidValue;
    if (lds_path_global(a) && !a.ws) return hipErrorInvalidValue;
    note_kernel(lds_path_global(a) ? "lds_path_gs" : "lds_path");
    return a.soft ? launch_soft<true>(a) : launch_soft<false>(a);
}

}  // namespace vtb
