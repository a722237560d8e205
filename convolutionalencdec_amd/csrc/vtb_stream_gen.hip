// Streaming decode (vtb_stream_*) for every constraint length the K=7 / K=9
// stream kernels do not cover (K = 3..9), on the generic trellis layout of vtb_lds_path.hip.
//
// The reference's chunked protocol (viterbiDecoderHardButterflyk1 with last=false, then
// last=true, src/viterbiDecoderButterflyk1.c:82-263) keeps metrics and survivors between
// calls and traces back only at `last`; its windowed traceback is a TODO (:195, 199).  Here a
// batch of streams advances in lockstep, one launch per call, and every stream emits the bits
// that became final during the call:
//   * ACS over the call's segments (all of them: no 48-step granularity, so no carry), one
//     wave per F = 64 / G streams on the register-resident trellis of vtb_gen_trellis.h
//     (locations rotate with the step; centred int32 metrics, strict '>' ties to the lower
//     predecessor, :129-130), decisions as one ballot word per register per step into a
//     per-wave survivor ring in global memory (step t at t mod W, bit = lane of the location);
//     a call may start at any phase (t_begin mod S), the metrics kept between calls by lane;
//   * not last: walks from all N states at the call's end go back one step at a time until
//     they stand on one state (step m); every survivor path passes through it, so no later
//     input can change the bits below m: they equal the whole-frame decode's and are emitted
//     by the verified block-parallel traceback of vtb_lds_path.hip over [e, hi), hi = m rounded
//     down to a whole number of bytes past e and at most the call's end minus K-1 (so the
//     terminating zero tail is never emitted early);
//   * last: the terminated traceback from state 0 at T emits [e, T - K + 1).
// Metrics are renormalised against state 0 at the end of every call (their spread is bounded),
// so a stream may run for any number of steps (< 2^30).  A stream that goes W steps without a
// merge has lost survivors it still needs: it reports -1 until `last`, then restarts.

#include "vtb_gen_trellis.h"

namespace vtb {
namespace {

using namespace gen;

template <int S>
using SGeo = Geometry<S>;

constexpr int kStage = 64;  // steps of input staged into LDS per round

template <int S, bool SOFT>
__global__ __launch_bounds__(64) void gen_stream_kernel(const uint8_t* __restrict__ in, size_t in_stride,
                                                        uint8_t* __restrict__ out, size_t out_stride, size_t streams,
                                                        Launch table, StreamArgs sa, uint64_t* __restrict__ ring,
                                                        int32_t* __restrict__ state) {
    using Gm = SGeo<S>;
    constexpr int N = Gm::N, G = Gm::G, R = Gm::R, F = Gm::F;
    constexpr int Q = SOFT ? 255 : 1;
    constexpr int INIT = int(uint8_t(N + 1)) * Q;  // (uint8_t)(NUM_STATES+1), reference :62
    constexpr int SB = SOFT ? 2 : 1;
    extern __shared__ uint8_t sm[];  // F x kStage x SB staged input bytes
    const int lane = threadIdx.x, fi = lane / G, lam = lane % G;
    const size_t f0 = size_t(blockIdx.x) * F, myf = f0 + fi;
    const bool real = myf < streams;
    const int W = sa.ring;
    uint64_t* rg = ring + size_t(blockIdx.x) * size_t(W) * R;
    int32_t* st = state + size_t(blockIdx.x) * gen_stream_state_words(S);
    const int C = sa.t_end - sa.t_begin;  // steps of this call

    // the lane's trellis constants; metrics by location (the carried ones were stored by lane at
    // the previous call's end, the same phase as this call's start)
    const unsigned l0 = lane_of<S>(unsigned(lam));
    Coef<S, R, SOFT> coef;
    setup_coef<S, R, SOFT>(table, l0, coef);
    int m[R];
#pragma unroll
    for (int r = 0; r < R; r++) m[r] = sa.t_begin == 0 ? ((unsigned(r) * 64u + l0 == 0) ? 0 : INIT) : st[r * 64 + lane];

    // ---- ACS over the call's steps ----
    // The call starts at phase t_begin mod S: a first chunk of the (S - phase) mod S steps up to
    // phase 0, then chunks of kChunk steps (whole phase cycles) run as static-phase cycles with
    // the next cycle's received pairs read ahead; the call's last partial cycle and the first
    // chunk step one at a time, the phase chosen per step.  The lane owning chunk step i keeps
    // its R decision words (v_writelane); one ring store per chunk.
    constexpr int kChunk = S * (kStage / S);
    uint32_t klo[R], khi[R];
#pragma unroll
    for (int r = 0; r < R; r++) klo[r] = khi[r] = 0;
    auto keep = [&](const uint64_t (&bal)[R], int i) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            klo[r] = uint32_t(vtb_writelane(int(uint32_t(bal[r])), i, int(klo[r])));
            khi[r] = uint32_t(vtb_writelane(int(uint32_t(bal[r] >> 32)), i, int(khi[r])));
        }
    };
    const int pro = (S - sa.t_begin % S) % S;
    for (int c0 = 0; c0 < C;) {
        const int n = c0 == 0 && pro > 0 ? (pro < C ? pro : C) : (C - c0 < kChunk ? C - c0 : kChunk);
        __syncthreads();
        for (int idx = lane; idx < F * n * SB; idx += 64) {
            const int f = idx / (n * SB), o = idx - f * (n * SB);
            const uint8_t v = f0 + f < streams ? in[(f0 + f) * in_stride + size_t(c0) * SB + o] : 0;
            sm[f * kStage * SB + o] = SOFT ? v : uint8_t(hard_offset(v));
        }
        __syncthreads();
        const uint8_t* my = sm + fi * kStage * SB;
        int i = 0;
        if ((sa.t_begin + c0) % S == 0 && n >= S) {
            auto load_q = [&](int at, int (&q)[S]) {
#pragma unroll
                for (int ph = 0; ph < S; ph++) q[ph] = rx_raw<SOFT>(my + (at + ph) * SB);
            };
            const int ncyc = n / S * S;
            int q[S];
            load_q(0, q);
#pragma unroll
            for (int ph = 0; ph < S; ph++) q[ph] = rx_pair<SOFT>(q[ph]);
            for (; i < ncyc; i += S) {
                int qn[S];
                load_q(i + S < ncyc ? i + S : i, qn);
                acs_cycle<S, R, SOFT>(m, q, coef, klo, khi, i);
#pragma unroll
                for (int ph = 0; ph < S; ph++) q[ph] = rx_pair<SOFT>(qn[ph]);
            }
        }
        for (; i < n; i++) {
            const int ph = (sa.t_begin + c0 + i) % S;
            const int qp = rx_pair<SOFT>(rx_raw<SOFT>(my + i * SB));
            uint64_t bal[R];
            gen_static_for(std::make_integer_sequence<int, S>{}, [&](auto pc) {
                constexpr int PH = decltype(pc)::value;
                if (ph == PH) rot_step<S, PH, R, SOFT>(m, qp, coef, bal);
            });
            keep(bal, i);
        }
        if (lane < n) {
            const size_t slot = size_t((sa.t_begin + c0 + lane) % W) * R;
#pragma unroll
            for (int r = 0; r < R; r++) rg[slot + r] = uint64_t(klo[r]) | (uint64_t(khi[r]) << 32);
        }
        c0 += n;
    }
    // renormalise against state 0 of the lane's stream, keep the metrics for the next call
    const int ref = __shfl(m[0], fi * G);
#pragma unroll
    for (int r = 0; r < R; r++) {
        m[r] -= ref;
        if (!sa.last) st[r * 64 + lane] = m[r];
    }
    __threadfence_block();  // the ring words of this call before any walk reads them
    __syncthreads();

    // the predecessor of state s after step t: the decision bit of s's location after step t
    auto pred = [&](unsigned s, int t) -> unsigned {
        const unsigned loc = rotr_s<S>(s, (t + 1) % S);
        const uint64_t w = rg[size_t(t % W) * R + (loc >> 6)];
        return (s >> 1) | (unsigned((w >> (fi * G + lane_of<S>(loc & unsigned(G - 1)))) & 1u) << (S - 1));
    };
    // the same from step t's R words (each word's bit taken before the select: no scratch array)
    auto pred_w = [&](unsigned s, int t, const uint64_t (&w)[R]) -> unsigned {
        const unsigned loc = rotr_s<S>(s, (t + 1) % S);
        const unsigned sh = unsigned(fi * G) + lane_of<S>(loc & unsigned(G - 1));
        unsigned x[R];
#pragma unroll
        for (int r = 0; r < R; r++) x[r] = unsigned(w[r] >> sh) & 1u;
        unsigned d = x[0];
        if constexpr (R == 2) d = (loc & 64u) ? x[1] : x[0];
        if constexpr (R == 4) {
            const unsigned lo2 = (loc & 64u) ? x[1] : x[0], hi2 = (loc & 64u) ? x[3] : x[2];
            d = (loc & 128u) ? hi2 : lo2;
        }
        return (s >> 1) | (d << (S - 1));
    };
    const int e0 = st[64 * R + fi];
    const int flags = st[64 * R + 32 + fi];
    const bool lost = flags != 0 || sa.t_end - e0 > W;
    const uint64_t fmask = (G == 64 ? ~uint64_t(0) : ((uint64_t(1) << G) - 1)) << (fi * G);

    int hi = e0;
    unsigned kloc = 0;
    if (sa.last) {
        hi = sa.t_end;
    } else {
        // merge test: walkers from every state at the call's end, one step back at a time,
        // until all walkers of a stream stand on one state (its last S steps excluded: the
        // zero tail of a frame that ends in the next call must not be emitted early)
        const int cap = sa.t_end - S;
        unsigned wk[R];
#pragma unroll
        for (int r = 0; r < R; r++) wk[r] = unsigned(r * G + lam);
        bool walking = real && !lost && cap > e0;
        int t = sa.t_end, sl = t % W;  // sl: ring slot of step t
        // the walkers' words of kMB steps loaded at once (they do not depend on the states, only
        // the bits taken from them do), then the kMB steps one at a time with their merge checks
        constexpr int kMB = R == 1 ? 8 : 4;
        while (__ballot(walking) != 0) {
            uint64_t w[kMB][R];
#pragma unroll
            for (int j = 0, s2 = sl; j < kMB; j++) {
                s2 = s2 == 0 ? W - 1 : s2 - 1;
#pragma unroll
                for (int r = 0; r < R; r++) w[j][r] = rg[size_t(s2) * R + r];
            }
#pragma unroll
            for (int j = 0; j < kMB; j++) {
                if (walking) {
                    t--;
                    sl = sl == 0 ? W - 1 : sl - 1;
#pragma unroll
                    for (int r = 0; r < R; r++) wk[r] = pred_w(wk[r], t, w[j]);
                }
                const unsigned r0 = unsigned(__shfl(int(wk[0]), fi * G));
                bool same = true;
#pragma unroll
                for (int r = 0; r < R; r++) same = same && wk[r] == r0;
                const bool merged = (__ballot(same) & fmask) == fmask;
                if (walking && merged) {
                    // every survivor path passes through state r0 at step t: bits below it are
                    // final; walk on to a whole number of bytes past e0 (and below the tail cap)
                    const int lim = t < cap ? t : cap;
                    const int h = e0 + (lim - e0) / 8 * 8;
                    unsigned s0 = r0;
                    for (int u = t - 1; u >= h; u--) s0 = pred(s0, u);
                    hi = h, kloc = s0;
                    walking = false;
                }
                if (walking && t <= e0) walking = false;
            }
        }
    }
    // emission of [e0, hi): the verified block-parallel traceback over the stream's G lanes
    // (vtb_gen_trellis.h traceback_span, location walks with the words of several steps loaded at
    // once; every lane calls it, so the cross-lane checks see the whole wave).  It ends in the
    // location of state kloc after step hi - 1 (state 0 at `last`); e0 is a multiple of 8.
    const int emit_end = sa.last ? sa.t_end - S : hi;  // bits past the terminated tail are not output
    const bool emits = real && !lost && hi > e0;
    // ring slot of step t in [e0, hi): t - wb, less W once past the ring's end (hi - e0 <= W)
    const int wb = e0 - e0 % W;
    traceback_span<S, R>(e0, emits ? hi : e0, emit_end, rotr_s<S>(kloc, hi % S), G, unsigned(fi * G),
                         out + myf * out_stride, (table.dbg & kDbgTbCap) != 0, table.guard_hits,
                         [&](int t, uint64_t (&w)[R]) {
                             const int d = t - wb;
                             const size_t slot = size_t(d >= W ? d - W : d) * R;
#pragma unroll
                             for (int r = 0; r < R; r++) w[r] = rg[slot + r];
                         });
    if (real && lam == 0) {
        sa.out_bits[myf] = lost ? -1 : (sa.last ? emit_end - e0 : hi - e0);
        st[64 * R + fi] = sa.last ? 0 : (lost ? e0 : hi);
        st[64 * R + 32 + fi] = sa.last ? 0 : (lost ? 1 : 0);
    }
}

template <int S, bool SOFT>
hipError_t launch_typed(const Launch& a, const StreamArgs& s) {
    using Gm = SGeo<S>;
    const size_t waves = (a.frames + Gm::F - 1) / Gm::F;
    const size_t lds = size_t(Gm::F) * kStage * (SOFT ? 2 : 1);
    hipLaunchKernelGGL((gen_stream_kernel<S, SOFT>), dim3(unsigned(waves)), dim3(64), lds, a.stream, a.in, a.in_stride,
                       a.out, a.out_stride, a.frames, a, s, static_cast<uint64_t*>(a.ws),
                       reinterpret_cast<int32_t*>(s.state));
    return hipGetLastError();
}

template <bool SOFT>
hipError_t launch_soft(const Launch& a, const StreamArgs& s) {
    switch (a.S) {
        case 2: return launch_typed<2, SOFT>(a, s);
        case 3: return launch_typed<3, SOFT>(a, s);
        case 4: return launch_typed<4, SOFT>(a, s);
        case 5: return launch_typed<5, SOFT>(a, s);
        case 6: return launch_typed<6, SOFT>(a, s);
        case 7: return launch_typed<7, SOFT>(a, s);
        case 8: return launch_typed<8, SOFT>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

size_t gen_stream_waves(int S, size_t streams) {
    const int N = 1 << S, G = N < 64 ? N : 64, F = 64 / G;
    return (streams + F - 1) / F;
}

size_t gen_stream_ring_bytes_per_step(int S) {
    const int N = 1 << S, G = N < 64 ? N : 64;
    return size_t(N / G) * 8;
}

hipError_t launch_gen_stream(const Launch& a, const StreamArgs& s) {
    if (a.frames == 0) return hipSuccess;
    if (!a.ws || !s.state || !s.out_bits || s.ring < 48 || a.S < 2 || a.S > kMaxS) return hipErrorInvalidValue;
    note_kernel("gen_stream");
    return a.soft ? launch_soft<true>(a, s) : launch_soft<false>(a, s);
}

}  // namespace vtb
