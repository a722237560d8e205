// Generic gfx950 decoder for every K = 3..9 ("LDS path" kernel family): batch frames
// (lds_path_kernel) and single frames as segments (gen_seg_kernel), on the register-resident
// trellis of vtb_gen_trellis.h (DPP / permlane partners, one VALU compare per decision).
//
// Survivor words: the lane that owns step t mod C (C = P floor(64/P), P = the loop body's steps,
// a multiple of S: whole phase cycles) keeps the step's R words in registers (v_writelane) and
// the wave stores C steps' words at once, coalesced.  Two variants (template parameter GS;
// lds_path_global picks one):
//   * GS (global survivors, the default): the survivor words in a global workspace (8 R T bytes
//     per wave), the input staged through LDS C steps at a time (the next chunk loaded into
//     registers while this one runs), the traceback reading the words back from L2 / HBM.  Every
//     frame up to VTB_MAX_FRAME_BITS (the reference's MAX_PKT_LEN_UNCODED_BITS,
//     viterbiDecoder.h:18), at any K, hard or soft;
//   * LDS: the survivor words and the wave's whole input in LDS, 8 R T + F T B bytes per wave
//     (B = 1 hard, 2 soft), VTB_DEBUG bit 20 only.
// Decisions, metrics and traceback are the same code in both: the outputs are identical.
//
#include "vtb_gen_trellis.h"

namespace vtb {
namespace {

using namespace gen;

constexpr int kWavesPerBlock = 4;

template <int S, bool SOFT, bool GS>
__global__ __launch_bounds__(64 * kWavesPerBlock) void lds_path_kernel(const uint8_t* __restrict__ in, size_t in_stride,
                                                                        uint8_t* __restrict__ out, size_t out_stride,
                                                                        int T, int L, size_t frames, int waves_per_block,
                                                                        Launch table) {
    using Gm = Geometry<S>;
    constexpr int N = Gm::N, G = Gm::G, R = Gm::R, F = Gm::F, C = Gm::C;
    constexpr int Q = SOFT ? 255 : 1;
    constexpr int INIT = int(uint8_t(N + 1)) * Q;  // (uint8_t)(NUM_STATES+1), reference :62
    constexpr int B = SOFT ? 2 : 1;

    extern __shared__ uint64_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int fi = lane / G;
    const int lam = lane % G;

    constexpr int P = Gm::P, U = Gm::U;
    const int TS = (T + P - 1) / P * P;  // steps run: whole loop bodies (decisions past T unused)
    const size_t dec_words = (size_t)TS * R;
    uint64_t* dec;
    uint8_t* inbuf;
    int in_row;  // staged bytes per frame
    if constexpr (GS) {
        // one wave per block: the block's slot of the launch's workspace, the staging buffer in LDS
        dec = static_cast<uint64_t*>(table.ws) + (size_t)blockIdx.x * dec_words;
        inbuf = reinterpret_cast<uint8_t*>(smem);
        in_row = C * B;
    } else {
        in_row = TS * B;
        const size_t in_bytes = ((size_t)F * in_row + 7) & ~size_t(7);
        dec = smem + (size_t)wave * (dec_words + in_bytes / 8);
        inbuf = reinterpret_cast<uint8_t*>(dec + dec_words);
    }

    const size_t frame0 = ((size_t)blockIdx.x * waves_per_block + wave) * F;
    const size_t myframe = frame0 + fi;
    const bool valid = myframe < frames;

    const unsigned l0 = lane_of<S>(unsigned(lam));  // this lane's location (register 0)
    Coef<S, R, SOFT> coef;
    setup_coef<S, R, SOFT>(table, l0, coef);
    int m[R];
#pragma unroll
    for (int r = 0; r < R; r++) m[r] = unsigned(r) * 64u + l0 == 0 ? 0 : INIT;  // phase 0: location = state

    uint32_t klo[R], khi[R];  // lane i keeps the words of step c0 + i
#pragma unroll
    for (int r = 0; r < R; r++) klo[r] = khi[r] = 0;
    // the received pairs of the P steps at p (read one loop body ahead of their use: the LDS
    // latency off the recursion's chain)
    auto load_q = [&](const uint8_t* p, int (&q)[P]) {
#pragma unroll
        for (int j = 0; j < P; j++) q[j] = rx_raw<SOFT>(p + j * B);
    };

    const uint8_t* myin = inbuf + fi * in_row;
    if constexpr (!GS) {
        // the wave's input frames into LDS (coalesced byte loads; zero past T)
        for (int idx = lane; idx < F * in_row; idx += 64) {
            const int f = idx / in_row, off = idx - f * in_row;
            uint8_t v = 0;
            if (frame0 + f < frames && off < T * B) v = in[(frame0 + f) * in_stride + off];
            inbuf[idx] = SOFT ? v : uint8_t(hard_offset(v));
        }
        __syncthreads();
    }
    // GS: the input of the next C steps is loaded into registers (kPf bytes per lane) while this
    // chunk's steps run, and written to the other half of the staging buffer after them
    constexpr int kPf = (F * C * B + 63) / 64;
    uint32_t pf[GS ? kPf : 1];
    auto fetch = [&](int c0) {
#pragma unroll
        for (int j = 0; j < kPf; j++) {
            const int idx = lane + 64 * j, f = idx / (C * B), off = idx - f * (C * B), src = c0 * B + off;
            pf[j] = f < F && frame0 + f < frames && src < T * B ? in[(frame0 + f) * in_stride + (size_t)src] : 0u;
        }
    };
    auto commit = [&](uint8_t* buf) {
#pragma unroll
        for (int j = 0; j < kPf; j++)
            if (lane + 64 * j < F * C * B) buf[lane + 64 * j] = uint8_t(SOFT ? pf[j] : hard_offset(pf[j]));
    };
    if constexpr (GS) {
        fetch(0);
        commit(inbuf);
        __syncthreads();
    }
    for (int c0 = 0, k = 0; c0 < TS; c0 += C, k ^= 1) {
        const int n = TS - c0 < C ? TS - c0 : C;  // a multiple of S
        const uint8_t* base;
        if constexpr (GS) {
            if (c0 + C < TS) fetch(c0 + C);
            base = myin + k * (F * C * B);
        } else {
            base = myin + c0 * B;
        }
        int q[P];
        load_q(base, q);
#pragma unroll
        for (int j = 0; j < P; j++) q[j] = rx_pair<SOFT>(q[j]);
        for (int i = 0; i < n; i += P) {  // (n: a multiple of P)
            int qn[P];
            load_q(base + (i + P < n ? i + P : i) * B, qn);
#pragma unroll
            for (int u = 0; u < U; u++) acs_cycle<S, R, SOFT>(m, q + u * S, coef, klo, khi, i + u * S);
#pragma unroll
            for (int j = 0; j < P; j++) q[j] = rx_pair<SOFT>(qn[j]);
        }
        if (lane < n) {
#pragma unroll
            for (int r = 0; r < R; r++) dec[(size_t)(c0 + lane) * R + r] = uint64_t(klo[r]) | (uint64_t(khi[r]) << 32);
        }
        if constexpr (GS) {
            if (c0 + C < TS) {
                commit(inbuf + (k ^ 1) * (F * C * B));
                __syncthreads();
            }
        }
    }
    if constexpr (GS) __threadfence_block();  // the survivor words before any lane's traceback reads them

    __syncthreads();
    if (!valid) return;

    // the frame's G lanes trace it back (vtb_gen_trellis.h traceback_chains)
    traceback_chains<S, R>(T, L, G, unsigned(fi * G), out + myframe * out_stride, (table.dbg & kDbgTbCap) != 0,
                           table.guard_hits, [&](int t, uint64_t (&w)[R]) {
#pragma unroll
                               for (int r = 0; r < R; r++) w[r] = dec[(size_t)t * R + r];
                           });
}

template <int S>
size_t lds_bytes_per_wave(int soft, int T) {
    using Gm = Geometry<S>;
    const size_t TS = size_t(T + Geometry<S>::P - 1) / Geometry<S>::P * Geometry<S>::P;  // whole loop bodies
    size_t dec = TS * Gm::R * 8;
    size_t inb = ((size_t)Gm::F * TS * (soft ? 2 : 1) + 7) & ~size_t(7);
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
size_t gs_bytes_per_wave(const Launch& a) {
    const size_t P = size_t(body_steps(a.S));
    return (size_t(a.T) + P - 1) / P * P * states_per_lane(a.S) * 8;
}
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
        const size_t lds = 2 * (size_t)Gm::F * Gm::C * (SOFT ? 2 : 1);  // two staging halves
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


// ---------------- single-frame latency path for every K (gen_seg_kernel) ----------------
//
// vtb_decode_frame_sync for the codes without a SEG kernel of their own (K = 3..6, 8; K = 7 and
// K = 9 have k7_seg / k9_seg): one frame at a time is one dependent chain of T steps, so the frame
// is cut into G segments decoded at once by the F = 64 / min(N, 64) frame slots of each of up to
// eight waves of one workgroup -- or, for K = 6, 8, of several workgroups on one XCD whose rows and
// metric vectors go through a workspace to the last one to arrive (vtb_k9.hip's hand-over) -- on
// the batch kernel's trellis layout and arithmetic (vtb_gen_trellis.h).  Segment
// i runs n steps from g_i = i (n - warm); segment 0 starts from the reference's start metrics,
// the others from equal metrics.  Segment i's decisions are the frame's from s_i = g_i + warm on
// when its metric vector there equals segment i - 1's final one up to a constant (the trellis
// compares differences only; segment i - 1 is exact up to s_i by induction) -- vtb_k7_lds.hip's
// SEG argument.  n and warm are whole loop bodies (P steps, a multiple of S: every g_i is one, all
// slots of a wave share the phase, and the boundary compares happen at phase 0, where location =
// state).
// If every boundary holds, wave 0 traces the frame back over all segments' words (64 blocks,
// verified chains, completeness guard) and writes the bytes; else nothing is
// written and *done = 2 (the host decodes the frame with the batch kernel).  Input from and
// output to host-mapped memory, *done = 1 with a system-scope release at the end.
struct GenSeg {
    int n = 0, warm = 0, G = 0, W = 0;  // steps per segment, warm-up, segments, waves per workgroup
    int in_lds = 0;                     // LDS byte offset of the staged input, later the decoded bytes
                                        // (the frame's survivor rows, T R 8 bytes, from offset 0)
    int x_lds = 0;                      // exchange: final metrics [G][N], warm-up metrics [G][N], ok [G]
    uint32_t* done = nullptr;           // completion word (host-mapped) or null
    // several workgroups (nwg > 1): rows and metrics handed over in a workspace
    int nwg = 1;
    uint32_t* counter = nullptr;  // workgroups arrived; the last one resets it
    int32_t* gmet = nullptr;      // final metrics [G][N], warm-up metrics [G][N]
    uint64_t* grows = nullptr;    // the frame's survivor rows [T][R]
};

// Words handed from one workgroup to another inside a launch: global agent-scope relaxed
// accesses, i.e. sc1 stores and loads that bypass the per-CU L1 (cdna_hip_programming.md
// Guideline 16; vtb_k9.hip k9_seg_kernel)
typedef __attribute__((address_space(1))) uint32_t gen_gu32;
typedef __attribute__((address_space(1))) uint64_t gen_gu64;
__device__ __forceinline__ void st_agent32(int32_t* p, int32_t v) {
    __hip_atomic_store((gen_gu32*)(p), uint32_t(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t ld_agent32(const int32_t* p) {
    return int32_t(__hip_atomic_load((const gen_gu32*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_agent64(uint64_t* p, uint64_t v) {
    __hip_atomic_store((gen_gu64*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent64(const uint64_t* p) {
    return __hip_atomic_load((const gen_gu64*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kGenSegStage = 4;  // 16-byte staging loads per thread issued before their stores (v0..v3)

template <int S, bool SOFT>
__global__ __launch_bounds__(512) void gen_seg_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int T,
                                                      int L, Launch table, GenSeg sg) {
    using Gm = Geometry<S>;
    constexpr int N = Gm::N, G = Gm::G, R = Gm::R, F = Gm::F, C = Gm::C;
    constexpr int Q = SOFT ? 255 : 1;
    constexpr int INIT = int(uint8_t(N + 1)) * Q;  // reference :62
    constexpr int B = SOFT ? 2 : 1;
    extern __shared__ uint64_t smem[];
    uint8_t* sm = reinterpret_cast<uint8_t*>(smem);
    // several workgroups: all working ones on one XCD (grid stride 8, one L2 for the hand-over);
    // the others return at once
    const bool multi = sg.nwg > 1;
    if (multi && (blockIdx.x & 7u)) return;
    const int wg = multi ? int(blockIdx.x >> 3) : 0;
    const int wv = int(threadIdx.x >> 6), lane = int(threadIdx.x & 63);
    const int fi = lane / G, lam = lane % G;
    // Measurement only (Launch::tstamp, tools/tstamp_seg.py): wave 0's phase times, 100 MHz
    // ticks: 0 entry, 1 input staged, 2 steps done, 3 boundaries checked, 5 traceback done,
    // 6 output written; 7 = core clocks 0 to 6
    const uint64_t clk0 = table.tstamp ? __builtin_amdgcn_s_memtime() : 0;
    auto ts = [&](int k) {  // (several workgroups: 0-2 from workgroup 0, the rest from the last to arrive)
        if (table.tstamp && threadIdx.x == 0 && (k >= 3 || wg == 0)) table.tstamp[k] = __builtin_amdgcn_s_memrealtime();
    };
    ts(0);

    // the frame's input into LDS: rounds of up to four 16-byte loads per thread, all issued before
    // their stores (the host-mapped buffer is padded to 16 bytes)
    {
        const int nin = B * T, step = 16 * int(blockDim.x);
        // (loads past the frame read the buffer's last chunk again: clamped, never stored; named
        // registers, not an array, which the compiler placed in scratch)
        const int last = (nin - 1) & ~15;
        auto ld = [&](int o) { return *reinterpret_cast<const uint4*>(in + (o < nin ? o : last)); };
        auto stl = [&](int o, uint4 v) {
            if (!SOFT) v = make_uint4(hard_offset4(v.x), hard_offset4(v.y), hard_offset4(v.z), hard_offset4(v.w));
            if (o < nin) *reinterpret_cast<uint4*>(sm + sg.in_lds + o) = v;
        };
        for (int base = 16 * int(threadIdx.x); base < nin; base += kGenSegStage * step) {
            const uint4 v0 = ld(base), v1 = ld(base + step), v2 = ld(base + 2 * step), v3 = ld(base + 3 * step);
            stl(base, v0), stl(base + step, v1), stl(base + 2 * step, v2), stl(base + 3 * step, v3);
        }
    }
    __syncthreads();
    ts(1);

    const int gwv = wg * sg.W + wv;  // the wave's index over the workgroups
    const int seg = gwv * F + fi;    // this slot's segment
    const int sstep = sg.n - sg.warm;
    const int g0 = seg * sstep;  // a multiple of S
    const unsigned l0 = lane_of<S>(unsigned(lam));
    Coef<S, R, SOFT> coef;
    setup_coef<S, R, SOFT>(table, l0, coef);
    int m[R], mw[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        m[r] = seg == 0 ? (unsigned(r) * 64u + l0 == 0 ? 0 : INIT) : 0;
        mw[r] = m[r];
    }
    // survivor rows of the frame: step t's R words (this frame's G bits from bit 0) at row t,
    // written by the one segment whose decisions are the frame's there (segment 0: local steps
    // [0, n), segment i: [warm, n), i.e. [s_i, s_(i+1)))
    uint64_t* rows = reinterpret_cast<uint64_t*>(sm);
    const uint8_t* inb = sm + sg.in_lds;
    uint32_t klo[R], khi[R];
#pragma unroll
    for (int r = 0; r < R; r++) klo[r] = khi[r] = 0;
    // the received pairs of local steps t .. t + P - 1, read one loop body ahead of their use
    // (steps past the frame: any input, their decisions unused)
    constexpr int P = Gm::P, U = Gm::U;
    auto load_q = [&](int t, int (&q)[P]) {
#pragma unroll
        for (int j = 0; j < P; j++) {
            const int tg = g0 + t + j;
            q[j] = rx_raw<SOFT>(inb + (tg < T ? tg : T - 1) * B);
        }
    };
    int q[P];
    load_q(0, q);
#pragma unroll
    for (int j = 0; j < P; j++) q[j] = rx_pair<SOFT>(q[j]);
    for (int c0 = 0; c0 < sg.n; c0 += C) {
        const int nn = sg.n - c0 < C ? sg.n - c0 : C;  // a multiple of P
        for (int i = 0; i < nn; i += P) {
            int qn[P];
            load_q(c0 + i + P, qn);
#pragma unroll
            for (int u = 0; u < U; u++) acs_cycle<S, R, SOFT>(m, q + u * S, coef, klo, khi, i + u * S);
#pragma unroll
            for (int j = 0; j < P; j++) q[j] = rx_pair<SOFT>(qn[j]);
            if (c0 + i + P == sg.warm) {
#pragma unroll
                for (int r = 0; r < R; r++) mw[r] = m[r];
            }
        }
        // each of the wave's F slots' G bits of the words of steps c0 .. c0 + nn - 1
#pragma unroll
        for (int f = 0; f < F; f++) {
            const int si = gwv * F + f, lt = c0 + lane, t = si * sstep + lt;
            if (si < sg.G && lane < nn && (si == 0 || lt >= sg.warm) && t < T) {
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const uint64_t w = uint64_t(klo[r]) | (uint64_t(khi[r]) << 32);
                    const uint64_t v = G == 64 ? w : (w >> (f * G)) & ((uint64_t(1) << (G & 63)) - 1);
                    if (multi) {
                        st_agent64(sg.grows + size_t(t) * R + r, v);
                    } else {
                        rows[size_t(t) * R + r] = v;
                    }
                }
            }
        }
    }

    ts(2);
    // boundary checks: segment i's metrics after its warm-up against segment i - 1's final
    // metrics, equal up to a constant (both at phase 0: index = location = state)
    int32_t* xf = reinterpret_cast<int32_t*>(sm + sg.x_lds);
    int32_t* xw = xf + sg.G * N;
    uint32_t* okf = reinterpret_cast<uint32_t*>(xw + sg.G * N);
    bool all = true;
    if (!multi) {
        // one workgroup: the vectors exchanged in LDS, one check per slot
        if (seg < sg.G) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                xf[seg * N + r * 64 + int(l0)] = m[r];
                xw[seg * N + r * 64 + int(l0)] = mw[r];
            }
        }
        __syncthreads();
        const uint64_t fmask = (G == 64 ? ~uint64_t(0) : ((uint64_t(1) << (G & 63)) - 1)) << (fi * G);
        {
            bool same = true;
            if (seg >= 1 && seg < sg.G) {
                const int d0 = xf[(seg - 1) * N] - xw[seg * N];  // state 0
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const int d = r * 64 + int(l0);
                    same = same && xf[(seg - 1) * N + d] - xw[seg * N + d] == d0;
                }
            }
            const bool ok = (__ballot(same) & fmask) == fmask;
            if (lam == 0 && seg < sg.G) okf[seg] = ok ? 1u : 0u;
        }
        __syncthreads();
        if (wv != 0) return;  // (no barrier follows)
        for (int i = 0; i < sg.G; i++) all = all && okf[i] != 0u;
    } else {
        // several workgroups: the vectors and the rows go through the workspace (sc1 stores,
        // drained before the barrier); the last workgroup to arrive (one atomic add per
        // workgroup, nobody waits) copies the rows into its LDS and checks every boundary
        if (seg < sg.G) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                st_agent32(sg.gmet + size_t(seg) * N + r * 64 + int(l0), m[r]);
                st_agent32(sg.gmet + size_t(sg.G + seg) * N + r * 64 + int(l0), mw[r]);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
            okf[0] = __hip_atomic_fetch_add((gen_gu32*)(sg.counter), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                             uint32_t(sg.nwg - 1)
                         ? 1u
                         : 0u;
        __syncthreads();
        if (okf[0] == 0u) return;  // (the whole workgroup: no barrier follows for it)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (orders the loads after the election)
        // (every load of the hand-over issued before any use: one L2 round trip in all -- the
        // boundary metrics of up to kBw boundaries per wave, then the rows into LDS)
        constexpr int kBw = 8;  // boundaries a wave checks at once
        bool ok = true;
        for (int i0 = 1 + wv; i0 < sg.G; i0 += kBw * sg.W) {
            int dx[kBw][R];
#pragma unroll
            for (int k = 0; k < kBw; k++) {
                const int i = i0 + k * sg.W;
                const int32_t* pf = sg.gmet + size_t(i - 1) * N;     // segment i - 1: final
                const int32_t* pw = sg.gmet + size_t(sg.G + i) * N;  // segment i: warm-up end
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const int l = r * 64 + lane;
                    dx[k][r] = i < sg.G && l < N ? ld_agent32(pf + l) - ld_agent32(pw + l) : 0;
                }
            }
            if (i0 == 1 + wv) {  // (the first group's loads in flight: the rows too)
                const int bd = int(blockDim.x), TR = T * R;
                for (int k = int(threadIdx.x); k < TR; k += 4 * bd) {
                    uint64_t v[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) v[j] = k + j * bd < TR ? ld_agent64(sg.grows + k + j * bd) : 0;
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (k + j * bd < TR) rows[k + j * bd] = v[j];
                }
            }
#pragma unroll
            for (int k = 0; k < kBw; k++) {
                const int d0 = __shfl(dx[k][0], 0);  // state 0
                bool same = true;
#pragma unroll
                for (int r = 0; r < R; r++) same = same && (r * 64 + lane >= N || dx[k][r] == d0);
                ok = ok && (i0 + k * sg.W >= sg.G || __ballot(!same) == 0);
            }
        }
        if (1 + wv >= sg.G) {  // (a wave without boundaries still copies its share of the rows)
            const int bd = int(blockDim.x), TR = T * R;
            for (int k = int(threadIdx.x); k < TR; k += 4 * bd) {
                uint64_t v[4];
#pragma unroll
                for (int j = 0; j < 4; j++) v[j] = k + j * bd < TR ? ld_agent64(sg.grows + k + j * bd) : 0;
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (k + j * bd < TR) rows[k + j * bd] = v[j];
            }
        }
        if (lane == 0) okf[1 + wv] = ok ? 1u : 0u;
        __syncthreads();
        if (wv != 0) return;  // (no barrier follows)
        for (int i = 0; i < sg.W; i++) all = all && okf[1 + i] != 0u;
        if (lane == 0) __hip_atomic_store((gen_gu32*)(sg.counter), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    ts(3);
    if (!all) {
        if (sg.done && lane == 0) __hip_atomic_store(sg.done, 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }

    // ---- traceback, wave 0: one chain of 64 blocks over [0, T) (the global phase of a step is
    // its local one: g_i = 0 mod S), the bytes into LDS (the input is no longer needed) ----
    uint8_t* ob = sm + sg.in_lds;
    traceback_chains<S, R>(T, L, 64, 0u, ob, (table.dbg & kDbgTbCap) != 0, table.guard_hits,
                           [&](int t, uint64_t (&w)[R]) {
#pragma unroll
                               for (int r = 0; r < R; r++) w[r] = rows[size_t(t) * R + r];
                           });
    ts(5);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int nbytes = (L + 7) >> 3;
    if (((nbytes | int(size_t(out) & 3)) & 3) == 0) {
        for (int i = lane; i < (nbytes >> 2); i += 64) reinterpret_cast<uint32_t*>(out)[i] = reinterpret_cast<const uint32_t*>(ob)[i];
    } else {
        for (int i = lane; i < nbytes; i += 64) out[i] = ob[i];
    }
    if (table.tstamp) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ts(6);
        if (threadIdx.x == 0) table.tstamp[7] = __builtin_amdgcn_s_memtime() - clk0;
    }
    if (sg.done) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(sg.done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Segments and LDS of the single-frame path for S = a.S at `waves` waves per workgroup, `nwg`
// workgroups and warm-up `warm` (rounded up to whole loop bodies): the most segments (up to
// nwg x waves x F, at most gen_seg_max, whose boundaries must all converge) that leave each at
// least kGenSegMin new steps.  One workgroup: K <= 4 codes forget their start within a few
// steps, 64 segments (K = 3 2,048-bit frames: 80 steps per segment instead of 112), 32 above.
// Several workgroups (K = 6, 8: the slots of one workgroup give 16 / 8 segments): up to 64.
constexpr int kGenSegMin = 32;
constexpr int gen_seg_max(int S, int nwg) { return nwg > 1 || S <= 3 ? 64 : 32; }
bool gen_seg_geometry(const Launch& a, int waves, int nwg, int warm, GenSeg& g, size_t& lds) {
    if (a.S < 2 || a.S > kMaxS || a.S == 6 || a.S == 8 || waves < 1 || waves > 8 || nwg < 1 || nwg > 8 || warm < 1)
        return false;
    const int S = a.S, T = a.T, F = frames_per_wave(S), R = states_per_lane(S), N = 1 << S;
    const int P = body_steps(S);
    warm = (warm + P - 1) / P * P;
    int G = waves * F * nwg;
    if (G > gen_seg_max(S, nwg)) G = gen_seg_max(S, nwg);
    const int cap = (T - warm) / kGenSegMin;
    if (G > cap) G = cap;
    if (G < 2) return false;  // (too short to be worth segments: the batch kernel)
    int sstep = (T - warm + G - 1) / G;
    sstep = (sstep + P - 1) / P * P;
    G = (T - warm + sstep - 1) / sstep;  // (the rounding may leave the last segments nothing to cover: dropped,
    if (G < 2) return false;             // a segment past the frame would run on clamped input and need not converge)
    const int n = sstep + warm;
    if (G * sstep + warm < T) return false;
    const int tw = (G + F - 1) / F;  // waves the segments need
    g.n = n, g.warm = warm, g.G = G;
    if (nwg > 1) {
        g.W = waves, g.nwg = (tw + waves - 1) / waves;
        if (g.nwg < 2) return false;  // (one workgroup holds them: the single-workgroup form)
    } else {
        g.W = tw, g.nwg = 1;
    }
    g.in_lds = (T * R * 8 + 15) / 16 * 16;
    const int nin = (a.soft ? 2 : 1) * T;
    g.x_lds = g.in_lds + (nin + 15) / 16 * 16;
    const size_t x = size_t(2 * G * N) * 4 + size_t(G) * 4;  // (several workgroups: 1 + W flags)
    lds = size_t(g.x_lds) + (x > 36 ? x : 36);
    if (lds > kLdsLimit || (T + 7) / 8 > nin) return false;
    // several workgroups: more than half a CU's LDS each, so that no two share a CU's SIMDs
    if (g.nwg > 1 && lds < kLdsLimit / 2 + 1024) lds = kLdsLimit / 2 + 1024;
    return true;
}

// workspace of the several-workgroup form: arrival counter, metrics, the frame's rows
size_t gen_seg_ws_bytes(const Launch& a, const GenSeg& g) {
    const size_t N = size_t(1) << a.S;
    return 256 + (size_t(2) * g.G * N * 4 + 255) / 256 * 256 + size_t(a.T) * states_per_lane(a.S) * 8;
}

template <int S, bool SOFT>
hipError_t launch_gen_seg_typed(const Launch& a, const GenSeg& g, size_t lds) {
    auto kern = gen_seg_kernel<S, SOFT>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                           int(lds));
        if (e != hipSuccess) return e;
    }
    // several workgroups: placed 8 apart (round-robin over the XCDs: all on one XCD)
    const unsigned grid = g.nwg > 1 ? unsigned(8 * g.nwg) : 1u;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * g.W), lds, a.stream, a.in, a.out, a.T, a.L, a, g);
    return hipGetLastError();
}

}  // namespace

bool gen_seg_supported(const Launch& a, int waves, int nwg, int warm) {
    GenSeg g;
    size_t lds = 0;
    return gen_seg_geometry(a, waves, nwg, warm, g, lds);
}

size_t gen_seg_workspace_bytes(const Launch& a, int waves, int nwg, int warm) {
    GenSeg g;
    size_t lds = 0;
    if (nwg < 2 || !gen_seg_geometry(a, waves, nwg, warm, g, lds)) return 0;
    return gen_seg_ws_bytes(a, g);
}

hipError_t launch_gen_seg(const Launch& a, int waves, int nwg, int warm, uint32_t* done) {
    GenSeg g;
    size_t lds = 0;
    if (a.frames != 1 || !gen_seg_geometry(a, waves, nwg, warm, g, lds)) return hipErrorInvalidValue;
    g.done = done;
    if (g.nwg > 1) {
        if (!a.ws) return hipErrorInvalidValue;
        uint8_t* base = static_cast<uint8_t*>(a.ws);
        const size_t N = size_t(1) << a.S;
        g.counter = reinterpret_cast<uint32_t*>(base);
        g.gmet = reinterpret_cast<int32_t*>(base + 256);
        g.grows = reinterpret_cast<uint64_t*>(base + 256 + (size_t(2) * g.G * N * 4 + 255) / 256 * 256);
    }
    note_kernel("gen_seg");
    switch (a.S * 2 + (a.soft ? 1 : 0)) {
        case 4: return launch_gen_seg_typed<2, false>(a, g, lds);
        case 5: return launch_gen_seg_typed<2, true>(a, g, lds);
        case 6: return launch_gen_seg_typed<3, false>(a, g, lds);
        case 7: return launch_gen_seg_typed<3, true>(a, g, lds);
        case 8: return launch_gen_seg_typed<4, false>(a, g, lds);
        case 9: return launch_gen_seg_typed<4, true>(a, g, lds);
        case 10: return launch_gen_seg_typed<5, false>(a, g, lds);
        case 11: return launch_gen_seg_typed<5, true>(a, g, lds);
        case 14: return launch_gen_seg_typed<7, false>(a, g, lds);
        case 15: return launch_gen_seg_typed<7, true>(a, g, lds);
        default: return hipErrorInvalidValue;
    }
}

bool lds_path_supported(const Launch& a) {
    // the GS variant takes every frame the LDS variant cannot hold
    return a.S >= 2 && a.S <= kMaxS && a.T > a.S && a.T <= VTB_MAX_FRAME_BITS + a.S;
}

// Which variant runs (measured on MI355X, 4,096-frame batches, K = 3..8 x L = 1,024..16,384,
// tools/generic_sweep.py): with the bpermute trellis (profiles/r06/generic/
// sweep_r06c_batched_walk_noscratch.jsonl) the LDS variant won for K = 3, 4 frames of 2,048+ steps;
// with the register-resident trellis and the prefetched staging (sweep_r06f_rot_pf.jsonl) GS runs
// at or above it everywhere (K = 3, L = 4,096 hard: 48.3 against 34.5 Gbit/s; K = 4: 57.3 against
// 45.9) -- the LDS survivors cap the waves per CU, GS's few KB do not.  So GS, and the LDS variant
// only when VTB_DEBUG bit 20 asks for it (tests; it stays exact and selectable).
bool lds_path_global(const Launch& a) {
    if (a.dbg & kDbgGenericGs) return true;
    if (!(a.dbg & kDbgGenericLds)) return true;
    const size_t w = bytes_per_wave(a.S, a.soft, a.T);
    return w == 0 || w > kLdsLimit;
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
