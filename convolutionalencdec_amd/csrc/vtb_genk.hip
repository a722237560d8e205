// General rate-k/n decoder (k input bits per trellis step).
//
// The reference's generic decoder (src/viterbiDecoder.c:52-234) defines the trellis: state =
// the last S = K-1 input segments (k bits each, newest in the low bits); destination d has
// 2^k predecessors src = d / 2^k + e * 2^((S-1)k) (:101-110), the edge label is the encoder
// output for delay (src << k) | (d mod 2^k) (:32-49 with convEncode.c:19-44, 132-161), the
// branch metric the Hamming distance to the received segment (:85-90), the survivor the
// first minimum (argmin2/4/8 with <=, convHelpers.h:40-63).  Its 5K-step register-exchange
// traceback in uint8 registers (:119-229) loses bits for k*5K > 8, so this decoder is
// terminated maximum likelihood with a full traceback from state 0 instead, exact int32
// metrics and the reference's start metrics 0 / (uint8)(N+1) (:236-262); the checker is
// oracle_genk_decode, and k = 1 reproduces the k=1 decoder bit for bit.
//
// One wave64 per frame.  The N = 2^(kS) <= 256 states spread over the lanes (state d in
// lane d % 64, register d / 64); metrics double-buffered in LDS (each lane gathers its 2^k
// predecessors with ds_read), decisions as k ballot words per register per step in LDS,
// edge labels from an LDS table of the N * 2^k delays.  A completeness kernel: these codes
// are not on the headline path, so it favours generality over the K=7 kernel's tricks.

#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include "viterbi_amd.h"
#include "vtb_internal.h"

namespace vtb {
namespace {

int gen_status() { return hipGetLastError() == hipSuccess ? VTB_OK : VTB_ERR_DEVICE; }

uint32_t gen_rev(uint64_t v, int bits) {  // convEncode.c:163-174
    uint32_t r = 0;
    for (int i = 0; i < bits; i++) r = (r << 1) | uint32_t((v >> i) & 1u);
    return r;
}

struct GenArgs {
    int k, S, n, N, T, L, R;
    int u8;          // VTB_GENK_K1_REFERENCE_U8: the reference's k=1 butterfly arithmetic (below)
    uint32_t rg[8];  // generators bit-reversed over k*K bits (convEncode.c:163-174)
};

// Wave-wide minimum of one value per lane (the U8 renormalisation, every 121 steps).
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, uint32_t(__shfl_xor(int(v), o)));
    return v;
}

struct GenLayout {  // LDS byte offsets
    size_t tab, met, inb, outb, dec, total;
};

GenLayout gen_layout(int N, int E, int T, int L, int R, int k, bool gdec) {
    GenLayout l;
    l.dec = 0;                                             // T * R * k u64 words (in LDS unless gdec)
    l.met = l.dec + (gdec ? 0 : 8 * size_t(T) * R * k);   // 2 * N int32
    l.tab = l.met + 8 * size_t(N);                   // N * E bytes
    l.inb = (l.tab + size_t(N) * E + 15) & ~size_t(15);  // T bytes
    l.outb = (l.inb + size_t(T) + 15) & ~size_t(15);     // ceil(L / 8) bytes
    l.total = (l.outb + size_t((L + 7) / 8) + 15) & ~size_t(15);
    return l;
}

// N <= 64 states: one state per lane, its metric in a register, the 2^k predecessors gathered
// with ds_bpermute, the lane's 2^k edge labels (time-invariant) in registers; k is a template
// parameter so every per-edge loop is unrolled.
//
// U8 (k = 1 only): the reference's k=1 butterfly arithmetic (viterbiDecoderButterflyk1.c:101-183)
// -- the upper predecessor's branch metric is n minus the lower's, whatever the generators
// (:104-107), sums wrap mod 256 (uint8 METRIC_TYPE), the strict '>' keeps the lower predecessor
// on ties (:129-130), and when the counter reaches 120 the minimum is subtracted (:159-183) --
// so that codes whose uint8 sums can wrap (n >= 4) decode exactly as the reference does.
template <int KB, bool U8 = false>
__device__ __forceinline__ void acs_r1(int N, int kS, int T, const uint8_t* inb, uint32_t nmask, const uint8_t* tab,
                                       int32_t* met, uint64_t* dec, int lane) {
    constexpr int E = 1 << KB;
    const int d = lane;
    const bool live = d < N;
    int32_t m = live ? met[d] : 0;
    uint32_t lab[E];
    int srcl[E];
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int src = live ? (d >> KB) | (e << (kS - KB)) : 0;
        srcl[e] = src << 2;
        if (U8)  // butterfly j = d >> 1: symm[j] = label of delay (j << 1) | 0, complemented for ec
            lab[e] = live ? uint32_t(tab[(d >> 1) << 1]) ^ ((((d & 1) ^ e) & 1) ? nmask : 0u) : 0u;
        else
            lab[e] = live ? uint32_t(tab[(src << KB) | (d & (E - 1))]) : 0u;
    }
    uint32_t renorm = 0;
    for (int t = 0; t < T; t++) {
        const uint32_t rx = inb[t] & nmask;
        uint32_t best = 0xFFFFFFFFu;
#pragma unroll
        for (int e = 0; e < E; e++) {
            uint32_t pm = uint32_t(__builtin_amdgcn_ds_bpermute(srcl[e], m)) + uint32_t(__popc(lab[e] ^ rx));
            if (U8) pm &= 0xFFu;
            best = min(best, (pm << 4) | uint32_t(e));
        }
        m = int32_t(best >> 4);
        if (U8) {
            if (renorm >= 120) {
                m -= int32_t(wave_min(live ? uint32_t(m) : 0xFFu));
                renorm = 0;
            } else {
                renorm++;
            }
        }
        const int be = int(best & 15u);
#pragma unroll
        for (int j = 0; j < KB; j++) {
            const uint64_t w = __ballot(live && ((be >> j) & 1));
            if (lane == j) dec[size_t(t) * KB + j] = w;
        }
    }
}

// N = 256 states (k * S = 8: k = 1, 2 or 4), four states per lane: d = 64 r + lane.  The
// 4 * 2^k edge labels of a lane's states are time-invariant and sit in registers (compile-time
// indices: k is a template parameter), the previous metrics in LDS (double-buffered).
template <int KB, bool U8 = false>
__device__ __forceinline__ void acs_r4(const GenArgs& a, int T, const uint8_t* inb, uint32_t nmask, const uint8_t* tab,
                                       int32_t* met, uint64_t* dec, int lane) {
    constexpr int E = 1 << KB, kS = 8, N = 256;
    uint32_t lab[4][E];
    int sbase[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int d = r * 64 + lane;
        sbase[r] = d >> KB;
#pragma unroll
        for (int e = 0; e < E; e++) {
            if (U8)  // the butterfly identity of acs_r1 U8
                lab[r][e] = uint32_t(tab[(d >> 1) << 1]) ^ ((((d & 1) ^ e) & 1) ? nmask : 0u);
            else
                lab[r][e] = uint32_t(tab[(((d >> KB) | (e << (kS - KB))) << KB) | (d & (E - 1))]);
        }
    }
    int cur = 0;
    uint32_t renorm = 0;
    for (int t = 0; t < T; t++) {
        const uint32_t rx = inb[t] & nmask;
        const int32_t* mc = met + cur * N;
        int32_t* mn = met + (cur ^ 1) * N;
        uint32_t nm[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            uint32_t best = 0xFFFFFFFFu;
#pragma unroll
            for (int e = 0; e < E; e++) {
                uint32_t pm = uint32_t(mc[sbase[r] | (e << (kS - KB))]) + uint32_t(__popc(lab[r][e] ^ rx));
                if (U8) pm &= 0xFFu;
                best = min(best, (pm << 4) | uint32_t(e));
            }
            nm[r] = best >> 4;
            const int be = int(best & 15u);
#pragma unroll
            for (int j = 0; j < KB; j++) {
                const uint64_t w = __ballot((be >> j) & 1);
                if (lane == j) dec[(size_t(t) * 4 + r) * KB + j] = w;
            }
        }
        if (U8) {
            if (renorm >= 120) {
                const uint32_t mn4 = wave_min(min(min(nm[0], nm[1]), min(nm[2], nm[3])));
#pragma unroll
                for (int r = 0; r < 4; r++) nm[r] -= mn4;
                renorm = 0;
            } else {
                renorm++;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; r++) mn[r * 64 + lane] = int32_t(nm[r]);
        cur ^= 1;
        __syncthreads();
    }
    (void)a;
}

// GDEC: decision words in a global workspace (one slot per frame of the launch) instead of
// LDS, for trellises whose words would hold the CU to one or two waves.
template <bool GDEC>
__global__ __launch_bounds__(64) void genk_kernel(const uint8_t* __restrict__ in, size_t in_stride,
                                                  uint8_t* __restrict__ out, size_t out_stride, size_t frames,
                                                  GenArgs a, GenLayout ly, uint64_t* __restrict__ ws) {
    extern __shared__ uint64_t gsm[];
    uint8_t* sm = reinterpret_cast<uint8_t*>(gsm);
    uint64_t* dec = GDEC ? ws + size_t(blockIdx.x) * size_t(a.T) * a.R * a.k : reinterpret_cast<uint64_t*>(sm + ly.dec);
    int32_t* met = reinterpret_cast<int32_t*>(sm + ly.met);
    uint8_t* tab = sm + ly.tab;
    uint8_t* inb = sm + ly.inb;
    uint8_t* outb = sm + ly.outb;
    const int lane = threadIdx.x;
    const size_t f = blockIdx.x;
    if (f >= frames) return;
    const int k = a.k, N = a.N, E = 1 << k, kS = k * a.S, T = a.T, R = a.R;
    const uint32_t nmask = (1u << a.n) - 1u;

    for (int i = lane; i < N * E; i += 64) {  // edge labels, index = delay (src << k) | bits
        uint32_t o = 0;
        for (int j = 0; j < a.n; j++) o |= (uint32_t(__popc(uint32_t(i) & a.rg[j])) & 1u) << j;
        tab[i] = uint8_t(o);
    }
    const uint8_t* row = in + f * in_stride;
    for (int i = lane; i < T; i += 64) inb[i] = row[i];
    for (int i = lane; i < (a.L + 7) / 8; i += 64) outb[i] = 0;
    const int32_t init = int32_t(uint8_t(N + 1));
    for (int d = lane; d < N; d += 64) met[d] = d == 0 ? 0 : init;
    __syncthreads();

    // Candidates carry their predecessor index: cand = (pm << 4) | e, so one min gives the
    // metric and the first minimum (lowest e among equal metrics, the reference's argmin).
    if (R == 1) {
        switch (k) {
            case 1:
                if (a.u8)
                    acs_r1<1, true>(N, kS, T, inb, nmask, tab, met, dec, lane);
                else
                    acs_r1<1>(N, kS, T, inb, nmask, tab, met, dec, lane);
                break;
            case 2: acs_r1<2>(N, kS, T, inb, nmask, tab, met, dec, lane); break;
            case 3: acs_r1<3>(N, kS, T, inb, nmask, tab, met, dec, lane); break;
            default: acs_r1<4>(N, kS, T, inb, nmask, tab, met, dec, lane); break;
        }
        __syncthreads();
    } else if (k == 1) {
        if (a.u8)
            acs_r4<1, true>(a, T, inb, nmask, tab, met, dec, lane);
        else
            acs_r4<1>(a, T, inb, nmask, tab, met, dec, lane);
    } else if (k == 2) {
        acs_r4<2>(a, T, inb, nmask, tab, met, dec, lane);
    } else {
        acs_r4<4>(a, T, inb, nmask, tab, met, dec, lane);
    }

    // Traceback from state 0 (terminated frame), block-parallel and verified (the K=7
    // kernel's scheme, vtb_k7_lds.hip): lane b walks steps [b tbb, (b+1) tbb) back from
    // kGenWarm steps past its block's end, starting from state 0 there (exact when the walk
    // starts at T).  A block is right if it entered on its successor's exit state and that
    // successor is proven; failed blocks re-walk from a proven successor until all are
    // proven.  Then every lane emits its block's bits (LDS atomic OR: blocks share bytes).
    {
        constexpr int kGenWarm = 96;
        auto pred = [&](int s, int t) {
            const uint64_t* w = dec + (size_t(t) * R + (s >> 6)) * k;
            int e = 0;
            for (int j = 0; j < k; j++) e |= int((w[j] >> (s & 63)) & 1u) << j;
            return (s >> k) | (e << (kS - k));
        };
        const int tbb = (T + 63) / 64, lo = lane * tbb, top = min(lo + tbb, T);
        const bool active = lo < T;
        const int start = min(top + kGenWarm, T);
        int s = 0;
        for (int t = start - 1; active && t >= top; t--) s = pred(s, t);
        int s_top = s;
        for (int t = top - 1; active && t >= lo; t--) s = pred(s, t);
        int fin = s;
        bool fixed = !active || start == T;
        for (int round = 0; round < 65; round++) {
            const int sf = __shfl_down(fin, 1);
            const bool ok = fixed || s_top == sf;
            const uint64_t bad = ~__ballot(ok);
            if (bad == 0) break;
            if (!ok && (bad >> (lane + 1)) == 0) {
                s_top = s = sf;
                for (int t = top - 1; t >= lo; t--) s = pred(s, t);
                fin = s;
                fixed = true;
            }
        }
        uint32_t* ow = reinterpret_cast<uint32_t*>(outb);
        uint32_t acc = 0;
        int wcur = -1;
        s = s_top;
        for (int t = top - 1; active && t >= lo; t--) {
            if (t < T - a.S) {
                const int seg = s & (E - 1);
                for (int j = 0; j < k; j++) {
                    if ((seg >> (k - 1 - j)) & 1) {
                        const int pos = t * k + j;
                        if ((pos >> 5) != wcur) {
                            if (acc) atomicOr(ow + wcur, acc);
                            wcur = pos >> 5, acc = 0;
                        }
                        acc |= 1u << (8 * ((pos >> 3) & 3) + 7 - (pos & 7));
                    }
                }
            }
            s = pred(s, t);
        }
        if (acc) atomicOr(ow + wcur, acc);
    }
    __syncthreads();
    uint8_t* orow = out + f * out_stride;  // (GDEC: each lane read the decision words its walks need)
    for (int i = lane; i < (a.L + 7) / 8; i += 64) orow[i] = outb[i];
}

}  // namespace
}  // namespace vtb

extern "C" {

int vtb_genk_decode_device(const vtb_genk_code_t* code, int32_t info_bits, const uint8_t* d_in, size_t in_stride,
                           uint8_t* d_out, size_t out_stride, size_t frames, void* stream) {
    if (!code || !d_in || !d_out) return VTB_ERR_INVALID;
    const int k = code->input_bits, K = code->constraint_length, n = code->coded_bits;
    if (k < 1 || K < 2 || n < 1 || n > 8) return VTB_ERR_INVALID;
    const int S = K - 1;
    if (k * S > 8 || k * K > 12) return VTB_ERR_UNSUPPORTED;  // N <= 256 states, N * 2^k <= 4096 labels
    for (int i = 0; i < n; i++)
        if (code->generators[i] == 0 || (code->generators[i] >> (k * K))) return VTB_ERR_INVALID;
    if (code->flags & ~int32_t(VTB_GENK_K1_REFERENCE_U8)) return VTB_ERR_INVALID;
    const bool u8 = code->flags & VTB_GENK_K1_REFERENCE_U8;
    if (u8 && k != 1) return VTB_ERR_INVALID;
    if (info_bits < 1 || info_bits % k || info_bits > VTB_MAX_FRAME_BITS) return VTB_ERR_INVALID;
    const int T = info_bits / k + S, N = 1 << (k * S), E = 1 << k, R = (N + 63) / 64;
    if (in_stride < size_t(T) || out_stride < size_t((info_bits + 7) / 8)) return VTB_ERR_INVALID;
    if (frames == 0) return VTB_OK;
    vtb::GenArgs a{};
    a.k = k, a.S = S, a.n = n, a.N = N, a.T = T, a.L = info_bits, a.R = R, a.u8 = u8 ? 1 : 0;
    for (int i = 0; i < n; i++) a.rg[i] = vtb::gen_rev(code->generators[i], k * K);
    // decision words in LDS while they leave room for 4 waves per CU, else in a workspace
    const size_t dec_bytes = 8 * size_t(T) * R * k;
    const bool gdec = dec_bytes > 32 * 1024;
    const vtb::GenLayout ly = vtb::gen_layout(N, E, T, info_bits, R, k, gdec);
    if (ly.total > 160 * 1024 || frames > 0x7fffffffu) return VTB_ERR_UNSUPPORTED;
    hipStream_t st = (hipStream_t)stream;
    vtb::note_kernel("genk");
    if (!gdec) {
        if (ly.total > 64 * 1024 &&
            hipFuncSetAttribute(reinterpret_cast<const void*>(vtb::genk_kernel<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, int(ly.total)) != hipSuccess)
            return VTB_ERR_DEVICE;
        hipLaunchKernelGGL(vtb::genk_kernel<false>, dim3(unsigned(frames)), dim3(64), ly.total, st, d_in, in_stride,
                           d_out, out_stride, frames, a, ly, nullptr);
        return vtb::gen_status();
    }
    // workspace from the stream's pool, up to 1 GiB per launch (frames in launches of that)
    const size_t per = std::max<size_t>(1, (size_t(1) << 30) / dec_bytes);
    const size_t chunk = std::min(frames, per);
    // (the per-device pool that keeps its memory between launches, vtb_api.hip workspace_alloc)
    void* ws = nullptr;
    if (vtb::workspace_alloc(&ws, chunk * dec_bytes, st) != hipSuccess) return VTB_ERR_NOMEM;
    int rc = VTB_OK;
    for (size_t f0 = 0; f0 < frames && rc == VTB_OK; f0 += chunk) {
        const size_t nf = std::min(chunk, frames - f0);
        hipLaunchKernelGGL(vtb::genk_kernel<true>, dim3(unsigned(nf)), dim3(64), ly.total, st, d_in + f0 * in_stride,
                           in_stride, d_out + f0 * out_stride, out_stride, nf, a, ly, static_cast<uint64_t*>(ws));
        rc = vtb::gen_status();
    }
    if (vtb::workspace_free(ws, st) != hipSuccess && rc == VTB_OK) rc = VTB_ERR_DEVICE;
    return rc;
}

}  // extern "C"
