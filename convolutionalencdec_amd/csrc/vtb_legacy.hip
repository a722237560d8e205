// Kernels and entry points behind the legacy API's per-call semantics
// (include/viterbiDecoder.h, csrc/legacy/viterbiDecoder.c):
//
//  * vtb_legacy_metrics_k1 / vtb_legacy_metrics_genk: the reference decoder's forward pass
//    over one last=false chunk, so that a caller reading nodeMetricsCur between calls
//    (handTracedTest/handTraced.c:72-111 reads it; viterbiDecoderButterflyk1.c:189-191 and
//    viterbiDecoder.c:91-131 keep it current) sees the reference's values.  The k=1 form
//    keeps the reference's uint8 arithmetic exactly -- wrapping sums, the strict '>' select
//    (:129-130) and the subtract-the-minimum renormalisation when the counter reaches 120
//    (:159-183) -- because those uint8 values, not the exact metrics, are what the caller
//    sees.  The generic form is the destination-indexed update with exact metrics and the
//    first minimum over the 2^k predecessors (argminPathMetrics, convHelpers.h:40-63).
//  * vtb_genk_decode_frame_legacy: one general-k frame from host memory for
//    VITERBI_DECODER_HARD with k > 1 (viterbiDecoder.h:91-94 -> viterbiDecoderHard).
//
// Latency-bound single-stream work: one workgroup of up to 256 lanes (one per state),
// metrics double-buffered in LDS, a barrier per trellis step.  The hot batch path is
// vtb_k7_lds.hip / vtb_k9.hip; these kernels only serve callers of the per-frame API.

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "viterbi_amd.h"
#include "vtb_internal.h"

namespace vtb {
namespace {

struct FwdArgs {
    int butterfly;   // 1: k=1 butterfly in uint8 with renormalisation; 0: generic, exact
    int k, S, n, N;  // input bits per step, state segments, coded bits, states
    int count;       // segments this call
    uint32_t rg[8];  // generators bit-reversed over k*K bits (convEncode.c:163-174)
};

__global__ __launch_bounds__(256) void legacy_forward_kernel(const uint8_t* __restrict__ seg, uint32_t* met,
                                                             uint32_t* counter, FwdArgs a) {
    __shared__ uint32_t m[2][256];
    __shared__ uint8_t lab[4096];  // edge label of delay (src << k) | e
    __shared__ uint32_t mn;
    const int tid = threadIdx.x, N = a.N, k = a.k, E = 1 << k, kS = k * a.S;
    const uint32_t nmask = (1u << a.n) - 1u;
    for (int i = tid; i < N * E; i += blockDim.x) {
        uint32_t o = 0;
        for (int j = 0; j < a.n; j++) o |= (uint32_t(__popc(uint32_t(i) & a.rg[j])) & 1u) << j;
        lab[i] = uint8_t(o);
    }
    if (tid < N) m[0][tid] = met[tid];
    uint32_t cnt = a.butterfly ? *counter : 0;
    __syncthreads();
    int cur = 0;
    for (int t = 0; t < a.count; t++) {
        const uint32_t rx = seg[t];
        const uint32_t* mc = m[cur];
        if (tid < N) {
            uint32_t nm;
            if (a.butterfly) {
                // destination d = 2j + b of butterfly j (sources j, j + N/2); edge metric of the
                // symmetric label (viterbiDecoderButterflyk1.c:104-107), all sums in uint8
                const int j = tid >> 1;
                const uint32_t em = uint32_t(__popc((uint32_t(lab[j << 1]) ^ rx) & nmask));
                const uint32_t ec = (uint32_t(a.n) - em) & 0xFFu;
                const uint32_t x0 = (mc[j] + ((tid & 1) ? ec : em)) & 0xFFu;
                const uint32_t x1 = (mc[j + N / 2] + ((tid & 1) ? em : ec)) & 0xFFu;
                nm = x0 > x1 ? x1 : x0;
            } else {
                const int bits = tid & (E - 1);
                nm = 0;
                for (int e = 0; e < E; e++) {
                    const int src = (tid >> k) | (e << (kS - k));
                    const uint32_t pm = mc[src] + uint32_t(__popc((uint32_t(lab[(src << k) | bits]) ^ rx) & nmask));
                    if (e == 0 || pm < nm) nm = pm;  // first minimum
                }
            }
            m[cur ^ 1][tid] = nm;
        }
        if (a.butterfly) {
            if (tid == 0) mn = 0xFFu;
            __syncthreads();
            if (cnt >= 120) {  // renormalise: subtract the minimum of the new metrics
                if (tid < N) atomicMin(&mn, m[cur ^ 1][tid]);
                __syncthreads();
                if (tid < N) m[cur ^ 1][tid] -= mn;
                cnt = 0;
            } else {
                cnt++;
            }
        }
        cur ^= 1;
        __syncthreads();
    }
    if (tid < N) {
        met[tid] = m[cur][tid];
        met[N + tid] = m[cur ^ 1][tid];  // one step earlier (count >= 1)
    }
    if (a.butterfly && tid == 0) *counter = cnt;
}

uint32_t rev_bits(uint64_t v, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; i++) r = (r << 1) | uint32_t((v >> i) & 1u);
    return r;
}

// Per-host-thread device context of the legacy entry points (the reference API is reentrant
// per state struct; one context per calling thread keeps threads independent).
struct Ctx {
    int device = -1;
    hipStream_t stream = nullptr;
    uint8_t* d_seg = nullptr;  // segments, grown on demand
    size_t seg_cap = 0;
    uint32_t* d_met = nullptr;  // 2 * 256 metrics + counter
    uint8_t* d_out = nullptr;   // general-k frame output
    size_t out_cap = 0;
    void release() {
        if (device >= 0) {
            int prev = -1;
            (void)hipGetDevice(&prev);
            (void)hipSetDevice(device);
            if (stream) (void)hipStreamSynchronize(stream);
            if (d_seg) (void)hipFree(d_seg);
            if (d_met) (void)hipFree(d_met);
            if (d_out) (void)hipFree(d_out);
            if (stream) (void)hipStreamDestroy(stream);
            if (prev >= 0) (void)hipSetDevice(prev);
        }
        device = -1;
        stream = nullptr;
        d_seg = d_out = nullptr;
        d_met = nullptr;
        seg_cap = out_cap = 0;
    }
    ~Ctx() { release(); }
};

int legacy_device() {
    const char* s = std::getenv("VTB_LEGACY_DEVICE");
    return s ? std::atoi(s) : 0;
}

// Bind the calling thread's context to the legacy device with room for `segs` segments and
// `outb` output bytes.  On any failure the context is released (no half-built state).
int ctx_ready(Ctx& c, size_t segs, size_t outb) {
    const int dev = legacy_device();
    if (c.device != dev) {
        c.release();
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || dev < 0 || dev >= ndev) return VTB_ERR_DEVICE;
        if (!device_is_gfx950(dev)) return VTB_ERR_DEVICE;
        if (hipSetDevice(dev) != hipSuccess) return VTB_ERR_DEVICE;
        c.device = dev;
        if (hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) != hipSuccess ||
            hipMalloc(&c.d_met, (2 * 256 + 1) * sizeof(uint32_t)) != hipSuccess) {
            c.release();
            return VTB_ERR_NOMEM;
        }
    } else if (hipSetDevice(dev) != hipSuccess) {
        return VTB_ERR_DEVICE;
    }
    if (segs > c.seg_cap) {
        if (c.d_seg) (void)hipFree(c.d_seg);
        c.d_seg = nullptr;
        c.seg_cap = 0;
        if (hipMalloc(&c.d_seg, segs) != hipSuccess) {
            c.release();
            return VTB_ERR_NOMEM;
        }
        c.seg_cap = segs;
    }
    if (outb > c.out_cap) {
        if (c.d_out) (void)hipFree(c.d_out);
        c.d_out = nullptr;
        c.out_cap = 0;
        if (hipMalloc(&c.d_out, outb) != hipSuccess) {
            c.release();
            return VTB_ERR_NOMEM;
        }
        c.out_cap = outb;
    }
    return VTB_OK;
}

thread_local Ctx g_ctx;

struct PrevDevice {
    int prev = -1;
    PrevDevice() {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~PrevDevice() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Run the forward kernel over host segments; metrics (N in, N + N out) and the counter
// through the context's device buffer.
int run_forward(const FwdArgs& a, const uint8_t* segments, uint32_t* met_io, uint32_t* prev, uint32_t* counter) {
    PrevDevice keep;
    Ctx& c = g_ctx;
    int r = ctx_ready(c, size_t(a.count > 0 ? a.count : 1), 0);
    if (r != VTB_OK) return r;
    const size_t mb = size_t(a.N) * sizeof(uint32_t);
    uint32_t* d_cnt = c.d_met + 2 * 256;
    uint32_t tmp[512];
    // every error exit after the first asynchronous copy drains the stream first: queued copies
    // still read the caller's buffers and write tmp (this frame)
    auto fail = [&]() {
        (void)hipStreamSynchronize(c.stream);
        return VTB_ERR_DEVICE;
    };
    if (hipMemcpyAsync(c.d_seg, segments, size_t(a.count), hipMemcpyHostToDevice, c.stream) != hipSuccess ||
        hipMemcpyAsync(c.d_met, met_io, mb, hipMemcpyHostToDevice, c.stream) != hipSuccess ||
        (counter && hipMemcpyAsync(d_cnt, counter, sizeof(uint32_t), hipMemcpyHostToDevice, c.stream) != hipSuccess))
        return fail();
    const int threads = a.N < 64 ? 64 : a.N;
    hipLaunchKernelGGL(legacy_forward_kernel, dim3(1), dim3(threads), 0, c.stream, c.d_seg, c.d_met, d_cnt, a);
    if (hipGetLastError() != hipSuccess) return fail();
    if (hipMemcpyAsync(tmp, c.d_met, 2 * mb, hipMemcpyDeviceToHost, c.stream) != hipSuccess ||
        (counter && hipMemcpyAsync(counter, d_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream) != hipSuccess) ||
        hipStreamSynchronize(c.stream) != hipSuccess)
        return fail();
    std::memcpy(met_io, tmp, mb);
    if (prev) std::memcpy(prev, tmp + a.N, mb);
    return VTB_OK;
}

}  // namespace
}  // namespace vtb

extern "C" {

int vtb_legacy_metrics_k1(const vtb_code_t* code, const uint8_t* segments, int32_t count, uint8_t* metrics,
                          uint32_t* renorm_counter) {
    if (!code || !metrics || !renorm_counter || count < 0 || (count > 0 && !segments)) return VTB_ERR_INVALID;
    const int K = code->constraint_length;
    if (K < VTB_MIN_K || K > VTB_MAX_K || code->coded_bits != 2) return VTB_ERR_UNSUPPORTED;
    for (int i = 0; i < 2; i++)
        if (code->generators[i] >> K) return VTB_ERR_INVALID;
    if (count == 0) return VTB_OK;
    vtb::FwdArgs a{};
    a.butterfly = 1, a.k = 1, a.S = K - 1, a.n = 2, a.N = 1 << (K - 1), a.count = count;
    for (int i = 0; i < 2; i++) a.rg[i] = vtb::rev_bits(code->generators[i], K);
    uint32_t m[256];
    for (int s = 0; s < a.N; s++) m[s] = metrics[s];
    int r = vtb::run_forward(a, segments, m, nullptr, renorm_counter);
    if (r != VTB_OK) return r;
    for (int s = 0; s < a.N; s++) metrics[s] = uint8_t(m[s]);
    return VTB_OK;
}

int vtb_legacy_metrics_k1n(const vtb_genk_code_t* code, const uint8_t* segments, int32_t count, uint8_t* metrics,
                           uint32_t* renorm_counter) {
    if (!code || !metrics || !renorm_counter || count < 0 || (count > 0 && !segments)) return VTB_ERR_INVALID;
    const int K = code->constraint_length, n = code->coded_bits;
    if (code->input_bits != 1 || n < 1 || n > 8) return VTB_ERR_INVALID;
    if (K < VTB_MIN_K || K > VTB_MAX_K) return VTB_ERR_UNSUPPORTED;
    for (int i = 0; i < n; i++)
        if (code->generators[i] >> K) return VTB_ERR_INVALID;
    if (count == 0) return VTB_OK;
    vtb::FwdArgs a{};
    a.butterfly = 1, a.k = 1, a.S = K - 1, a.n = n, a.N = 1 << (K - 1), a.count = count;
    for (int i = 0; i < n; i++) a.rg[i] = vtb::rev_bits(code->generators[i], K);
    uint32_t m[256];
    for (int s = 0; s < a.N; s++) m[s] = metrics[s];
    int r = vtb::run_forward(a, segments, m, nullptr, renorm_counter);
    if (r != VTB_OK) return r;
    for (int s = 0; s < a.N; s++) metrics[s] = uint8_t(m[s]);
    return VTB_OK;
}

int vtb_legacy_metrics_genk(const vtb_genk_code_t* code, const uint8_t* segments, int32_t count, uint32_t* metrics,
                            uint32_t* prev_metrics) {
    if (!code || !metrics || count < 0 || (count > 0 && !segments)) return VTB_ERR_INVALID;
    const int k = code->input_bits, K = code->constraint_length, n = code->coded_bits;
    if (k < 1 || K < 2 || n < 1 || n > 8) return VTB_ERR_INVALID;
    if (k * (K - 1) > 8 || k * K > 12) return VTB_ERR_UNSUPPORTED;
    for (int i = 0; i < n; i++)
        if (code->generators[i] >> (k * K)) return VTB_ERR_INVALID;
    if (count == 0) return VTB_OK;
    vtb::FwdArgs a{};
    a.butterfly = 0, a.k = k, a.S = K - 1, a.n = n, a.N = 1 << (k * (K - 1)), a.count = count;
    for (int i = 0; i < n; i++) a.rg[i] = vtb::rev_bits(code->generators[i], k * K);
    return vtb::run_forward(a, segments, metrics, prev_metrics, nullptr);
}

int vtb_genk_decode_frame_legacy(const vtb_genk_code_t* code, const uint8_t* coded, int32_t segments, uint8_t* out) {
    if (!code || !coded || !out) return VTB_ERR_INVALID;
    const int k = code->input_bits, S = code->constraint_length - 1;
    const int64_t info = int64_t(segments - S) * k;
    // k > 1: whole bytes (the reference's own requirement, viterbiDecoder.c:222-227); k = 1 any
    // length (its butterfly decoder pads the last byte, viterbiDecoderButterflyk1.c:226-249)
    if (segments <= S || info < 1 || (k > 1 && info % 8) || info > VTB_MAX_FRAME_BITS) return VTB_ERR_INVALID;
    const size_t ob = size_t(info + 7) / 8;
    vtb::PrevDevice keep;
    vtb::Ctx& c = vtb::g_ctx;
    int r = vtb::ctx_ready(c, size_t(segments), ob);
    if (r != VTB_OK) return r;
    if (hipMemcpyAsync(c.d_seg, coded, size_t(segments), hipMemcpyHostToDevice, c.stream) != hipSuccess) {
        (void)hipStreamSynchronize(c.stream);
        return VTB_ERR_DEVICE;
    }
    r = vtb_genk_decode_device(code, int32_t(info), c.d_seg, size_t(segments), c.d_out, ob, 1, c.stream);
    if (r != VTB_OK) {
        (void)hipStreamSynchronize(c.stream);
        return r;
    }
    if (hipMemcpyAsync(out, c.d_out, ob, hipMemcpyDeviceToHost, c.stream) != hipSuccess ||
        hipStreamSynchronize(c.stream) != hipSuccess) {
        (void)hipStreamSynchronize(c.stream);
        return VTB_ERR_DEVICE;
    }
    return int(ob);
}

}  // extern "C"
