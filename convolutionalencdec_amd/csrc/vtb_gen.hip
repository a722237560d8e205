// Device-side synthetic frames: payload bytes, terminated
// convolutional encoding and the channel (BSC bit flips for hard input, BPSK AWGN plus the
// 8-bit soft quantiser for soft input), so large batches never cross PCIe.
//
// All three are integer-exact: a counter-based hash keyed by (seed, frame, counter) is the
// only source of randomness and the Gaussian is an Irwin-Hall sum in fixed point, so the
// test oracle (oracle/viterbi_oracle.c, oracle_gen_*) reproduces every byte.  The RNG
// stream is build-defined; the reference's own harness (berTestK7.c:22-43) draws from
// glibc rand(), which the oracle restates separately for its known-answer test.
//
// Encoder semantics follow convEnc (src/convEncode.c:46-130) for whole terminated frames:
// information bits MSB-first, the tapped delay line takes the newest bit in its LSB, output
// bit j of a segment is the parity of the delay line under the bit-reversed generator j
// (convEncode.c:19-44, 132-161), and K-1 zero tail segments close the frame.
//
// HBM-bound byte work: one thread per 8 payload bytes, per 4 coded segments, per segment of
// channel output; no LDS, no cross-lane traffic.

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "viterbi_amd.h"
#include "vtb_internal.h"

namespace vtb {
namespace {

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finalizer
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

// The counter-based stream (include/viterbi_amd.h, "Synthetic frames").
__host__ __device__ __forceinline__ uint64_t rand64(uint64_t seed, uint64_t frame, uint64_t ctr) {
    return mix64(mix64(seed + 0x9E3779B97F4A7C15ull * (frame + 1)) ^ (0xD1B54A32D192ED03ull * (ctr + 1)));
}

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void payload_kernel(uint64_t seed, int nbytes, uint32_t last_mask,
                                                           uint8_t* __restrict__ out, size_t stride,
                                                           size_t frames) {
    const int groups = (nbytes + 7) >> 3;
    const size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= frames * (size_t)groups) return;
    const size_t f = i / groups;
    const int g = int(i - f * groups);
    const uint64_t r = rand64(seed, f, (uint64_t)g);
    uint8_t* o = out + f * stride + 8 * g;
    const int nb = min(8, nbytes - 8 * g);
    for (int b = 0; b < nb; b++) {
        uint32_t v = uint32_t(r >> (8 * b)) & 0xffu;
        if (8 * g + b == nbytes - 1) v &= last_mask;
        o[b] = uint8_t(v);
    }
}

// Four coded segments t0..t0+3 per thread.  Segment t's delay line holds information bits
// t-K+1..t (bit i = bit t-i; bits outside [0, L) are zero), read from a 24-bit big-endian
// window of payload bytes starting at byte floor((t0 - 8) / 8).
__global__ __launch_bounds__(kThreads) void encode_kernel(int K, uint32_t rg0, uint32_t rg1, int L,
                                                          const uint8_t* __restrict__ unc, size_t in_stride,
                                                          uint8_t* __restrict__ coded, size_t out_stride,
                                                          size_t frames) {
    const int T = L + K - 1;
    const int quads = (T + 3) >> 2;
    const size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= frames * (size_t)quads) return;
    const size_t f = i / quads;
    const int t0 = 4 * int(i - f * quads);
    const uint8_t* u = unc + f * in_stride;
    const int b0 = (t0 - 8) >> 3;  // arithmetic shift: floor
    uint32_t W = 0;
    for (int k = 0; k < 3; k++) {
        const int b = b0 + k;
        uint32_t v = 0;
        if (b >= 0 && 8 * b < L) {
            v = u[b];
            const int valid = L - 8 * b;  // bits of this byte inside the frame
            if (valid < 8) v &= (0xFFu << (8 - valid)) & 0xFFu;
        }
        W = (W << 8) | v;
    }
    const uint32_t mask = (1u << K) - 1u;
    uint8_t* o = coded + f * out_stride;
    for (int s = 0; s < 4; s++) {
        const int t = t0 + s;
        if (t >= T) break;
        const int pos = 23 - (t - 8 * b0);  // bit position of information bit t in W
        const uint32_t st = (W >> pos) & mask;
        o[t] = uint8_t((__builtin_popcount(st & rg0) & 1) | ((__builtin_popcount(st & rg1) & 1) << 1));
    }
}

// BSC: one hash per segment, its low / high 32 bits decide the flips of coded bits 0 / 1.
__global__ __launch_bounds__(kThreads) void bsc_kernel(uint64_t seed, uint32_t p32, int T,
                                                       const uint8_t* __restrict__ coded, size_t in_stride,
                                                       uint8_t* __restrict__ rx, size_t out_stride, size_t frames) {
    const size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= frames * (size_t)T) return;
    const size_t f = i / T;
    const int t = int(i - f * T);
    const uint64_t r = rand64(seed, f, (uint64_t)t);
    const uint32_t flips = (uint32_t(r) < p32 ? 1u : 0u) | (uint32_t(r >> 32) < p32 ? 2u : 0u);
    rx[f * out_stride + t] = uint8_t((coded[f * in_stride + t] & 3u) ^ flips);
}

// AWGN + quantiser: per coded bit, z = (sum of 12 uniform 21-bit draws - 6 * 2^21) / 2^21
// (Irwin-Hall, unit variance; four hashes at counters 8t + 4i + h, three draws each), then
// q = clamp(floor(b * 255 * 2^16 - floor(kq * z_fx / 2^21) + 2^15) / 2^16, 0, 255) with
// kq = round(sigma * 127.5 * 2^16): q = round((1 - y) * 127.5) for y = (1 - 2b) + sigma z.
__global__ __launch_bounds__(kThreads) void awgn_kernel(uint64_t seed, int64_t kq, int T,
                                                        const uint8_t* __restrict__ coded, size_t in_stride,
                                                        uint8_t* __restrict__ rx, size_t out_stride, size_t frames) {
    const size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= frames * (size_t)T) return;
    const size_t f = i / T;
    const int t = int(i - f * T);
    const uint32_t c = coded[f * in_stride + t];
    uint32_t qq[2];
    for (int b = 0; b < 2; b++) {
        int64_t z = -(6ll << 21);
        for (int h = 0; h < 4; h++) {
            const uint64_t r = rand64(seed, f, 8ull * t + 4 * b + h);
            z += int64_t(r & 0x1FFFFF) + int64_t((r >> 21) & 0x1FFFFF) + int64_t((r >> 42) & 0x1FFFFF);
        }
        const int64_t v = (kq * z) >> 21;  // floor
        const int64_t qf = (((c >> b) & 1u) ? (255ll << 16) : 0ll) - v;
        int64_t q = (qf + 32768) >> 16;
        q = q < 0 ? 0 : (q > 255 ? 255 : q);
        qq[b] = uint32_t(q);
    }
    uint8_t* o = rx + f * out_stride + 2 * (size_t)t;
    o[0] = uint8_t(qq[0]);
    o[1] = uint8_t(qq[1]);
}

unsigned blocks_for(size_t n) { return unsigned((n + kThreads - 1) / kThreads); }

int launch_status() { return hipGetLastError() == hipSuccess ? VTB_OK : VTB_ERR_DEVICE; }

uint32_t rev_bits(uint64_t v, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; i++) r = (r << 1) | uint32_t((v >> i) & 1u);
    return r;
}

}  // namespace
}  // namespace vtb

extern "C" {

uint64_t vtb_rand64(uint64_t seed, uint64_t frame, uint64_t ctr) { return vtb::rand64(seed, frame, ctr); }

int64_t vtb_awgn_kq(double snr_db) {
    const double esn0 = std::pow(10.0, (snr_db + 10.0 * std::log10(4.0)) / 10.0);
    const double sigma = std::sqrt(1.0 / (2.0 * esn0));
    return (int64_t)std::llround(sigma * 127.5 * 65536.0);
}

uint32_t vtb_bsc_p32(double p) {
    if (!(p > 0.0)) return 0u;
    if (p >= 1.0) return 0xFFFFFFFFu;
    return (uint32_t)std::floor(p * 4294967296.0);
}

int vtb_payload_device(uint64_t seed, int32_t frame_bits, uint8_t* d_out, size_t stride, size_t frames,
                       void* stream) {
    if (frame_bits < 1 || !d_out) return VTB_ERR_INVALID;
    const int nbytes = (frame_bits + 7) >> 3;
    if (stride < (size_t)nbytes) return VTB_ERR_INVALID;
    if (frames == 0) return VTB_OK;
    const uint32_t last_mask = (frame_bits & 7) ? ((0xFFu << (8 - (frame_bits & 7))) & 0xFFu) : 0xFFu;
    const size_t n = frames * (size_t)((nbytes + 7) >> 3);
    hipLaunchKernelGGL(vtb::payload_kernel, dim3(vtb::blocks_for(n)), dim3(vtb::kThreads), 0, (hipStream_t)stream,
                       seed, nbytes, last_mask, d_out, stride, frames);
    return vtb::launch_status();
}

int vtb_encode_device(const vtb_code_t* code, int32_t frame_bits, const uint8_t* d_uncoded, size_t in_stride,
                      uint8_t* d_coded, size_t out_stride, size_t frames, void* stream) {
    if (!code || !d_uncoded || !d_coded || frame_bits < 1) return VTB_ERR_INVALID;
    if (code->coded_bits != 2) return VTB_ERR_UNSUPPORTED;
    const int K = code->constraint_length;
    if (K < VTB_MIN_K || K > VTB_MAX_K) return VTB_ERR_UNSUPPORTED;
    if ((code->generators[0] >> K) || (code->generators[1] >> K)) return VTB_ERR_INVALID;
    const int T = frame_bits + K - 1;
    if (in_stride < (size_t)((frame_bits + 7) >> 3) || out_stride < (size_t)T) return VTB_ERR_INVALID;
    if (frames == 0) return VTB_OK;
    const size_t n = frames * (size_t)((T + 3) >> 2);
    hipLaunchKernelGGL(vtb::encode_kernel, dim3(vtb::blocks_for(n)), dim3(vtb::kThreads), 0, (hipStream_t)stream, K,
                       vtb::rev_bits(code->generators[0], K), vtb::rev_bits(code->generators[1], K), frame_bits,
                       d_uncoded, in_stride, d_coded, out_stride, frames);
    return vtb::launch_status();
}

int vtb_channel_device(vtb_input_t output, double param, uint64_t seed, const uint8_t* d_coded, size_t in_stride,
                       int32_t segments, uint8_t* d_rx, size_t out_stride, size_t frames, void* stream) {
    if (!d_coded || !d_rx || segments < 1 || in_stride < (size_t)segments) return VTB_ERR_INVALID;
    if (frames == 0) return VTB_OK;
    const size_t n = frames * (size_t)segments;
    if (output == VTB_INPUT_HARD) {
        if (out_stride < (size_t)segments || !(param >= 0.0 && param <= 1.0)) return VTB_ERR_INVALID;
        hipLaunchKernelGGL(vtb::bsc_kernel, dim3(vtb::blocks_for(n)), dim3(vtb::kThreads), 0, (hipStream_t)stream,
                           seed, vtb_bsc_p32(param), segments, d_coded, in_stride, d_rx, out_stride, frames);
    } else if (output == VTB_INPUT_SOFT8) {
        if (out_stride < 2 * (size_t)segments || !std::isfinite(param)) return VTB_ERR_INVALID;
        hipLaunchKernelGGL(vtb::awgn_kernel, dim3(vtb::blocks_for(n)), dim3(vtb::kThreads), 0, (hipStream_t)stream,
                           seed, vtb_awgn_kq(param), segments, d_coded, in_stride, d_rx, out_stride, frames);
    } else {
        return VTB_ERR_INVALID;
    }
    return vtb::launch_status();
}

}  // extern "C"
