// Measurement only: round-trip latency of ONE synchronous single-frame call (the legacy
// VITERBI_DECODER_HARD contract), by how the host hands the frame over and learns that the
// kernel is done.  Each variant runs N calls back to back from one host thread; the kernel
// does no decoding, only the data movement of a 2,054-byte hard frame in / 256 bytes out.
//   sync      launch, hipStreamSynchronize
//   h2d+sync  hipMemcpyAsync (pinned -> device) + launch + hipStreamSynchronize
//   flag      launch; the kernel reads the frame from pinned host memory itself (zero copy),
//             writes the output bytes and then a completion word into coherent host memory;
//             the host spins on the word
//   graph     the flag variant launched as a one-node hipGraph
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                          \
        }                                                                      \
    } while (0)

constexpr int kIn = 2054, kOut = 256;

__global__ __launch_bounds__(256) void frame_kernel(const uint8_t* in, uint8_t* out, unsigned* flag, unsigned seq) {
    __shared__ uint8_t buf[kIn + 64];
    const int t = threadIdx.x;
    // one 8-byte load per thread (the frame in one round trip)
    if (8 * t < kIn) {
        for (int i = 0; i < 8 && 8 * t + i < kIn; i++) buf[8 * t + i] = in[8 * t + i];
    }
    __syncthreads();
    if (t < kOut) out[t] = buf[t] ^ buf[kIn - 1 - t];
    if (flag) {
        __syncthreads();
        if (t == 0) {
            __threadfence_system();
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

int main() {
    uint8_t *h_in, *h_out, *d_in, *d_out, *dh_in, *dh_out;
    unsigned *h_flag, *dh_flag;
    CK(hipHostMalloc((void**)&h_in, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc((void**)&h_out, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc((void**)&h_flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void**)&dh_in, h_in, 0));
    CK(hipHostGetDevicePointer((void**)&dh_out, h_out, 0));
    CK(hipHostGetDevicePointer((void**)&dh_flag, h_flag, 0));
    CK(hipMalloc(&d_in, 4096));
    CK(hipMalloc(&d_out, 4096));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int i = 0; i < kIn; i++) h_in[i] = uint8_t(i * 7);
    const int N = 2000;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    volatile unsigned* vf = h_flag;

    for (int rep = 0; rep < 2; rep++) {
        // sync
        auto t0 = now();
        for (int i = 0; i < N; i++) {
            hipLaunchKernelGGL(frame_kernel, dim3(1), dim3(256), 0, s, d_in, d_out, (unsigned*)nullptr, 0u);
            CK(hipStreamSynchronize(s));
        }
        auto t1 = now();
        // h2d + sync (output straight to pinned memory)
        for (int i = 0; i < N; i++) {
            CK(hipMemcpyAsync(d_in, h_in, kIn, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(frame_kernel, dim3(1), dim3(256), 0, s, d_in, dh_out, (unsigned*)nullptr, 0u);
            CK(hipStreamSynchronize(s));
        }
        auto t2 = now();
        // zero copy in, spin on the completion word
        unsigned seq = 1;
        long spins = 0;
        for (int i = 0; i < N; i++, seq++) {
            hipLaunchKernelGGL(frame_kernel, dim3(1), dim3(256), 0, s, dh_in, dh_out, dh_flag, seq);
            while (*vf != seq) spins++;
            std::atomic_thread_fence(std::memory_order_acquire);
        }
        auto t3 = now();
        CK(hipStreamSynchronize(s));
        // graph of the flag variant (the seq value is baked in: spin for a change instead)
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        hipLaunchKernelGGL(frame_kernel, dim3(1), dim3(256), 0, s, dh_in, dh_out, dh_flag, 7u);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        auto t4 = now();
        for (int i = 0; i < N; i++) {
            *vf = 0;
            std::atomic_thread_fence(std::memory_order_seq_cst);
            CK(hipGraphLaunch(ge, s));
            while (*vf != 7u) spins++;
        }
        auto t5 = now();
        CK(hipStreamSynchronize(s));
        // sync, 4 waves of 64 (latency of a 256-thread single-block dispatch is the same kernel)
        std::printf("rep %d: sync %.2f us/call, h2d+sync %.2f, zero-copy+flag %.2f, graph+flag %.2f (spins %ld)\n", rep,
                    us(t0, t1) / N, us(t1, t2) / N, us(t2, t3) / N, us(t4, t5) / N, spins);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    // output correctness of the zero-copy variant
    int bad = 0;
    for (int t = 0; t < kOut; t++) bad += h_out[t] != uint8_t(h_in[t] ^ h_in[kIn - 1 - t]);
    std::printf("zero-copy output mismatches: %d\n", bad);
    return 0;
}
