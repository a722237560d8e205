// Measurement only: per-launch cost of back-to-back kernels on one stream (HIP events around
// N launches), by grid size and dynamic LDS, plain launches vs one hipGraph of N launches,
// and two streams alternating.  Explains the fixed ~6 us of the K=7 launch (VTB_DEBUG=16).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__global__ __launch_bounds__(64) void empty_kernel(int* p, int flag) {
    extern __shared__ int lds[];
    if (flag) {
        lds[threadIdx.x] = threadIdx.x;
        __syncthreads();
        p[blockIdx.x * 64 + threadIdx.x] = lds[63 - threadIdx.x];
    }
}

int main() {
    int* d;
    CK(hipMalloc(&d, 64 * 65536 * sizeof(int)));
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int N = 200;
    for (int grid : {1, 256, 2048, 8192}) {
        for (int lds : {0, 20480}) {
            for (int flag : {0, 1}) {
                for (int w = 0; w < 10; w++) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(64), lds, s, d, flag);
                CK(hipStreamSynchronize(s));
                CK(hipEventRecord(e0, s));
                for (int i = 0; i < N; i++) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(64), lds, s, d, flag);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                // the same N launches captured in one graph
                hipGraph_t g;
                hipGraphExec_t ge;
                CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
                for (int i = 0; i < N; i++) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(64), lds, s, d, flag);
                CK(hipStreamEndCapture(s, &g));
                CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
                CK(hipGraphLaunch(ge, s));
                CK(hipStreamSynchronize(s));
                CK(hipEventRecord(e0, s));
                CK(hipGraphLaunch(ge, s));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float gms;
                CK(hipEventElapsedTime(&gms, e0, e1));
                CK(hipGraphExecDestroy(ge));
                CK(hipGraphDestroy(g));
                // two streams alternating
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0, s));
                CK(hipStreamWaitEvent(s2, e0, 0));
                for (int i = 0; i < N; i++)
                    hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(64), lds, (i & 1) ? s2 : s, d, flag);
                hipEvent_t e2;
                CK(hipEventCreate(&e2));
                CK(hipEventRecord(e2, s2));
                CK(hipStreamWaitEvent(s, e2, 0));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ams;
                CK(hipEventElapsedTime(&ams, e0, e1));
                CK(hipEventDestroy(e2));
                std::printf("grid %5d lds %5d work %d: plain %.2f us/launch, graph %.2f, two streams %.2f\n", grid, lds,
                            flag, 1000.f * ms / N, 1000.f * gms / N, 1000.f * ams / N);
            }
        }
    }
    return 0;
}
