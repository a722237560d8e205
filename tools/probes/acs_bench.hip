// Probe: cost of the K=7 ACS step (vtb_k7_lds.hip) in isolation -- registers only, no LDS
// -- with variants that drop one ingredient each.  Prints wall cycles per step per SIMD
// (at the measured clock) for 1, 2 and 4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "../../convolutionalencdec_amd/csrc/vtb_k7_common.h"

using namespace vtb::k7;

// V: 0 full step; 1 no decision extraction; 2 XOR16/32 via DPP (wrong, cost only);
//    3 no renorm; 4 decision via two SDWA compares into SGPRs (old kernel);
//    5 no min (A only); 6 XOR4 via one DPP (wrong, cost only)
template <int V, int PH>
__device__ __forceinline__ void step(uint32_t& M, uint32_t& acc, uint2 vw, uint64_t& sink) {
    constexpr int P = 5 - PH;
    const uint32_t A = M + vw.x;
    uint32_t B;
    if constexpr ((V == 2 && P >= 4) || (V == 6 && P == 2)) {
        B = __builtin_amdgcn_update_dpp(0u, M, 0x128, 0xF, 0xF, true) + vw.y;
    } else {
        B = partner_plus<P>(M, vw.y);
    }
    const uint32_t nw = V == 5 ? A : pk_min(A, B);
    if constexpr (V == 4) {
        uint64_t ca, cb;
        asm volatile("v_cmp_gt_u16_sdwa %0, %1, %2 src0_sel:WORD_0 src1_sel:WORD_0" : "=s"(ca) : "v"(A), "v"(B));
        asm volatile("v_cmp_gt_u16_sdwa %0, %1, %2 src0_sel:WORD_1 src1_sel:WORD_1" : "=s"(cb) : "v"(A), "v"(B));
        sink ^= ca ^ cb;
    } else if constexpr (V != 1) {
        const uint32_t d = pk_sub(B, A);
        acc = (d & 0x80008000u) | ((acc >> 1) & 0x7FFF7FFFu);
    } else {
        acc ^= B;
    }
    M = nw & 0xFFFEFFFEu;
}

template <int V>
__global__ __launch_bounds__(64) void k(uint64_t* out, int iters, uint32_t seed) {
    const int lane = threadIdx.x;
    uint32_t M = 8192u * 0x10001u + lane;
    uint32_t acc = 0;
    uint64_t sink = 0;
    uint2 vw[6];
    for (int i = 0; i < 6; i++) vw[i] = make_uint2((seed * (i + 1) + lane) & 0x01ff01ffu, (seed ^ (lane * 77 + i)) & 0x01ff01ffu);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int g = 0; g < 8; g++) {
            step<V, 0>(M, acc, vw[0], sink);
            step<V, 1>(M, acc, vw[1], sink);
            step<V, 2>(M, acc, vw[2], sink);
            step<V, 3>(M, acc, vw[3], sink);
            step<V, 4>(M, acc, vw[4], sink);
            step<V, 5>(M, acc, vw[5], sink);
            if ((g % 8) == 2 || (g % 8) == 5 || (g % 8) == 7) sink += acc;  // every 16 steps (48 = 3 x 16)
            if (V != 3 && (g & 1)) {
                const uint32_t ref = __builtin_amdgcn_readlane(M, 0);
                const uint32_t dd = ((kBias - (ref & 0xffffu)) & 0xffffu) | ((kBias - (ref >> 16)) << 16);
                M = pk_add(M, dd);
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if ((M ^ acc ^ (uint32_t)sink) == 0x12345678u) out[1 << 20] = M;
}

// Same step with the table pairs read from an LDS ring as in vtb_k7_lds.hip (two groups
// ahead), W = 1: plus the 16-step decision-word stores to LDS.
template <int W>
__global__ __launch_bounds__(64) void kl(uint64_t* out, int iters, uint32_t seed) {
    __shared__ uint4 tab4[48 * 4];
    __shared__ uint32_t dec[64 * 64];
    uint8_t* tab = reinterpret_cast<uint8_t*>(tab4);
    const int lane = threadIdx.x;
    for (int i = lane; i < 48 * 4; i += 64) tab4[i] = make_uint4(seed * i, seed ^ i, i * 7, i * 13);
    __syncthreads();
    uint32_t off[6];
    for (int k = 0; k < 6; k++) off[k] = 8 * ((lane * (k + 3)) & 7);
    uint32_t M = 8192u * 0x10001u + lane, acc = 0;
    uint64_t sink = 0;
    uint2 cur[6], nx1[6];
    for (int k = 0; k < 6; k++) {
        cur[k] = *reinterpret_cast<const uint2*>(tab + k * 64 + off[k]);
        nx1[k] = *reinterpret_cast<const uint2*>(tab + (6 + k) * 64 + off[k]);
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        const uint2* ap[6];
        for (int k = 0; k < 6; k++) ap[k] = reinterpret_cast<const uint2*>(tab + off[k]);
        uint32_t* dchunk = dec + (it & 15) * 3 * 64 + lane;
#pragma unroll
        for (int g = 0; g < 8; g++) {
            uint2 nx2[6];
#pragma unroll
            for (int k = 0; k < 6; k++) nx2[k] = ap[k][((6 * (g + 2) + k) % 48) * 8];
            step<0, 0>(M, acc, cur[0], sink);
            step<0, 1>(M, acc, cur[1], sink);
            step<0, 2>(M, acc, cur[2], sink);
            step<0, 3>(M, acc, cur[3], sink);
            step<0, 4>(M, acc, cur[4], sink);
            step<0, 5>(M, acc, cur[5], sink);
            if ((g % 8) == 2 || (g % 8) == 5 || (g % 8) == 7) {
                if (W) dchunk[((g * 6) / 16) * 64] = acc;
                else sink += acc;
            }
            if (g & 1) {
                const uint32_t ref = __builtin_amdgcn_readlane(M, 0);
                const uint32_t dd = ((kBias - (ref & 0xffffu)) & 0xffffu) | ((kBias - (ref >> 16)) << 16);
                M = pk_add(M, dd);
            }
#pragma unroll
            for (int k = 0; k < 6; k++) {
                cur[k] = nx1[k];
                nx1[k] = nx2[k];
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if ((M ^ acc ^ (uint32_t)sink ^ dec[lane]) == 0x12345678u) out[1 << 20] = M;
}

template <int V>
void run(const char* name, uint64_t* d) {
    const int iters = 400, steps = iters * 48;
    printf("%-40s", name);
    for (int wps : {1, 2, 4}) {
        const int blocks = 1024 * wps;
        hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(64), 0, 0, d, iters, 12345u);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(64), 0, 0, d, iters, 12345u);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        static uint64_t h[4096];
        (void)hipMemcpy(h, d, 8 * blocks, hipMemcpyDeviceToHost);
        double cyc = 0;
        for (int b = 0; b < blocks; b++) cyc += h[b];
        cyc /= blocks;
        // per SIMD: wps waves each doing `steps` steps in the wave's lifetime (cycles from s_memtime)
        printf("  %d w/SIMD: %6.1f cyc/step/SIMD (wave %6.1f) %.1f GHz", wps, cyc / (steps * wps), cyc / steps,
               cyc / (ms * 1e-3) / 1e9);
    }
    printf("\n");
}

template <int W>
void runl(const char* name, uint64_t* d) {
    const int iters = 400, steps = iters * 48;
    printf("%-40s", name);
    for (int wps : {1, 2, 4}) {
        const int blocks = 1024 * wps;
        hipLaunchKernelGGL(kl<W>, dim3(blocks), dim3(64), 0, 0, d, iters, 12345u);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(kl<W>, dim3(blocks), dim3(64), 0, 0, d, iters, 12345u);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        static uint64_t h[4096];
        (void)hipMemcpy(h, d, 8 * blocks, hipMemcpyDeviceToHost);
        double cyc = 0;
        for (int b = 0; b < blocks; b++) cyc += h[b];
        cyc /= blocks;
        printf("  %d w/SIMD: %6.1f cyc/step/SIMD (wave %6.1f) %.1f GHz", wps, cyc / (steps * wps), cyc / steps,
               cyc / (ms * 1e-3) / 1e9);
    }
    printf("\n");
}

int main(int argc, char** argv) {
    uint64_t* d;
    (void)hipMalloc(&d, ((1 << 20) + 8) * 8);
    if (argc > 1) {  // counter runs: the full step only, 2 waves per SIMD
        hipLaunchKernelGGL(k<0>, dim3(2048), dim3(64), 0, 0, d, 400, 12345u);
        (void)hipDeviceSynchronize();
        return 0;
    }
    run<0>("full step", d);
    run<1>("no decision extraction", d);
    run<2>("XOR16/32 by DPP (cost only)", d);
    run<6>("XOR4 by one DPP (cost only)", d);
    run<3>("no renorm", d);
    run<4>("decisions by 2 SDWA cmps", d);
    run<5>("no min", d);
    runl<0>("table from LDS", d);
    runl<1>("table from LDS + word stores", d);
    return 0;
}
