// Probe: cycles per trellis step of the generic register-resident recursion (vtb_lds_path.hip)
// by variant, one wave alone (latency) and 4 waves per SIMD (issue).  Measurement only.
//   V0 shipped: two compares, the decision word combined on the SALU, two v_writelane
//   V1 the decision on the VALU (sub, xor, one compare), two v_writelane
//   V2 shipped without the v_writelane (decision words folded into an SGPR)
//   V3 metric chain only (add, DPP sub, min) + one compare folded into an SGPR
// hipcc --offload-arch=gfx950 -O3 -o genstep_probe genstep_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <utility>

__device__ int wl(int value, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

template <int P>
__device__ __forceinline__ int partner(int m) {
    if constexpr (P == 0) return __builtin_amdgcn_update_dpp(0, m, 0xB1, 0xF, 0xF, true);
    else if constexpr (P == 1) return __builtin_amdgcn_update_dpp(0, m, 0x4E, 0xF, 0xF, true);
    else if constexpr (P == 2) return __builtin_amdgcn_update_dpp(0, m, 0x141, 0xF, 0xF, true);
    else if constexpr (P == 3) return __builtin_amdgcn_update_dpp(0, m, 0x128, 0xF, 0xF, true);
    else {
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %0\n\ts_nop 0" : "+v"(m));
        return m;
    }
}

typedef short short2_t __attribute__((ext_vector_type(2)));

template <int... Is, class Fn>
__device__ __forceinline__ void sfor(std::integer_sequence<int, Is...>, Fn&& fn) {
    (fn(std::integral_constant<int, Is>{}), ...);
}

template <int S, int V>
__global__ __launch_bounds__(64) void k(const int* __restrict__ qin, unsigned long long* out, int steps) {
    const int lane = threadIdx.x;
    int m = lane * 3;
    int sig[S], kap[S], rs[S];
    uint64_t um[S];
    for (int ph = 0; ph < S; ph++) {
        sig[ph] = qin[(lane + ph) & 63] | 1;
        kap[ph] = qin[(lane * 7 + ph) & 63];
        rs[ph] = ((lane >> (S - 1 - ph)) & 1) ? -1 : 0;
        um[ph] = __ballot(rs[ph] != 0);
    }
    uint32_t klo = 0, khi = 0;
    uint64_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int t = 0; t < steps; t += S) {
        sfor(std::make_integer_sequence<int, S>{}, [&](auto pc) {
            constexpr int PH = decltype(pc)::value;
            const int q = (((t + PH) & 3) * 0x8001) & 0x00010001;  // (uniform: SALU, off the chain)
            const int mu = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, sig[PH]), __builtin_bit_cast(short2_t, q),
                                                  kap[PH], false);
            const int pm = partner<S - 1 - PH>(m);
            const int a = m + mu, b = pm - mu;
            uint64_t bal;
            if constexpr (V == 0 || V == 2) {
                const uint64_t gt = __ballot(a > b), lt = __ballot(b > a);
                bal = (gt & ~um[PH]) | (lt & um[PH]);
            } else if constexpr (V == 1) {
                bal = __ballot(((a - b) ^ rs[PH]) > rs[PH]);
            } else {
                bal = __ballot(a > b);
            }
            if constexpr (V <= 1) {
                const int i = (t + PH) & 63;
                klo = uint32_t(wl(int(uint32_t(bal)), i, int(klo)));
                khi = uint32_t(wl(int(uint32_t(bal >> 32)), i, int(khi)));
            } else {
                acc ^= bal;
            }
            m = a < b ? a : b;
        });
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 2] = t1 - t0;
    out[blockIdx.x * 2 + 1] = uint64_t(m) + klo + khi + acc;  // (keeps the work live)
}

template <int S, int V>
void run(int* dq, unsigned long long* dout, int blocks, const char* name) {
    const int steps = 8192 / S * S;
    unsigned long long h[2 * 4096];
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL((k<S, V>), dim3(blocks), dim3(64), 0, 0, dq, dout, steps);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, dout, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost);
    double s = 0;
    for (int b = 0; b < blocks; b++) s += double(h[2 * b]);
    printf("{\"S\": %d, \"variant\": \"%s\", \"waves\": %d, \"cycles_per_step\": %.1f}\n", S, name, blocks,
           s / blocks / steps);
}

int main() {
    int* dq;
    unsigned long long* dout;
    int hq[64];
    for (int i = 0; i < 64; i++) hq[i] = (i * 37) & 0x00010001;
    (void)hipMalloc(&dq, sizeof(hq));
    (void)hipMalloc(&dout, sizeof(unsigned long long) * 2 * 4096);
    (void)hipMemcpy(dq, hq, sizeof(hq), hipMemcpyHostToDevice);
    for (int blocks : {1, 4096}) {
        run<2, 0>(dq, dout, blocks, "V0 shipped");
        run<2, 1>(dq, dout, blocks, "V1 valu-decision");
        run<2, 2>(dq, dout, blocks, "V2 no-writelane");
        run<2, 3>(dq, dout, blocks, "V3 chain+cmp");
        run<5, 0>(dq, dout, blocks, "V0 shipped");
        run<5, 1>(dq, dout, blocks, "V1 valu-decision");
        run<5, 2>(dq, dout, blocks, "V2 no-writelane");
        run<5, 3>(dq, dout, blocks, "V3 chain+cmp");
    }
    return 0;
}
