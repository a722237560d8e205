// Probe: the K=7 ACS step with two metric registers per lane (32 lanes per frame pair, four
// frames per wave64) against the shipped layout (one register per lane, 64 lanes per frame
// pair).  With two registers, one of the six location bits is the register index (the
// butterfly runs inside the lane with plain adds) and XOR 32 disappears; the XOR-16 phase
// exchanges rows between the two registers with one v_permlane16_swap (a transposition:
// afterwards each lane holds a partner pair) and then also runs inside the lane.  Bits 5
// and 4 take turns as the register bit, so each six-step period has two transpositions.
// Table values live in registers (no LDS), so this isolates VALU/DPP/permlane issue.
// Prints cycles per frame-pair-step per SIMD at the nominal clock.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_add(uint32_t m, uint32_t w) {
    return __builtin_amdgcn_update_dpp(0u, m, CTRL, 0xF, 0xF, true) + w;
}

// In-lane butterfly of a partner pair (r0, r1): 4 plain adds, 2 mins.
__device__ __forceinline__ void inlane(uint32_t& r0, uint32_t& r1, uint4 t) {
    const uint32_t a0 = r0 + t.x, b0 = r1 + t.y, a1 = r1 + t.z, b1 = r0 + t.w;
    r0 = pk_min(a0, b0);
    r1 = pk_min(a1, b1);
}
template <int CTRL>
__device__ __forceinline__ void dppstep(uint32_t& r, uint2 t) {
    r = pk_min(r + t.x, dpp_add<CTRL>(r, t.y));
}

// Two registers per lane: 6 steps = reg phase, x16 phase, 4 DPP phases (x8, x7, x2, x1).
__global__ __launch_bounds__(64) void k2(uint64_t* out, int iters, uint32_t seed) {
    const int lane = threadIdx.x;
    uint32_t r0 = 8192u * 0x10001u + lane, r1 = r0 + 3;
    uint4 tq[2];
    uint2 td[4][2];
    for (int i = 0; i < 2; i++) tq[i] = make_uint4(seed * (i + 1) + lane, seed ^ lane, seed + 7 * lane, lane * 13);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 2; j++) td[i][j] = make_uint2((seed * (i + 3) + lane + j) & 0x01ff01ffu, (seed ^ (lane * 77 + i + j)) & 0x01ff01ffu);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int g = 0; g < 4; g++) {
            // bits 5 and 4 alternate between the register and the lane row: a transposition
            // before each of the two in-lane steps
            asm volatile("s_nop 0\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 0" : "+v"(r0), "+v"(r1));
            inlane(r0, r1, tq[0]);
            asm volatile("s_nop 0\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 0" : "+v"(r0), "+v"(r1));
            inlane(r0, r1, tq[1]);
            r0 &= 0xFFFCFFFCu, r1 &= 0xFFFCFFFCu;
            dppstep<0x128>(r0, td[0][0]), dppstep<0x128>(r1, td[0][1]);
            dppstep<0x141>(r0, td[1][0]), dppstep<0x141>(r1, td[1][1]);
            r0 &= 0xFFFCFFFCu, r1 &= 0xFFFCFFFCu;
            dppstep<0x4E>(r0, td[2][0]), dppstep<0x4E>(r1, td[2][1]);
            dppstep<0xB1>(r0, td[3][0]), dppstep<0xB1>(r1, td[3][1]);
            r0 &= 0xFFFCFFFCu, r1 &= 0xFFFCFFFCu;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if ((r0 ^ r1) == 0x12345678u) out[1 << 20] = r0;
}

// Shipped layout, one register per lane: 6 steps = x32, x16 (in-place permlane swaps),
// x8, x7, x2, x1 (DPP); C independent chains per wave.
template <int C>
__global__ __launch_bounds__(64) void k1(uint64_t* out, int iters, uint32_t seed) {
    const int lane = threadIdx.x;
    uint32_t M[C];
    uint2 vw[6][C];
    for (int c = 0; c < C; c++) {
        M[c] = 8192u * 0x10001u + lane + c;
        for (int i = 0; i < 6; i++)
            vw[i][c] = make_uint2((seed * (i + 1) + lane + c) & 0x01ff01ffu, (seed ^ (lane * 77 + i + c)) & 0x01ff01ffu);
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int g = 0; g < 4; g++) {
#pragma unroll
            for (int c = 0; c < C; c++) {
                uint32_t A = M[c] + vw[0][c].x, m = M[c];
                asm volatile("v_permlane32_swap_b32 %0, %0\n\ts_nop 0" : "+v"(m));
                M[c] = pk_min(A, m + vw[0][c].y);
            }
#pragma unroll
            for (int c = 0; c < C; c++) {
                uint32_t A = M[c] + vw[1][c].x, m = M[c];
                asm volatile("v_permlane16_swap_b32 %0, %0\n\ts_nop 0" : "+v"(m));
                M[c] = pk_min(A, m + vw[1][c].y);
                M[c] &= 0xFFFCFFFCu;
            }
#pragma unroll
            for (int c = 0; c < C; c++) dppstep<0x128>(M[c], vw[2][c]);
#pragma unroll
            for (int c = 0; c < C; c++) {
                dppstep<0x141>(M[c], vw[3][c]);
                M[c] &= 0xFFFCFFFCu;
            }
#pragma unroll
            for (int c = 0; c < C; c++) dppstep<0x4E>(M[c], vw[4][c]);
#pragma unroll
            for (int c = 0; c < C; c++) {
                dppstep<0xB1>(M[c], vw[5][c]);
                M[c] &= 0xFFFCFFFCu;
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
    for (int c = 0; c < C; c++) x ^= M[c];
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if (x == 0x12345678u) out[1 << 20] = x;
}


// Round 5: the same two layouts with the real loop's per-state overhead (vtb_k7_lds.hip, per 48
// steps and register: 24 history clears (above), 14 v_perm + 9 v_bfi + 12 shifts of survivor
// packing, 3 survivor-word stores, table pairs read from LDS two groups ahead, the chunk's
// staging writes), so the per-frame-pair-step cost includes what does not shrink with the
// layout.  Per 6-step period and register: 2 v_perm, 1 v_bfi, 1 shift, 3 table reads (8 B per
// state-step); per 24 steps and register: 2 survivor stores (1.5 in the kernel) and 2 staging
// writes.  The two-register kernel holds two states per lane, so it does all of that twice per
// lane: equal work per state.
__device__ __forceinline__ void hist_ops(uint32_t m, uint32_t& pw, uint32_t& acc) {
    uint32_t t;
    asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(t) : "v"(m), "v"(pw), "s"(0x06020400u));
    asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(pw) : "v"(t), "v"(m), "s"(0x07030501u));
    asm volatile("v_bfi_b32 %0, %3, %1, %2" : "=v"(acc) : "v"(pw), "v"(acc), "s"(0x03030303u));
    asm volatile("v_lshlrev_b32 %0, 2, %0" : "+v"(acc));
}
// Table pairs come from LDS as in the kernel: read two periods (12 steps) ahead into a
// four-slot register ring, the read address rotating per iteration (not loop-invariant).
__global__ __launch_bounds__(64) void k1f(uint64_t* out, int iters, uint32_t seed) {
    __shared__ uint2 tab[64 * 32];
    const int lane = threadIdx.x;
    for (int i = lane; i < 64 * 32; i += 64) tab[i] = make_uint2((seed * i) & 0x01ff01ffu, (seed ^ (i * 77)) & 0x01ff01ffu);
    __syncthreads();
    uint32_t M = 8192u * 0x10001u + lane, pw = lane, acc = 0;
    uint2 vb[4][6];
    for (int g = 0; g < 4; g++)
        for (int i = 0; i < 6; i++) vb[g][i] = tab[lane + 64 * ((6 * g + i) & 31)];
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        const int rot = (it & 7) * 4;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            uint2* vw = vb[g];
            {
                uint32_t A = M + vw[0].x, m = M;
                asm volatile("v_permlane32_swap_b32 %0, %0\n\ts_nop 0" : "+v"(m));
                M = pk_min(A, m + vw[0].y);
            }
            {
                uint32_t A = M + vw[1].x, m = M;
                asm volatile("v_permlane16_swap_b32 %0, %0\n\ts_nop 0" : "+v"(m));
                M = pk_min(A, m + vw[1].y);
                hist_ops(M, pw, acc);
                M &= 0xFFFCFFFCu;
            }
#pragma unroll
            for (int i = 0; i < 6; i++) vb[(g + 2) & 3][i] = tab[lane + 64 * ((rot + 6 * g + i) & 31)];
            dppstep<0x128>(M, vw[2]);
            dppstep<0x141>(M, vw[3]);
            M &= 0xFFFCFFFCu;
            dppstep<0x4E>(M, vw[4]);
            dppstep<0xB1>(M, vw[5]);
            M &= 0xFFFCFFFCu;
        }
        asm volatile("ds_write_b32 %0, %1 offset:16384\n\tds_write_b32 %0, %2 offset:16640" ::"v"(lane * 4), "v"(acc), "v"(pw));
        asm volatile("ds_write_b32 %0, %1 offset:20480\n\tds_write_b32 %0, %2 offset:20736" ::"v"(lane * 4), "v"(M), "v"(acc));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if ((M ^ acc) == 0x12345678u) out[1 << 20] = M;
}

// Round 6: the half-partner layout (two frames per wave as lanes 0-31 / 32-63, a lane's two u16
// halves holding one frame's locations l and l ^ 32): the bit-5 butterfly is inside the register
// (no v_permlane32_swap), bits 0-3 DPP and bit 4 the permlane16 swap as shipped; everything else
// (history, table reads from LDS, stores) as k1f.  OPSEL: the partner candidate as one VOP3P
// v_pk_add_u16 with the source halves swapped (true), or a plain add of a half-swapped table
// value with the min taking the sum back through op_sel (false).
__device__ __forceinline__ uint32_t pk_min_sw(uint32_t a, uint32_t b) {
    const u16x2 bv = __builtin_bit_cast(u16x2, b);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a), __builtin_shufflevector(bv, bv, 1, 0)));
}
template <bool OPSEL>
__global__ __launch_bounds__(64) void k1h(uint64_t* out, int iters, uint32_t seed) {
    __shared__ uint2 tab[64 * 32];
    const int lane = threadIdx.x;
    for (int i = lane; i < 64 * 32; i += 64) tab[i] = make_uint2((seed * i) & 0x01ff01ffu, (seed ^ (i * 77)) & 0x01ff01ffu);
    __syncthreads();
    uint32_t M = 8192u * 0x10001u + lane, pw = lane, acc = 0;
    uint2 vb[4][6];
    for (int g = 0; g < 4; g++)
        for (int i = 0; i < 6; i++) vb[g][i] = tab[lane + 64 * ((6 * g + i) & 31)];
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        const int rot = (it & 7) * 4;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            uint2* vw = vb[g];
            {
                const uint32_t A = M + vw[0].x;
                if (OPSEL) {
                    uint32_t B;
                    asm("v_pk_add_u16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(B) : "v"(M), "v"(vw[0].y));
                    M = pk_min(A, B);
                } else {
                    M = pk_min_sw(A, M + vw[0].y);
                }
            }
            {
                uint32_t A = M + vw[1].x, m = M;
                asm volatile("v_permlane16_swap_b32 %0, %0\n\ts_nop 0" : "+v"(m));
                M = pk_min(A, m + vw[1].y);
                hist_ops(M, pw, acc);
                M &= 0xFFFCFFFCu;
            }
#pragma unroll
            for (int i = 0; i < 6; i++) vb[(g + 2) & 3][i] = tab[lane + 64 * ((rot + 6 * g + i) & 31)];
            dppstep<0x128>(M, vw[2]);
            dppstep<0x141>(M, vw[3]);
            M &= 0xFFFCFFFCu;
            dppstep<0x4E>(M, vw[4]);
            dppstep<0xB1>(M, vw[5]);
            M &= 0xFFFCFFFCu;
        }
        asm volatile("ds_write_b32 %0, %1 offset:16384\n\tds_write_b32 %0, %2 offset:16640" ::"v"(lane * 4), "v"(acc), "v"(pw));
        asm volatile("ds_write_b32 %0, %1 offset:20480\n\tds_write_b32 %0, %2 offset:20736" ::"v"(lane * 4), "v"(M), "v"(acc));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if ((M ^ acc) == 0x12345678u) out[1 << 20] = M;
}

__global__ __launch_bounds__(64) void k2f(uint64_t* out, int iters, uint32_t seed) {
    __shared__ uint2 tab[64 * 32];
    const int lane = threadIdx.x;
    for (int i = lane; i < 64 * 32; i += 64) tab[i] = make_uint2((seed * i) & 0x01ff01ffu, (seed ^ (i * 77)) & 0x01ff01ffu);
    __syncthreads();
    uint32_t r0 = 8192u * 0x10001u + lane, r1 = r0 + 3, pw0 = lane, pw1 = lane + 1, acc0 = 0, acc1 = 0;
    uint2 vb[4][12];  // per period: tq[0], tq[1] as 2 x 2 pairs, td[0..3][0..1]
    for (int g = 0; g < 4; g++)
        for (int i = 0; i < 12; i++) vb[g][i] = tab[lane + 64 * ((12 * g + i) & 31)];
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        const int rot = (it & 7) * 4;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            uint2* v = vb[g];
            asm volatile("s_nop 0\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 0" : "+v"(r0), "+v"(r1));
            inlane(r0, r1, make_uint4(v[0].x, v[0].y, v[1].x, v[1].y));
            asm volatile("s_nop 0\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 0" : "+v"(r0), "+v"(r1));
            inlane(r0, r1, make_uint4(v[2].x, v[2].y, v[3].x, v[3].y));
            hist_ops(r0, pw0, acc0);
            hist_ops(r1, pw1, acc1);
            r0 &= 0xFFFCFFFCu, r1 &= 0xFFFCFFFCu;
#pragma unroll
            for (int i = 0; i < 12; i++) vb[(g + 2) & 3][i] = tab[lane + 64 * ((rot + 12 * g + i) & 31)];
            dppstep<0x128>(r0, v[4]), dppstep<0x128>(r1, v[5]);
            dppstep<0x141>(r0, v[6]), dppstep<0x141>(r1, v[7]);
            r0 &= 0xFFFCFFFCu, r1 &= 0xFFFCFFFCu;
            dppstep<0x4E>(r0, v[8]), dppstep<0x4E>(r1, v[9]);
            dppstep<0xB1>(r0, v[10]), dppstep<0xB1>(r1, v[11]);
            r0 &= 0xFFFCFFFCu, r1 &= 0xFFFCFFFCu;
        }
        asm volatile("ds_write_b32 %0, %1 offset:16384\n\tds_write_b32 %0, %2 offset:16640" ::"v"(lane * 4), "v"(acc0), "v"(pw0));
        asm volatile("ds_write_b32 %0, %1 offset:20480\n\tds_write_b32 %0, %2 offset:20736" ::"v"(lane * 4), "v"(r0), "v"(acc0));
        asm volatile("ds_write_b32 %0, %1 offset:24576\n\tds_write_b32 %0, %2 offset:24832" ::"v"(lane * 4), "v"(acc1), "v"(pw1));
        asm volatile("ds_write_b32 %0, %1 offset:28672\n\tds_write_b32 %0, %2 offset:28928" ::"v"(lane * 4), "v"(r1), "v"(acc1));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if ((r0 ^ r1 ^ acc0 ^ acc1) == 0x12345678u) out[1 << 20] = r0;
}

template <typename F>
double run(F kern, int cus, int wps, int pairs_per_wave, double mhz) {
    uint64_t* d;
    (void)hipMalloc(&d, (size_t(1) << 20) * 8 + 8);
    const int iters = 2000, steps = iters * 24;
    const int blocks = cus * 4 * wps;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, d, iters, 12345u);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, d, iters, 12345u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(d);
    return ms * 1e-3 * mhz * 1e6 / (double(steps) * pairs_per_wave * wps);
}

int main(int argc, char** argv) {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const double mhz = 2400.0;
    const int cus = p.multiProcessorCount;
    if (argc > 1 && argv[1][0] == 'h') {
        // round 6: shipped vs the half-partner layout, interleaved, five rounds
        for (int r = 0; r < 5; r++)
            for (int wps : {2, 4})
                printf("round %d W=%d: shipped %.2f  half-partner (VOP3P add) %.2f  half-partner (op_sel min) %.2f  "
                       "cycles per frame-pair-step per SIMD\n",
                       r, wps, run(k1f, cus, wps, 1, mhz), run(k1h<true>, cus, wps, 1, mhz), run(k1h<false>, cus, wps, 1, mhz));
        return 0;
    }
    for (int wps : {1, 2, 4}) {
        printf("W=%d waves/SIMD: shipped C=1 %.2f  shipped C=2 %.2f  two-register %.2f  cycles per frame-pair-step per SIMD\n",
               wps, run(k1<1>, cus, wps, 1, mhz), run(k1<2>, cus, wps, 2, mhz), run(k2, cus, wps, 2, mhz));
    }
    // Round 5: the two-register layout fed with split halves for the 4,096 x
    // 1,024 soft launch.  4,096 frames = 8,192 half-frames, four per wave, two waves per SIMD;
    // each half runs t1 = 576 steps (split_t1(1030, 96): frame A [0, 576), frame B [480, 1056)),
    // i.e. 1,152 steps per frame against the pair kernel's 1,032.
    for (int wps : {1, 2}) {
        const double c1 = run(k1f, cus, wps, 1, mhz), c2 = run(k2f, cus, wps, 2, mhz);
        printf("with overhead, W=%d: shipped %.2f  two-register %.2f  cycles per frame-pair-step per SIMD\n", wps, c1, c2);
    }
    const double ship = run(k1f, cus, 2, 1, mhz), two = run(k2f, cus, 2, 2, mhz);
    const double per_frame_ship = 1032.0 * ship, per_frame_halves = 2.0 * 576.0 * two;
    printf("4096 x 1024 soft, ACS per frame pair (SIMD cycles): pair kernel %.0f (1032 steps x %.2f), two-register halves "
           "%.0f (2 x 576 steps x %.2f): %+.1f %%\n",
           per_frame_ship, ship, per_frame_halves, two, 100.0 * (per_frame_halves / per_frame_ship - 1.0));
    return 0;
}
