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
// One wave64 per frame.  The N = 2^(kS) <= 256 states spread over the lanes (N <= 64: state d
// in lane d, predecessors by ds_bpermute; N = 256: states 4 lane .. 4 lane + 3, values
// double-buffered in LDS), survivor pointers every S steps instead of per-step decisions
// (below), a verified block-parallel traceback over them.  A completeness kernel: these codes
// are not on the headline path.

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
    int ptr_bytes;   // survivor-pointer bytes per frame (gen_ptr_bytes)
    int u8;          // VTB_GENK_K1_REFERENCE_U8: the reference's k=1 butterfly arithmetic (below)
    int warm;        // traceback warm-up steps per block (any value is exact: the walk is verified)
    int dbg;         // the knobs' $VTB_DEBUG: bit 17 caps the verification; -DVTB_MEASURE builds: bit 0 skips the traceback, 1 the ACS
    uint32_t* hits;  // testing: completeness-guard counter (Launch::guard_hits), null in production
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

// Survivor pointers (round 3).  Every state carries V = (m << 12) | (e << 8) | ptr: m its path
// metric (20 bits: at most n T < 2^18), e its own top k bits -- the edge index under which all
// its successors see it (src = d / 2^k + e 2^((S-1)k)) -- and ptr the state its survivor path
// passed through at the last boundary.  A candidate is then V_src + (bm << 12): one min over
// the 2^k candidates gives the metric, the first minimum (lowest e among equal metrics, the
// reference's argmin: e sits below the metric) and the survivor's pointer in one value, so the
// per-step decisions are never stored.  Boundaries are the steps t = t_b (mod S), t_b = (T-1)
// mod S: there each state's ptr (8 bits) is written out and reset to the state itself.  A
// state's S steps of inputs are its own bits, so the traceback jumps S steps per read and
// emits the state at each boundary as the kS output bits of that window.
constexpr int kMetShift = 12;

// Boundaries of a frame of T steps (S steps apart, the last at step T-1) and their pointer bytes.
__host__ __device__ constexpr int gen_boundaries(int T, int S) { return (T - 1) / S + 1; }
size_t gen_ptr_bytes(int T, int S, int N) { return size_t(gen_boundaries(T, S)) * size_t(N < 4 ? 4 : N); }

GenLayout gen_layout(int N, int E, int T, int L, int S, bool gdec) {
    GenLayout l;
    l.dec = 0;                                                         // pointer bytes (in LDS unless gdec)
    l.met = (l.dec + (gdec ? 0 : gen_ptr_bytes(T, S, N)) + 15) & ~size_t(15);  // 2 * N uint32
    l.tab = l.met + 8 * size_t(N);                                     // N * E bytes
    l.inb = (l.tab + size_t(N) * E + 15) & ~size_t(15);               // T + 1 bytes
    l.outb = (l.inb + size_t(T) + 1 + 15) & ~size_t(15);              // ceil(L / 8) bytes
    l.total = (l.outb + size_t((L + 7) / 8) + 15) & ~size_t(15);
    return l;
}

// The state's constant low 12 bits: e << 8 | (d & 0xFF) (the pointer reset value).
__device__ __forceinline__ uint32_t own_tag(int d, int kS, int KB) {
    return (uint32_t(d >> (kS - KB)) << 8) | uint32_t(d & 0xFF);
}

// Branch metrics.  PK (n <= 3): the branch metrics of all 2^n labels for the step's received
// segment rx packed 4 bits per label in one word (ptab: lane x holds the word for rx = x, read
// back with v_readlane), so a candidate is V + (bfe(P, 4 lab, 4) << 12): two instructions per
// edge.  Otherwise popc(lab ^ rx): three.
template <bool PK>
__device__ __forceinline__ uint32_t gen_cand(uint32_t v, uint32_t lab, uint32_t rx, uint32_t P) {
    if (PK) return (__builtin_amdgcn_ubfe(P, lab, 4) << kMetShift) + v;
    return (uint32_t(__popc(lab ^ rx)) << kMetShift) + v;
}

__device__ __forceinline__ uint32_t gen_ptab(int n, int lane) {
    uint32_t p = 0;
    for (int x = 0; x < (1 << n); x++) p |= uint32_t(__popc(uint32_t(x) ^ uint32_t(lane))) << (4 * x);
    return p;
}

// The new state value: the winning candidate with its e field (and at a boundary its pointer)
// replaced by the state's own.
__device__ __forceinline__ uint32_t gen_next(uint32_t best, uint32_t tag, bool bnd) {
    const uint32_t mask = bnd ? 0xFFFu : 0xF00u;
    return (best & ~mask) | (tag & mask);
}

// N <= 64 states: one state per lane, its value in a register, the 2^k predecessors gathered
// with ds_bpermute, the lane's 2^k edge labels (time-invariant) in registers; k is a template
// parameter so every per-edge loop is unrolled.  Pointers: one byte per state and boundary.
//
// U8 (k = 1 only): the reference's k=1 butterfly arithmetic (viterbiDecoderButterflyk1.c:101-183)
// -- the upper predecessor's branch metric is n minus the lower's, whatever the generators
// (:104-107), sums wrap mod 256 (uint8 METRIC_TYPE), the strict '>' keeps the lower predecessor
// on ties (:129-130), and when the counter reaches 120 the minimum is subtracted (:159-183) --
// so that codes whose uint8 sums can wrap (n >= 4) decode exactly as the reference does.
template <int KB, bool U8 = false, bool PK = false>
__device__ __forceinline__ void acs_r1(int N, int S, int T, int n, const uint8_t* inb, uint32_t nmask,
                                       const uint8_t* tab, const int32_t* met, uint8_t* ptrs, int lane) {
    constexpr int E = 1 << KB;
    const int kS = KB * S;
    const int d = lane;
    const bool live = d < N;
    const uint32_t tag = live ? own_tag(d, kS, KB) : 0u;
    uint32_t v = live ? (uint32_t(met[d]) << kMetShift) | tag : 0u;
    constexpr bool LIN = !PK && !U8;  // as in acs_rn below
    uint32_t lab[E], be[E];
    int srcl[E];
    const uint32_t labd = live ? uint32_t(tab[d]) : 0u;
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int src = live ? (d >> KB) | (e << (kS - KB)) : 0;
        srcl[e] = src << 2;
        be[e] = LIN ? __builtin_amdgcn_readfirstlane(uint32_t(tab[e << kS])) : 0u;
        if (LIN)
            lab[e] = 0;
        else if (U8)  // butterfly j = d >> 1: symm[j] = label of delay (j << 1) | 0, complemented for ec
            lab[e] = live ? uint32_t(tab[(d >> 1) << 1]) ^ ((((d & 1) ^ e) & 1) ? nmask : 0u) : 0u;
        else
            lab[e] = live ? uint32_t(tab[(src << KB) | (d & (E - 1))]) : 0u;
        if (PK) lab[e] *= 4;  // bit offset of the label's field in the packed word
    }
    const uint32_t ptab = PK ? gen_ptab(n, lane) : 0u;
    uint32_t renorm = 0;
    int cnt = S - 1 - (T - 1) % S, bi = 0;  // steps into the current window, boundary index
    for (int t = 0; t < T; t++) {
        const uint32_t rx = inb[t] & nmask;
        const uint32_t P = PK ? __builtin_amdgcn_readlane(ptab, __builtin_amdgcn_readfirstlane(rx)) : 0u;
        uint32_t best = 0xFFFFFFFFu;
#pragma unroll
        for (int e = 0; e < E; e++) {
            const uint32_t pv = uint32_t(__builtin_amdgcn_ds_bpermute(srcl[e], int(v)));
            uint32_t c = LIN ? gen_cand<false>(pv, labd, be[e] ^ __builtin_amdgcn_readfirstlane(rx), 0u)
                             : gen_cand<PK>(pv, lab[e], rx, P);
            if (U8) c &= 0xFFFFFu;  // (pm + bm) mod 256
            best = min(best, c);
        }
        const bool bnd = cnt == S - 1;
        cnt = bnd ? 0 : cnt + 1;
        if (bnd) {
            if (live) ptrs[size_t(bi) * size_t(N < 4 ? 4 : N) + d] = uint8_t(best);
            bi++;
        }
        v = gen_next(best, tag, bnd);
        if (U8) {
            if (renorm >= 120) {
                v -= wave_min(live ? v : 0xFFFFFFFFu) & ~0xFFFu;
                renorm = 0;
            } else {
                renorm++;
            }
        }
    }
}

// N = 64 R states, R = 2 (k = 1, K = 8) or 4 (k S = 8: k = 1, 2 or 4), R consecutive states per
// lane: d = R lane + r.  Their predecessors src = d / 2^k + e 2^(kS-k) then coincide: at
// R = 4 and k = 2, 4 all four states of a lane share the same 2^k predecessors (lane + 64 e;
// lane / 4 + 16 e), at k = 1 pairs do (2 lane + r / 2 + 128 e; R = 2: lane + 64 e), so a lane
// reads 4, 4, 16 or 2 values per step instead of R 2^k, and writes its R new values as one
// 16- or 8-byte store.  The values live in LDS (double-buffered, state s at s); the R 2^k
// edge labels of a lane's states are time-invariant and sit in registers (k is a template
// parameter: every per-edge loop unrolls).  Pointers: the lane's R bytes form one dword or
// halfword, so boundary i's N bytes are in state order.
template <int KB, int R, bool U8 = false, bool PK = false>
__device__ __forceinline__ void acs_rn(int T, int n, const uint8_t* inb, uint32_t nmask, const uint8_t* tab,
                                       uint32_t* met, uint8_t* ptrs, int lane) {
    static_assert(R == 4 || (R == 2 && KB == 1), "N = 128 only at k = 1");
    constexpr int E = 1 << KB, kS = R == 4 ? 8 : 7, N = 64 * R, S = kS / KB;
    constexpr int G = (R >> KB) > 1 ? (R >> KB) : 1;  // distinct predecessor sets per lane
    // LIN (neither packed nor U8): the label of edge (e -> d) is tab[d | e << kS] = tab[d] ^
    // tab[e << kS] (the encoder is linear over GF(2)), so a lane keeps its states' tab[d] (4
    // registers) and the step's uniform y_e = tab[e << kS] ^ rx sits in scalar registers,
    // instead of 4 * 2^k label registers (64 at k = 4: the wave count per SIMD)
    constexpr bool LIN = !PK && !U8;
    uint32_t lab[R][LIN ? 1 : E], tag[R], be[E];
    const int base = (R * lane) >> KB;  // + g: the lane's predecessor sets
#pragma unroll
    for (int e = 0; e < E; e++) be[e] = LIN ? __builtin_amdgcn_readfirstlane(uint32_t(tab[e << kS])) : 0u;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int d = R * lane + r;
        tag[r] = own_tag(d, kS, KB);
        met[d] = (met[d] << kMetShift) | tag[r];
        if (LIN) {
            lab[r][0] = tab[d];
            continue;
        }
#pragma unroll
        for (int e = 0; e < (LIN ? 1 : E); e++) {
            if (U8)  // the butterfly identity of acs_r1 U8
                lab[r][e] = uint32_t(tab[(d >> 1) << 1]) ^ ((((d & 1) ^ e) & 1) ? nmask : 0u);
            else
                lab[r][e] = uint32_t(tab[d | (e << kS)]);
            if (PK) lab[r][e] *= 4;
        }
    }
    const uint32_t ptab = PK ? gen_ptab(n, lane) : 0u;
    int cur = 0;
    uint32_t renorm = 0;
    int cnt = S - 1 - (T - 1) % S, bi = 0;
    // (PK: the next step's packed word is fetched a step ahead, off the metric chain; inb[T] is
    // inside the LDS layout, its value unused)
    uint32_t Pn = PK ? __builtin_amdgcn_readlane(ptab, __builtin_amdgcn_readfirstlane(inb[0] & nmask)) : 0u;
    for (int t = 0; t < T; t++) {
        const uint32_t rx = inb[t] & nmask;
        const uint32_t P = Pn;
        if (PK) Pn = __builtin_amdgcn_readlane(ptab, __builtin_amdgcn_readfirstlane(inb[t + 1] & nmask));
        const uint32_t* mc = met + cur * N;
        uint32_t* mn = met + (cur ^ 1) * N;
        const bool bnd = cnt == S - 1;
        cnt = bnd ? 0 : cnt + 1;
        uint32_t pv[G][E], y[E], nm[R];
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
            for (int e = 0; e < E; e++) pv[g][e] = mc[base + g + (e << (kS - KB))];
#pragma unroll
        for (int e = 0; e < E; e++) y[e] = LIN ? be[e] ^ __builtin_amdgcn_readfirstlane(rx) : 0u;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int g = G > 1 ? r >> KB : 0;
            uint32_t best = 0xFFFFFFFFu;
#pragma unroll
            for (int e = 0; e < E; e++) {
                uint32_t c = LIN ? gen_cand<false>(pv[g][e], lab[r][0], y[e], 0u)
                                 : gen_cand<PK>(pv[g][e], lab[r][e], rx, P);
                if (U8) c &= 0xFFFFFu;
                best = min(best, c);
            }
            nm[r] = best;
        }
        if (bnd) {
            const uint32_t lo = __builtin_amdgcn_perm(nm[1], nm[0], 0x0c0c0400u);
            if constexpr (R == 4)
                reinterpret_cast<uint32_t*>(ptrs)[size_t(bi) * 64 + lane] =
                    lo | __builtin_amdgcn_perm(nm[R - 1], nm[R - 2], 0x04000c0cu);
            else
                reinterpret_cast<uint16_t*>(ptrs)[size_t(bi) * 64 + lane] = uint16_t(lo);
            bi++;
        }
#pragma unroll
        for (int r = 0; r < R; r++) nm[r] = gen_next(nm[r], tag[r], bnd);
        if (U8) {
            if (renorm >= 120) {
                uint32_t mr = nm[0];
#pragma unroll
                for (int r = 1; r < R; r++) mr = min(mr, nm[r]);
                mr = wave_min(mr) & ~0xFFFu;
#pragma unroll
                for (int r = 0; r < R; r++) nm[r] -= mr;
                renorm = 0;
            } else {
                renorm++;
            }
        }
        if constexpr (R == 4)
            reinterpret_cast<uint4*>(mn)[lane] = make_uint4(nm[0], nm[1], nm[R - 2], nm[R - 1]);
        else
            reinterpret_cast<uint2*>(mn)[lane] = make_uint2(nm[0], nm[1]);
        cur ^= 1;
        // one wave per workgroup: its LDS accesses complete in issue order, so the next step's
        // reads see these writes without a workgroup barrier (a compiler fence keeps the order)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// GDEC: pointer bytes in a global workspace (one slot per frame of the launch) instead of
// LDS, for trellises whose pointers would hold the CU to few waves.
template <bool GDEC, int KB>
__global__ __launch_bounds__(64) void genk_kernel(const uint8_t* __restrict__ in, size_t in_stride,
                                                  uint8_t* __restrict__ out, size_t out_stride, size_t frames,
                                                  GenArgs a, GenLayout ly, uint8_t* __restrict__ ws) {
    extern __shared__ uint64_t gsm[];
    uint8_t* sm = reinterpret_cast<uint8_t*>(gsm);
    uint8_t* ptrs = GDEC ? ws + size_t(blockIdx.x) * size_t(a.ptr_bytes) : sm + ly.dec;
    uint32_t* met = reinterpret_cast<uint32_t*>(sm + ly.met);
    uint8_t* tab = sm + ly.tab;
    uint8_t* inb = sm + ly.inb;
    uint8_t* outb = sm + ly.outb;
    const int lane = threadIdx.x;
    const size_t f = blockIdx.x;
    if (f >= frames) return;
    constexpr int k = KB, E = 1 << KB;  // one instance per k: each gets its own register budget
    const int N = a.N, S = a.S, kS = k * S, T = a.T, R = a.R, n = a.n;
    const uint32_t nmask = (1u << n) - 1u;

    for (int i = lane; i < N * E; i += 64) {  // edge labels, index = delay (src << k) | bits
        uint32_t o = 0;
        for (int j = 0; j < n; j++) o |= (uint32_t(__popc(uint32_t(i) & a.rg[j])) & 1u) << j;
        tab[i] = uint8_t(o);
    }
    const uint8_t* row = in + f * in_stride;
#pragma unroll 1
    for (int i = lane; i <= T; i += 64) inb[i] = i < T ? row[i] : 0;
#pragma unroll 1
    for (int i = lane; i < (a.L + 7) / 8; i += 64) outb[i] = 0;
    const uint32_t init = uint8_t(N + 1);
    for (int d = lane; d < N; d += 64) met[d] = d == 0 ? 0 : init;
    __syncthreads();

    const bool pk = n <= 3;
    if (a.dbg & 2) {
    } else if (R == 1) {
        const int32_t* m0 = reinterpret_cast<const int32_t*>(met);
        if (KB == 1 && a.u8)
            pk ? acs_r1<KB, true, true>(N, S, T, n, inb, nmask, tab, m0, ptrs, lane)
               : acs_r1<KB, true>(N, S, T, n, inb, nmask, tab, m0, ptrs, lane);
        else
            pk ? acs_r1<KB, false, true>(N, S, T, n, inb, nmask, tab, m0, ptrs, lane)
               : acs_r1<KB, false>(N, S, T, n, inb, nmask, tab, m0, ptrs, lane);
    } else if (R == 2) {  // k = 1, K = 8
        if constexpr (KB == 1) {
            if (a.u8)
                pk ? acs_rn<1, 2, true, true>(T, n, inb, nmask, tab, met, ptrs, lane)
                   : acs_rn<1, 2, true>(T, n, inb, nmask, tab, met, ptrs, lane);
            else
                pk ? acs_rn<1, 2, false, true>(T, n, inb, nmask, tab, met, ptrs, lane)
                   : acs_rn<1, 2, false>(T, n, inb, nmask, tab, met, ptrs, lane);
        }
    } else if constexpr (KB == 1 || KB == 2 || KB == 4) {
        // (k = 4: 64 packed-label registers would cost waves; the linear labels need 4)
        if (KB == 1 && a.u8)
            pk ? acs_rn<KB, 4, true, true>(T, n, inb, nmask, tab, met, ptrs, lane)
               : acs_rn<KB, 4, true>(T, n, inb, nmask, tab, met, ptrs, lane);
        else
            pk && KB != 4 ? acs_rn<KB, 4, false, KB != 4>(T, n, inb, nmask, tab, met, ptrs, lane)
                          : acs_rn<KB, 4, false>(T, n, inb, nmask, tab, met, ptrs, lane);
    }
    __syncthreads();

    // Traceback over the boundaries (i = 0 .. nb-1, boundary i at step t_b + i S, the last at
    // T-1 where the terminated frame is in state 0), block-parallel and verified (the K=7
    // kernel's scheme, vtb_k7_lds.hip): lane b walks boundaries [b tbb, (b+1) tbb) back from
    // a warm-up past its block's end, starting from state 0 there (exact when the walk starts
    // at the last boundary).  A block is right if it entered on its successor's exit state and
    // that successor is proven; failed blocks re-walk from a proven successor until all are
    // proven.  Then every lane emits its block's windows (LDS atomic OR: windows share words).
    if (!(a.dbg & 1)) {
        const int nb = gen_boundaries(T, S), pstride = N < 4 ? 4 : N;
        const int warm = (a.warm + S - 1) / S;
        auto ptr = [&](int i, int s) -> int {  // state at boundary i-1 on the survivor of s at i
            return ptrs[size_t(i) * size_t(pstride) + s];  // (R > 1: the lanes' words are in state order)
        };
        const int tbb = (nb + 63) / 64, lo = lane * tbb, top = min(lo + tbb, nb);
        const bool active = lo < nb;
        const int start = min(top + warm, nb);
        int s = 0;
        for (int i = start - 1; active && i >= top; i--) s = ptr(i, s);
        int s_top = s;
        for (int i = top - 1; active && i >= lo; i--) s = ptr(i, s);
        // (one chain of up to 64 blocks: at most 63 re-walk rounds.)  Completeness guard: a block
        // still unproven after the cap (VTB_DEBUG bit 17: every chain with a walked block) sends the frame to its
        // serial walk -- lane 0 emits every window from state 0 at the last boundary
        int fin = s;
        bool fixed = !active || start == nb;
        const bool tbforce = (a.dbg & kDbgTbCap) != 0;
        const int rounds = tbforce ? 0 : 65;
        bool unproven = false;
        for (int round = 0;; round++) {
            const int sf = __shfl_down(fin, 1);
            const bool ok = fixed || (s_top == sf && !tbforce);
            const uint64_t bad = ~__ballot(ok);
            if (bad == 0) break;
            if (round == rounds) {
                unproven = true;
                break;
            }
            if (!ok && (bad >> (lane + 1)) == 0) {
                s_top = s = sf;
                for (int i = top - 1; i >= lo; i--) s = ptr(i, s);
                fin = s;
                fixed = true;
            }
        }
        int elo = lo, etop = top;  // emitted boundaries [elo, etop), from s_top at etop - 1
        bool emit = active;
        if (unproven) {
            emit = lane == 0, elo = 0, etop = nb, s_top = 0;
            if (lane == 0) note_guard(a.hits);
        }
        // window i holds the inputs of steps t_b + (i-1) S + 1 .. t_b + i S: the kS bits of the
        // state at boundary i, oldest (its top bits) first, at stream bit p0 = (t_b + (i-1) S + 1) k
        // (the first window's bits before step 0 are the start state's and dropped; the last
        // window is the S flush steps and not emitted)
        uint32_t* ow = reinterpret_cast<uint32_t*>(outb);
        const int tb0 = (T - 1) % S;
        uint32_t acc = 0;
        int wcur = -1;
        auto put = [&](int byte, uint32_t v) {
            if ((byte >> 2) != wcur) {
                if (acc) atomicOr(ow + wcur, acc);
                wcur = byte >> 2, acc = 0;
            }
            acc |= v << (8 * (byte & 3));
        };
        s = s_top;
        for (int i = etop - 1; emit && i >= elo; i--) {
            if (i < nb - 1) {
                int p0 = (tb0 + (i - 1) * S + 1) * k, w = kS;
                uint32_t fv = uint32_t(s);
                if (p0 < 0) {
                    w += p0;
                    fv &= (1u << w) - 1u;
                    p0 = 0;
                }
                const uint32_t v16 = fv << (16 - w - (p0 & 7));
                const int byte = p0 >> 3;
                if (v16 & 0xFFu) put(byte + 1, v16 & 0xFFu);
                if (v16 >> 8) put(byte, v16 >> 8);
            }
            s = ptr(i, s);
        }
        if (acc) atomicOr(ow + wcur, acc);
    }
    __syncthreads();
    uint8_t* orow = out + f * out_stride;  // (GDEC: each lane read the pointer bytes its walks need)
#pragma unroll 1  // (unrolled, the byte copy would set the kernel's register count)
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
    hipStream_t st = (hipStream_t)stream;
    // testing knobs (vtb_internal.h), read per call: this entry point has no plan to hold them
    const vtb::Knobs kn = vtb::read_knobs();
    // k = 1, K = 7 or 9, rate 1/3, hard segments: the K=7 LDS pair kernel / the K=9 frame kernel
    // with a 16-column table (vtb_k7_lds.hip k7_pair NB = 3, vtb_k9.hip k9_pair NB = 3).  Its butterfly takes the upper predecessor's branch
    // metric as n - e (reference viterbiDecoderButterflyk1.c:104-107): the reference's own
    // arithmetic for any generators, and the exact one when every generator taps both ends.
    // Its exact metrics equal the reference's uint8 ones at n = 3 (the minimum grows by at most
    // one per step, so nothing wraps: DESIGN.md §3, §4.7).  VTB_KERNEL=genk keeps this kernel.
    if (k == 1 && (K == 7 || K == 9) && n == 3 && kn.force != vtb::Force::Genk) {
        bool ends = true;
        for (int i = 0; i < n; i++) ends = ends && ((code->generators[i] >> (K - 1)) & 1u) && (code->generators[i] & 1u);
        vtb::Launch la;
        la.S = S, la.soft = 0, la.T = T, la.L = info_bits;
        la.in = d_in, la.in_stride = in_stride, la.out = d_out, la.out_stride = out_stride;
        la.frames = frames, la.stream = st, la.cus = vtb::current_device_cus(), la.dbg = kn.dbg;
        la.guard_hits = vtb::debug_guard_hits();
        uint32_t rg[3];
        for (int i = 0; i < 3; i++) rg[i] = vtb::gen_rev(code->generators[i], K);
        for (int j = 0; j < (1 << (K - 2)); j++) {  // label of butterfly j: the encoder on delay (j << 1) | 0 (reference :24-29)
            uint32_t c = 0;
            for (int i = 0; i < 3; i++) c |= uint32_t(__builtin_popcount((uint32_t(j) << 1) & rg[i]) & 1) << i;
            la.symm[j] = uint8_t(c);
        }
        if ((u8 || ends) && K == 7 && vtb::k7_n3_supported(la)) {
            const hipError_t e = vtb::launch_k7_lds_n3(la);
            return e == hipSuccess ? VTB_OK : e == hipErrorOutOfMemory ? VTB_ERR_NOMEM : VTB_ERR_DEVICE;
        }
        // K = 9 (the K=9 frame kernel, survivors in a workspace from the stream's pool)
        if ((u8 || ends) && K == 9 && vtb::k9_n3_supported(la)) {
            void* ws = nullptr;
            if (vtb::workspace_alloc(&ws, vtb::k9_n3_workspace_bytes(la), st) != hipSuccess) return VTB_ERR_NOMEM;
            la.ws = ws;
            const hipError_t e = vtb::launch_k9_n3(la);
            const bool freed = vtb::workspace_free(ws, st) == hipSuccess;
            if (e != hipSuccess) return e == hipErrorOutOfMemory ? VTB_ERR_NOMEM : VTB_ERR_DEVICE;
            return freed ? VTB_OK : VTB_ERR_DEVICE;
        }
    }
    vtb::GenArgs a{};
    a.k = k, a.S = S, a.n = n, a.N = N, a.T = T, a.L = info_bits, a.R = R, a.u8 = u8 ? 1 : 0;
    a.dbg = kn.dbg;
    a.hits = vtb::debug_guard_hits();
    a.warm = kn.genk_warm >= 0 ? kn.genk_warm : 96;  // ($VTB_GENK_WARM: measurement only)
    for (int i = 0; i < n; i++) a.rg[i] = vtb::gen_rev(code->generators[i], k * K);
    // survivor pointers in LDS while they leave room for 4 waves per CU, else in a workspace
    const size_t dec_bytes = (vtb::gen_ptr_bytes(T, S, N) + 15) & ~size_t(15);
    a.ptr_bytes = int(dec_bytes);
    const bool gdec = dec_bytes > 32 * 1024;
    const vtb::GenLayout ly = vtb::gen_layout(N, E, T, info_bits, S, gdec);
    if (ly.total > 160 * 1024 || frames > 0x7fffffffu) return VTB_ERR_UNSUPPORTED;
    vtb::note_kernel("genk");
    const auto kern = [&](bool g) -> const void* {
        switch (k) {
            case 1: return g ? reinterpret_cast<const void*>(vtb::genk_kernel<true, 1>)
                             : reinterpret_cast<const void*>(vtb::genk_kernel<false, 1>);
            case 2: return g ? reinterpret_cast<const void*>(vtb::genk_kernel<true, 2>)
                             : reinterpret_cast<const void*>(vtb::genk_kernel<false, 2>);
            case 3: return g ? reinterpret_cast<const void*>(vtb::genk_kernel<true, 3>)
                             : reinterpret_cast<const void*>(vtb::genk_kernel<false, 3>);
            default: return g ? reinterpret_cast<const void*>(vtb::genk_kernel<true, 4>)
                              : reinterpret_cast<const void*>(vtb::genk_kernel<false, 4>);
        }
    };
    const auto launch = [&](bool g, size_t f0, size_t nf, uint8_t* ws) {
        const uint8_t* pin = d_in + f0 * in_stride;
        uint8_t* pout = d_out + f0 * out_stride;
        void* args[] = {&pin, const_cast<size_t*>(&in_stride), &pout, const_cast<size_t*>(&out_stride), &nf,
                        &a, const_cast<vtb::GenLayout*>(&ly), &ws};
        if (hipLaunchKernel(kern(g), dim3(unsigned(nf)), dim3(64), args, ly.total, st) != hipSuccess)
            return VTB_ERR_DEVICE;
        return vtb::gen_status();
    };
    if (!gdec) {
        if (ly.total > 64 * 1024 &&
            hipFuncSetAttribute(kern(false), hipFuncAttributeMaxDynamicSharedMemorySize, int(ly.total)) != hipSuccess)
            return VTB_ERR_DEVICE;
        return launch(false, 0, frames, nullptr);
    }
    // workspace from the stream's pool, up to 1 GiB per launch (frames in launches of that)
    const size_t per = std::max<size_t>(1, (size_t(1) << 30) / dec_bytes);
    const size_t chunk = std::min(frames, per);
    // (the per-device pool that keeps its memory between launches, vtb_api.hip workspace_alloc)
    void* ws = nullptr;
    if (vtb::workspace_alloc(&ws, chunk * dec_bytes, st) != hipSuccess) return VTB_ERR_NOMEM;
    int rc = VTB_OK;
    for (size_t f0 = 0; f0 < frames && rc == VTB_OK; f0 += chunk)
        rc = launch(true, f0, std::min(chunk, frames - f0), static_cast<uint8_t*>(ws));
    if (vtb::workspace_free(ws, st) != hipSuccess && rc == VTB_OK) rc = VTB_ERR_DEVICE;
    return rc;
}

}  // extern "C"
