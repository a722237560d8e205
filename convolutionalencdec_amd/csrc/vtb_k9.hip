// K=9 (256 states) decoder, hard and 8-bit soft input: BASELINE config C4.
//
// The K=7 kernel's design (vtb_k7_lds.hip header) scaled to 256 states:
//
// Layout.  One wave64 decodes two frames, A and B, packed in the u16 halves of every
// register.  Location l (8 bits) = r * 64 + lambda lives in register M[r] of lane
// lane_of(lambda): location bits 0..5 are lane bits (lane XOR 1, 2, 7, 8, 16, 32 through
// the same involution as K=7), bits 6..7 select one of four registers.
//
// In-place state relabelling (reference butterfly viterbiDecoderButterflyk1.c:101-152).
// Location l holds state rotl8(l, t mod 8) at step t; the two sources of a butterfly sit
// at locations differing in bit p = 7 - (t mod 8).  For p = 7, 6 the partner is another
// register of the same lane (no cross-lane op at all); for p = 5, 4 an in-place
// v_permlane32/16_swap per register; for p = 3..0 a DPP row_ror:8 / row_half_mirror /
// quad_perm folded into the add.
//
// Metrics carry their decisions exactly as in the K=7 kernel: a stored metric is 4m + h,
// the tie bit R << b / (1 - R) << b (b = t & 1) enters both candidates from the
// branch-metric table, so M' = pk_min(A, B) keeps the decision D (the location bit p of
// the survivor's predecessor) in bit b; after each odd step the two history bits are
// gathered into per-register survivor words (one v_perm per two windows, three v_bfi per
// 16 steps) and cleared.  Ties go to the lower predecessor (strict '>', reference
// :129-130).
//
// Start metrics: the reference's K=9 start value is (uint8)(NUM_STATES+1) = 1 (x255 soft,
// reference viterbiDecoderButterflyk1.c:62), kept exactly (the K=7 kernel's larger
// equivalent start value does not apply).
//
// Renormalisation every 12 steps against location 0 (state 0) with bias B = 16Q (= nQS):
// for every t, m_t(s) - m_t(0) >= -nQS, and the spread plus 12 steps of growth keeps
// 4m + 3 + a candidate's table value below 2^16 (DESIGN.md §3, K=9 figures).
//
// Survivors.  64 B per step per wave do not fit LDS at useful occupancy, so they go to a
// per-wave global workspace: per 16 steps a 1-KB column of 256 words, the word of
// location l at byte 4 rev6(lambda) + 256 rev2(r) -- i.e. address bits 2..7 carry bits
// 2..7 of l' = rev8(l) and address bits 8..9 its bits 0..1.  Each register's store is one
// contiguous 256-B wave store.  In l' numbering step t's pairing bit is bit t mod 8, so a
// window's two decisions are adjacent address bits and the traceback edits the word
// address in place (one global_load_ushort, one shift, one bit-field insert per window).
//
// Frame ends.  Windows pair an even and an odd step, so the kernel runs Tq = T + delta
// steps with delta = T & 1: for odd T one extra own-keeping step at the start (its table
// row makes every location keep its own predecessor, which leaves the start metrics
// unchanged) and the decoded bit stream is shifted back by one bit at the copy-out.  Steps
// past Tq up to the 48-step chunk grid run on clamped input; afterwards their survivor
// bits are overwritten with own-keeping decisions, so a walk from location 0 at the end of
// the padding reaches location 0 (the terminated state) at Tq.
//
// Traceback (reference :200-256): the K=7 kernel's verified block-parallel chains, with
// 8-bit locations (an octet's eight decoded bits are its end location l', oldest step at
// bit 0).

#include <utility>

#include "vtb_k7_common.h"

namespace vtb {
namespace {

using k7::pk_min;
using k7::uniform64;

constexpr int kCh = 48;                  // ACS steps per unrolled chunk (multiple of 8 and 16)
constexpr int kCol = 49;                 // 8-byte slots per table column (48 rows + bank skew)
constexpr int kRingBytes = 8 * kCol * 8;  // branch-metric ring: 8 (label, R) columns
constexpr int kAH = 2;                  // table rows read this many steps ahead
constexpr int kRS = 3;                  // register ring slots (48 % kRS == 0)
constexpr int kTbWarm = 48;              // traceback warm-up steps past a block's end
constexpr uint32_t kR1 = 0x10001u;
constexpr int kColBytes = 1024;          // survivor column: 256 words per 16 steps

// History bits per u16 half (as vtb_k7_lds.hip): soft input keeps 4m + h (2 history bits);
// hard input, whose metrics stay below 256, keeps 256m + h with 8 history
// bits -- tie bit at t mod 8, survivor byte and clear every 8 steps, renormalisation once per
// 48-step chunk, and an octet (8 steps, all of l') per traceback read.
template <bool SOFT>
struct Hist {
    static constexpr int HB = SOFT ? 2 : 8;
    static constexpr uint32_t SC = 1u << HB;
    static constexpr uint32_t MASK = (SC - 1) * 0x10001u;
};

int tb_block(int Tq) {
    const int per = (Tq + 31) / 32;  // 32 blocks per frame, multiple of 48 steps
    return (per + 47) / 48 * 48;
}
int t_pad(int Tq) { return (Tq + kCh - 1) / kCh * kCh; }
// NB = 3 (k = 1 rate 1/3, hard input, vtb_genk_decode_device): 16 (label, R) columns
constexpr int ring_bytes(int NB) { return (2 << NB) * kCol * 8; }
int region0(int Tq, int NB = 2) {  // table ring, later the decoded bytes of both frames
    const int r = 8 * tb_block(Tq) > ring_bytes(NB) ? 8 * tb_block(Tq) : ring_bytes(NB);
    return (r + 255) / 256 * 256;
}
size_t ws_wave_bytes(int Tq) { return (size_t)kColBytes * (t_pad(Tq) / 16); }

__device__ __forceinline__ uint32_t lane_of(uint32_t l) { return l ^ (((l >> 2) & 1u) * 3u); }
__device__ __forceinline__ uint32_t rev6(uint32_t l) {
    return ((l & 1) << 5) | ((l & 2) << 3) | ((l & 4) << 1) | ((l & 8) >> 1) | ((l & 16) >> 3) | ((l & 32) >> 5);
}
__host__ __device__ constexpr int rev2(int r) { return ((r & 1) << 1) | (r >> 1); }
__device__ __forceinline__ int rotl8(int x, int r) { return ((x << r) | (x >> (8 - r))) & 255; }

__device__ __forceinline__ uint32_t bfi_op(uint32_t mask, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(mask), "v"(a), "v"(b));
    return r;
}

// One coalesced wave store of survivor words (saddr form: wave base in SGPRs); SC: write-through
// (sc1), the words another workgroup reads in the same launch (k9_seg_kernel).
template <int OFF, bool SC = false>
__device__ __forceinline__ void gstore(uint32_t vo, uint32_t z, uint64_t base) {
    if constexpr (SC)
        asm volatile("global_store_dword %0, %1, %2 offset:%3 sc1" ::"v"(vo), "v"(z), "s"(base), "i"(OFF) : "memory");
    else
        asm volatile("global_store_dword %0, %1, %2 offset:%3" ::"v"(vo), "v"(z), "s"(base), "i"(OFF) : "memory");
}

// Words handed from one workgroup to another inside a launch: global (never flat) agent-scope
// relaxed accesses, i.e. sc1 stores and loads that bypass the per-CU L1.
typedef __attribute__((address_space(1))) uint32_t gu32;
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store((gu32*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load((const gu32*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int... Is, class F>
__device__ __forceinline__ void static_for(std::integer_sequence<int, Is...>, F&& f) {
    (f(std::integral_constant<int, Is>{}), ...);
}

// Candidates of one step for the four registers: A = own + V, B = partner (across location
// bit P) + W.
template <int P>
__device__ __forceinline__ void candidates(uint32_t (&M)[4], const uint2 (&vw)[4], uint32_t (&A)[4], uint32_t (&B)[4]) {
    if constexpr (P >= 6) {
        constexpr int x = 1 << (P - 6);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            A[r] = M[r] + vw[r].x;
            B[r] = M[r ^ x] + vw[r].y;
        }
    } else if constexpr (P == 5 || P == 4) {
        // The adds separate the last VALU write of each M[r] from its swap; the s_nop the
        // last swap from the first read of a result (one wait state each way).
        if constexpr (P == 5) {
            asm volatile(
                "v_add_u32 %0, %4, %8\n\tv_add_u32 %1, %5, %9\n\tv_add_u32 %2, %6, %10\n\tv_add_u32 %3, %7, %11\n\t"
                "v_permlane32_swap_b32 %4, %4\n\tv_permlane32_swap_b32 %5, %5\n\t"
                "v_permlane32_swap_b32 %6, %6\n\tv_permlane32_swap_b32 %7, %7\n\ts_nop 0"
                : "=&v"(A[0]), "=&v"(A[1]), "=&v"(A[2]), "=&v"(A[3]), "+v"(M[0]), "+v"(M[1]), "+v"(M[2]), "+v"(M[3])
                : "v"(vw[0].x), "v"(vw[1].x), "v"(vw[2].x), "v"(vw[3].x));
        } else {
            asm volatile(
                "v_add_u32 %0, %4, %8\n\tv_add_u32 %1, %5, %9\n\tv_add_u32 %2, %6, %10\n\tv_add_u32 %3, %7, %11\n\t"
                "v_permlane16_swap_b32 %4, %4\n\tv_permlane16_swap_b32 %5, %5\n\t"
                "v_permlane16_swap_b32 %6, %6\n\tv_permlane16_swap_b32 %7, %7\n\ts_nop 0"
                : "=&v"(A[0]), "=&v"(A[1]), "=&v"(A[2]), "=&v"(A[3]), "+v"(M[0]), "+v"(M[1]), "+v"(M[2]), "+v"(M[3])
                : "v"(vw[0].x), "v"(vw[1].x), "v"(vw[2].x), "v"(vw[3].x));
        }
#pragma unroll
        for (int r = 0; r < 4; r++) B[r] = M[r] + vw[r].y;
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            A[r] = M[r] + vw[r].x;
            if constexpr (P == 3) B[r] = __builtin_amdgcn_update_dpp(0u, M[r], 0x128, 0xF, 0xF, true) + vw[r].y;  // row_ror:8
            if constexpr (P == 2) B[r] = __builtin_amdgcn_update_dpp(0u, M[r], 0x141, 0xF, 0xF, true) + vw[r].y;  // XOR 7
            if constexpr (P == 1) B[r] = __builtin_amdgcn_update_dpp(0u, M[r], 0x4E, 0xF, 0xF, true) + vw[r].y;   // XOR 2
            if constexpr (P == 0) B[r] = __builtin_amdgcn_update_dpp(0u, M[r], 0xB1, 0xF, 0xF, true) + vw[r].y;   // XOR 1
        }
    }
}

// Address bit of l' bit e inside a survivor column (bits 2..7 in place, bits 0..1 at 8..9).
__host__ __device__ constexpr int addr_pos(int e) { return e >= 2 ? e : e + 8; }
__device__ __forceinline__ uint32_t lprime_of(uint32_t a) { return (a & 0xFCu) | ((a >> 8) & 3u); }

// 48 traceback steps over [tlo, tlo + 48), newest first (see vtb_k7_lds.hip tb_body).  cb is
// the byte offset of the block's first survivor column plus 2f (bits 2..9 clear); la the
// address field of the survivor's location.  Returns the 48 decoded bits, bit 0 = step tlo.
template <bool SC = false>
__device__ __forceinline__ uint64_t tb_body(uint32_t cb, uint32_t& la, uint64_t gbase) {
    uint32_t a = cb | la;
    uint64_t bits = 0;
#pragma unroll
    for (int j = 0; j < 24; j++) {
        const int todd = 47 - 2 * j;
        if (j % 4 == 0) bits |= uint64_t(lprime_of(a)) << (8 * (5 - j / 4));  // octet ending at tlo + todd + 1
        const int wi = (todd & 15) >> 1, sh = 8 * (wi & 1) + 2 * (wi >> 1);
        uint32_t v;
        if constexpr (SC)
            asm volatile("global_load_ushort %0, %1, %2 offset:%3 sc1\n\ts_waitcnt vmcnt(0)"
                         : "=v"(v) : "v"(a), "s"(gbase), "i"((todd >> 4) * kColBytes));
        else
            asm volatile("global_load_ushort %0, %1, %2 offset:%3\n\ts_waitcnt vmcnt(0)"
                         : "=v"(v) : "v"(a), "s"(gbase), "i"((todd >> 4) * kColBytes));
        const int pos = addr_pos((todd - 1) & 7);
        const uint32_t fld = pos >= sh ? (v << (pos - sh)) : (v >> (sh - pos));
        a = (a & ~(3u << pos)) | (fld & (3u << pos));
    }
    la = a & 0x3FCu;
    return bits;
}

// Hard input: 48 traceback steps as six octets, one byte read each.  The byte of octet k
// (steps tlo + 8k + b) at the survivor's location holds the decisions D_b along its path, and
// D_b is l' bit b (step t's pairing bit is bit t mod 8 of l'), so the location eight steps
// back is the byte itself and the octet's eight decoded bits are its end location l'.
template <bool SC = false>
__device__ __forceinline__ uint64_t tb_body8(uint32_t cb, uint32_t& la, uint64_t gbase) {
    uint32_t a = cb | la;
    uint64_t bits = 0;
#pragma unroll
    for (int k = 5; k >= 0; k--) {
        bits |= uint64_t(lprime_of(a)) << (8 * k);
        uint32_t v;
        if constexpr (SC)
            asm volatile("global_load_ubyte %0, %1, %2 offset:%3 sc1\n\ts_waitcnt vmcnt(0)"
                         : "=v"(v) : "v"(a), "s"(gbase), "i"(kColBytes * (k >> 1) + (k & 1)));
        else
            asm volatile("global_load_ubyte %0, %1, %2 offset:%3\n\ts_waitcnt vmcnt(0)"
                         : "=v"(v) : "v"(a), "s"(gbase), "i"(kColBytes * (k >> 1) + (k & 1)));
        a = (a & ~0x3FCu) | (v & 0xFCu) | ((v & 3u) << 8);
    }
    la = a & 0x3FCu;
    return bits;
}

__device__ __forceinline__ void put_bits48(uint8_t* ob, int tlo, uint64_t bits) {
    unsigned short* o = reinterpret_cast<unsigned short*>(ob + (tlo >> 3));
    const uint32_t r = __builtin_bitreverse32(uint32_t(bits)), rh = __builtin_bitreverse32(uint32_t(bits >> 32));
    o[0] = (unsigned short)((r >> 24) | ((r >> 8) & 0xff00u));
    o[1] = (unsigned short)(((r >> 8) & 0xffu) | ((r & 0xffu) << 8));
    o[2] = (unsigned short)((rh >> 24) | ((rh >> 8) & 0xff00u));
}

// Decoded bits of steps [tlo, tlo + 48) to global memory at o (byte stores: a stream row has
// no alignment guarantee).
__device__ __forceinline__ void put_bits48_global(uint8_t* o, uint64_t bits) {
    const uint32_t r = __builtin_bitreverse32(uint32_t(bits)), rh = __builtin_bitreverse32(uint32_t(bits >> 32));
    o[0] = uint8_t(r >> 24), o[1] = uint8_t(r >> 16), o[2] = uint8_t(r >> 8), o[3] = uint8_t(r);
    o[4] = uint8_t(rh >> 24), o[5] = uint8_t(rh >> 16);
}

// Eight survivor walks of 48 steps each (the location part of tb_body / tb_body8 only), all
// eight loads of a window issued before one wait: the streaming merge test walks all 256 end
// locations of a frame, eight per lane, and each walk is a chain of dependent loads.
template <bool SOFT>
__device__ __forceinline__ void tb_walk48_x8(uint32_t cb, uint32_t (&la)[8], uint64_t gbase) {
    uint32_t a[8], v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = cb | la[k];
    if constexpr (SOFT) {
#pragma unroll
        for (int j = 0; j < 24; j++) {
            const int todd = 47 - 2 * j;
            const int wi = (todd & 15) >> 1, sh = 8 * (wi & 1) + 2 * (wi >> 1);
#pragma unroll
            for (int k = 0; k < 8; k++)
                asm volatile("global_load_ushort %0, %1, %2 offset:%3" : "=v"(v[k]) : "v"(a[k]), "s"(gbase),
                             "i"((todd >> 4) * kColBytes));
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]),
                         "+v"(v[6]), "+v"(v[7]));
            const int pos = addr_pos((todd - 1) & 7);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t fld = pos >= sh ? (v[k] << (pos - sh)) : (v[k] >> (sh - pos));
                a[k] = (a[k] & ~(3u << pos)) | (fld & (3u << pos));
            }
        }
    } else {
#pragma unroll
        for (int o = 5; o >= 0; o--) {
#pragma unroll
            for (int k = 0; k < 8; k++)
                asm volatile("global_load_ubyte %0, %1, %2 offset:%3" : "=v"(v[k]) : "v"(a[k]), "s"(gbase),
                             "i"(kColBytes * (o >> 1) + (o & 1)));
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]),
                         "+v"(v[6]), "+v"(v[7]));
#pragma unroll
            for (int k = 0; k < 8; k++) a[k] = (a[k] & ~0x3FCu) | (v[k] & 0xFCu) | ((v[k] & 3u) << 8);
        }
    }
#pragma unroll
    for (int k = 0; k < 8; k++) la[k] = a[k] & 0x3FCu;
}

// Traceback of one streaming call (vtb_stream_decode, K = 9): vtb_k7_lds.hip
// stream_traceback with 256 locations.  Frame f of the wave (lanes 32f .. 32f + 31) has
// emitted the bits of steps [0, e_f) before the call.
//  * Not last: walks from all 256 locations at t_end (eight per lane) go back 48 steps at a
//    time until they stand on one location (step m): no later input can change the path
//    below m, so the bits of [e_f, m) equal the whole-frame decode's and are emitted.
//    m <= t_end - 48, so the zero tail is never emitted early.
//  * Last: the terminated traceback from location 0 at T (the padding steps keep location 0)
//    emits [e_f, T - 8).
// The emission is the frame decoder's verified block-parallel traceback, 32 blocks per frame.
// If the ring no longer holds step e_f (no merge within sa.ring steps) the frame is flagged:
// -1 bits until last.
template <bool SOFT>
__device__ void stream_traceback9(const StreamArgs& sa, uint8_t* out, size_t out_stride, int T, int t_end,
                                  uint64_t gbase, size_t fa, bool has_b, size_t wp, int dbg, uint32_t* hits) {
    const int lane = threadIdx.x, f = lane >> 5, blk = lane & 31;
    uint32_t* st = sa.state + wp * kStreamStateWords9;
    const int e0 = int(st[256 + f]);
    const uint32_t flags0 = __builtin_amdgcn_readfirstlane(st[258]);
    const bool real = f == 0 || has_b;
    const bool lost = ((flags0 >> f) & 1u) || t_end - e0 > sa.ring;
    auto colb = [&](int tlo) { return uint32_t(2 * f + kColBytes * ((tlo % sa.ring) >> 4)); };
    auto tb48 = [&](int tlo, uint32_t& la) -> uint64_t {
        if constexpr (SOFT) return tb_body(colb(tlo), la, gbase);
        else return tb_body8(colb(tlo), la, gbase);
    };
    int hi = e0, kfrom = e0;
    uint32_t kloc = 0;
    if (sa.last) {
        hi = t_end, kfrom = T;
    } else {
        // merge test: lane j of frame f walks the locations l' = j + 32 k, k = 0..7
        uint32_t la[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t lp = uint32_t(blk + 32 * k);
            la[k] = (lp & 0xFCu) | ((lp & 3u) << 8);
        }
        bool walking = !lost && real;
        for (int tlo = t_end - 48; __builtin_amdgcn_readfirstlane(__ballot(walking && tlo >= e0) != 0); tlo -= 48) {
            const bool here = walking && tlo >= e0;
            if (here) tb_walk48_x8<SOFT>(colb(tlo), la, gbase);
            const uint32_t ref = __shfl(la[0], 32 * f);
            bool all = true;
#pragma unroll
            for (int k = 0; k < 8; k++) all = all && la[k] == ref;
            const uint64_t same = __ballot(all);
            const bool merged = uint32_t(same >> (32 * f)) == 0xFFFFFFFFu;
            if (here && merged) {
                hi = kfrom = tlo, kloc = ref;
                walking = false;
            }
            if (tlo < e0) walking = false;
        }
    }
    if (!lost && real && hi > e0) {
        const int n = hi - e0;                           // multiple of 48
        const int tbb = ((n + 31) / 32 + 47) / 48 * 48;  // 32 blocks per frame
        const int bot = e0 + blk * tbb;
        const bool active = bot < hi;
        const int start_full = bot + tbb + kTbWarm;
        const int start = min(start_full, hi);
        const bool known = start >= kfrom;
        const int nbody = (kTbWarm + tbb) / 48;
        uint8_t* ob = out + (fa + f) * out_stride;  // byte (tlo - e0) / 8 of the call's bits
        uint32_t loc = known ? kloc : 0u, loc_top = loc;
        if (active) {
            for (int g = 0; g < nbody; g++) {
                const int tlo = start_full - 48 * (g + 1);
                if (g == kTbWarm / 48) loc_top = loc;
                if (tlo < start) {
                    const uint64_t bits = tb48(tlo, loc);
                    if (g >= kTbWarm / 48) put_bits48_global(ob + ((tlo - e0) >> 3), bits);
                }
            }
        }
        // (chains of 32 blocks: at most 31 re-walk rounds) completeness guard: a frame still
        // unproven after the cap (VTB_DEBUG bit 17: every chain with a walked block) is walked serially from its known
        // location at hi by lane 32f
        uint32_t fin = loc;
        bool fixed = known || !active;
        const bool tbforce = (dbg & kDbgTbCap) != 0;
        if (tbforce) loc_top = ~0u;  // (bit 17: no check passes)
        const int rounds = tbforce ? 0 : 33;
        uint64_t unproven = 0;
        for (int round = 0;; round++) {
            const uint32_t sf = __shfl_down(fin, 1);
            const bool ok = fixed || loc_top == sf;
            const uint64_t bad = ~__ballot(ok);
            const uint32_t badf = uint32_t(bad >> (32 * f));
            if (badf == 0 && uint32_t(bad >> (32 * (1 - f))) == 0) break;
            if (round == rounds) {
                unproven = bad;
                break;
            }
            const bool succ_proven = (uint64_t(badf) >> (blk + 1)) == 0;
            if (!ok && succ_proven) {
                loc = sf;
                for (int g = kTbWarm / 48; g < nbody; g++) {
                    const int tlo = start_full - 48 * (g + 1);
                    put_bits48_global(ob + ((tlo - e0) >> 3), tb48(tlo, loc));
                }
                fin = loc;
                fixed = true;
            }
        }
        if (blk == 0 && real && uint32_t(unproven >> (32 * f)) != 0) {  // (no stream B: nothing to walk)
            note_guard(hits);
            uint32_t l = kloc;
            for (int tlo = hi - 48; tlo >= e0; tlo -= 48) put_bits48_global(ob + ((tlo - e0) >> 3), tb48(tlo, l));
        }
    }
    const int bits_out = lost ? -1 : sa.last ? T - 8 - e0 : hi - e0;
    if (real && blk == 0) sa.out_bits[fa + f] = bits_out;
    const uint64_t lostmask = __ballot(lost && real && blk == 0);
    const uint32_t flags = sa.last ? 0u : uint32_t((lostmask & 1u) | ((lostmask >> 32) & 1u) << 1);
    const int e_next = sa.last || lost ? (sa.last ? 0 : e0) : hi;
    if (blk == 0) st[256 + f] = uint32_t(e_next);
    if (lane == 0) st[258] = flags;
}

// Per register and phase: byte offset of the (V, W) column (edge label c of the butterfly's
// upper state, R = bit p of the location); the same for every frame pair of the wave.
template <int NB = 2>
__device__ __forceinline__ void column_offsets(const Launch& table, uint32_t (&off)[4][8], int lane) {
    const uint32_t lam = lane_of(uint32_t(lane));
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int ph = 0; ph < 8; ph++) {
            const int l = r * 64 + int(lam), p = 7 - ph;
            off[r][ph] = 8u * kCol * (table.symm[rotl8(l & ~(1 << p), ph)] + (1u << NB) * ((l >> p) & 1u));
        }
}

// One frame pair (wave-pair index wp: frames 2wp, 2wp + 1), survivors in workspace slot
// `slot` (this wave's).
// STREAM: one call of the streaming decoder (vtb_stream_decode): steps [sa.t_begin, Tpad =
// sa.t_end) continue from the metrics in sa.state (delta = 0, Tq = T = the steps received so
// far), survivor words go to a ring of sa.ring steps (ws_wave = 64 sa.ring bytes per wave), and
// stream_traceback9 emits the bits that became final.
// SEG (k9_seg_kernel, the single-frame latency path): the waves of several workgroups decode
// one frame as segments, two per wave in the u16 halves; segment i runs sg->n kernel steps
// from g_i = i (n - warm), the frame's input is staged in LDS at sg->in_lds, survivor words go
// to the wave's slot, and the final and warm-up metrics come back in seg_out[0..7].
struct Seg9 {
    int n = 0, warm = 0, G = 0;  // steps per segment, warm-up, segments in use
    int ring_bytes = 0;          // LDS bytes per wave (table ring)
    int in_lds = 0;              // LDS byte offset of the staged frame
};

// NB: coded bits per step (2; 3 for the hard rate-1/3 frame kernel, launch_k9_n3)
template <bool SOFT, bool STREAM = false, bool SEG = false, int NB = 2>
__device__ __forceinline__ void k9_pair(const uint8_t* __restrict__ in, size_t in_stride, uint8_t* __restrict__ out,
                                        size_t out_stride, int T, int L, int delta, int Tq, int Tpad, int tbb,
                                        size_t frames, int dbg, uint8_t* __restrict__ ws, size_t ws_wave, size_t wp,
                                        size_t slot, const uint32_t (&off)[4][8], const StreamArgs& sa = StreamArgs(),
                                        const Seg9* sg = nullptr, uint32_t* seg_out = nullptr, uint32_t* hits = nullptr) {
    static_assert(NB == 2 || (!SOFT && !STREAM && !SEG), "rate 1/3: the hard frame kernel only");
    constexpr uint32_t Q = SOFT ? 255 : 1;
    constexpr int NL = 1 << NB;  // edge labels
    using H = Hist<SOFT>;
    // renormalised metric of location 0 (scaled): the metric spread bound n Q S (n = NB, S = 8)
    constexpr uint32_t B4 = H::SC * 8 * NB * Q;
    extern __shared__ uint4 smem4[];
    const int wv = SEG ? int(threadIdx.x >> 6) : 0;
    uint8_t* tab = reinterpret_cast<uint8_t*>(smem4) + (SEG ? wv * sg->ring_bytes : 0);
    const int lane = SEG ? int(threadIdx.x & 63) : int(threadIdx.x);
    // SEG: this wave's segments (half B a copy of half A when unused) and their first kernel step
    const int segA = SEG ? 2 * int(slot) : 0, segB = SEG && 2 * int(slot) + 1 < sg->G ? 2 * int(slot) + 1 : segA;
    const int gA = SEG ? segA * (sg->n - sg->warm) : 0, gB = SEG ? segB * (sg->n - sg->warm) : 0;
    const size_t fa = wp * 2, fb = fa + 1;
    const bool has_b = fb < frames;
    const uint8_t* inA = in + fa * in_stride;
    const uint8_t* inB = in + (has_b ? fb : fa) * in_stride;
    const uint64_t gbase = uniform64(reinterpret_cast<uint64_t>(ws + slot * ws_wave));
    const uint32_t lam = lane_of(lane);  // this lane's 6 low location bits

    // Table staging (as vtb_k7_lds.hip): lane r < 48 builds ring row r of a chunk from the
    // raw input of kernel step 48c + r, i.e. input step 48c + r - delta.
    const int srow = lane < kCh ? lane : lane - kCh;
    const uint64_t baseA = uniform64(reinterpret_cast<uint64_t>(inA)), baseB = uniform64(reinterpret_cast<uint64_t>(inB));
    auto load_raw = [&](int c, uint32_t& ra, uint32_t& rb) {
        int t = c * kCh + srow - delta;
        t = t < 0 ? 0 : (t < T ? t : T - 1);
        if constexpr (SEG) {
            // kernel step g + 48c + r of each half, input step (that - delta), from the LDS copy
            constexpr int SB = SOFT ? 2 : 1;
            int ta = gA + c * kCh + srow - delta, tb = gB + c * kCh + srow - delta;
            ta = ta < 0 ? 0 : (ta < T ? ta : T - 1);
            tb = tb < 0 ? 0 : (tb < T ? tb : T - 1);
            const uint32_t la = uint32_t(sg->in_lds + SB * ta), lb = uint32_t(sg->in_lds + SB * tb);
            if constexpr (SOFT) {
                asm volatile("ds_read_u16 %0, %2\n\tds_read_u16 %1, %3" : "=&v"(ra), "=&v"(rb) : "v"(la), "v"(lb));
            } else {
                asm volatile("ds_read_u8 %0, %2\n\tds_read_u8 %1, %3" : "=&v"(ra), "=&v"(rb) : "v"(la), "v"(lb));
            }
        } else if constexpr (STREAM) {
            // row r of this call: the carry's held-back rows first, then the new input
            constexpr int SB = SOFT ? 2 : 1;
            const int r = t - sa.t_begin;
            const uint8_t* pa = r < sa.carry_len ? sa.carry + fa * kStreamCarryStride + SB * r : inA + SB * (r - sa.carry_len);
            const uint8_t* pb = r < sa.carry_len ? sa.carry + (has_b ? fb : fa) * kStreamCarryStride + SB * r
                                                 : inB + SB * (r - sa.carry_len);
            if constexpr (SOFT) {
                asm volatile("global_load_ushort %0, %2, off\n\tglobal_load_ushort %1, %3, off"
                             : "=&v"(ra), "=&v"(rb) : "v"(pa), "v"(pb));
            } else {
                asm volatile("global_load_ubyte %0, %2, off\n\tglobal_load_ubyte %1, %3, off"
                             : "=&v"(ra), "=&v"(rb) : "v"(pa), "v"(pb));
            }
        } else if constexpr (SOFT) {
            asm volatile("global_load_ushort %0, %2, %3\n\tglobal_load_ushort %1, %2, %4"
                         : "=&v"(ra), "=&v"(rb) : "v"(2u * uint32_t(t)), "s"(baseA), "s"(baseB));
        } else {
            asm volatile("global_load_ubyte %0, %2, %3\n\tglobal_load_ubyte %1, %2, %4"
                         : "=&v"(ra), "=&v"(rb) : "v"(uint32_t(t)), "s"(baseA), "s"(baseB));
        }
    };
    auto stage_compute = [&](uint32_t ra, uint32_t rb, uint32_t (&e)[NL], uint32_t (&et)[NL]) {
        uint32_t q0 = __builtin_amdgcn_perm(rb, ra, 0x0C040C00u);
        uint32_t q1 = __builtin_amdgcn_perm(rb, ra, 0x0C050C01u), q2 = 0;
        if constexpr (!SOFT) {
            q1 = (q0 >> 1) & kR1;
            if constexpr (NB == 3) q2 = (q0 >> 2) & kR1;  // (bits above coded bit NB-1 are ignored)
            q0 &= kR1;
        }
        q0 <<= H::HB;
        q1 <<= H::HB;
        constexpr uint32_t QQ = H::SC * Q * kR1;
        e[0] = q0 + q1, e[1] = (QQ + q1) - q0, e[2] = 2 * QQ - e[1], e[3] = 2 * QQ - e[0];
        if constexpr (NB == 3) {  // labels 4..7 set coded bit 2 (vtb_k7_lds.hip stage_compute)
            q2 <<= H::HB;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                e[4 + k] = e[k] + (QQ - q2);
                e[k] += q2;
            }
        }
        const uint32_t tie = (1u << (srow & (H::HB - 1))) * kR1;
#pragma unroll
        for (int k = 0; k < NL; k++) et[k] = e[k] + tie;
    };
    // Column k = c + 4R holds (V, W) = (4e(c) + R tie, 4e(~c) + (1 - R) tie).
    const uint32_t wbase0 = uint32_t(SEG ? wv * sg->ring_bytes : 0) + 8u * uint32_t(srow), wbase1 = wbase0 + 24u * kCol,
                   wbase2 = wbase0 + 48u * kCol;
    auto stage_write = [&](int c, const uint32_t (&e)[NL], const uint32_t (&et)[NL]) {
#define VTB_W2(base, k, v, w)                                                                         \
    asm volatile("ds_write2_b32 %0, %1, %2 offset0:%3 offset1:%4" ::"v"(base), "v"(v), "v"(w),        \
                 "i"(2 * kCol * ((k) % 3)), "i"(2 * kCol * ((k) % 3) + 1) : "memory");
        if constexpr (NB == 3) {
            // 16 columns k = c + 8R: (V, W) = (e(c) + R tie, e(7 - c) + (1 - R) tie), the
            // complement's metric 3Q - e(c) as the reference's n - e (viterbiDecoderButterflyk1.c:104-107);
            // three columns per base address (offsets below 256 dwords)
            const uint32_t wb3 = wbase2 + 24u * kCol, wb4 = wb3 + 24u * kCol, wb5 = wb4 + 24u * kCol;
            VTB_W2(wbase0, 0, e[0], et[7]) VTB_W2(wbase0, 1, e[1], et[6]) VTB_W2(wbase0, 2, e[2], et[5])
            VTB_W2(wbase1, 3, e[3], et[4]) VTB_W2(wbase1, 4, e[4], et[3]) VTB_W2(wbase1, 5, e[5], et[2])
            VTB_W2(wbase2, 6, e[6], et[1]) VTB_W2(wbase2, 7, e[7], et[0]) VTB_W2(wbase2, 8, et[0], e[7])
            VTB_W2(wb3, 9, et[1], e[6]) VTB_W2(wb3, 10, et[2], e[5]) VTB_W2(wb3, 11, et[3], e[4])
            VTB_W2(wb4, 12, et[4], e[3]) VTB_W2(wb4, 13, et[5], e[2]) VTB_W2(wb4, 14, et[6], e[1])
            VTB_W2(wb5, 15, et[7], e[0])
        } else {
            VTB_W2(wbase0, 0, e[0], et[3]) VTB_W2(wbase0, 1, e[1], et[2]) VTB_W2(wbase0, 2, e[2], et[1])
            VTB_W2(wbase1, 3, e[3], et[0]) VTB_W2(wbase1, 4, et[0], e[3]) VTB_W2(wbase1, 5, et[1], e[2])
            VTB_W2(wbase2, 6, et[2], e[1]) VTB_W2(wbase2, 7, et[3], e[0])
        }
#undef VTB_W2
        // Own-keeping rows: the start step of odd T; for hard input also the padding steps
        // past Tq (W = the metric spread nQS + 1 keeps every survivor at its own location,
        // so the octet that straddles Tq holds the true path's bits; for soft input that W
        // would overflow u16, and the padding survivor bits are overwritten after the ACS).
        // SEG: per half (kernel steps g + 48c + r).
        if constexpr (SEG) {
            const int sa_ = gA + c * kCh + srow, sb_ = gB + c * kCh + srow;
            const bool ka = sa_ < delta || (!SOFT && sa_ >= Tq), kb = sb_ < delta || (!SOFT && sb_ >= Tq);
            if (ka || kb) {
                uint2* col = reinterpret_cast<uint2*>(tab) + srow;
                constexpr uint32_t PADW = H::SC * ((SOFT ? 2 : 16) * Q + 1) * kR1;
                const uint32_t keep = (ka ? 0u : 0xFFFFu) | (kb ? 0u : 0xFFFF0000u);
                const uint32_t tie = et[0] - e[0];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    col[k * kCol] = make_uint2(e[k] & keep, (et[3 - k] & keep) | ((PADW + tie) & ~keep));
                    col[(4 + k) * kCol] = make_uint2((et[k] & keep) | (tie & ~keep), (e[3 - k] & keep) | (PADW & ~keep));
                }
            }
            return;
        }
        const bool pad_row = !SOFT && (c + 1) * kCh > Tq && c * kCh + srow >= Tq;
        if ((c == 0 && srow < delta) || pad_row) {
            uint2* col = reinterpret_cast<uint2*>(tab) + srow;
            constexpr uint32_t PADW = H::SC * ((SOFT ? 2 : 8 * NB) * Q + 1) * kR1;
            const uint32_t tie = et[0] - e[0];
#pragma unroll
            for (int k = 0; k < NL; k++) {
                col[k * kCol] = make_uint2(0u, PADW + tie);
                col[(NL + k) * kCol] = make_uint2(tie, PADW);
            }
        }
    };

    uint32_t M[4];
    M[0] = (lane == 0) ? B4 * kR1 : (B4 + H::SC * Q) * kR1;
    M[1] = M[2] = M[3] = (B4 + H::SC * Q) * kR1;
    const int tbeg = STREAM ? sa.t_begin : 0;  // first step of this launch
    if constexpr (STREAM) {
        if (tbeg > 0)
#pragma unroll
            for (int r = 0; r < 4; r++) M[r] = sa.state[wp * kStreamStateWords9 + 64 * r + lane];
    }
    if constexpr (SEG) {  // segments after the first start from equal metrics
#pragma unroll
        for (int r = 0; r < 4; r++) M[r] = segA > 0 ? B4 * kR1 : (M[r] & 0xFFFFu) | (B4 << 16);
    }
    uint32_t ra, rb;
    if (!STREAM || Tpad > tbeg) {
        uint32_t e[NL], et[NL];
        load_raw(tbeg / kCh, ra, rb);
        if constexpr (SEG) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ra), "+v"(rb));
        else asm volatile("s_waitcnt vmcnt(0)" : "+v"(ra), "+v"(rb));
        stage_compute(ra, rb, e, et);
        stage_write(tbeg / kCh, e, et);
    }
    uint2 buf[kRS][4];
#pragma unroll
    for (int s = 0; s < kAH; s++)
#pragma unroll
        for (int r = 0; r < 4; r++) buf[s][r] = *reinterpret_cast<const uint2*>(tab + off[r][s] + 8 * s);

    const uint32_t wlane = 4u * rev6(lam);  // survivor word byte offset of the lane within a column
    uint32_t dd = 0, m_prev[4] = {0, 0, 0, 0}, pw[4][4] = {}, se[NL], set[NL], msave[4] = {0, 0, 0, 0};
    const int tacs = (dbg & 2) ? 0 : SEG ? sg->n : Tpad;
    // STREAM, soft, last call with odd T: the window of step T - 1 (the last real step, even)
    // also holds padding step T, whose ACS runs on clamped input; the metrics right after step
    // T - 1 hold each location's own even decision (bit 0 of each half), kept in msave for the
    // survivor fix-up below (the ACS of step T may carry another location's bit 0 into l)
    const int tsave = (STREAM && SOFT && sa.last && (T & 1)) ? T - 1 : -1;
    for (int t0 = tbeg; t0 < tacs; t0 += kCh) {
        const int c0 = t0 / kCh;
        // survivor column of step t0 (streaming: position in the ring)
        const uint32_t gvo = uint32_t(kColBytes) * uint32_t((STREAM ? t0 % sa.ring : t0) >> 4) + wlane;
        static_for(std::make_integer_sequence<int, kCh>{}, [&](auto ic) {
            constexpr int I = decltype(ic)::value;
            constexpr int PH = I % 8;
            if constexpr (I == 0) load_raw(c0 + 1, ra, rb);  // next chunk's raw input
            if constexpr (I == 20) {
                // one survivor store batch (step 15) was issued after the loads (SEG: LDS loads)
                if constexpr (SEG) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ra), "+v"(rb));
                else asm volatile("s_waitcnt vmcnt(4)" : "+v"(ra), "+v"(rb));
                stage_compute(ra, rb, se, set);
            }
            if constexpr (I == kCh - kAH) stage_write(c0 + 1, se, set);  // all rows of this chunk read
            // renormalisation reference: location 0 at a step whose history is clear
            constexpr bool RN_READ = SOFT ? (I % 12) == 10 : I == 40;
            constexpr bool RN_APPLY = SOFT ? (I % 12) == 11 : I == 47;
            if constexpr (RN_READ) {
                const uint32_t ref = __builtin_amdgcn_readfirstlane(M[0]);
                asm("s_sub_u32 %0, %1, %2" : "=s"(dd) : "s"(B4 * kR1), "s"(ref) : "scc");
            }
            uint32_t A[4], Bc[4];
            candidates<7 - PH>(M, buf[I % kRS], A, Bc);
            // table rows kAH steps ahead (ring row (I + kAH) % 48: next chunk's rows wrap)
            {
                constexpr int IN = (I + kAH) % kCh, PN = IN % 8;
#pragma unroll
                for (int r = 0; r < 4; r++)
                    buf[(I + kAH) % kRS][r] = *reinterpret_cast<const uint2*>(tab + off[r][PN] + 8 * IN);
            }
#pragma unroll
            for (int r = 0; r < 4; r++) M[r] = pk_min(A[r], Bc[r]);
            if constexpr (STREAM && SOFT && (I & 1) == 0) {
                if (t0 + I == tsave)
#pragma unroll
                    for (int r = 0; r < 4; r++) msave[r] = M[r];
            }
            if constexpr (!SOFT && (I & 7) == 7) {
                // octet history bytes: [A oct 0, A oct 1, B oct 0, B oct 1] per 16 steps
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    if constexpr ((I & 15) == 7) m_prev[r] = M[r];
                    else pw[r][0] = __builtin_amdgcn_perm(M[r], m_prev[r], 0x06020400u);
                    M[r] = RN_APPLY ? ((M[r] & ~H::MASK) + dd) : (M[r] & ~H::MASK);
                }
                if constexpr ((I & 15) == 15) {
                    constexpr int W = I >> 4;
                    gstore<W * kColBytes + 256 * rev2(0), SEG>(gvo, pw[0][0], gbase);
                    gstore<W * kColBytes + 256 * rev2(1), SEG>(gvo, pw[1][0], gbase);
                    gstore<W * kColBytes + 256 * rev2(2), SEG>(gvo, pw[2][0], gbase);
                    gstore<W * kColBytes + 256 * rev2(3), SEG>(gvo, pw[3][0], gbase);
                }
            }
            if constexpr (SOFT && (I & 1)) {
                constexpr int w = (I & 15) >> 1;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    if constexpr (w & 1) pw[r][w >> 1] = __builtin_amdgcn_perm(M[r], m_prev[r], 0x06020400u);
                    else m_prev[r] = M[r];
                    M[r] = RN_APPLY ? ((M[r] & ~H::MASK) + dd) : (M[r] & ~H::MASK);
                }
                if constexpr ((I & 15) == 15) {
                    constexpr int W = I >> 4;
                    uint32_t z[4];
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        z[r] = bfi_op(0x03030303u, pw[r][0], pw[r][1] << 2);
                        z[r] = bfi_op(0x0F0F0F0Fu, z[r], pw[r][2] << 4);
                        z[r] = bfi_op(0x3F3F3F3Fu, z[r], pw[r][3] << 6);
                    }
                    gstore<W * kColBytes + 256 * rev2(0), SEG>(gvo, z[0], gbase);
                    gstore<W * kColBytes + 256 * rev2(1), SEG>(gvo, z[1], gbase);
                    gstore<W * kColBytes + 256 * rev2(2), SEG>(gvo, z[2], gbase);
                    gstore<W * kColBytes + 256 * rev2(3), SEG>(gvo, z[3], gbase);
                }
            }
        });
        if constexpr (SEG) {
            if (t0 == sg->warm - kCh)
#pragma unroll
                for (int r = 0; r < 4; r++) msave[r] = M[r];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    if constexpr (SEG) {
        // soft input: the last segment's padding steps (kernel steps >= Tq) get own-keeping
        // survivor bits, one bit per step, in that segment's half of the words
        if (SOFT && !(dbg & 2)) {
            uint32_t* wsw = reinterpret_cast<uint32_t*>(ws + slot * ws_wave);
            for (int h = 0; h < 2; h++) {
                const int g0 = h ? gB : gA;
                if (h == 1 && segB == segA) break;
                const int lo = Tq - g0;  // first local padding step
                if (lo >= sg->n) continue;
                for (int g = (lo > 0 ? lo : 0) >> 4; g < (sg->n >> 4); g++) {
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const uint32_t lp = (rev6(lam) << 2) | uint32_t(rev2(r));
                        uint32_t own = 0, mask = 0;
                        for (int t = (16 * g > lo ? 16 * g : lo); t < 16 * g + 16; t++) {
                            const int w = (t & 15) >> 1, bit = 8 * (w & 1) + 2 * (w >> 1) + (t & 1);
                            own |= ((lp >> ((g0 + t) & 7)) & 1u) << bit;
                            mask |= 1u << bit;
                        }
                        own <<= 16 * h;
                        mask <<= 16 * h;
                        uint32_t* p = wsw + (kColBytes / 4) * g + (wlane >> 2) + 64 * rev2(r);
                        st_agent(p, (ld_agent(p) & ~mask) | (own & mask));
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
#pragma unroll
        for (int r = 0; r < 4; r++) seg_out[r] = M[r], seg_out[4 + r] = msave[r];
        return;
    }

    if constexpr (STREAM) {
        if (!sa.last)
#pragma unroll
            for (int r = 0; r < 4; r++) sa.state[wp * kStreamStateWords9 + 64 * r + lane] = M[r];
        // Soft input, last call, padding steps [T, Tpad): own-keeping survivor bits, one bit per
        // step.  For odd T the window of step T - 1 gets the location's own even decision
        // (msave, captured after step T - 1), not the bit step T's ACS carried in.
        if (SOFT && sa.last) {
            uint32_t* wsw = reinterpret_cast<uint32_t*>(ws + slot * ws_wave);
            for (int g = T >> 4; g < (Tpad >> 4); g++) {
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const uint32_t lp = (rev6(lam) << 2) | uint32_t(rev2(r));
                    uint32_t own = 0, mask = 0;
                    for (int t = (16 * g > T ? 16 * g : T); t < 16 * g + 16; t++) {
                        const int w = (t & 15) >> 1, bit = 8 * (w & 1) + 2 * (w >> 1) + (t & 1);
                        own |= ((lp >> (t & 7)) & 1u) << bit;
                        mask |= 1u << bit;
                    }
                    own |= own << 16;
                    mask |= mask << 16;
                    if ((T & 1) && ((T - 1) >> 4) == g) {
                        const int w = ((T - 1) & 15) >> 1, bit = 8 * (w & 1) + 2 * (w >> 1);
                        own |= ((msave[r] & 1u) << bit) | (((msave[r] >> 16) & 1u) << (bit + 16));
                        mask |= (1u << bit) | (1u << (bit + 16));
                    }
                    uint32_t* p = wsw + (kColBytes / 4) * ((16 * g % sa.ring) >> 4) + (wlane >> 2) + 64 * rev2(r);
                    *p = (*p & ~mask) | (own & mask);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (dbg & 1) return;
        stream_traceback9<SOFT>(sa, out, out_stride, T, Tpad, gbase, fa, has_b, wp, dbg, hits);
        return;
    }
    // Soft input, padding steps [Tq, Tpad): overwrite their survivor bits with own-keeping
    // decisions (both history bits = the location's own bits t_even mod 8, +1 of l').
    if (SOFT && !(dbg & 2)) {
        uint32_t* wsw = reinterpret_cast<uint32_t*>(ws + slot * ws_wave);
        for (int g = Tq >> 4; g < (Tpad >> 4); g++) {
            const int w0 = Tq > 16 * g ? (Tq - 16 * g) >> 1 : 0;  // first padding window of the word
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const uint32_t lp = (rev6(lam) << 2) | uint32_t(rev2(r));
                uint32_t own = 0, mask = 0;
                for (int w = w0; w < 8; w++) {
                    const int sh = 8 * (w & 1) + 2 * (w >> 1);
                    own |= ((lp >> (2 * (w & 3))) & 3u) << sh;
                    mask |= 3u << sh;
                }
                own |= own << 16;
                mask |= mask << 16;
                uint32_t* p = wsw + (kColBytes / 4) * g + (wlane >> 2) + 64 * rev2(r);
                *p = (*p & ~mask) | (own & mask);
            }
        }
    }
    __syncthreads();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (dbg & 1) return;

    // ---------------- traceback: verified block-parallel chains (vtb_k7_lds.hip) ----------------
    const int f = lane >> 5, blk = lane & 31;
    const uint32_t cb0 = uint32_t(2 * f);
    uint8_t* ob = tab + f * 4 * tbb;
    const int top = (blk + 1) * tbb;
    const int start_full = top + kTbWarm;
    const int start = min(start_full, Tpad);
    const bool known = start >= Tq;
    const int nbody = (dbg & 8) ? 1 : (kTbWarm + tbb) / 48;
    auto tb48 = [&](uint32_t cb, uint32_t& la) {
        if constexpr (SOFT) return tb_body(cb, la, gbase);
        else return tb_body8(cb, la, gbase);
    };
    uint32_t loc = 0, loc_top = 0;
    for (int g = 0; g < nbody; g++) {
        const int tlo = start_full - 48 * (g + 1);
        if (g == kTbWarm / 48) loc_top = loc;
        if (tlo < start) {
            const uint64_t bits = tb48(cb0 + kColBytes * (tlo >> 4), loc);
            if (g >= kTbWarm / 48) put_bits48(ob, tlo, bits);
        }
    }
    // (chains of 32 blocks, the last known: at most 31 re-walk rounds.)  Completeness guard:
    // a frame with a block still unproven after the cap (VTB_DEBUG bit 17: every chain with a walked block) is traced
    // back serially by lane 32f from location 0 at Tpad, the reference's own walk
    // (viterbiDecoderButterflyk1.c:200-256)
    uint32_t fin = loc;
    bool fixed = known || (dbg & 4);
    const bool tbforce = (dbg & kDbgTbCap) != 0;
    if (tbforce) loc_top = ~0u;  // (bit 17: no check passes)
    const int rounds = tbforce ? 0 : 33;
    uint64_t unproven = 0;
    for (int round = 0;; round++) {
        const uint32_t sf = __shfl_down(fin, 1);
        const bool ok = fixed || loc_top == sf;
        const uint64_t bad = ~__ballot(ok);
        if (bad == 0) break;
        if (round == rounds) {
            unproven = bad;
            break;
        }
        const uint32_t badf = uint32_t(bad >> (32 * f));
        const bool succ_proven = (uint64_t(badf) >> (blk + 1)) == 0;
        if (!ok && succ_proven) {
            loc = sf;
            for (int g = kTbWarm / 48; g < nbody; g++) {
                const int tlo = start_full - 48 * (g + 1);
                put_bits48(ob, tlo, tb48(cb0 + kColBytes * (tlo >> 4), loc));
            }
            fin = loc;
            fixed = true;
        }
    }
    if (blk == 0 && (f == 0 || has_b) && uint32_t(unproven >> (32 * f)) != 0) {  // (a lone last frame: no B)
        note_guard(hits);
        uint32_t l = 0;
        for (int tlo = Tpad - 48; tlo >= 0; tlo -= 48) put_bits48(ob, tlo, tb48(cb0 + kColBytes * (tlo >> 4), l));
    }
    __syncthreads();

    // copy out; with delta = 1 kernel step t' is input step t' - 1 (shift the stream one bit)
    const int nbytes = (L + 7) >> 3;
    for (int i = lane; i < 2 * nbytes; i += 64) {
        const int fr = i >= nbytes, j = i - fr * nbytes;
        if (fr && !has_b) break;
        const uint8_t* s = tab + fr * 4 * tbb;
        const uint8_t v = delta ? uint8_t((s[j] << 1) | (s[j + 1] >> 7)) : s[j];
        out[(fr ? fb : fa) * out_stride + j] = v;
    }
}

// Single-frame latency path for K = 9 (vtb_decode_frame_sync): the frame is cut into up to
// 2 x waves segments over several workgroups of W waves (one per SIMD), each workgroup
// stages the whole frame from (host-mapped) memory into LDS once, every wave runs the ACS of
// its two segments (k9_pair SEG, survivor words in its workspace slot) and publishes its
// final and warm-up metric vectors; the last workgroup to arrive (atomic counter) checks
// every segment boundary (metrics equal up to a constant, vtb_k7_lds.hip §SEG), and its wave 0
// traces the frame back over all segments' words and writes the bytes, then *done = 1 (2: a
// boundary did not converge, nothing written: the caller decodes the frame whole).
struct Seg9Args {
    Seg9 s;
    uint32_t* met;      // per global wave: final [4][64], warm-up [4][64] (packed pairs)
    uint32_t* counter;  // workgroups arrived; the last one resets it
    uint32_t* done;     // completion word (host-mapped) or null
    int nwg;            // workgroups
    int ob_lds;         // LDS byte offset of the decoded bytes
    int flag_lds;       // LDS byte offset of the election flag and the per-wave check results
    int xcd;            // grid stride of the working workgroups (8: all on one XCD, one L2)
};

template <bool SOFT>
__global__ __launch_bounds__(512) void k9_seg_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int T,
                                                     int L, int delta, int Tq, int dbg, Launch table,
                                                     uint8_t* __restrict__ ws, size_t ws_wave, Seg9Args a) {
    extern __shared__ uint4 smem4[];
    uint8_t* sm = reinterpret_cast<uint8_t*>(smem4);
    if (int(blockIdx.x) % a.xcd) return;  // placeholder workgroups of the XCD-local grid
    const int wv = int(threadIdx.x >> 6), lane = int(threadIdx.x & 63), W = int(blockDim.x >> 6);
    const int gw = int(blockIdx.x) / a.xcd * W + wv;  // global wave: segments 2gw, 2gw + 1
    {
        // the frame into LDS: up to four 16-byte loads per thread, all issued before any store
        const int nin = (SOFT ? 2 : 1) * T, step = 16 * int(blockDim.x), i0 = 16 * int(threadIdx.x);
        uint4 v0 = make_uint4(0, 0, 0, 0), v1 = v0, v2 = v0, v3 = v0;
        if (i0 < nin) v0 = *reinterpret_cast<const uint4*>(in + i0);
        if (i0 + step < nin) v1 = *reinterpret_cast<const uint4*>(in + i0 + step);
        if (i0 + 2 * step < nin) v2 = *reinterpret_cast<const uint4*>(in + i0 + 2 * step);
        if (i0 + 3 * step < nin) v3 = *reinterpret_cast<const uint4*>(in + i0 + 3 * step);
        uint8_t* dst = sm + a.s.in_lds + i0;
        if (i0 < nin) *reinterpret_cast<uint4*>(dst) = v0;
        if (i0 + step < nin) *reinterpret_cast<uint4*>(dst + step) = v1;
        if (i0 + 2 * step < nin) *reinterpret_cast<uint4*>(dst + 2 * step) = v2;
        if (i0 + 3 * step < nin) *reinterpret_cast<uint4*>(dst + 3 * step) = v3;
    }
    __syncthreads();
    const int G = a.s.G;
    if (2 * gw < G) {
        uint32_t off[4][8];
        column_offsets(table, off, lane);
        uint32_t fm[8];
        k9_pair<SOFT, false, true>(in, 0, out, 0, T, L, delta, Tq, 0, 0, 1, dbg, ws, ws_wave, 0, size_t(gw), off,
                                   StreamArgs(), &a.s, fm);
        uint32_t* mw = a.met + size_t(gw) * 512;
#pragma unroll
        for (int r = 0; r < 4; r++) st_agent(mw + 64 * r + lane, fm[r]), st_agent(mw + 256 + 64 * r + lane, fm[4 + r]);
    }
    // the last workgroup to arrive does the rest.  Hand-off (cdna_hip_programming.md Guideline
    // 16, write-through form): every word another workgroup reads (survivor words, metrics) is
    // stored sc1 and drained by its wave before the barrier, one lane adds to the counter, and
    // every load of those words in the last workgroup is an sc1 load (no fences)
    uint32_t* flag = reinterpret_cast<uint32_t*>(sm + a.flag_lds);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        flag[0] = __hip_atomic_fetch_add((gu32*)(a.counter), 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) == uint32_t(a.nwg - 1) ? 1u : 0u;
    __syncthreads();
    if (flag[0] == 0u) return;  // (the whole workgroup: no barrier follows for it)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (orders the loads after the election)
    // boundaries i = 1 .. G-1: segment i's metrics at the end of its warm-up against segment
    // i - 1's final metrics (the same step), equal up to a constant over all 256 states
    using H = Hist<SOFT>;
    constexpr uint32_t KEEP = 0xFFFFu & ~(H::SC - 1);
    bool ok = true;
    for (int i = 1 + wv; i < G; i += W) {
        const uint32_t* pf = a.met + size_t((i - 1) >> 1) * 512;        // segment i - 1: final
        const uint32_t* pw = a.met + size_t(i >> 1) * 512 + 256;        // segment i: warm-up end
        const int sf = 16 * ((i - 1) & 1), sw = 16 * (i & 1);
        uint32_t x[4], y[4];
#pragma unroll
        for (int r = 0; r < 4; r++) x[r] = (ld_agent(pf + 64 * r + lane) >> sf) & KEEP, y[r] = (ld_agent(pw + 64 * r + lane) >> sw) & KEEP;
        const uint32_t x0 = __builtin_amdgcn_readfirstlane(x[0]), y0 = __builtin_amdgcn_readfirstlane(y[0]);
        bool same = true;
#pragma unroll
        for (int r = 0; r < 4; r++) same = same && ((x[r] - x0) & 0xFFFFu) == ((y[r] - y0) & 0xFFFFu);
        ok = ok && __ballot(same) == ~0ull;
    }
    if (lane == 0) flag[1 + wv] = ok ? 1u : 0u;
    __syncthreads();
    bool all = true;
    for (int i = 0; i < W; i++) all = all && flag[1 + i] != 0u;
    if (dbg & 2) all = true;  // (VTB_DEBUG 2, 1: no ACS / no traceback, phase timing only)
    if (wv != 0) return;
    if (lane == 0) st_agent(a.counter, 0u);  // for the next launch (stream-ordered after this one)
    if (dbg & 1) {
        if (a.done && lane == 0) __hip_atomic_store(a.done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    if (!all) {
        if (a.done && lane == 0) __hip_atomic_store(a.done, 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    // traceback, wave 0: blocks of tbp kernel steps (a multiple of 48), lane b = block b; the
    // 48 steps at tlo read the words of the segment that owns them (one workspace for all
    // segments: slot * ws_wave is a multiple of the 1-KB column, so the in-place address edits
    // of tb_body stay inside the column)
    const int n = a.s.n, warm = a.s.warm, stp = n - warm, Tpad = (Tq + kCh - 1) / kCh * kCh;
    const uint64_t gbase = uniform64(reinterpret_cast<uint64_t>(ws));
    auto col_at = [&](int tlo) -> uint32_t {
        int i = tlo < warm ? 0 : (tlo - warm) / stp;
        if (i > G - 1) i = G - 1;
        const int lt = tlo - i * stp;
        return uint32_t(size_t(i >> 1) * ws_wave) + uint32_t(2 * (i & 1)) + uint32_t(kColBytes * (lt >> 4));
    };
    auto tb48 = [&](uint32_t cb, uint32_t& la) {
        if constexpr (SOFT) return tb_body<true>(cb, la, gbase);
        else return tb_body8<true>(cb, la, gbase);
    };
    uint8_t* ob = sm + a.ob_lds;
    const int nb48 = Tpad / kCh;
    const int tbp = (nb48 + 63) / 64 * kCh;
    const bool active = lane * tbp < Tpad;
    const int start_full = (lane + 1) * tbp + kTbWarm;
    const int start = min(start_full, Tpad);
    const bool known = start >= Tq;
    const int nbody = (kTbWarm + tbp) / 48;
    uint32_t loc = 0, loc_top = 0;
    if (active) {
        for (int g = 0; g < nbody; g++) {
            const int tlo = start_full - 48 * (g + 1);
            if (g == kTbWarm / 48) loc_top = loc;
            if (tlo < start) {
                const uint64_t bits = tb48(col_at(tlo), loc);
                if (g >= kTbWarm / 48) put_bits48(ob, tlo, bits);
            }
        }
    }
    // one chain of up to 64 blocks (at most 63 re-walk rounds), with the completeness guard:
    // unproven after the cap (VTB_DEBUG bit 17: every chain with a walked block), lane 0 walks the frame serially
    // from location 0 at Tpad
    uint32_t fin = loc;
    bool fixed = known || !active;
    const bool tbforce = (dbg & kDbgTbCap) != 0;
    if (tbforce) loc_top = ~0u;  // (bit 17: no check passes)
    const int rounds = tbforce ? 0 : 65;
    bool unproven = false;
    for (int round = 0;; round++) {
        const uint32_t sfin = __shfl_down(fin, 1);
        const bool okb = fixed || loc_top == sfin;
        const uint64_t bad = ~__ballot(okb);
        if (bad == 0) break;
        if (round == rounds) {
            unproven = true;
            break;
        }
        if (!okb && (bad >> (lane + 1)) == 0) {
            loc = sfin;
            for (int g = kTbWarm / 48; g < nbody; g++) {
                const int tlo = start_full - 48 * (g + 1);
                put_bits48(ob, tlo, tb48(col_at(tlo), loc));
            }
            fin = loc;
            fixed = true;
        }
    }
    if (unproven && lane == 0) {
        note_guard(table.guard_hits);
        uint32_t l = 0;
        for (int tlo = Tpad - 48; tlo >= 0; tlo -= 48) put_bits48(ob, tlo, tb48(col_at(tlo), l));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // copy out; with delta = 1 kernel step t' is input step t' - 1 (shift the stream one bit)
    const int nbytes = (L + 7) >> 3;
    for (int j = lane; j < nbytes; j += 64) out[j] = delta ? uint8_t((ob[j] << 1) | (ob[j + 1] >> 7)) : ob[j];
    if (a.done) {
        // every lane's output stores complete, then the system-scope release store (its
        // own fence writes back; no acquire needed here, so no __threadfence_system)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(a.done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// LOOP: persistent over frame pairs (as vtb_k7_lds.hip), wave b decodes pairs b, b + grid, ...;
// !LOOP: one wave per pair, for batches the CUs hold in one round (fewer live registers).
template <bool SOFT, bool LOOP, bool STREAM = false, int NB = 2>
__global__ __launch_bounds__(64) void k9_kernel(const uint8_t* __restrict__ in, size_t in_stride,
                                                uint8_t* __restrict__ out, size_t out_stride, int T, int L, int delta,
                                                int Tq, int Tpad, int tbb, size_t frames, int dbg, Launch table,
                                                uint8_t* __restrict__ ws, size_t ws_wave, StreamArgs sa = StreamArgs()) {
    static_assert(!(STREAM && LOOP), "streaming calls keep per-pair state: one wave per pair");
    uint32_t off[4][8];
    column_offsets<NB>(table, off, threadIdx.x);
    if constexpr (STREAM) {
        k9_pair<SOFT, true>(in, in_stride, out, out_stride, T, L, 0, T, Tpad, 0, frames, dbg, ws, ws_wave, blockIdx.x,
                            blockIdx.x, off, sa, nullptr, nullptr, table.guard_hits);
    } else if constexpr (!LOOP) {
        k9_pair<SOFT, false, false, NB>(in, in_stride, out, out_stride, T, L, delta, Tq, Tpad, tbb, frames, dbg, ws,
                                        ws_wave, blockIdx.x, blockIdx.x, off, StreamArgs(), nullptr, nullptr, table.guard_hits);
    } else {
        const size_t pairs = (frames + 1) / 2;
        for (size_t wp = blockIdx.x; wp < pairs; wp += gridDim.x) {
            k9_pair<SOFT, false, false, NB>(in, in_stride, out, out_stride, T, L, delta, Tq, Tpad, tbb, frames, dbg, ws,
                                            ws_wave, wp, blockIdx.x, off, StreamArgs(), nullptr, nullptr, table.guard_hits);
            __syncthreads();  // LDS (decoded bytes) before the next pair's table ring
        }
    }
}

// ---------------- one frame per wave (k9s) ----------------
//
// A batch of F frames gives the pair kernel F / 2 waves: 2 per SIMD at config C4's 4,096, where
// the SIMD still idles (VALU active 78 % of its cycles; 4 waves per SIMD of the same kernel run
// +15 % faster per wave-step, profiles/r05/pricing/k9_waves_ab.jsonl).  Here every wave decodes
// one frame, so the same batch fills 4 waves per SIMD with the same work per state-step.
//
// Layout: location l = 128 h + 64 r + lambda -- bits 0..5 lane bits (lane_of, as k9_pair), bit 6
// the register M[r] (r = 0, 1), bit 7 the u16 half h.  In l' = rev8(l) numbering h is bit 0, r
// bit 1 and rev6(lambda) bits 2..7, so a survivor column of 16 steps is 256 u16 words at byte 2 l'
// (512 B; the word of register r at 8 rev6(lambda) + 4 r holds h = 0 in its low half), and a
// window's two decisions (l' bits t mod 8, t mod 8 + 1) are address bits 1 + t mod 8 and above.
// Per step the butterfly partner is the other half (p = 7: one v_pk_add_u16 with the source
// halves swapped), the other register (p = 6), a v_permlane32/16_swap (p = 5, 4) or DPP (3..0).
//
// Branch metrics: the pair kernel's ring with both halves from this frame.  Column k = c + 4R
// of row t holds in its low half the value of location l (upper state label c, R = bit p of l)
// and in its high half that of l ^ 128:
//  * t mod 8 = ph >= 1: l ^ 128's upper state is l's with bit ph - 1 flipped, whose label is
//    c ^ d(ph) (labels are linear in the state: checked on the host, k9s_dpack); the staging
//    lane computes the high half from its input with the coded bits in d(ph) complemented;
//  * ph = 0 (p = 7): l and l ^ 128 are the butterfly itself, same c, R flipped: the tie bit goes
//    into the other half (tieE / tieT below).
constexpr int kColS = 512;  // survivor column: 256 u16 words per 16 steps
constexpr uint32_t kDbgK9Pair = 1u << 18;  // VTB_DEBUG bit 18 (exact): K=9 frames on the pair kernel

int tb_block_s(int Tq) {
    const int per = (Tq + 63) / 64;  // 64 blocks per frame, multiple of 48 steps
    return (per + 47) / 48 * 48;
}
int region0_s(int Tq) {  // table ring, later the decoded bytes of the frame
    const int r = 8 * tb_block_s(Tq) > kRingBytes ? 8 * tb_block_s(Tq) : kRingBytes;
    return (r + 255) / 256 * 256;
}
size_t ws_wave_bytes_s(int Tq) { return (size_t)kColS * (t_pad(Tq) / 16); }

// Candidates of one step for the two registers (as candidates<P>).
template <int P>
__device__ __forceinline__ void candidates_s(uint32_t (&M)[2], const uint2 (&vw)[2], uint32_t (&A)[2], uint32_t (&B)[2]) {
    if constexpr (P == 7) {
#pragma unroll
        for (int r = 0; r < 2; r++) {
            A[r] = M[r] + vw[r].x;
            asm("v_pk_add_u16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(B[r]) : "v"(M[r]), "v"(vw[r].y));
        }
    } else if constexpr (P == 6) {
        A[0] = M[0] + vw[0].x, B[0] = M[1] + vw[0].y;
        A[1] = M[1] + vw[1].x, B[1] = M[0] + vw[1].y;
    } else if constexpr (P == 5 || P == 4) {
        // s_nop: one wait state between the last VALU write of M[r] and its swap (the adds may be
        // fewer than the hazard needs when the compiler puts M[1]'s write right before), and
        // between the last swap and the first read of a result
        if constexpr (P == 5) {
            asm volatile(
                "v_add_u32 %0, %2, %4\n\tv_add_u32 %1, %3, %5\n\ts_nop 0\n\t"
                "v_permlane32_swap_b32 %2, %2\n\tv_permlane32_swap_b32 %3, %3\n\ts_nop 0"
                : "=&v"(A[0]), "=&v"(A[1]), "+v"(M[0]), "+v"(M[1])
                : "v"(vw[0].x), "v"(vw[1].x));
        } else {
            asm volatile(
                "v_add_u32 %0, %2, %4\n\tv_add_u32 %1, %3, %5\n\ts_nop 0\n\t"
                "v_permlane16_swap_b32 %2, %2\n\tv_permlane16_swap_b32 %3, %3\n\ts_nop 0"
                : "=&v"(A[0]), "=&v"(A[1]), "+v"(M[0]), "+v"(M[1])
                : "v"(vw[0].x), "v"(vw[1].x));
        }
#pragma unroll
        for (int r = 0; r < 2; r++) B[r] = M[r] + vw[r].y;
    } else {
#pragma unroll
        for (int r = 0; r < 2; r++) {
            A[r] = M[r] + vw[r].x;
            if constexpr (P == 3) B[r] = __builtin_amdgcn_update_dpp(0u, M[r], 0x128, 0xF, 0xF, true) + vw[r].y;  // row_ror:8
            if constexpr (P == 2) B[r] = __builtin_amdgcn_update_dpp(0u, M[r], 0x141, 0xF, 0xF, true) + vw[r].y;  // XOR 7
            if constexpr (P == 1) B[r] = __builtin_amdgcn_update_dpp(0u, M[r], 0x4E, 0xF, 0xF, true) + vw[r].y;   // XOR 2
            if constexpr (P == 0) B[r] = __builtin_amdgcn_update_dpp(0u, M[r], 0xB1, 0xF, 0xF, true) + vw[r].y;   // XOR 1
        }
    }
}

// 48 traceback steps over [tlo, tlo + 48), newest first (tb_body / tb_body8 in the k9s column
// layout): cb the byte offset of the block's first survivor column (bits 0..8 clear), la = 2 l'
// of the survivor's location.  Returns the 48 decoded bits, bit 0 = step tlo.
template <bool SOFT>
__device__ __forceinline__ uint64_t tbs_body(uint32_t cb, uint32_t& la, uint64_t gbase) {
    uint32_t a = cb | la;
    uint64_t bits = 0;
    if constexpr (SOFT) {
#pragma unroll
        for (int j = 0; j < 24; j++) {
            const int todd = 47 - 2 * j;
            if (j % 4 == 0) bits |= uint64_t((a >> 1) & 0xFFu) << (8 * (5 - j / 4));
            const int wi = (todd & 15) >> 1, sh = 8 * (wi & 1) + 2 * (wi >> 1);
            uint32_t v;
            asm volatile("global_load_ushort %0, %1, %2 offset:%3\n\ts_waitcnt vmcnt(0)"
                         : "=v"(v) : "v"(a), "s"(gbase), "i"((todd >> 4) * kColS));
            const int pos = ((todd - 1) & 7) + 1;
            const uint32_t fld = pos >= sh ? (v << (pos - sh)) : (v >> (sh - pos));
            a = (a & ~(3u << pos)) | (fld & (3u << pos));
        }
    } else {
#pragma unroll
        for (int k = 5; k >= 0; k--) {
            bits |= uint64_t((a >> 1) & 0xFFu) << (8 * k);
            uint32_t v;
            asm volatile("global_load_ubyte %0, %1, %2 offset:%3\n\ts_waitcnt vmcnt(0)"
                         : "=v"(v) : "v"(a), "s"(gbase), "i"(kColS * (k >> 1) + (k & 1)));
            a = (a & ~0x1FEu) | (v << 1);
        }
    }
    la = a & 0x1FEu;
    return bits;
}

// One frame (index fr) per wave, survivors in workspace slot `slot`.  dpack: d(ph) of the
// header, 2 bits per phase.
template <bool SOFT>
__device__ __forceinline__ void k9_single(const uint8_t* __restrict__ in, size_t in_stride, uint8_t* __restrict__ out,
                                          size_t out_stride, int T, int L, int delta, int Tq, int Tpad, int tbb,
                                          int dbg, uint8_t* __restrict__ ws, size_t ws_wave, size_t fr, size_t slot,
                                          const uint32_t (&off)[2][8], uint32_t dpack, uint32_t* hits) {
    constexpr uint32_t Q = SOFT ? 255 : 1;
    using H = Hist<SOFT>;
    constexpr uint32_t B4 = H::SC * 8 * 2 * Q;  // as k9_pair (NB = 2)
    extern __shared__ uint4 smem4[];
    uint8_t* tab = reinterpret_cast<uint8_t*>(smem4);
    const int lane = int(threadIdx.x);
    const uint64_t gbase = uniform64(reinterpret_cast<uint64_t>(ws + slot * ws_wave));
    const uint32_t lam = lane_of(uint32_t(lane));

    // Table staging: lane r < 48 builds ring row r of a chunk (k9_pair), both halves from this
    // frame's input (header: the high half's coded bits complemented by d(ph), its tie bit in
    // the other half at ph = 0).
    const int srow = lane < kCh ? lane : lane - kCh;
    const int sph = srow & 7;
    const uint32_t d = (dpack >> (2 * sph)) & 3u;
    const uint32_t xmask = SOFT ? ((d & 1u) ? 0xFFu : 0u) | ((d & 2u) ? 0xFF00u : 0u) : d;
    const uint32_t tie16 = 1u << (srow & (H::HB - 1));
    const uint32_t tieE = sph == 0 ? tie16 << 16 : 0u, tieT = sph == 0 ? tie16 : tie16 * kR1;
    const uint64_t base = uniform64(reinterpret_cast<uint64_t>(in + fr * in_stride));
    auto load_raw = [&](int c, uint32_t& ra) {
        int t = c * kCh + srow - delta;
        t = t < 0 ? 0 : (t < T ? t : T - 1);
        if constexpr (SOFT)
            asm volatile("global_load_ushort %0, %1, %2" : "=v"(ra) : "v"(2u * uint32_t(t)), "s"(base));
        else
            asm volatile("global_load_ubyte %0, %1, %2" : "=v"(ra) : "v"(uint32_t(t)), "s"(base));
    };
    auto stage_compute = [&](uint32_t ra, uint32_t (&e)[4], uint32_t (&et)[4]) {
        const uint32_t rb = ra ^ xmask;
        uint32_t q0 = __builtin_amdgcn_perm(rb, ra, 0x0C040C00u);
        uint32_t q1 = __builtin_amdgcn_perm(rb, ra, 0x0C050C01u);
        if constexpr (!SOFT) {
            q1 = (q0 >> 1) & kR1;
            q0 &= kR1;
        }
        q0 <<= H::HB;
        q1 <<= H::HB;
        constexpr uint32_t QQ = H::SC * Q * kR1;
        e[0] = q0 + q1, e[1] = (QQ + q1) - q0, e[2] = 2 * QQ - e[1], e[3] = 2 * QQ - e[0];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            et[k] = e[k] + tieT;
            e[k] += tieE;
        }
    };
    const uint32_t wbase0 = 8u * uint32_t(srow), wbase1 = wbase0 + 24u * kCol, wbase2 = wbase0 + 48u * kCol;
    auto stage_write = [&](int c, const uint32_t (&e)[4], const uint32_t (&et)[4]) {
#define VTB_W2(base, k, v, w)                                                                         \
    asm volatile("ds_write2_b32 %0, %1, %2 offset0:%3 offset1:%4" ::"v"(base), "v"(v), "v"(w),        \
                 "i"(2 * kCol * ((k) % 3)), "i"(2 * kCol * ((k) % 3) + 1) : "memory");
        VTB_W2(wbase0, 0, e[0], et[3]) VTB_W2(wbase0, 1, e[1], et[2]) VTB_W2(wbase0, 2, e[2], et[1])
        VTB_W2(wbase1, 3, e[3], et[0]) VTB_W2(wbase1, 4, et[0], e[3]) VTB_W2(wbase1, 5, et[1], e[2])
        VTB_W2(wbase2, 6, et[2], e[1]) VTB_W2(wbase2, 7, et[3], e[0])
#undef VTB_W2
        // own-keeping rows (k9_pair): the start step of odd T, for hard input the padding steps
        const bool pad_row = !SOFT && (c + 1) * kCh > Tq && c * kCh + srow >= Tq;
        if ((c == 0 && srow < delta) || pad_row) {
            uint2* col = reinterpret_cast<uint2*>(tab) + srow;
            constexpr uint32_t PADW = H::SC * ((SOFT ? 2 : 16) * Q + 1) * kR1;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                col[k * kCol] = make_uint2(tieE, PADW + tieT);
                col[(4 + k) * kCol] = make_uint2(tieT, PADW + tieE);
            }
        }
    };

    // start metrics (k9_pair): location 0 (register 0, low half, lane 0) at B4, the rest B4 + Q
    uint32_t M[2];
    M[0] = (lane == 0) ? B4 | ((B4 + H::SC * Q) << 16) : (B4 + H::SC * Q) * kR1;
    M[1] = (B4 + H::SC * Q) * kR1;
    uint32_t ra;
    {
        uint32_t e[4], et[4];
        load_raw(0, ra);
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(ra));
        stage_compute(ra, e, et);
        stage_write(0, e, et);
    }
    uint2 buf[kRS][2];
#pragma unroll
    for (int s = 0; s < kAH; s++)
#pragma unroll
        for (int r = 0; r < 2; r++) buf[s][r] = *reinterpret_cast<const uint2*>(tab + off[r][s] + 8 * s);

    const uint32_t wlane = 8u * rev6(lam);  // survivor word byte offset of the lane within a column
    uint32_t dd = 0, m_prev[2] = {0, 0}, pw[2][4] = {}, se[4], set[4];
    const int tacs = (dbg & 2) ? 0 : Tpad;
    for (int t0 = 0; t0 < tacs; t0 += kCh) {
        const int c0 = t0 / kCh;
        const uint32_t gvo = uint32_t(kColS) * uint32_t(t0 >> 4) + wlane;
        static_for(std::make_integer_sequence<int, kCh>{}, [&](auto ic) {
            constexpr int I = decltype(ic)::value;
            constexpr int PH = I % 8;
            if constexpr (I == 0) load_raw(c0 + 1, ra);  // next chunk's raw input
            if constexpr (I == 20) {
                // one survivor store batch (step 15, two stores) was issued after the load
                asm volatile("s_waitcnt vmcnt(2)" : "+v"(ra));
                stage_compute(ra, se, set);
            }
            if constexpr (I == kCh - kAH) stage_write(c0 + 1, se, set);
            // renormalisation against location 0 (low half of lane 0's M[0]), both halves
            constexpr bool RN_READ = SOFT ? (I % 12) == 10 : I == 40;
            constexpr bool RN_APPLY = SOFT ? (I % 12) == 11 : I == 47;
            if constexpr (RN_READ) {
                const uint32_t ref = __builtin_amdgcn_readfirstlane(M[0]) & 0xFFFFu;
                dd = B4 * kR1 - ref * kR1;
            }
            uint32_t A[2], Bc[2];
            candidates_s<7 - PH>(M, buf[I % kRS], A, Bc);
            {
                constexpr int IN = (I + kAH) % kCh, PN = IN % 8;
#pragma unroll
                for (int r = 0; r < 2; r++)
                    buf[(I + kAH) % kRS][r] = *reinterpret_cast<const uint2*>(tab + off[r][PN] + 8 * IN);
            }
#pragma unroll
            for (int r = 0; r < 2; r++) M[r] = pk_min(A[r], Bc[r]);
            if constexpr (!SOFT && (I & 7) == 7) {
                // octet history bytes: [h0 oct 0, h0 oct 1, h1 oct 0, h1 oct 1] per 16 steps
#pragma unroll
                for (int r = 0; r < 2; r++) {
                    if constexpr ((I & 15) == 7) m_prev[r] = M[r];
                    else pw[r][0] = __builtin_amdgcn_perm(M[r], m_prev[r], 0x06020400u);
                    M[r] = RN_APPLY ? ((M[r] & ~H::MASK) + dd) : (M[r] & ~H::MASK);
                }
                if constexpr ((I & 15) == 15) {
                    constexpr int W = I >> 4;
                    gstore<W * kColS>(gvo, pw[0][0], gbase);
                    gstore<W * kColS + 4>(gvo, pw[1][0], gbase);
                }
            }
            if constexpr (SOFT && (I & 1)) {
                constexpr int w = (I & 15) >> 1;
#pragma unroll
                for (int r = 0; r < 2; r++) {
                    if constexpr (w & 1) pw[r][w >> 1] = __builtin_amdgcn_perm(M[r], m_prev[r], 0x06020400u);
                    else m_prev[r] = M[r];
                    M[r] = RN_APPLY ? ((M[r] & ~H::MASK) + dd) : (M[r] & ~H::MASK);
                }
                if constexpr ((I & 15) == 15) {
                    constexpr int W = I >> 4;
                    uint32_t z[2];
#pragma unroll
                    for (int r = 0; r < 2; r++) {
                        z[r] = bfi_op(0x03030303u, pw[r][0], pw[r][1] << 2);
                        z[r] = bfi_op(0x0F0F0F0Fu, z[r], pw[r][2] << 4);
                        z[r] = bfi_op(0x3F3F3F3Fu, z[r], pw[r][3] << 6);
                    }
                    gstore<W * kColS>(gvo, z[0], gbase);
                    gstore<W * kColS + 4>(gvo, z[1], gbase);
                }
            }
        });
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // Soft input, padding steps [Tq, Tpad): own-keeping survivor bits (k9_pair), per half
    if (SOFT && !(dbg & 2)) {
        uint32_t* wsw = reinterpret_cast<uint32_t*>(ws + slot * ws_wave);
        for (int g = Tq >> 4; g < (Tpad >> 4); g++) {
            const int w0 = Tq > 16 * g ? (Tq - 16 * g) >> 1 : 0;  // first padding window of the word
#pragma unroll
            for (int r = 0; r < 2; r++) {
                const uint32_t lp = (rev6(lam) << 2) | (uint32_t(r) << 1);  // l' of the low half
                uint32_t own = 0, mask = 0;
                for (int w = w0; w < 8; w++) {
                    const int sh = 8 * (w & 1) + 2 * (w >> 1);
                    own |= ((lp >> (2 * (w & 3))) & 3u) << sh;
                    own |= (((lp | 1u) >> (2 * (w & 3))) & 3u) << (sh + 16);
                    mask |= 3u << sh;
                }
                mask |= mask << 16;
                uint32_t* p = wsw + (kColS / 4) * g + (wlane >> 2) + r;
                *p = (*p & ~mask) | (own & mask);
            }
        }
    }
    __syncthreads();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (dbg & 1) return;

    // ---------------- traceback: verified block-parallel chains, 64 blocks ----------------
    const int blk = lane;
    uint8_t* ob = tab;
    const int top = (blk + 1) * tbb;
    const int start_full = top + kTbWarm;
    const int start = min(start_full, Tpad);
    const bool known = start >= Tq;
    const int nbody = (dbg & 8) ? 1 : (kTbWarm + tbb) / 48;
    uint32_t loc = 0, loc_top = 0;
    for (int g = 0; g < nbody; g++) {
        const int tlo = start_full - 48 * (g + 1);
        if (g == kTbWarm / 48) loc_top = loc;
        if (tlo < start) {
            const uint64_t bits = tbs_body<SOFT>(uint32_t(kColS) * uint32_t(tlo >> 4), loc, gbase);
            if (g >= kTbWarm / 48) put_bits48(ob, tlo, bits);
        }
    }
    // (chains of at most 64 blocks, the last known: at most 63 re-walk rounds.)  Completeness
    // guard as k9_pair: a frame with a block still unproven after the cap (VTB_DEBUG bit 17: every
    // chain with a walked block) is traced back serially by lane 0 from location 0 at Tpad
    uint32_t fin = loc;
    bool fixed = known || (dbg & 4);
    const bool tbforce = (dbg & kDbgTbCap) != 0;
    if (tbforce) loc_top = ~0u;  // (bit 17: no check passes)
    const int rounds = tbforce ? 0 : 65;
    uint64_t unproven = 0;
    for (int round = 0;; round++) {
        const uint32_t sf = __shfl_down(fin, 1);
        const bool ok = fixed || loc_top == sf;
        const uint64_t bad = ~__ballot(ok);
        if (bad == 0) break;
        if (round == rounds) {
            unproven = bad;
            break;
        }
        const bool succ_proven = blk == 63 || (bad >> (blk + 1)) == 0;
        if (!ok && succ_proven) {
            loc = sf;
            for (int g = kTbWarm / 48; g < nbody; g++) {
                const int tlo = start_full - 48 * (g + 1);
                put_bits48(ob, tlo, tbs_body<SOFT>(uint32_t(kColS) * uint32_t(tlo >> 4), loc, gbase));
            }
            fin = loc;
            fixed = true;
        }
    }
    if (blk == 0 && unproven != 0) {
        note_guard(hits);
        uint32_t l = 0;
        for (int tlo = Tpad - 48; tlo >= 0; tlo -= 48)
            put_bits48(ob, tlo, tbs_body<SOFT>(uint32_t(kColS) * uint32_t(tlo >> 4), l, gbase));
    }
    __syncthreads();

    // copy out; with delta = 1 kernel step t' is input step t' - 1 (shift the stream one bit)
    const int nbytes = (L + 7) >> 3;
    for (int j = lane; j < nbytes; j += 64) {
        const uint8_t v = delta ? uint8_t((ob[j] << 1) | (ob[j + 1] >> 7)) : ob[j];
        out[fr * out_stride + j] = v;
    }
}

// One wave per frame, for batches the CUs hold in one round (launch_k9).
template <bool SOFT>
__global__ __launch_bounds__(64) void k9s_kernel(const uint8_t* __restrict__ in, size_t in_stride,
                                                 uint8_t* __restrict__ out, size_t out_stride, int T, int L, int delta,
                                                 int Tq, int Tpad, int tbb, int dbg, Launch table,
                                                 uint8_t* __restrict__ ws, size_t ws_wave, uint32_t dpack) {
    uint32_t off[2][8];
    const uint32_t lam = lane_of(threadIdx.x);
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
        for (int ph = 0; ph < 8; ph++) {
            const int l = r * 64 + int(lam), p = 7 - ph;
            off[r][ph] = 8u * kCol * (table.symm[rotl8(l & ~(1 << p), ph)] + 4u * ((l >> p) & 1u));
        }
    k9_single<SOFT>(in, in_stride, out, out_stride, T, L, delta, Tq, Tpad, tbb, dbg, ws, ws_wave, blockIdx.x,
                    blockIdx.x, off, dpack, table.guard_hits);
}

// d(ph) of the k9s header packed 2 bits per phase, or false if the code's butterfly labels are
// not linear in the state (symm[s ^ e] = symm[s] ^ d for every s): then the pair kernel runs.
bool k9s_dpack(const Launch& a, uint32_t& dpack) {
    dpack = 0;
    for (int ph = 1; ph < 8; ph++) {
        const int e = 1 << (ph - 1);
        const int d = a.symm[e] ^ a.symm[0];
        if (d > 3) return false;
        for (int s = 0; s < 128; s++)
            if ((a.symm[s ^ e] ^ a.symm[s]) != d) return false;
        dpack |= uint32_t(d) << (2 * ph);
    }
    return true;
}

// k9s runs a batch the CUs hold in one round (one wave per frame, resident waves and 1 GiB of
// survivor slots); a larger batch goes to the persistent pair kernel, whose waves carry two
// frames each: a persistent k9s grid leaves its last round part-empty (16,384 soft frames: 0.345
// ms against the pair kernel's 0.309, profiles/r05/k9s/ab.jsonl).  False also for codes whose
// labels are not linear in the state (k9s_dpack) and under VTB_DEBUG bit 18.
bool k9s_use(const Launch& a, uint32_t& dpack) {
    const int Tq = a.T + (a.T & 1);
    if ((a.dbg & kDbgK9Pair) || (size_t)region0_s(Tq) > 64 * 1024 || !k9s_dpack(a, dpack)) return false;
    auto kern = a.soft ? k9s_kernel<true> : k9s_kernel<false>;
    const int per_cu = resident_per_cu(reinterpret_cast<const void*>(kern), (size_t)region0_s(Tq));
    const size_t resident = size_t(per_cu > 0 ? per_cu : 8) * size_t(a.cus > 0 ? a.cus : 1);
    const size_t cap = (size_t(1) << 30) / ws_wave_bytes_s(Tq);
    return a.frames <= resident && a.frames <= cap;
}

// Grid: the frame pairs, at most what the CUs hold at once and at most 1 GiB of survivor
// slots (one per wave).
size_t grid_waves(const Launch& a, int Tq, int NB = 2) {
    const size_t pairs = (a.frames + 1) / 2;
    size_t grid = pairs;
    auto kern = NB == 3 ? k9_kernel<false, true, false, 3> : a.soft ? k9_kernel<true, true> : k9_kernel<false, true>;
    const int per_cu =
        (a.dbg & 32) ? 0 : resident_per_cu(reinterpret_cast<const void*>(kern), (size_t)region0(Tq, NB));
    if (per_cu > 0) {
        const size_t resident = size_t(per_cu) * size_t(a.cus > 0 ? a.cus : 1);
        if (resident < grid) grid = resident;
    }
    size_t cap = (size_t(1) << 30) / ws_wave_bytes(Tq);
    if (cap < 1) cap = 1;
    return cap < grid ? cap : grid;
}

// K = 9 single-frame geometry: W waves per workgroup, up to `wgs` workgroups; n = ACS steps per
// segment (multiple of 48) so that 2 W wgs segments cover Tq, G = the segments whose exact part
// starts before Tq.
bool k9_seg_geometry(int Tq, int W, int wgs, int warm, Seg9& sg, int& nwg) {
    if (W < 1 || W > 8 || wgs < 1 || wgs > 64 || warm < kCh || warm % kCh) return false;
    const int G2 = 2 * W * wgs;
    int n = (Tq + (G2 - 1) * warm + G2 - 1) / G2;
    n = (n + kCh - 1) / kCh * kCh;
    if (n < warm + kCh) n = warm + kCh;
    int G = 1;
    while (G < G2 && G * (n - warm) + warm < Tq) G++;
    if ((G - 1) * (n - warm) + n < Tq) return false;
    sg.n = n, sg.warm = warm, sg.G = G;
    nwg = ((G + 1) / 2 + W - 1) / W;
    return true;
}

size_t k9_seg_lds(int T, int Tq, bool soft, int W, int& in_lds, int& ob_lds, int& flag_lds) {
    in_lds = W * ((kRingBytes + 15) / 16 * 16);
    ob_lds = in_lds + ((soft ? 2 : 1) * T + 15) / 16 * 16;
    flag_lds = ob_lds + (t_pad(Tq) / 8 + 16 + 15) / 16 * 16;
    return size_t(flag_lds) + 4 * (1 + W);
}
}  // namespace

bool k9_seg_supported(const Launch& a, int waves, int wgs, int warm) {
    const int delta = a.T & 1, Tq = a.T + delta;
    Seg9 sg;
    int nwg, il, ol, fl;
    if (a.S != 8 || a.T < 240 || !k9_seg_geometry(Tq, waves, wgs, warm, sg, nwg)) return false;
    const int nin = (a.soft ? 2 : 1) * a.T;
    return nin <= 16 * 4 * 64 * waves && k9_seg_lds(a.T, Tq, a.soft, waves, il, ol, fl) <= 64 * 1024;
}

size_t k9_seg_workspace_bytes(const Launch& a, int waves, int wgs, int warm) {
    const int Tq = a.T + (a.T & 1);
    Seg9 sg;
    int nwg;
    if (!k9_seg_geometry(Tq, waves, wgs, warm, sg, nwg)) return 0;
    const size_t nw = size_t(nwg) * waves;
    return 256 + nw * 512 * 4 + nw * size_t(kColBytes) * (sg.n / 16);  // counter, metrics, words
}

hipError_t launch_k9_seg(const Launch& a, int waves, int wgs, int warm, uint32_t* done) {
    const int delta = a.T & 1, Tq = a.T + delta;
    Seg9Args g;
    int nwg;
    if (!a.ws || !k9_seg_geometry(Tq, waves, wgs, warm, g.s, nwg)) return hipErrorInvalidValue;
    int il, ol, fl;
    const size_t lds = k9_seg_lds(a.T, Tq, a.soft, waves, il, ol, fl);
    g.s.ring_bytes = (kRingBytes + 15) / 16 * 16;
    g.s.in_lds = il;
    g.ob_lds = ol;
    g.flag_lds = fl;
    g.nwg = nwg;
    g.done = done;
    // all working workgroups on one XCD (workgroups go round-robin over the 8 XCDs): the
    // arrival fences and the traceback's word reads stay within one L2 (72.7 against 67.4
    // Mbit/s for speedDecode K=9); $VTB_SEG9_XCD=0 spreads them (measurement)
    g.xcd = a.seg9_xcd == 0 ? 1 : 8;
    uint8_t* base = static_cast<uint8_t*>(a.ws);
    g.counter = reinterpret_cast<uint32_t*>(base);
    g.met = reinterpret_cast<uint32_t*>(base + 256);
    const size_t nw = size_t(nwg) * waves, ws_wave = size_t(kColBytes) * (g.s.n / 16);
    uint8_t* words = base + 256 + nw * 512 * 4;
    auto kern = a.soft ? k9_seg_kernel<true> : k9_seg_kernel<false>;
    note_kernel("k9_seg");
    hipLaunchKernelGGL(kern, dim3(unsigned(nwg * g.xcd)), dim3(64 * waves), lds, a.stream, a.in, a.out, a.T, a.L, delta, Tq,
                       a.dbg, a, words, ws_wave, g);
    return hipGetLastError();
}

bool k9_supported(const Launch& a) {
    return a.S == 8 && a.T > a.S && (size_t)region0(a.T + (a.T & 1)) <= 160 * 1024;
}

size_t k9_workspace_bytes(const Launch& a) {
    const int Tq = a.T + (a.T & 1);
    uint32_t dpack;
    if (k9s_use(a, dpack)) return a.frames * ws_wave_bytes_s(Tq);
    return grid_waves(a, Tq) * ws_wave_bytes(Tq);
}

// One streaming call (see launch_k7_stream): every wave (two streams) continues its trellis
// over [s.t_begin, s.t_end) and emits the final bits (stream_traceback9).
hipError_t launch_k9_stream(const Launch& a, const StreamArgs& s) {
    if (a.frames == 0) return hipSuccess;
    if (!a.ws || !s.state || !s.out_bits || s.ring < 48 || s.ring % 48 || s.t_begin % 48 || s.t_end % 48)
        return hipErrorInvalidValue;
    auto kern = a.soft ? k9_kernel<true, false, true> : k9_kernel<false, false, true>;
    const size_t waves = (a.frames + 1) / 2;
    note_kernel("k9_stream");
    hipLaunchKernelGGL(kern, dim3(unsigned(waves)), dim3(64), (size_t)kRingBytes, a.stream, a.in, a.in_stride, a.out,
                       a.out_stride, a.T, a.L, 0, a.T, s.t_end, 0, a.frames, a.dbg, a, static_cast<uint8_t*>(a.ws),
                       size_t(kColBytes) / 16 * size_t(s.ring), s);
    return hipGetLastError();
}

// k = 1 rate 1/3, hard input (a.symm: 3-bit butterfly labels): the K=9 frame kernel with a
// 16-column branch-metric table (k9_pair NB = 3); survivors in a.ws (k9_n3_workspace_bytes).
bool k9_n3_supported(const Launch& a) {
    return a.S == 8 && !a.soft && a.T > a.S && (size_t)region0(a.T + (a.T & 1), 3) <= 160 * 1024;
}
size_t k9_n3_workspace_bytes(const Launch& a) {
    const int Tq = a.T + (a.T & 1);
    return grid_waves(a, Tq, 3) * ws_wave_bytes(Tq);
}
hipError_t launch_k9_n3(const Launch& a) {
    if (a.frames == 0) return hipSuccess;
    if (!a.ws || !k9_n3_supported(a)) return hipErrorInvalidValue;
    const int delta = a.T & 1, Tq = a.T + delta;
    const size_t lds = (size_t)region0(Tq, 3);
    const size_t grid = grid_waves(a, Tq, 3);
    const bool lp = grid < (a.frames + 1) / 2;
    auto kern = lp ? k9_kernel<false, true, false, 3> : k9_kernel<false, false, false, 3>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
    }
    note_kernel(lp ? "k9_n3_loop" : "k9_n3");
    hipLaunchKernelGGL(kern, dim3(unsigned(grid)), dim3(64), lds, a.stream, a.in, a.in_stride, a.out,
                       a.out_stride, a.T, a.L, delta, Tq, t_pad(Tq), tb_block(Tq), a.frames, a.dbg, a,
                       static_cast<uint8_t*>(a.ws), ws_wave_bytes(Tq), StreamArgs());
    return hipGetLastError();
}

hipError_t launch_k9(const Launch& a) {
    if (a.frames == 0) return hipSuccess;
    if (!a.ws) return hipErrorInvalidValue;
    const int delta = a.T & 1, Tq = a.T + delta;
    uint32_t dpack;
    if (k9s_use(a, dpack)) {
        note_kernel("k9s");
        hipLaunchKernelGGL(a.soft ? k9s_kernel<true> : k9s_kernel<false>, dim3(unsigned(a.frames)), dim3(64),
                           (size_t)region0_s(Tq), a.stream, a.in, a.in_stride, a.out, a.out_stride, a.T, a.L, delta,
                           Tq, t_pad(Tq), tb_block_s(Tq), a.dbg, a, static_cast<uint8_t*>(a.ws),
                           ws_wave_bytes_s(Tq), dpack);
        return hipGetLastError();
    }
    const size_t lds = (size_t)region0(Tq);
    const size_t grid = grid_waves(a, Tq);
    auto kern = grid < (a.frames + 1) / 2 ? (a.soft ? k9_kernel<true, true> : k9_kernel<false, true>)
                                          : (a.soft ? k9_kernel<true, false> : k9_kernel<false, false>);
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
    }
    note_kernel(grid < (a.frames + 1) / 2 ? "k9_loop" : "k9");
    hipLaunchKernelGGL(kern, dim3(unsigned(grid)), dim3(64), lds, a.stream, a.in, a.in_stride, a.out,
                       a.out_stride, a.T, a.L, delta, Tq, t_pad(Tq), tb_block(Tq), a.frames, a.dbg, a,
                       static_cast<uint8_t*>(a.ws), ws_wave_bytes(Tq), StreamArgs());
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipSuccess;
}

}  // namespace vtb
