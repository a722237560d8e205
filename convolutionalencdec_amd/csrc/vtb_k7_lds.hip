// K=7 (64 states) decoder with LDS-resident survivors: the fast path for frames whose
// survivor words fit in LDS at two waves per SIMD (L up to ~1000 at 8 waves/CU; longer
// frames run at lower occupancy).  Hard and 8-bit soft input.
//
// Layout.  One wave64 decodes two frames, A and B.  Lane l holds the path metric of the
// trellis state living at "location" l for both frames as one packed u16 pair
// [m_A, m_B]: every packed instruction advances both frames.
//
// In-place state relabelling.  Instead of moving state s to lane s every step (the
// reference's destination-indexed butterfly, viterbiDecoderButterflyk1.c:101-152), each
// butterfly writes its two destinations back into the two locations its sources came
// from.  Location l then holds state rotl6(l, t mod 6) at step t, and the two sources of
// a butterfly (states j and j+32) sit in lanes that differ in one bit, p = 5 - (t mod 6).
// Location l is kept in lane L(l) = l ^ (3 if bit 2 of l else 0), a linear involution
// chosen so that every pairing bit maps to an XOR of the lane index that one cross-lane op
// performs: location bits 0..5 -> lane XOR 1, 2, 7, 8, 16, 32 = DPP quad_perm,
// quad_perm, row_half_mirror, row_ror:8 (folded into the add), in-place
// v_permlane16_swap, v_permlane32_swap.
//
// Metrics carry their decisions.  A stored metric is 4m + h: the exact integer path
// metric m (renormalised) times four, plus two low "history" bits h.  Step t puts a tie
// bit at position b = t & 1 into both candidates: the own candidate gets R << b and the
// partner's (1 - R) << b, where R = bit p of the lane's location (R = 1: the lane's own
// state is the upper predecessor j+32).  So the two candidates never compare equal, an
// exact tie goes to the lower predecessor j as in the reference (strict '>',
// viterbiDecoderButterflyk1.c:129-130), and bit b of the minimum is the decision
// D = R xor [partner won] = the location bit p of the survivor's predecessor.  The ACS is
// three instructions per step for two frames:
//     A = M + V;  B = partner(M) + W;  M' = pk_min(A, B)
// with (V, W) = (4e(c) + R << b, 4e(~c) + (1 - R) << b) read from a branch-metric table
// row in LDS (c = the butterfly's edge label).  History bits below b never reach a
// comparison's outcome (candidate metrics differ by multiples of 4).  After the odd step
// of each two-step window the history holds [D_odd at this location, D_even at the
// survivor's predecessor] -- exactly the two decisions a traceback through this location
// reads -- so the two bits are appended to the lane's survivor word and cleared.
//
// Table rows (one per step): eight (V, W) u32 pairs for (c, R), both frames packed, staged
// for a whole 48-step chunk at a time by 48 lanes from raw input bytes loaded a chunk
// earlier, into a 48-row LDS ring stored column-major: pair k of ring row r at 8-byte slot
// 49k + r.  Staging writes (lane = row) are then contiguous ds_write_b64s and the eight
// pairs of one row sit in distinct banks for the broadcast ds_read_b64 of a step.  Steps past T (padding up to the chunk size) use
// rows V = tie, W = 4(12Q + 1) + tie that make every lane keep its own predecessor, so
// the survivor at location 0 stays at location 0 through the padding.
//
// Initial metrics: the reference starts state 0 at 0 and every other state at
// (uint8)(N+1) = 65 (x255 soft).  For K=7 any start value above 12Q (six steps of the
// largest branch metric) yields the same decisions -- during the first six steps a path
// from state 0 always beats one from another state, paths from other states compare
// with equal offsets, and from step 6 on every state descends from state 0 -- so this
// kernel uses 12Q + 1.
//
// Renormalisation every 12 steps (subtract location 0's metric taken at the start of the
// window, add a bias) rides on the history clear; it replaces the reference's uint8 renorm
// (exact metrics have a bounded spread).
//
// Survivors.  Two windows' history bytes are gathered by one v_perm, and every 16 steps
// three v_bfi pack the 8 windows into one word per lane (frame A in bits 0..15, frame B in
// 16..31; window w at bits 8(w & 1) + 2(w >> 1)), which the wave writes (256 B, one
// ds_write_b32) to the slot of the lane's bit-reversed location l' = rev6(l).
//
// Traceback (reference :200-256), two steps per LDS read: in l' numbering step t's
// pairing bit is bit t mod 6, so a window's two decisions are the new bits
// (t_even mod 6, t_odd mod 6) of l', adjacent; the walk keeps the LDS address of the
// survivor's word and a window is one read, one shift and one bit-field insert.  A
// sextet's six decoded bits are its end location (oldest step at bit 0 of l').  Lanes
// 0-31 trace blocks of frame A, lanes 32-63 of frame B, each block of TBB steps (a
// multiple of 48) walking back from 48 steps past its end.  A block whose walk starts at
// or beyond T starts at the known location 0 (the terminated path ends in state 0).  The
// others are verified together: a block is right if it entered on its successor's exit
// location and its successor is proven; failed blocks re-walk from a proven successor
// until all are proven.  So the output is exactly the reference's for every input; only
// the time depends on how fast survivor paths merge.

#include <type_traits>
#include <utility>

#include "vtb_k7_common.h"

namespace vtb {
namespace {

using namespace k7;

constexpr int kCol = 49;                   // 8-byte slots per table column (48 rows + bank skew)
__host__ __device__ constexpr int ring_slot(int r) { return r; }
constexpr int kRingBytes = 8 * kCol * 8;   // branch-metric ring: 8 (label, R) columns
// Rate 1/3 (NB = 3): 16 (label, R) columns of a 24-row ring (25 slots: the 16 columns of a row
// in distinct bank pairs), refilled half a chunk at a time (k7_pair), so that the ring, 3.2 KB,
// leaves 8 waves per CU at L = 1,024 like the rate-1/2 ring.
template <int NB>
constexpr int kColN = NB == 3 ? 25 : kCol;   // 8-byte slots per table column
template <int NB>
constexpr int kRowsN = NB == 3 ? 24 : kChunk;  // ring rows
constexpr int ring_bytes(int NB) { return (2 << NB) * (NB == 3 ? kColN<3> : kCol) * 8; }
constexpr int kTbWarm = 48;  // traceback warm-up steps past a block's end (multiple of 48)
// Share of its chunks the second-dispatched wave of a SIMD runs at priority 1 (wave balance,
// k7_pair).  Round 2: 55 / 59 / 63 measured alike (31.06 / 31.1 / 31.0 us per 4,096-frame launch);
// round 4, ten interleaved rounds over two boxes (profiles/r04/first/ab_prio_*.txt): 67 is
// 0.4-0.6 % faster than 59, 50 / 71 / 75 slower.
constexpr int kPrioPct = 67;
constexpr uint32_t kR1 = 0x10001u;
// Soft renormalisation period in steps (divides the 48-step chunk).  16 would overflow the u16
// metrics on padding rows (PERF_LOG.md §5; tests/test_metric_bounds.py).
constexpr int kRenormSoft = 12;

// History bits per u16 half: soft input keeps 4m + h (2 history bits, the
// exact metric needs 14 bits); hard input, whose metrics stay below 128, keeps 256m + h
// with 8 history bits (tie bit at t mod 8, clear and survivor byte every 8 steps, eight
// decisions per traceback read).
// NB (k = 1 codes of rate 1/NB; 3 only for hard input, through vtb_genk_decode_device): the
// spread bound and the start value scale with the largest branch metric NB Q.
template <bool SOFT, int NB = 2>
struct Hist {
    static_assert(NB == 2 || (NB == 3 && !SOFT), "rate 1/3: hard input only");
    static constexpr int HB = SOFT ? 2 : 8;                  // history bits
    static constexpr uint32_t SC = 1u << HB;                 // metric scale
    static constexpr uint32_t MASK = (SC - 1) * 0x10001u;    // history bits of both frames
    static constexpr uint32_t BIAS = SC * (SOFT ? 3060 : 6 * NB);  // renormalised location-0 metric (scaled)
};

int tb_block(int T) {
    const int per = (T + 31) / 32;  // 32 blocks per frame, multiple of 48 steps
    return (per + 47) / 48 * 48;
}
int t_pad(int T) { return (T + kChunk - 1) / kChunk * kChunk; }
// SPLIT: frame A's half ends at t1 (a multiple of 48), frame B's starts `warm` steps
// earlier, and both run t1 steps: t1 = the smallest multiple of 48 with 2 t1 - warm >= T
// (ceil((T + warm) / 2): with the floor, T + warm odd and (T + warm - 1) / 2 a multiple of 48
// left frame B one step short of T - 1 -- fixed in round 2, tests/test_gpu_parity.py
// test_split_frames_vs_oracle L = 1051, 2203 and test_split_loop_odd_tail).
// kSplitWarm = 96: frame B's metrics then equal frame A's up to a constant at t1 in all of
// 2,000 simulated soft frames at SNR -5 dB (48: 98.2 %, and every miss costs its wave a
// second, unsplit pass).
constexpr int kSplitWarm = 96;
// SPLIT fix-up: chunks frame B's half may re-run from frame A's metrics before the frame falls
// back to its slow path (k7_pair)
constexpr int kFix = 4;
__host__ __device__ constexpr int split_t1(int T, int warm = kSplitWarm) {
    return ((T + warm + 1) / 2 + kChunk - 1) / kChunk * kChunk;
}
// LDS: [0, r0) table ring, later the decoded bytes of both frames; [r0, r0 + 16*Tpad)
// survivor words.
int region0(int T, int NB = 2) {  // multiple of 256: the traceback edits survivor-word addresses in place
    const int r = 8 * tb_block(T) > ring_bytes(NB) ? 8 * tb_block(T) : ring_bytes(NB);
    return (r + 255) / 256 * 256;
}
size_t lds_bytes(int T, int NB = 2) { return (size_t)region0(T, NB) + 16 * (size_t)t_pad(T); }

// Measurement only: phase timestamp k of this wave (Launch::tstamp, 8 u64 per wave).
__device__ __forceinline__ void tstamp(const Launch& table, int k) {
    if (table.tstamp && threadIdx.x == 0) table.tstamp[8 * blockIdx.x + k] = __builtin_amdgcn_s_memrealtime();
}

// LDS byte address of a pointer into the shared-memory aperture
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return uint32_t(size_t((const __attribute__((address_space(3))) uint8_t*)p));
}
// a table column by its LDS byte address: col[i] is the i-th 8-byte (V, W) slot
struct LdsCol {
    uint32_t a;
    __device__ __forceinline__ uint2 operator[](int i) const {
        const unsigned long long v = *(const __attribute__((address_space(3))) unsigned long long*)size_t(a + 8u * uint32_t(i));
        return make_uint2(uint32_t(v), uint32_t(v >> 32));
    }
};

// lane <-> location map (an involution)
__host__ __device__ __forceinline__ uint32_t lane_of(uint32_t l) { return l ^ (((l >> 2) & 1u) * 3u); }

// The candidates of a step: A = own metric + V, B = partner's metric (across location bit
// P: lane XOR 1, 2, 7, 8, 16, 32) + W.  For the permlane phases the add of A separates the
// last VALU write of m from the swap and an s_nop separates the swap from the read of its
// result (one wait state each way: tools/probes/permlane_hazard.hip).
template <int P>
__device__ __forceinline__ void candidates(uint32_t m, uint2 vw, uint32_t& A, uint32_t& B) {
    if constexpr (P == 4 || P == 5) {
        if constexpr (P == 4) {
            asm volatile("v_add_u32 %0, %1, %2\n\tv_permlane16_swap_b32 %1, %1\n\ts_nop 0"
                         : "=&v"(A), "+v"(m) : "v"(vw.x));
        } else {
            asm volatile("v_add_u32 %0, %1, %2\n\tv_permlane32_swap_b32 %1, %1\n\ts_nop 0"
                         : "=&v"(A), "+v"(m) : "v"(vw.x));
        }
        B = m + vw.y;
    } else {
        A = m + vw.x;
        if constexpr (P == 2) {
            B = __builtin_amdgcn_update_dpp(0u, m, 0x141, 0xF, 0xF, true) + vw.y;  // row_half_mirror: XOR 7
        } else {
            B = partner_plus<P>(m, vw.y);
        }
    }
}

// One v_bfi_b32 (the compiler otherwise splits a constant-mask select into and/and/or).
__device__ __forceinline__ uint32_t bfi_op(uint32_t mask, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(mask), "v"(a), "v"(b));
    return r;
}

// Reversed location numbering for the survivor words and the traceback: l' = rev6(l), so
// step t's pairing bit is bit t mod 6 of l' and a window's two decisions (even step at
// the lower history bit) land on the adjacent bits (t_even mod 6, t_odd mod 6) of l'.
__host__ __device__ __forceinline__ uint32_t rev6(uint32_t l) {
    return ((l & 1) << 5) | ((l & 2) << 3) | ((l & 4) << 1) | ((l & 8) >> 1) | ((l & 16) >> 3) | ((l & 32) >> 5);
}

// 48 traceback steps over [tlo, tlo + 48) (tlo a multiple of 48), newest first.  cb is the
// LDS byte address of the block's first survivor-word column (dec + 256 (tlo / 16) + 2f:
// bits 2..7 clear) and l4 = 4 l' of the survivor's location, so cb | l4 addresses its word
// and each window is one read, one shift and one bit-field insert on the address.
// Returns the 48 decoded bits with bit 0 = step tlo (a sextet's bits are its end location
// in l' numbering, oldest step at bit 0).
// One dependent read per window.
template <bool GS>
__device__ __forceinline__ uint64_t tb_body_serial(uint32_t cb, uint32_t& l4, uint64_t gbase) {
    uint32_t a = cb | l4;
    uint64_t bits = 0;
#pragma unroll
    for (int j = 0; j < 24; j++) {
        const int todd = 47 - 2 * j;  // odd step of the window, relative to tlo
        if (j % 3 == 0) bits |= uint64_t((a >> 2) & 63u) << (6 * (7 - j / 3));  // sextet end tlo + todd + 1
        const int wi = (todd & 15) >> 1, sh = 8 * (wi & 1) + 2 * (wi >> 1);      // window's bits in its half-word
        uint32_t v;  // survivor half-word (smem is LDS address 0: dynamic LDS only)
        if constexpr (GS) {
            asm volatile("global_load_ushort %0, %1, %2 offset:%3\n\ts_waitcnt vmcnt(0)"
                         : "=v"(v) : "v"(a), "s"(gbase), "i"((todd >> 4) * 256));
        } else {
            asm volatile("ds_read_u16 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a), "i"((todd >> 4) * 256));
        }
        const int pos = 2 + (todd - 1) % 6;  // address bit of l' bit (t_even mod 6)
        const uint32_t fld = pos >= sh ? (v << (pos - sh)) : (v >> (sh - pos));
        a = (a & ~(3u << pos)) | (fld & (3u << pos));
    }
    l4 = a & 0xFCu;
    return bits;
}

// Two windows per dependent read: window j's two decisions are the only address bits in
// which window j+1's word can differ, so the read of window j and the four candidate words
// of window j+1 (one base address with those bits clear, the bits as immediate offsets) are
// issued together, and window j's bits then pick window j+1's word.
template <bool GS>
__device__ __forceinline__ uint64_t tb_body_spec(uint32_t cb, uint32_t& l4, uint64_t gbase) {
    uint32_t a = cb | l4;
    uint64_t bits = 0;
#pragma unroll
    for (int j = 0; j < 24; j += 2) {
        const int todd = 47 - 2 * j, todd1 = todd - 2;  // odd steps of windows j, j+1 (relative to tlo)
        const int wi = (todd & 15) >> 1, sh = 8 * (wi & 1) + 2 * (wi >> 1);
        const int wi1 = (todd1 & 15) >> 1, sh1 = 8 * (wi1 & 1) + 2 * (wi1 >> 1);
        const int pos = 2 + (todd - 1) % 6, pos1 = 2 + (todd1 - 1) % 6;  // address bits of the decisions
        if (j % 3 == 0) bits |= uint64_t((a >> 2) & 63u) << (6 * (7 - j / 3));
        const uint32_t base = a & ~(3u << pos);  // window j+1's word address without window j's bits
        const int o = (todd >> 4) * 256, o1 = (todd1 >> 4) * 256, d = 1 << pos;
        uint32_t v, c0, c1, c2, c3;
        if constexpr (GS) {
            asm volatile(
                "global_load_ushort %0, %5, %7 offset:%8\n\t"
                "global_load_ushort %1, %6, %7 offset:%9\n\tglobal_load_ushort %2, %6, %7 offset:%10\n\t"
                "global_load_ushort %3, %6, %7 offset:%11\n\tglobal_load_ushort %4, %6, %7 offset:%12\n\t"
                "s_waitcnt vmcnt(0)"
                : "=&v"(v), "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3)
                : "v"(a), "v"(base), "s"(gbase), "i"(o), "i"(o1), "i"(o1 + d), "i"(o1 + 2 * d), "i"(o1 + 3 * d));
        } else {
            asm volatile(
                "ds_read_u16 %0, %5 offset:%7\n\t"
                "ds_read_u16 %1, %6 offset:%8\n\tds_read_u16 %2, %6 offset:%9\n\t"
                "ds_read_u16 %3, %6 offset:%10\n\tds_read_u16 %4, %6 offset:%11\n\t"
                "s_waitcnt lgkmcnt(0)"
                : "=&v"(v), "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3)
                : "v"(a), "v"(base), "i"(o), "i"(o1), "i"(o1 + d), "i"(o1 + 2 * d), "i"(o1 + 3 * d));
        }
        const uint32_t f = (v >> sh) & 3u;  // window j's decisions = address bits pos, pos + 1
        a = base | (f << pos);
        if ((j + 1) % 3 == 0) bits |= uint64_t((a >> 2) & 63u) << (6 * (7 - (j + 1) / 3));
        const uint32_t lo = (f & 1u) ? c1 : c0, hi = (f & 1u) ? c3 : c2;
        const uint32_t v1 = (f & 2u) ? hi : lo;
        a = (a & ~(3u << pos1)) | (((v1 >> sh1) & 3u) << pos1);
    }
    l4 = a & 0xFCu;
    return bits;
}

// The serial form is the shipped one.  The speculative form (round 1, measurement only)
// measured slower where it matters: LDS words 6 % per 4,096-frame launch (2.5 random
// reads per window cost more LDS bandwidth than the latency they hide, with 8 waves per CU
// tracing back at once), global words 2 % slower on config C3 (65,536 x 2,048 bits: the
// extra loads queue behind other waves' traffic), 2 % faster only for one 4,096-frame round
// with global words.
template <bool GS>
__device__ __forceinline__ uint64_t tb_body(uint32_t cb, uint32_t& l4, uint64_t gbase) {
    return tb_body_serial<GS>(cb, l4, gbase);
}

__device__ __forceinline__ uint32_t rotl6c(uint32_t x, int r) { return r == 0 ? x : ((x << r) | (x >> (6 - r))) & 63u; }
__device__ __forceinline__ uint32_t rotr6c(uint32_t x, int r) { return r == 0 ? x : ((x >> r) | (x << (6 - r))) & 63u; }

// Hard input (8 history bits): 48 traceback steps as six octets, one byte read each.  The
// byte of octet k (steps tlo + 8k + b, b = 0..7) at the survivor's location holds the
// decisions D_b along its path; D_b replaces l' bit r_b = (8k + b) mod 6, so the location
// eight steps back is rotl6(byte & 63, r_0) (bits b = 6, 7 are overwritten by b = 0, 1) and
// the decoded bits are [byte bit 6, byte bit 7, u2, u3, u4, u5, u0, u1] with
// u = rotr6(end location l', r_0).
template <bool GS>
__device__ __forceinline__ uint64_t tb_body8(uint32_t cb, uint32_t& l4, uint64_t gbase) {
    uint32_t a = cb | l4;
    uint64_t bits = 0;
#pragma unroll
    for (int k = 5; k >= 0; k--) {
        const int r0 = (8 * k) % 6;
        const uint32_t u = rotr6c((a >> 2) & 63u, r0);
        uint32_t v;
        if constexpr (GS) {
            asm volatile("global_load_ubyte %0, %1, %2 offset:%3\n\ts_waitcnt vmcnt(0)"
                         : "=v"(v) : "v"(a), "s"(gbase), "i"(256 * (k >> 1) + (k & 1)));
        } else {
            asm volatile("ds_read_u8 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a), "i"(256 * (k >> 1) + (k & 1)));
        }
        bits |= uint64_t((u & 0x3Cu) | ((v >> 6) & 3u) | ((u & 3u) << 6)) << (8 * k);
        a = (a & ~0xFCu) | (rotl6c(v & 63u, r0) << 2);
    }
    l4 = a & 0xFCu;
    return bits;
}

// The same two walks for the global-survivor variant with its newest steps' words in LDS:
// a lane's block is in LDS (is_lds: word at LDS byte lds_off + a) or in the workspace (gbase
// + a).  Every window issues both an LDS read and a global load -- the one the lane does not
// need at a harmless address (low LDS bytes / the slot's first, cache-hot column) -- and waits
// for both once, so LDS lanes and global lanes of a wave walk at the same time (a per-lane
// branch would run the two kinds one after the other; flat loads measured 40 % slower).
template <int O>
__device__ __forceinline__ uint32_t dual_ld16(uint32_t a, bool is_lds, uint32_t lds_off, uint64_t gbase) {
    const uint32_t al = is_lds ? lds_off + a : (a & 0xFFu), ag = is_lds ? (a & 0xFFu) : a;
    uint32_t vl, vg;
    asm volatile("ds_read_u16 %0, %2 offset:%4\n\tglobal_load_ushort %1, %3, %5 offset:%4\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                 : "=&v"(vl), "=&v"(vg) : "v"(al), "v"(ag), "i"(O), "s"(gbase));
    return is_lds ? vl : vg;
}
template <int O>
__device__ __forceinline__ uint32_t dual_ld8(uint32_t a, bool is_lds, uint32_t lds_off, uint64_t gbase) {
    const uint32_t al = is_lds ? lds_off + a : (a & 0xFFu), ag = is_lds ? (a & 0xFFu) : a;
    uint32_t vl, vg;
    asm volatile("ds_read_u8 %0, %2 offset:%4\n\tglobal_load_ubyte %1, %3, %5 offset:%4\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                 : "=&v"(vl), "=&v"(vg) : "v"(al), "v"(ag), "i"(O), "s"(gbase));
    return is_lds ? vl : vg;
}
template <int... Is, class F>
__device__ __forceinline__ void static_for_k7(std::integer_sequence<int, Is...>, F&& f) {
    (f(std::integral_constant<int, Is>{}), ...);
}
__device__ __forceinline__ uint64_t tb_body_dual(uint32_t cb, uint32_t& l4, bool is_lds, uint32_t lds_off,
                                                 uint64_t gbase) {
    uint32_t a = cb | l4;
    uint64_t bits = 0;
    static_for_k7(std::make_integer_sequence<int, 24>{}, [&](auto jc) {
        constexpr int j = decltype(jc)::value, todd = 47 - 2 * j;
        if (j % 3 == 0) bits |= uint64_t((a >> 2) & 63u) << (6 * (7 - j / 3));
        constexpr int wi = (todd & 15) >> 1, sh = 8 * (wi & 1) + 2 * (wi >> 1);
        const uint32_t v = dual_ld16<(todd >> 4) * 256>(a, is_lds, lds_off, gbase);
        constexpr int pos = 2 + (todd - 1) % 6;
        uint32_t fld;
        if constexpr (pos >= sh) fld = v << (pos - sh);
        else fld = v >> (sh - pos);
        a = (a & ~(3u << pos)) | (fld & (3u << pos));
    });
    l4 = a & 0xFCu;
    return bits;
}
__device__ __forceinline__ uint64_t tb_body8_dual(uint32_t cb, uint32_t& l4, bool is_lds, uint32_t lds_off,
                                                  uint64_t gbase) {
    uint32_t a = cb | l4;
    uint64_t bits = 0;
    static_for_k7(std::make_integer_sequence<int, 6>{}, [&](auto kc) {
        constexpr int k = 5 - decltype(kc)::value, r0 = (8 * k) % 6;
        const uint32_t u = rotr6c((a >> 2) & 63u, r0);
        const uint32_t v = dual_ld8<256 * (k >> 1) + (k & 1)>(a, is_lds, lds_off, gbase);
        bits |= uint64_t((u & 0x3Cu) | ((v >> 6) & 3u) | ((u & 3u) << 6)) << (8 * k);
        a = (a & ~0xFCu) | (rotl6c(v & 63u, r0) << 2);
    });
    l4 = a & 0xFCu;
    return bits;
}

// Output bytes of steps [tlo, tlo + 48) (bit 0 of bits = step tlo; bytes MSB-first as the
// reference packs them, viterbiDecoderButterflyk1.c:243-249).
__device__ __forceinline__ void put_bits48(uint8_t* ob, int tlo, uint64_t bits) {
    unsigned short* o = reinterpret_cast<unsigned short*>(ob + (tlo >> 3));
    const uint32_t r = __builtin_bitreverse32(uint32_t(bits)), rh = __builtin_bitreverse32(uint32_t(bits >> 32));
    o[0] = (unsigned short)((r >> 24) | ((r >> 8) & 0xff00u));
    o[1] = (unsigned short)(((r >> 8) & 0xffu) | ((r & 0xffu) << 8));
    o[2] = (unsigned short)((rh >> 24) | ((rh >> 8) & 0xff00u));
}

// The completeness guard's slow path (k7_pair): one frame traced back serially, 48 steps per
// walk, from location 0 at Tpad -- the reference's own walk (viterbiDecoderButterflyk1.c:
// 200-256), exact whatever the block-parallel chains did; it runs only when a verified chain
// is left unproven.  (Inlined: the walks' asm takes the workspace base in SGPRs.)  cb0, hyb,
// tg, lds_off, gbase: k7_pair's traceback addressing.
template <bool SOFT, bool GS>
__device__ __forceinline__ void tb_serial_frame(uint8_t* ob, int Tpad, uint32_t cb0, bool hyb, int tg, uint32_t lds_off,
                                             uint64_t gbase) {
    uint32_t l = 0;
    for (int tlo = Tpad - 48; tlo >= 0; tlo -= 48) {
        const uint32_t cb = cb0 + 256 * (tlo >> 4);
        uint64_t bits;
        if (GS && hyb) bits = SOFT ? tb_body_dual(cb, l, tlo >= tg, lds_off, gbase) : tb_body8_dual(cb, l, tlo >= tg, lds_off, gbase);
        else bits = SOFT ? tb_body<GS>(cb, l, gbase) : tb_body8<GS>(cb, l, gbase);
        put_bits48(ob, tlo, bits);
    }
}

// One ACS step of the lane's location pair: both candidates, then the packed minimum.
#define VTB_ACS(P, M, vw)                                                                        \
    {                                                                                            \
        uint32_t A, B;                                                                           \
        candidates<P>(M, vw, A, B);                                                              \
        M = pk_min(A, B);                                                                        \
    }

// Survivor word W (of the chunk's three) of this lane: LDS store, or a global store at
// byte offset gvo + 256 W of the wave's workspace (one coalesced 256-B wave store).
template <bool GS>
__device__ __forceinline__ void store_word(uint32_t* dchunk, uint32_t gvo, uint64_t gbase, int W, uint32_t z) {
    if constexpr (GS) {
        if (W == 0) asm volatile("global_store_dword %0, %1, %2" ::"v"(gvo), "v"(z), "s"(gbase) : "memory");
        if (W == 1) asm volatile("global_store_dword %0, %1, %2 offset:256" ::"v"(gvo), "v"(z), "s"(gbase) : "memory");
        if (W == 2) asm volatile("global_store_dword %0, %1, %2 offset:512" ::"v"(gvo), "v"(z), "s"(gbase) : "memory");
    } else {
        dchunk[W * 64] = z;
    }
}

// Decoded bits of steps [tlo, tlo + 48) to global memory at o (byte stores: a stream row
// has no alignment guarantee).
__device__ __forceinline__ void put_bits48_global(uint8_t* o, uint64_t bits) {
    const uint32_t r = __builtin_bitreverse32(uint32_t(bits)), rh = __builtin_bitreverse32(uint32_t(bits >> 32));
    o[0] = uint8_t(r >> 24), o[1] = uint8_t(r >> 16), o[2] = uint8_t(r >> 8), o[3] = uint8_t(r);
    o[4] = uint8_t(rh >> 24), o[5] = uint8_t(rh >> 16);
}

// Two survivor walks of 48 steps each over the survivor words (the location part of tb_body
// / tb_body8 only), their loads issued together: the merge test's walks are latency-bound
// chains of dependent loads, so each lane carries two.  G: global words (saddr form at
// gbase), else LDS words.
template <bool SOFT, bool G = true>
__device__ __forceinline__ void tb_walk48_pair(uint32_t cb, uint32_t& l4a, uint32_t& l4b, uint64_t gbase) {
    uint32_t a = cb | l4a, b = cb | l4b;
    if constexpr (SOFT) {
#pragma unroll
        for (int j = 0; j < 24; j++) {
            const int todd = 47 - 2 * j;
            const int wi = (todd & 15) >> 1, sh = 8 * (wi & 1) + 2 * (wi >> 1);
            uint32_t va, vb;
            if constexpr (G) {
                asm volatile("global_load_ushort %0, %2, %4 offset:%5\n\tglobal_load_ushort %1, %3, %4 offset:%5\n\t"
                             "s_waitcnt vmcnt(0)"
                             : "=&v"(va), "=&v"(vb) : "v"(a), "v"(b), "s"(gbase), "i"((todd >> 4) * 256));
            } else {
                asm volatile("ds_read_u16 %0, %2 offset:%4\n\tds_read_u16 %1, %3 offset:%4\n\ts_waitcnt lgkmcnt(0)"
                             : "=&v"(va), "=&v"(vb) : "v"(a), "v"(b), "i"((todd >> 4) * 256));
            }
            const int pos = 2 + (todd - 1) % 6;
            const uint32_t fa = pos >= sh ? (va << (pos - sh)) : (va >> (sh - pos));
            const uint32_t fb = pos >= sh ? (vb << (pos - sh)) : (vb >> (sh - pos));
            a = (a & ~(3u << pos)) | (fa & (3u << pos));
            b = (b & ~(3u << pos)) | (fb & (3u << pos));
        }
    } else {
#pragma unroll
        for (int k = 5; k >= 0; k--) {
            const int r0 = (8 * k) % 6;
            uint32_t va, vb;
            if constexpr (G) {
                asm volatile("global_load_ubyte %0, %2, %4 offset:%5\n\tglobal_load_ubyte %1, %3, %4 offset:%5\n\t"
                             "s_waitcnt vmcnt(0)"
                             : "=&v"(va), "=&v"(vb) : "v"(a), "v"(b), "s"(gbase), "i"(256 * (k >> 1) + (k & 1)));
            } else {
                asm volatile("ds_read_u8 %0, %2 offset:%4\n\tds_read_u8 %1, %3 offset:%4\n\ts_waitcnt lgkmcnt(0)"
                             : "=&v"(va), "=&v"(vb) : "v"(a), "v"(b), "i"(256 * (k >> 1) + (k & 1)));
            }
            a = (a & ~0xFCu) | (rotl6c(va & 63u, r0) << 2);
            b = (b & ~0xFCu) | (rotl6c(vb & 63u, r0) << 2);
        }
    }
    l4a = a & 0xFCu;
    l4b = b & 0xFCu;
}

// Traceback of one streaming call (vtb_stream_decode).  Frame f of the wave (lanes 32f ..
// 32f + 31) has emitted the decoded bits of steps [0, e_f) before the call.
//  * Not last: walks from all 64 locations at t_end (two per lane) go back 48 steps at a
//    time until they stand on one location (step m).  Every survivor path then passes
//    through it, so no later input can change the path below m: the bits of [e_f, m) are
//    final -- equal to the whole-frame decode's, hence the reference's -- and are emitted.
//    m <= t_end - 48, so the zero tail (the last K - 1 steps of a frame) is never emitted
//    early.
//  * Last: the terminated traceback from location 0 at T (the padding rows keep location 0,
//    as in the frame decoder) emits [e_f, T - 6).
// The emission is the frame decoder's verified block-parallel traceback over [e_f, hi_f),
// 32 blocks per frame, entering at the location known at hi_f.  If the ring no longer holds
// step e_f (no merge within sa.ring steps) the frame is flagged: -1 bits until last.
// !GS: this call's survivor words [t_begin, t_end) are in LDS at r0 (the walks read them
// there, older steps from the ring), and afterwards the ones later calls may still walk --
// from the lower of the two frames' new emission points -- are copied into the ring.
template <bool SOFT, bool GS>
__device__ void stream_traceback(const StreamArgs& sa, uint8_t* out, size_t out_stride, int T, int t_end,
                                 uint64_t gbase, size_t fa, bool has_b, size_t wp, uint32_t r0, int dbg,
                                 uint32_t* hits) {
    const int lane = threadIdx.x, f = lane >> 5, blk = lane & 31;
    uint32_t* st = sa.state + wp * kStreamStateWords;
    const int e0 = int(st[64 + f]);  // this lane's frame
    const uint32_t flags0 = __builtin_amdgcn_readfirstlane(st[66]);
    const bool real = f == 0 || has_b;
    const bool lost = ((flags0 >> f) & 1u) || t_end - e0 > sa.ring;
    auto colb = [&](int tlo) { return uint32_t(2 * f + 256 * ((tlo % sa.ring) >> 4)); };
    auto coll = [&](int tlo) { return uint32_t(r0 + 2 * f + 256 * ((tlo - sa.t_begin) >> 4)); };
    auto tb48 = [&](int tlo, uint32_t& l4) -> uint64_t {
        if (!GS && tlo >= sa.t_begin) {
            if constexpr (SOFT) return tb_body<false>(coll(tlo), l4, 0);
            else return tb_body8<false>(coll(tlo), l4, 0);
        }
        if constexpr (SOFT) return tb_body<true>(colb(tlo), l4, gbase);
        else return tb_body8<true>(colb(tlo), l4, gbase);
    };

    int hi = e0, kfrom = e0;
    uint32_t kloc = 0;
    if (sa.last) {
        hi = t_end, kfrom = T;
    } else {
        // merge test: lane j of frame f walks locations l' = j and j + 32
        uint32_t la = 4u * uint32_t(blk), lb = la + 128u;
        bool walking = !lost && real;
        for (int tlo = t_end - 48; __builtin_amdgcn_readfirstlane(__ballot(walking && tlo >= e0) != 0); tlo -= 48) {
            const bool here = walking && tlo >= e0;
            if (here) {
                if (!GS && tlo >= sa.t_begin) tb_walk48_pair<SOFT, false>(coll(tlo), la, lb, 0);
                else tb_walk48_pair<SOFT, true>(colb(tlo), la, lb, gbase);
            }
            const uint32_t ref = __shfl(la, 32 * f);
            const uint64_t same = __ballot(la == ref && lb == ref);
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
        // verification, as in the frame decoder (the last active block of a frame is known; a
        // chain of 32 blocks needs at most 31 re-walk rounds), with its completeness guard: a
        // frame still unproven after the cap (VTB_DEBUG bit 17: every chain with a walked block) is walked serially
        // from its known location at hi by lane 32f
        uint32_t fin = loc;
        bool fixed = known || !active;
        const bool tbforce = (dbg & kDbgTbCap) != 0;
        if (tbforce) loc_top = ~0u;  // (bit 17: no check passes)
        const int rounds = tbforce ? 0 : 33;
        bool unproven = false;
        for (int round = 0;; round++) {
            const uint32_t sf = __shfl_down(fin, 1);
            const bool ok = fixed || loc_top == sf;
            const uint64_t bad = ~__ballot(ok);
            const uint32_t badf = uint32_t(bad >> (32 * f));
            if (badf == 0) break;
            if (round == rounds) {
                unproven = true;
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
        if (unproven && blk == 0) {
            note_guard(hits);
            uint32_t l = kloc;
            for (int tlo = hi - 48; tlo >= e0; tlo -= 48) put_bits48_global(ob + ((tlo - e0) >> 3), tb48(tlo, l));
        }
    }
    const int bits_out = lost ? -1 : sa.last ? T - 6 - e0 : hi - e0;
    if (real && blk == 0) sa.out_bits[fa + f] = bits_out;
    // new emission state; the streams restart after last
    const uint64_t lostmask = __ballot(lost && real && blk == 0);
    const uint32_t flags = sa.last ? 0u : uint32_t((lostmask & 1u) | ((lostmask >> 32) & 1u) << 1);
    const int e_next = sa.last || lost ? (sa.last ? 0 : e0) : hi;
    if (blk == 0) st[64 + f] = uint32_t(e_next);
    if (lane == 0) st[66] = flags;
    if (!GS && !sa.last) {
        // survivor columns later calls may walk: [max(t_begin, min_f e_next), t_end), 16 steps
        // (one 256-B column of both frames' words) per wave store
        const int eb = has_b ? __shfl(e_next, 32) : __shfl(e_next, 0);
        int lo = min(__shfl(e_next, 0), eb);
        lo = max(lo, sa.t_begin) & ~15;
        extern __shared__ uint4 smem4[];
        const uint32_t* words = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(smem4) + r0);
        uint32_t* ring = reinterpret_cast<uint32_t*>(gbase);
        for (int t = lo; t < t_end; t += 16)
            ring[((t % sa.ring) >> 4) * 64 + lane] = words[((t - sa.t_begin) >> 4) * 64 + lane];
    }
}

// GS = false: survivor words in LDS at [r0, r0 + 16 Tpad).  GS = true: survivor words in a
// global workspace, 16 Tpad bytes per wave at ws + slot * ws_wave (same addressing with
// r0 = 0), for frames whose survivors do not fit in LDS or would cut the occupancy.
// STREAM (with GS): one call of the streaming decoder (vtb_stream_decode): steps
// [sa.t_begin, Tpad = sa.t_end) continue from the metrics in sa.state, survivor words go to a
// ring of sa.ring steps, and the traceback emits the bits that became final (see
// stream_traceback below).
// Per phase: byte offset of the lane's (V, W) column in the table ring: its edge label c
// and R = bit p of its location (the same for every frame pair of the wave).
template <int NB = 2>
__device__ __forceinline__ void column_offsets(const Launch& table, uint32_t (&off)[6], int lane) {
    const int loc = int(lane_of(uint32_t(lane)));
#pragma unroll
    for (int ph = 0; ph < 6; ph++) {
        const int p = 5 - ph;
        off[ph] = 8u * kColN<NB> * (table.symm[rotl6(loc & ~(1 << p), ph)] + (1u << NB) * ((loc >> p) & 1u));
    }
}

// Raw input of chunk 0 of pair wp (load_raw(0) below, for the persistent loop's prefetch of
// the next pair during this pair's traceback).  Issued in asm, waited for by stage_compute.
template <bool SOFT>
__device__ __forceinline__ void load_raw0(const uint8_t* in, size_t in_stride, size_t frames, int T, size_t wp,
                                          uint32_t& ra, uint32_t& rb) {
    const int lane = threadIdx.x, srow = lane < kChunk ? lane : lane - kChunk;
    const size_t fa = 2 * wp, fb = fa + 1 < frames ? fa + 1 : fa;
    const uint64_t baseA = uniform64(reinterpret_cast<uint64_t>(in + fa * in_stride));
    const uint64_t baseB = uniform64(reinterpret_cast<uint64_t>(in + fb * in_stride));
    const uint32_t tc = uint32_t(srow < T ? srow : T - 1);
    if constexpr (SOFT) {
        asm volatile("global_load_ushort %0, %2, %3\n\tglobal_load_ushort %1, %2, %4"
                     : "=&v"(ra), "=&v"(rb) : "v"(2 * tc), "s"(baseA), "s"(baseB));
    } else {
        asm volatile("global_load_ubyte %0, %2, %3\n\tglobal_load_ubyte %1, %2, %4"
                     : "=&v"(ra), "=&v"(rb) : "v"(tc), "s"(baseA), "s"(baseB));
    }
}

// The same for the persistent split kernel: chunk 0 of both halves of frame f (A from step 0,
// B from step t1 - warm).  Plain loads, not asm: the split kernel's convergence branch sits
// between this prefetch and its use, and the register allocator copied asm-loaded registers
// at that join before the asm wait, i.e. while the loads were still in flight (rare,
// timing-dependent wrong frames, found by the round-2 fuzz sweep); for compiler-visible loads
// the compiler places the wait before any use, copies included.
template <bool SOFT>
__device__ __forceinline__ void load_raw0_split(const uint8_t* in, size_t in_stride, int T, int t1, int warm, size_t f,
                                                uint32_t& ra, uint32_t& rb) {
    const int lane = threadIdx.x, srow = lane < kChunk ? lane : lane - kChunk;
    constexpr uint32_t SB = SOFT ? 2 : 1;
    const uint8_t* a = in + f * in_stride;
    const uint8_t* b = a + SB * size_t(t1 - warm);
    const int Tb = T - t1 + warm;
    const uint32_t tc = SB * uint32_t(srow < T ? srow : T - 1), tcb = SB * uint32_t(srow < Tb ? srow : Tb - 1);
    if constexpr (SOFT) {
        ra = *reinterpret_cast<const unsigned short*>(a + tc);
        rb = *reinterpret_cast<const unsigned short*>(b + tcb);
    } else {
        ra = a[tc];
        rb = b[tcb];
    }
}

// SEG (the single-frame latency path, k7_seg_kernel): one frame over the waves of one
// workgroup, 2 segments per wave in the u16 halves.  Segment i runs sg.n steps from
// g_i = i (n - warm); its decisions are the frame's from s_i = g_i + warm on (s_0 = 0) once
// its metrics at s_i equal segment i-1's there up to a constant (checked after the ACS).
struct SegArgs {
    int n = 0;          // ACS steps per segment (multiple of 48)
    int warm = 0;       // warm-up steps of segments 1.. (multiple of 48, < n)
    int G = 0;          // segments in use (<= 2 x waves)
    int seg_bytes = 0;  // LDS bytes per wave: table ring + survivor words (multiple of 256)
    int in_lds = 0;     // LDS byte offset of the staged frame input
    int x_lds = 0;      // LDS byte offset of the metric exchange area
    uint32_t* done = nullptr;  // completion word: 1 decoded, 2 not converged (output not written)
};

// One frame pair (wave-pair index wp: frames 2wp, 2wp + 1); slot = this wave's survivor
// workspace (GS).  pre: chunk 0's raw input is already in (pra, prb); next: the pair this wave
// decodes after this one (its chunk 0 is prefetched into (pra, prb) before the traceback;
// LDS variant only, whose traceback issues no global loads that would wait behind it).

// LIST (global-survivor variant, persistent): pair wp is frames list[1 + 2wp], list[2 + 2wp] of
// table.fail_list (the frames a persistent split launch could not decode split), `frames` = the
// list's count.  SPLIT with LOOP (the persistent split kernel): a split pass that does not
// converge appends the frame to table.fail_list instead of decoding it again in the wave.
// NB: coded bits per step (2; 3 for the hard rate-1/3 pair kernel, k7_lds_n3)
template <bool SOFT, bool GS, bool STREAM, bool LOOP, bool SPLIT, bool SEG = false, bool LIST = false, int NB = 2>
__device__ __forceinline__ void k7_pair(const uint8_t* __restrict__ in, size_t in_stride, uint8_t* __restrict__ out,
                                        size_t out_stride, int T, int L, int Tpad, int tbb, int r0, size_t frames,
                                        int dbg, const Launch& table, uint8_t* __restrict__ ws, size_t ws_wave,
                                        const StreamArgs& sa, size_t wp, size_t slot, bool pre, size_t next,
                                        uint32_t& pra, uint32_t& prb, const uint32_t (&off)[6],
                                        const SegArgs* sgp = nullptr, uint32_t* seg_out = nullptr) {
    static_assert(!SEG || (SPLIT && !GS && !STREAM && !LOOP), "SEG runs the split pair on LDS survivors");
    static_assert(!LIST || (GS && LOOP && !SPLIT && !STREAM), "the list kernel is the persistent global variant");
    static_assert(NB == 2 || (!SOFT && !GS && !STREAM && !SPLIT && !SEG && !LIST), "rate 1/3: the hard LDS pair kernel only");

    constexpr uint32_t Q = SOFT ? 255 : 1;
    constexpr int NL = 1 << NB;                 // edge labels
    constexpr uint32_t INIT = 6 * NB * Q + 1;  // start metric of states != 0: above six steps of the largest branch metric (see header)
    using H = Hist<SOFT, NB>;
    extern __shared__ uint4 smem4[];
    const int wv = SEG ? int(threadIdx.x >> 6) : 0;  // SEG: wave of the workgroup
    uint8_t* smem = reinterpret_cast<uint8_t*>(smem4) + (SEG ? wv * sgp->seg_bytes : 0);
    uint8_t* tab = smem;
    uint32_t* dec = reinterpret_cast<uint32_t*>(smem + r0);
    const int lane = SEG ? int(threadIdx.x & 63) : int(threadIdx.x);
    if (dbg & 16) return;  // (-DVTB_MEASURE builds only) launch cost
    // SPLIT: one frame per wave, its two halves in the u16 halves of the registers: A = steps
    // [0, t1), B = steps [t1 - 96, T) (96 warm-up steps from equal start metrics).  If B's
    // metrics at t1 equal A's up to a constant, B's decisions from t1 on are the frame's
    // (the trellis only compares differences); otherwise the wave decodes the frame again
    // the normal way (pass 1).  Per-pass values:
    // SEG: wave wv runs segments 2wv (half A) and 2wv + 1 (half B; a copy of A if unused)
    const int segA = 2 * wv, segB = SEG && 2 * wv + 1 < sgp->G ? 2 * wv + 1 : 2 * wv;
    const int gA = SEG ? segA * (sgp->n - sgp->warm) : 0, gB = SEG ? segB * (sgp->n - sgp->warm) : 0;
    const int warm = SEG ? sgp->warm : table.split_warm;
    const int t1s = SEG ? sgp->n : SPLIT ? split_t1(T, warm) : 0;
    bool sp = SPLIT;                            // this pass runs split
    int Tb = SEG ? T - gB : SPLIT ? T - t1s + warm : T;  // frame B's steps (local)
    const int Ta = SEG ? T - gA : T;                     // frame A's steps (local)
    size_t fa = SPLIT ? wp : wp * 2, fb = fa + 1;
    bool has_b = !SPLIT && fb < frames;
    if constexpr (LIST) {
        fa = table.fail_list[1 + 2 * wp];
        fb = has_b ? table.fail_list[2 + 2 * wp] : fa;
    }
    const uint64_t gbase = (GS || STREAM) ? uniform64(reinterpret_cast<uint64_t>(ws + slot * ws_wave)) : 0;
    const uint8_t* inA = in + fa * in_stride;
    const uint8_t* inB = SPLIT ? inA + (SOFT ? 2 : 1) * size_t(t1s - warm)
                               : in + (has_b ? fb : fa) * in_stride;  // lone last frame: B decodes a copy

    // Table staging: lane r < 48 builds the row of step 48c + r from the raw input bytes of
    // that step (soft q0 | q1 << 8, hard the byte).  The loads are issued in asm at the start
    // of the chunk before (so no compiler-placed use -- e.g. a zero-extension -- can pull
    // their wait up) and waited for where the chunk is staged, 36+ steps later.
    const int srow = lane < kChunk ? lane : lane - kChunk;  // staging row (lanes 48-63 duplicate 0-15)
    // (wave-uniform frame bases in SGPRs, one 32-bit lane offset; SEG: LDS byte addresses of
    // the staged frame input)
    const uint32_t ldsA = SEG ? uint32_t(sgp->in_lds + (SOFT ? 2 : 1) * gA) : 0u;
    const uint32_t ldsB = SEG ? uint32_t(sgp->in_lds + (SOFT ? 2 : 1) * gB) : 0u;
    uint64_t baseA = uniform64(reinterpret_cast<uint64_t>(inA));
    uint64_t baseB = uniform64(reinterpret_cast<uint64_t>(inB));
    // SPLIT fix-up pass (below): both halves read frame B's rows (frame A's from baseB too,
    // clamped at B's end) and survivor words go to frame B's half only
    bool fixp = false;
    auto load_raw = [&](int c, uint32_t& ra, uint32_t& rb) {
        const int t = c * kChunk + srow;
        const uint32_t tc = uint32_t(t < T ? t : T - 1);
        if constexpr (STREAM) {
            // row r of this call: the carry's held-back rows first, then the new input
            constexpr int SB = SOFT ? 2 : 1;
            const int r = int(tc) - sa.t_begin;
            const uint8_t* pa = r < sa.carry_len ? sa.carry + fa * kStreamCarryStride + SB * r
                                                 : inA + SB * (r - sa.carry_len);
            const uint8_t* pb = r < sa.carry_len ? sa.carry + (has_b ? fb : fa) * kStreamCarryStride + SB * r
                                                 : inB + SB * (r - sa.carry_len);
            if constexpr (SOFT) {
                asm volatile("global_load_ushort %0, %2, off\n\tglobal_load_ushort %1, %3, off"
                             : "=&v"(ra), "=&v"(rb) : "v"(pa), "v"(pb));
            } else {
                asm volatile("global_load_ubyte %0, %2, off\n\tglobal_load_ubyte %1, %3, off"
                             : "=&v"(ra), "=&v"(rb) : "v"(pa), "v"(pb));
            }
        } else if constexpr (SEG) {
            constexpr uint32_t SB = SOFT ? 2 : 1;
            const uint32_t tca = ldsA + SB * uint32_t(t < Ta ? t : Ta - 1), tcb = ldsB + SB * uint32_t(t < Tb ? t : Tb - 1);
            if constexpr (SOFT) {
                asm volatile("ds_read_u16 %0, %2\n\tds_read_u16 %1, %3" : "=&v"(ra), "=&v"(rb) : "v"(tca), "v"(tcb));
            } else {
                asm volatile("ds_read_u8 %0, %2\n\tds_read_u8 %1, %3" : "=&v"(ra), "=&v"(rb) : "v"(tca), "v"(tcb));
            }
        } else if constexpr (SPLIT) {
            constexpr uint32_t SB = SOFT ? 2 : 1;
            const uint32_t tcb = uint32_t(t < Tb ? t : Tb - 1);
            const uint32_t tca = fixp ? tcb : tc;
            if constexpr (SOFT) {
                asm volatile("global_load_ushort %0, %2, %4\n\tglobal_load_ushort %1, %3, %5"
                             : "=&v"(ra), "=&v"(rb) : "v"(SB * tca), "v"(SB * tcb), "s"(baseA), "s"(baseB));
            } else {
                asm volatile("global_load_ubyte %0, %2, %4\n\tglobal_load_ubyte %1, %3, %5"
                             : "=&v"(ra), "=&v"(rb) : "v"(SB * tca), "v"(SB * tcb), "s"(baseA), "s"(baseB));
            }
        } else if constexpr (SOFT) {
            asm volatile("global_load_ushort %0, %2, %3\n\tglobal_load_ushort %1, %2, %4"
                         : "=&v"(ra), "=&v"(rb) : "v"(2 * tc), "s"(baseA), "s"(baseB));
        } else {
            asm volatile("global_load_ubyte %0, %2, %3\n\tglobal_load_ubyte %1, %2, %4"
                         : "=&v"(ra), "=&v"(rb) : "v"(tc), "s"(baseA), "s"(baseB));
        }
    };
    // Row values of the lane's step: e[c] = 4e(c) and et[c] = 4e(c) + tie (tie bit b = t & 1
    // in both halves).  Branch-free, so the compiler can interleave it with ACS steps.
    // first: no survivor stores outstanding.  In the loop (GS) one survivor-word store (step
    // 15 of the chunk) was issued after the loads; vmcnt retires in issue order.
    auto stage_compute = [&](uint32_t ra, uint32_t rb, uint32_t (&e)[NL], uint32_t (&et)[NL], bool first) {
        if constexpr (SEG) {
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ra), "+v"(rb));
        } else if (GS && !first) {
            asm volatile("s_waitcnt vmcnt(1)" : "+v"(ra), "+v"(rb));
        } else {
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(ra), "+v"(rb));
        }
        // packed [frame A, frame B] received values of coded bits 0 and 1, times four
        uint32_t q0 = __builtin_amdgcn_perm(rb, ra, 0x0C040C00u);
        uint32_t q1 = __builtin_amdgcn_perm(rb, ra, 0x0C050C01u), q2 = 0;
        if constexpr (!SOFT) {
            q1 = (q0 >> 1) & kR1;
            if constexpr (NB == 3) q2 = (q0 >> 2) & kR1;  // (bits above coded bit NB-1 are ignored)
            q0 &= kR1;
        }
        q0 <<= H::HB;
        q1 <<= H::HB;
        // 4e of labels 0..3 (bit 0 of a label <-> coded bit 0); halves never borrow
        constexpr uint32_t QQ = H::SC * Q * kR1;
        e[0] = q0 + q1, e[1] = (QQ + q1) - q0, e[2] = 2 * QQ - e[1], e[3] = 2 * QQ - e[0];
        if constexpr (NB == 3) {
            // labels 4..7 set coded bit 2: e(c) = e(c & 3) + (c & 4 ? Q - q2 : q2); e(~c) = 3Q - e(c)
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
    // Column k = c + 4R of the ring holds (V, W) = (4e(c) + R tie, 4e(~c) + (1 - R) tie).
    // (V, W) of a slot from two unrelated VGPRs by ds_write2_b32 (a ds_write_b64 would need
    // them in a register pair: 8 moves per chunk); three bases keep offsets below 256 dwords.
    // (LDS byte addresses: the ring starts at LDS address 0, SEG: at this wave's region)
    const uint32_t wbase0 = uint32_t(SEG ? wv * sgp->seg_bytes : 0) + 8u * uint32_t(ring_slot(srow)), wbase1 = wbase0 + 24u * kCol, wbase2 = wbase0 + 48u * kCol;
    // PADCHK: the chunk may hold padding rows (only the chunk containing step T; the ACS
    // loop is split so that the check stays out of its other iterations).
    auto stage_write = [&](int c, const uint32_t (&e)[NL], const uint32_t (&et)[NL], auto padchk, int half = 0) {
        constexpr bool PADCHK = decltype(padchk)::value;
        if constexpr (NB == 3) {
            // rows [24 half, 24 half + 24) of chunk c into the 24-row ring (slot = row mod 24);
            // 16 columns k = c + 8R: (V, W) = (4e(c) + R tie, 4e(7 - c) + (1 - R) tie), the
            // complement's metric 3Q - e(c) as the reference's n - e (viterbiDecoderButterflyk1.c:104-107).
            // (V, W) by ds_write2_b32 from two unrelated VGPRs, five columns per base address
            // (offsets below 256 dwords)
            constexpr int KC = kColN<3>;
            if (srow / 24 == half) {
                const uint32_t b0 = uint32_t(lds_addr(tab)) + 8u * uint32_t(srow % 24);
                const uint32_t bs[4] = {b0, b0 + 40u * KC, b0 + 80u * KC, b0 + 120u * KC};
#define VTB_W3(k, v, w)                                                                                 \
    asm volatile("ds_write2_b32 %0, %1, %2 offset0:%3 offset1:%4" ::"v"(bs[(k) / 5]), "v"(v), "v"(w),   \
                 "i"(2 * KC * ((k) % 5)), "i"(2 * KC * ((k) % 5) + 1) : "memory");
                VTB_W3(0, e[0], et[7]) VTB_W3(1, e[1], et[6]) VTB_W3(2, e[2], et[5]) VTB_W3(3, e[3], et[4])
                VTB_W3(4, e[4], et[3]) VTB_W3(5, e[5], et[2]) VTB_W3(6, e[6], et[1]) VTB_W3(7, e[7], et[0])
                VTB_W3(8, et[0], e[7]) VTB_W3(9, et[1], e[6]) VTB_W3(10, et[2], e[5]) VTB_W3(11, et[3], e[4])
                VTB_W3(12, et[4], e[3]) VTB_W3(13, et[5], e[2]) VTB_W3(14, et[6], e[1]) VTB_W3(15, et[7], e[0])
#undef VTB_W3
                if (PADCHK && c * kChunk + srow >= T) {  // padding rows: own-keeping (below), rare
                    uint2* col = reinterpret_cast<uint2*>(tab) + (srow % 24);  // column k at col[KC * k]
                    constexpr uint32_t PADW = H::SC * INIT * kR1;
                    const uint32_t tie = et[0] - e[0];
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        col[k * KC] = make_uint2(0u, PADW + tie);
                        col[(8 + k) * KC] = make_uint2(tie, PADW);
                    }
                }
            }
            asm volatile("" ::: "memory");  // (ordered against the table reads)
            return;
        }
        uint2* col = reinterpret_cast<uint2*>(tab) + ring_slot(srow);  // column k at col[kCol * k]
#define VTB_W2(base, k, v, w)                                                                         \
    asm volatile("ds_write2_b32 %0, %1, %2 offset0:%3 offset1:%4" ::"v"(base), "v"(v), "v"(w),        \
                 "i"(2 * kCol * ((k) % 3)), "i"(2 * kCol * ((k) % 3) + 1) : "memory");
        VTB_W2(wbase0, 0, e[0], et[3]) VTB_W2(wbase0, 1, e[1], et[2]) VTB_W2(wbase0, 2, e[2], et[1])
        VTB_W2(wbase1, 3, e[3], et[0]) VTB_W2(wbase1, 4, et[0], e[3]) VTB_W2(wbase1, 5, et[1], e[2])
        VTB_W2(wbase2, 6, et[2], e[1]) VTB_W2(wbase2, 7, et[3], e[0])
#undef VTB_W2
        if (SEG) {
            // either half may hold padding rows (steps >= Ta in A, >= Tb in B): own-keeping rows
            // there, as below
            const int tr = c * kChunk + srow;
            if (PADCHK && (tr >= Ta || tr >= Tb)) {
                constexpr uint32_t PADW = H::SC * INIT * kR1;
                const uint32_t keep = (tr >= Ta ? 0u : 0xFFFFu) | (tr >= Tb ? 0u : 0xFFFF0000u);
                const uint32_t tie = et[0] - e[0];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    col[k * kCol] = make_uint2(e[k] & keep, (et[3 - k] & keep) | ((PADW + tie) & ~keep));
                    col[(4 + k) * kCol] = make_uint2((et[k] & keep) | (tie & ~keep), (e[3 - k] & keep) | (PADW & ~keep));
                }
            }
        } else if (SPLIT && sp) {
            // split pass: padding rows of frame B only (step >= Tb); frame A's half is real
            if (PADCHK && c * kChunk + srow >= Tb) {
                constexpr uint32_t PADW = H::SC * INIT * kR1, LO = 0xFFFFu, HI = 0xFFFF0000u;
                const uint32_t tie = et[0] - e[0];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    col[k * kCol] = make_uint2(e[k] & LO, (et[3 - k] & LO) | ((PADW + tie) & HI));
                    col[(4 + k) * kCol] = make_uint2((et[k] & LO) | (tie & HI), (e[3 - k] & LO) | (PADW & HI));
                }
            }
        } else if (PADCHK && (c + 1) * kChunk > T && c * kChunk + srow >= T) {  // padding rows
            constexpr uint32_t PADW = H::SC * INIT * kR1;
            const uint32_t tie = et[0] - e[0];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                col[k * kCol] = make_uint2(0u, PADW + tie);
                col[(4 + k) * kCol] = make_uint2(tie, PADW);
            }
        }
    };
    // staged row values of the next chunk (computed at group 3, written at group 8 - AH; NB = 3:
    // its second half at group 1 of that chunk)
    uint32_t se[NL], set[NL];
    auto stage = [&](int c, uint32_t ra, uint32_t rb) {
        if constexpr (NB == 3) {  // the chunk's first half now, its second at its group 1 (from se/set)
            stage_compute(ra, rb, se, set, true);
            stage_write(c, se, set, std::true_type{}, 0);
            return;
        }
        uint32_t e[NL], et[NL];
        stage_compute(ra, rb, e, et, true);
        stage_write(c, e, et, std::true_type{});
    };

    for (int pass = 0; pass < (SPLIT ? 2 : 1); pass++) {
    if (SPLIT && pass == 1) {  // the split halves did not converge: the frame the normal way
        sp = false;
        Tb = T;
        baseB = baseA;
        __syncthreads();
    }
    uint32_t M = (lane == 0) ? H::BIAS * kR1 : (H::BIAS + H::SC * INIT) * kR1;
    if (SPLIT && sp) M = (M & 0xFFFFu) | (H::BIAS << 16);  // frame B's half: equal start metrics
    if (SEG && segA > 0) M = H::BIAS * kR1;                 // SEG: half A of waves 1.. too
    uint32_t msave = 0;                                      // (SPLIT) frame B's metrics at t1
    // first step of this launch: 0, or (streaming) where the previous call stopped
    const int tbeg = STREAM ? sa.t_begin : 0;
    // GS (frames): survivor words of steps [0, tg) in the global workspace, of [tg, Tpad) in
    // LDS at r0 (the newest steps: the traceback's first walks read LDS)
    const int tg = GS && !STREAM ? table.gs_steps : (1 << 30);
    const int lds_t0 = (STREAM && !GS) ? tbeg : GS ? tg : 0;  // step of the first LDS word column
    if constexpr (STREAM) {
        if (tbeg > 0) M = sa.state[wp * kStreamStateWords + lane];
    }
    uint32_t ra = 0, rb = 0;
    if (!STREAM || Tpad > tbeg) {  // (a streaming call may have no new step)
        if (LOOP && pre) {
            ra = pra, rb = prb;
        } else {
            load_raw(tbeg / kChunk, ra, rb);
        }
        stage(tbeg / kChunk, ra, rb);
    }
    // software pipeline: the table pairs of group G+3 are read while group G computes, into
    // the slot of a four-group register ring (8 groups per chunk: no copies at the loop edge)
    uint2 buf[4][6];
    constexpr int AH = 2;  // groups read ahead
    auto prime = [&]() {  // the first AH groups' table pairs of a freshly staged chunk
#pragma unroll
        for (int g = 0; g < AH; g++)
#pragma unroll
            for (int k = 0; k < 6; k++) buf[g][k] = *reinterpret_cast<const uint2*>(tab + off[k] + 8 * ring_slot(6 * g + k));
    };
    prime();
    // LDS byte addresses of the lane's six table columns, held in VGPRs across the chunks (the
    // compiler otherwise re-adds the ring base to each column offset in every chunk: 6 VALU per
    // chunk; round 3 A/B -0.3 % soft, -0.4 % hard per 4,096-frame launch)
    uint32_t tad[6];
#pragma unroll
    for (int k = 0; k < 6; k++) {
        tad[k] = lds_addr(tab) + off[k];
        asm volatile("" : "+v"(tad[k]));
    }
    const uint32_t widx = rev6(lane_of(lane));  // survivor word slot of this lane's location

    uint32_t dd = 0, m_prev = 0, pw[4] = {0, 0, 0, 0};
    const int tacs = (dbg & 2) ? 0 : (SPLIT && sp ? t1s : Tpad);
    // One 48-step chunk of the ACS (fully unrolled); PADTAG: this chunk stages the chunk that
    // holds step T (padding rows possible).
    // gtag: this chunk's survivor words go to the global workspace (else LDS)
    // lasttag: the frame's last chunk, which may stop after ng_last of its 8 groups (the steps
    // past T up to the chunk's end need no ACS: their survivor words are written as own-keeping
    // patterns afterwards, pad_words) and stages nothing
    int ng_last = 8;
    auto acs_chunk = [&](const int t0, auto padtag, auto gtag, auto lasttag) __attribute__((always_inline)) {
        constexpr bool GSC = decltype(gtag)::value;
        constexpr bool LASTC = decltype(lasttag)::value;
        const int c0 = t0 / kChunk;
        LdsCol ap[6];
#pragma unroll
        for (int k = 0; k < 6; k++) ap[k].a = tad[k];
        uint32_t* dchunk = dec + ((t0 - lds_t0) >> 4) * 64 + widx;  // (LDS words; stream: this call's)
        // GS: byte offset of the lane's words (streaming: position in the survivor ring)
        const uint32_t gvo = 4u * (((STREAM ? t0 % sa.ring : t0) >> 4) * 64 + widx);

// Renormalisation: reference = location 0 (lane 0) at a step whose history is clear, the
// subtraction folded into the history clear (soft: every 12 steps; hard: once per chunk).
#define VTB_RENORM_READ(I) (SOFT ? ((I) % kRenormSoft) == kRenormSoft - 2 : (I) == 40)
#define VTB_RENORM_APPLY(I) (SOFT ? ((I) % kRenormSoft) == kRenormSoft - 1 : (I) == 47)
// (SPLIT fix-up pass: frame B's 16-bit half of the word only, frame A's stays)
#define VTB_STORE(GSC_, W_, z_)                                                                   \
    {                                                                                            \
        if (SPLIT && fixp) reinterpret_cast<uint16_t*>(dchunk + (W_) * 64)[1] = uint16_t((z_) >> 16); \
        else store_word<GSC_>(dchunk, gvo, gbase, (W_), (z_));                                   \
    }
#define VTB_CLR(x) ((x) & ~H::MASK)
#define VTB_STEP(I, PH)                                                                          \
    {                                                                                            \
        if (VTB_RENORM_READ(I)) {                                                                \
            const uint32_t ref = __builtin_amdgcn_readfirstlane(M);                              \
            asm("s_sub_u32 %0, %1, %2" : "=s"(dd) : "s"(H::BIAS * kR1), "s"(ref) : "scc");       \
        }                                                                                        \
        VTB_ACS(5 - (PH), M, cur[PH])                                                            \
        if (SOFT && ((I) & 1)) {                                                                 \
            /* window (I) >> 1 & 7 of the word: history bytes of two windows by one v_perm */    \
            const int w = ((I) & 15) >> 1;                                                       \
            if (w & 1) pw[w >> 1] = __builtin_amdgcn_perm(M, m_prev, 0x06020400u);                \
            else m_prev = M;                                                                     \
            M = VTB_RENORM_APPLY(I) ? (VTB_CLR(M) + dd) : VTB_CLR(M);                            \
            if (((I) & 15) == 15) {                                                              \
                /* bits 2j..2j+1 of byte (w & 1): window w = 2j + (w & 1) */                     \
                uint32_t z = bfi_op(0x03030303u, pw[0], pw[1] << 2);                             \
                z = bfi_op(0x0F0F0F0Fu, z, pw[2] << 4);                                          \
                z = bfi_op(0x3F3F3F3Fu, z, pw[3] << 6);                                          \
                VTB_STORE(GSC, (I) >> 4, z);                                                     \
            }                                                                                    \
        }                                                                                        \
        if (!SOFT && ((I) & 7) == 7) {                                                           \
            /* octet history bytes: [A oct 0, A oct 1, B oct 0, B oct 1] per 16 steps */         \
            if (((I) & 15) == 7) {                                                               \
                m_prev = M;                                                                      \
            } else {                                                                             \
                const uint32_t z = __builtin_amdgcn_perm(M, m_prev, 0x06020400u);                \
                VTB_STORE(GSC, (I) >> 4, z);                                                     \
            }                                                                                    \
            M = VTB_RENORM_APPLY(I) ? (VTB_CLR(M) + dd) : VTB_CLR(M);                            \
        }                                                                                        \
    }
#define VTB_GROUP(G)                                                                              \
    if (!LASTC || (G) < ng_last) {                                                                \
        if ((G) == 0 && !LASTC) load_raw(c0 + 1, ra, rb);                                         \
        if ((G) == 3 && !LASTC) stage_compute(ra, rb, se, set, !GSC);            \
        if ((G) == 8 - AH && !LASTC) { /* all rows of this chunk are in registers */ \
            stage_write(c0 + 1, se, set, padtag);                                                 \
        }                                                                                         \
        if (NB == 3 && (G) == 1) { /* rows 24-47 of this chunk: rows 0-23 are read */ \
            stage_write(c0, se, set, std::true_type{}, 1);                                       \
        }                                                                                         \
        uint2* cur = buf[(G) & 3];                                                                \
        /* table reads AH groups ahead, issued after the two permlane steps */                     \
        VTB_STEP(6 * (G) + 0, 0) VTB_STEP(6 * (G) + 1, 1)                                         \
        VTB_RD(G, 0) VTB_RD(G, 1) VTB_RD(G, 2) VTB_RD(G, 3) VTB_RD(G, 4) VTB_RD(G, 5)             \
        VTB_STEP(6 * (G) + 2, 2) VTB_STEP(6 * (G) + 3, 3)                                         \
        VTB_STEP(6 * (G) + 4, 4) VTB_STEP(6 * (G) + 5, 5)                                         \
    }
// Even groups read the next two groups' pairs of one phase (rows 6 apart in one column of
// the ring): one ds_read2_b64 per phase and group pair, half the LDS read instructions of
// one ds_read_b64 per step (measured 2% faster).
#define VTB_RD(G, k)                                                                              \
    if (((G) & 1) == 0) {                                                                         \
        buf[((G) + 2) & 3][k] = ap[k][(6 * ((G) + 2) + (k)) % kChunk % kRowsN<NB>];               \
        buf[((G) + 3) & 3][k] = ap[k][(6 * ((G) + 3) + (k)) % kChunk % kRowsN<NB>];               \
    }
        VTB_GROUP(0) VTB_GROUP(1) VTB_GROUP(2) VTB_GROUP(3) VTB_GROUP(4) VTB_GROUP(5) VTB_GROUP(6) VTB_GROUP(7)
#undef VTB_GROUP
#undef VTB_STEP
#undef VTB_STORE
#undef VTB_RENORM_READ
#undef VTB_RENORM_APPLY
#undef VTB_RD
    };
    // Wave balance.  The two waves of a SIMD get VALU issue by priority, then
    // age: at equal priority the first-dispatched wave (HW_ID wave slot 0) ran its ACS 6.6 us
    // ahead of its partner, which then ran alone at the single-wave rate (tools/tstamp.py,
    // 4,096 frames: ACS ends at 22.0 / 28.5 us).  The second-dispatched wave takes priority 1
    // for the first kPrioPct % of its chunks, so both finish together (ends 27.2 / 27.4 us,
    // launch -3.5 %).  Scheduling only: decisions are unchanged.
    uint32_t hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    const bool second = (hwid & 1u) != 0;
    const int hi_chunks = kPrioPct * ((tacs - tbeg) / kChunk) / 100;
    auto prio = [&](int t0) {
        if (second && (t0 - tbeg) / kChunk < hi_chunks) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
    };
    // one chunk, its survivor words to the global workspace (GS, steps before tg) or to LDS
    auto run_chunk = [&](const int t0, auto padtag, auto lasttag) __attribute__((always_inline)) {
        if constexpr (GS) {
            if (t0 < tg) acs_chunk(t0, padtag, std::true_type{}, lasttag);
            else acs_chunk(t0, padtag, std::false_type{}, lasttag);
        } else {
            acs_chunk(t0, padtag, std::false_type{}, lasttag);
        }
    };
    // Survivor words of the last chunk's steps [t0 + n_end, t0 + 48) (n_end = 24, all past T):
    // every location keeps its own predecessor there (what the padding rows make the ACS
    // decide), so a decision is the location's own bit p = 5 - (t mod 6), i.e. bit t mod 6 of
    // l' = widx, and a walk from location 0 at Tpad stays at location 0 down to T.  The word
    // with steps [16, 24) computed keeps those (soft: windows 0-3 in pw[0..1]; hard: octet 0 in
    // m_prev) and takes the pattern for the rest.
    auto pad_words = [&](const int t0, auto gtag) __attribute__((always_inline)) {
        constexpr bool GSC = decltype(gtag)::value;
        uint32_t* dchunk = dec + ((t0 - lds_t0) >> 4) * 64 + widx;
        const uint32_t gvo = 4u * ((t0 >> 4) * 64 + widx);
        auto lbit = [&](int t) { return (widx >> (t % 6)) & 1u; };
        auto pattern = [&](int s16) {  // one frame's 16-bit half of the word of steps [s16, s16 + 16)
            uint32_t p = 0;
            if constexpr (SOFT) {
#pragma unroll
                for (int w = 0; w < 8; w++)
                    p |= (lbit(s16 + 2 * w) | (lbit(s16 + 2 * w + 1) << 1)) << (8 * (w & 1) + 2 * (w >> 1));
            } else {
#pragma unroll
                for (int b = 0; b < 16; b++) p |= lbit(s16 + b) << b;  // octets 0, 1 in bytes 0, 1
            }
            return p * kR1;  // both frames
        };
        const uint32_t p1 = pattern(t0 + 16), p2 = pattern(t0 + 32);
        uint32_t z1;
        if constexpr (SOFT) {
            const uint32_t z = bfi_op(0x03030303u, pw[0], pw[1] << 2);
            z1 = bfi_op(0x0F0F0F0Fu, z, p1);  // windows 0-3 computed, 4-7 the pattern
        } else {
            z1 = __builtin_amdgcn_perm(p1, m_prev, 0x07020500u);  // [A oct 0, A oct 1 (pattern), B oct 0, B oct 1]
        }
        store_word<GSC>(dchunk, gvo, gbase, 1, z1);
        store_word<GSC>(dchunk, gvo, gbase, 2, p2);
    };
    // SPLIT: frame B's metrics after its steps [0, warm + 48 j), j = 1..kFix (the fix-up pass's
    // comparison points)
    uint32_t ck[kFix] = {};
    if constexpr (SPLIT) {
        for (int t0 = 0; t0 < tacs; t0 += kChunk) {
            prio(t0);
            run_chunk(t0, std::true_type{}, std::false_type{});  // (frame B's padding may start in any chunk)
            if (t0 == warm - kChunk) msave = M;
#pragma unroll
            for (int j = 0; j < kFix; j++)
                if (t0 == warm + kChunk * j) ck[j] = M;
        }
    } else {
        // chunks in order; only the one before the last stages padding rows
        const int tstage = tacs - 2 * kChunk;  // the chunk that stages the last one
        int t0 = tbeg;
        for (; t0 < tstage; t0 += kChunk) {
            prio(t0);
            run_chunk(t0, std::false_type{}, std::false_type{});
        }
        if (t0 == tstage) {
            prio(t0);
            run_chunk(t0, std::true_type{}, std::false_type{});
            t0 += kChunk;
        }
        if (t0 < tacs) {
            // frames (not streams) whose last chunk holds at most 24 real steps run only its first
            // 24 (4 groups) and write the rest of its survivor words as patterns (pad_words)
            if (!STREAM && T - t0 <= 24 && !(dbg & 8192)) {  // VTB_DEBUG bit 13: full last chunk (measurement)
                ng_last = 4;
                run_chunk(t0, std::false_type{}, std::true_type{});
                if constexpr (GS) {
                    if (t0 < tg) pad_words(t0, std::true_type{});
                    else pad_words(t0, std::false_type{});
                } else {
                    pad_words(t0, std::false_type{});
                }
            } else {
                run_chunk(t0, std::false_type{}, std::false_type{});
            }
        }
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (GS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // survivor words written
    __syncthreads();
    if constexpr (SEG) {  // the caller checks the segments and traces back
        seg_out[0] = M, seg_out[1] = msave;
        return;
    }
    tstamp(table, 1);
    if constexpr (STREAM) {
        if (!sa.last) sa.state[wp * kStreamStateWords + lane] = M;
        stream_traceback<SOFT, GS>(sa, out, out_stride, T, Tpad, gbase, fa, has_b, wp, uint32_t(r0), dbg, table.guard_hits);
        return;
    }
    const size_t units = SPLIT ? frames : (frames + 1) / 2;  // (persistent loop: pairs, or split frames)
    // the next unit's chunk-0 input, waited for after this unit's traceback (split pass: after
    // the fix-up, whose own loads and waits would otherwise queue behind it)
    auto prefetch_next = [&]() {
        if (LOOP && !GS && next < units) {
            if constexpr (SPLIT) load_raw0_split<SOFT>(in, in_stride, T, t1s, warm, next, pra, prb);
            else load_raw0<SOFT>(in, in_stride, frames, T, next, pra, prb);
        }
    };
    if (!(SPLIT && sp)) prefetch_next();
    if (SPLIT && sp) {
        // frame A's metrics at t1 against frame B's at its step 96 (= t1), histories masked:
        // equal up to a constant -> B's decisions from t1 on are the frame's
        constexpr uint32_t KEEP = 0xFFFFu & ~(H::SC - 1);
        const uint32_t a = M & KEEP, b = (msave >> 16) & KEEP;
        const uint32_t a0 = __builtin_amdgcn_readfirstlane(a), b0 = __builtin_amdgcn_readfirstlane(b);
        bool conv = __ballot(((a - a0) & 0xFFFFu) == ((b - b0) & 0xFFFFu)) == ~0ull;
        // VTB_DEBUG bit 15 (testing): the fix-up runs on every split frame, converged or not;
        // bit 16 (testing): its checks never match, so every fix-up runs kFix chunks and the
        // frame then takes the slow path.  Output must stay exact under both.
        const bool fix_all = (dbg & 32768) != 0, fix_never = (dbg & 65536) != 0;
        if ((!conv || fix_all) && !SEG && !(dbg & 16384)) {  // VTB_DEBUG bit 14: no fix-up (measurement)
            conv = false;
            // Fix-up: frame B's half re-runs its steps from t1 on, now from frame A's metrics
            // at t1 (the frame's true metrics there), writing its survivor words over B's, one
            // chunk at a time until its metric vector equals B's own at the same step up to a
            // constant (ck): from there on B's decisions were the frame's already.  Decisions
            // are exact either way; only a fix-up that has not converged after kFix chunks
            // falls back to the slow path below.
            fixp = true;
            const uint64_t baseA0 = baseA;
            baseA = baseB;
            M = (M & 0xFFFFu) * kR1;  // frame A's metrics at t1 in both halves
            uint32_t fa_, fb_;
            load_raw(warm / kChunk, fa_, fb_);
            stage(warm / kChunk, fa_, fb_);
            prime();
#pragma unroll 1
            for (int j = 0; j < kFix && !conv; j++) {
                const int t0 = warm + kChunk * j;
                if (t0 + kChunk > t1s) break;  // past frame B's run: nothing left to compare
                run_chunk(t0, std::true_type{}, std::false_type{});
                uint32_t ckj = ck[0];  // (ck[j] by selects: a dynamic index would put ck in scratch)
#pragma unroll
                for (int k = 1; k < kFix; k++) ckj = j == k ? ck[k] : ckj;
                const uint32_t fm = (M >> 16) & KEEP, bm = (ckj >> 16) & KEEP;
                const uint32_t f0 = __builtin_amdgcn_readfirstlane(fm), bm0 = __builtin_amdgcn_readfirstlane(bm);
                conv = __ballot(((fm - f0) & 0xFFFFu) == ((bm - bm0) & 0xFFFFu)) == ~0ull && !fix_never;
            }
            fixp = false;
            baseA = baseA0;  // (the slow path below decodes frame A's rows again)
            __syncthreads();  // the rewritten words before the traceback reads them
        }
        prefetch_next();
        if (!conv) {
            if constexpr (LOOP) {
                // persistent split kernel: the list kernel decodes this frame afterwards
                if (lane == 0) {
                    const uint32_t i = atomicAdd(table.fail_list, 1u);
                    table.fail_list[1 + i] = uint32_t(fa);
                }
                if (!GS && next < units) asm volatile("s_waitcnt vmcnt(0)" : "+v"(pra), "+v"(prb));
                return;
            } else {
                continue;
            }
        }
    }
    if (dbg & 1) return;

    // ---------------- traceback: verified block-parallel chains ----------------
    const int f = lane >> 5, blk = lane & 31;
    const uint32_t cb0 = uint32_t((GS ? 0 : r0) + 2 * f);  // this frame's 16-bit half of the word columns
    uint8_t* ob = tab + f * 4 * tbb;                                      // decoded bytes, index t/8
    // (SPLIT pass: 48-step blocks over [0, t1) per half; frame A's last block (lane nA - 1)
    // enters at frame B's location at its step 96 (lane 34's exit), frame B's blocks 0 and 1
    // are warm-up only)
    const int tbp = (SPLIT && sp) ? kChunk : tbb, nA = t1s / kChunk;
    const int top = (blk + 1) * tbp;
    const int start_full = top + kTbWarm;
    const int start = min(start_full, (SPLIT && sp) ? t1s : Tpad);
    // walk starts on the known path (location 0 at and past T)
    const int kB0 = 32 + warm / kChunk;  // frame B's first decoded block (lane)
    const bool known = (SPLIT && sp) ? (f == 1 && start >= Tb) || (f == 0 && blk >= nA) || (f == 1 && lane < kB0)
                                     : start >= T;
    const int nbody = (dbg & 8) ? 1 : (kTbWarm + tbp) / 48;  // dbg bit 3: warm-up walk only
    // GS with LDS words for the newest steps: per block (lane) LDS or global, both walked at once
    const bool hyb = GS && tg < Tpad;
    const uint32_t lds_off = uint32_t(r0) - 16u * uint32_t(GS ? tg : 0);  // LDS byte of word offset a
    auto tb48 = [&](uint32_t cb, uint32_t& l4) {
        if constexpr (SOFT) return tb_body<GS>(cb, l4, gbase);
        else return tb_body8<GS>(cb, l4, gbase);
    };
    auto tb48t = [&](int tlo, uint32_t& l4) -> uint64_t {  // the 48 steps at tlo
        const uint32_t cb = cb0 + 256 * (tlo >> 4);
        if (GS && hyb) {
            if constexpr (SOFT) return tb_body_dual(cb, l4, tlo >= tg, lds_off, gbase);
            else return tb_body8_dual(cb, l4, tlo >= tg, lds_off, gbase);
        }
        return tb48(cb, l4);
    };
    // survivor location as 4 l'.  Walks that start from an unknown location start at
    // lane-dependent ones (any start is exact: the walk is verified), so that the first reads of
    // up to 44 blocks do not all hit one LDS bank (round 3: soft -0.3 % per 4,096-frame launch,
    // profiles/r03/ab_tbspread.txt)
    uint32_t loc = known ? 0u : 4u * ((uint32_t(lane) * 37u) & 63u), loc_top = 0;
    for (int g = 0; g < nbody; g++) {
        const int tlo = start_full - 48 * (g + 1);
        if (g == kTbWarm / 48) loc_top = loc;
        if (tlo < start) {  // lane's walk has begun (start is a multiple of 48)
            const uint64_t bits = tb48t(tlo, loc);
            if (g >= kTbWarm / 48) put_bits48(ob, tlo, bits);
        }
    }
    // Verification, all blocks at once: a block is right if it entered on its successor's
    // exit location and that successor is proven, i.e. every later block of the frame checks
    // (the last blocks are known).  Failed blocks whose successor is proven re-walk from it;
    // a re-walk can change their exit, so the checks repeat until every block is proven --
    // one round when all blocks merged within the warm-up.
    // Rounds: every round proves at least the last unproven block of each chain (its successor
    // is proven; the chain's last block is known), so a chain of n blocks needs at most n - 1
    // re-walk rounds plus the check that sees no failure.  Unsplit frames are chains of at most
    // 32 blocks; the split pass chains frame A's nA <= 32 blocks and frame B's blocks kB0..31
    // (kB0 = 32 + warm / 48 >= 33 for warm >= 48) into one chain of nA + 64 - kB0 <= 63.  (Round
    // 3 capped this loop at 33 rounds for both: a pure-noise split frame kept by the in-wave
    // fix-up left frame A's first blocks unverified -- fuzz case 1366, 6 wrong bits at 85-93,
    // DESIGN.md 4.2b.)
    // Completeness guard (round 5): the loop's last check runs after the cap's re-walks, and a
    // block still unproven there never reaches the output -- the split pass sends its frame to
    // the slow path (the unsplit pass, or the list kernel), an unsplit frame is traced back
    // serially from location 0 at Tpad (the reference's own walk, viterbiDecoderButterflyk1.c:
    // 200-256).  VTB_DEBUG bit 17 sends every chain with a walked block there (no check, no re-walk), to exercise both.
    uint32_t fin = loc;  // survivor's location at step blk * tbb
    bool fixed = known || (dbg & 4);  // dbg bit 2 (measurement builds only): skip verification
    const bool tbforce = (dbg & kDbgTbCap) != 0;
    if (tbforce) loc_top = ~0u;  // (bit 17: no check passes)
    const int rounds = tbforce ? 0 : (SPLIT && sp) ? 65 : 33;
    uint64_t unproven = 0;
    for (int round = 0;; round++) {
        // successor's exit (lane 31, frame A's last block, is known)
        const uint32_t sf = (SPLIT && sp) ? __shfl(fin, lane == nA - 1 ? kB0 : (lane + 1) & 63) : __shfl_down(fin, 1);
        const bool ok = fixed || loc_top == sf;
        const uint64_t bad = ~__ballot(ok);
        if (bad == 0) break;
        if (round == rounds) {
            unproven = bad;
            break;
        }
        bool succ_proven;
        if (SPLIT && sp) {  // one chain: frame A's blocks 0..nA-1, then frame B's blocks kB0-32..31
            const uint64_t cm = (bad & ((uint64_t(1) << nA) - 1)) | ((bad >> kB0) << nA);
            const int pos = f == 0 ? blk : nA + lane - kB0;
            succ_proven = (cm >> (pos + 1)) == 0;
        } else {
            const uint32_t badf = uint32_t(bad >> (32 * f));  // this frame's failed blocks
            succ_proven = (uint64_t(badf) >> (blk + 1)) == 0;
        }
        if (!ok && succ_proven) {
            loc = sf;
            for (int g = kTbWarm / 48; g < nbody; g++) {
                const int tlo = start_full - 48 * (g + 1);
                put_bits48(ob, tlo, tb48t(tlo, loc));
            }
            fin = loc;
            fixed = true;
        }
    }
    if (unproven) {
        if (lane == 0) note_guard(table.guard_hits);
        if (SPLIT && sp) {
            if constexpr (LOOP) {  // the list kernel decodes the frame afterwards
                if (lane == 0) {
                    const uint32_t i = atomicAdd(table.fail_list, 1u);
                    table.fail_list[1 + i] = uint32_t(fa);
                }
                if (!GS && next < units) asm volatile("s_waitcnt vmcnt(0)" : "+v"(pra), "+v"(prb));
                return;
            } else {
                continue;  // pass 1: the frame unsplit
            }
        }
        // an unsplit frame with an unproven block: lane 32f walks frame f whole
        // (f = 1 without a real frame B decodes a copy of A that is never written out: not walked)
        if (blk == 0 && (f == 0 || has_b) && uint32_t(unproven >> (32 * f)) != 0)
            tb_serial_frame<SOFT, GS>(ob, Tpad, cb0, hyb, tg, lds_off, gbase);
    }
    __syncthreads();
    tstamp(table, 2);

    // copy the decoded bytes out (bits past L are zero: the survivor ends in state 0)
    const int nbytes = (L + 7) >> 3;
    const bool words = ((nbytes | out_stride | (size_t)out) & 3) == 0;  // wave-uniform
    if (SPLIT && sp) {  // frame A's half up to t1, then frame B's from its step 96
        uint8_t* o = out + fa * out_stride;
        const int na = t1s >> 3;
        for (int i = lane; i < nbytes; i += 64) o[i] = i < na ? tab[i] : tab[4 * tbb + warm / 8 + (i - na)];
    } else if (words) {  // lanes 0-31 copy frame A, 32-63 frame B, one dword each per pass
        uint8_t* o = out + (f ? fb : fa) * out_stride;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(tab + f * 4 * tbb);
        if (f == 0 || has_b)
            for (int i = blk; i < (nbytes >> 2); i += 32) reinterpret_cast<uint32_t*>(o)[i] = src[i];
    } else {
        uint8_t* oa = out + fa * out_stride;
        for (int i = lane; i < nbytes; i += 64) oa[i] = tab[i];
        if (has_b) {
            uint8_t* o2 = out + fb * out_stride;
            for (int i = lane; i < nbytes; i += 64) o2[i] = tab[4 * tbb + i];
        }
    }
    // the prefetched registers are complete before they leave this function (no copy of an
    // in-flight load destination can happen past here)
    if (LOOP && !GS && next < units) asm volatile("s_waitcnt vmcnt(0)" : "+v"(pra), "+v"(prb));
    break;
    }
}

// LOOP: persistent over frame pairs, wave b decodes pairs b, b + grid, ... (the grid is what
// the CUs hold at once, so every SIMD keeps the same number of waves to the end instead of
// the dispatcher refilling freed slots unevenly).  !LOOP: one wave per pair, for batches the
// CUs hold in one round and for the streaming decoder (the loop's extra live state costs
// ~3 % there).  GS: survivor slot = the wave (streaming: the pair, whose ring persists).
template <bool SOFT, bool GS, bool STREAM, bool LOOP, bool SPLIT = false, bool LIST = false, int NB = 2>
#define VTB_K7_WPE
__global__ __launch_bounds__(64) VTB_K7_WPE void k7_lds_kernel(const uint8_t* __restrict__ in, size_t in_stride,
                                                    uint8_t* __restrict__ out, size_t out_stride, int T, int L,
                                                    int Tpad, int tbb, int r0, size_t frames, int dbg, Launch table,
                                                    uint8_t* __restrict__ ws, size_t ws_wave, StreamArgs sa) {
    static_assert(!(STREAM && LOOP), "streaming calls keep per-pair state: one wave per pair");
    static_assert(!SPLIT || (!GS && !STREAM), "split frames: LDS survivors");
    if constexpr (LIST) frames = __builtin_amdgcn_readfirstlane(table.fail_list[0]);  // the list's frames
    const size_t pairs = (frames + 1) / 2;
    uint32_t pra = 0, prb = 0;  // next pair's chunk-0 input, prefetched during the traceback (LDS variant)
    uint32_t off[6];
    uint64_t clk0 = 0;
    if (table.tstamp) {
        tstamp(table, 0);
        clk0 = __builtin_amdgcn_s_memtime();
    }
    column_offsets<NB>(table, off, threadIdx.x);
    if constexpr (!LOOP) {
        k7_pair<SOFT, GS, STREAM, false, SPLIT, false, false, NB>(in, in_stride, out, out_stride, T, L, Tpad, tbb, r0,
                                                                  frames, dbg, table, ws, ws_wave, sa, blockIdx.x,
                                                                  blockIdx.x, false, pairs, pra, prb, off);
    } else {
        // units: frame pairs, or (SPLIT) frames; every wave leaves the loop when the units run out
        const size_t units = SPLIT ? frames : pairs;
        for (size_t wp = blockIdx.x; wp < units; wp += gridDim.x) {
            k7_pair<SOFT, GS, STREAM, true, SPLIT, false, LIST, NB>(in, in_stride, out, out_stride, T, L, Tpad, tbb, r0, frames,
                                                                dbg, table, ws, ws_wave, sa, wp, blockIdx.x,
                                                                !GS && wp != blockIdx.x, wp + gridDim.x, pra, prb, off);
            __syncthreads();  // LDS of this pair (decoded bytes) before the next pair's table ring
        }
    }
    if (table.tstamp) {
        tstamp(table, 3);
        const uint64_t clk1 = __builtin_amdgcn_s_memtime();
        uint32_t hwid, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        if (threadIdx.x == 0) {
            table.tstamp[8 * blockIdx.x + 4] = clk0;
            table.tstamp[8 * blockIdx.x + 5] = clk1;
            table.tstamp[8 * blockIdx.x + 6] = hwid;
            table.tstamp[8 * blockIdx.x + 7] = xcc;
        }
    }
}

// Single-frame latency path (SEG): one workgroup of W waves per frame, 2W segments of the
// frame at once (one per u16 half; see SegArgs).  The frame's input is staged into LDS
// first (a host-mapped frame crosses PCIe once, in one round trip), the segments' ACS run
// in parallel, and segment i's metrics at s_i are checked against segment i - 1's (equal up
// to a constant: every later decision of segment i is the frame's).  If every check holds,
// wave 0 traces the frame back over all segments' survivor words (the frame decoder's
// verified block-parallel chains, one chain of 48-step blocks over the 64 lanes) and writes
// the bytes out; otherwise nothing is written and sg.done reports 2 (the caller decodes the
// frame again with the frame kernel).  sg.done (host-mapped) is written last, after a
// system-scope release, so a host thread can wait on it instead of synchronising the stream.
constexpr int kSegLoads = 4;  // 16-byte staging loads per thread: frames of up to 64 B per thread
template <bool SOFT>
__global__ __launch_bounds__(512) void k7_seg_kernel(const uint8_t* __restrict__ in, size_t in_stride,
                                                     uint8_t* __restrict__ out, size_t out_stride, int T, int L,
                                                     int Tpad, int r0, int dbg, Launch table, SegArgs sg) {
    extern __shared__ uint4 smem4[];
    uint8_t* smem = reinterpret_cast<uint8_t*>(smem4);
    const int wv = int(threadIdx.x >> 6), lane = int(threadIdx.x & 63), W = int(blockDim.x >> 6);
    // the frame's input bytes into LDS: up to four 16-byte loads per thread, all issued before
    // any store (one round trip; the input buffer is padded to 16 bytes)
    {
        const uint8_t* src = in + size_t(blockIdx.x) * in_stride;
        const int nin = (SOFT ? 2 : 1) * T;
        const int step = 16 * int(blockDim.x), i0 = 16 * int(threadIdx.x);
        uint4 v0 = make_uint4(0, 0, 0, 0), v1 = v0, v2 = v0, v3 = v0;
        static_assert(kSegLoads == 4, "four staging loads per thread");
        if (i0 < nin) v0 = *reinterpret_cast<const uint4*>(src + i0);
        if (i0 + step < nin) v1 = *reinterpret_cast<const uint4*>(src + i0 + step);
        if (i0 + 2 * step < nin) v2 = *reinterpret_cast<const uint4*>(src + i0 + 2 * step);
        if (i0 + 3 * step < nin) v3 = *reinterpret_cast<const uint4*>(src + i0 + 3 * step);
        uint8_t* dst = smem + sg.in_lds + i0;
        if (i0 < nin) *reinterpret_cast<uint4*>(dst) = v0;
        if (i0 + step < nin) *reinterpret_cast<uint4*>(dst + step) = v1;
        if (i0 + 2 * step < nin) *reinterpret_cast<uint4*>(dst + 2 * step) = v2;
        if (i0 + 3 * step < nin) *reinterpret_cast<uint4*>(dst + 3 * step) = v3;
    }
    __syncthreads();
    uint32_t off[6];
    column_offsets(table, off, lane);
    uint32_t pra = 0, prb = 0, fm[2] = {0, 0};
    k7_pair<SOFT, false, false, false, true, true>(in, in_stride, out, out_stride, T, L, Tpad, 0, r0, 1, dbg, table,
                                                    nullptr, 0, StreamArgs(), blockIdx.x, blockIdx.x, false, 1, pra,
                                                    prb, off, &sg, fm);
    if (dbg & 16) return;
    using H = Hist<SOFT>;
    // exchange: final metrics (both halves) and the metrics at the end of the warm-up
    uint32_t* xf = reinterpret_cast<uint32_t*>(smem + sg.x_lds);
    uint32_t* xs = xf + 64 * W;
    uint32_t* okw = xs + 64 * W;
    xf[64 * wv + lane] = fm[0];
    xs[64 * wv + lane] = fm[1];
    __syncthreads();
    constexpr uint32_t KEEP = 0xFFFFu & ~(H::SC - 1);
    auto same_up_to_const = [](uint32_t a, uint32_t b) {  // a, b: this lane's metrics (history masked)
        const uint32_t a0 = __builtin_amdgcn_readfirstlane(a), b0 = __builtin_amdgcn_readfirstlane(b);
        return __ballot(((a - a0) & 0xFFFFu) == ((b - b0) & 0xFFFFu)) == ~0ull;
    };
    bool ok = true;
    if (2 * wv + 1 < sg.G) ok = ok && same_up_to_const(fm[0] & KEEP, (fm[1] >> 16) & KEEP);  // half B vs half A
    if (wv > 0) ok = ok && same_up_to_const((xf[64 * (wv - 1) + lane] >> 16) & KEEP, fm[1] & KEEP);  // A vs wave - 1's B
    if (lane == 0) okw[wv] = ok ? 1u : 0u;
    __syncthreads();
    bool all = true;
    for (int i = 0; i < W; i++) all = all && okw[i] != 0u;
    if (wv != 0) return;  // (no barrier follows)
    if (!all) {
        if (sg.done && lane == 0) __hip_atomic_store(sg.done, 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    // ---- traceback, wave 0: blocks of tbp steps (a multiple of 48), lane b = block b ----
    const int step = sg.n - sg.warm;
    auto col_at = [&](int tlo) -> uint32_t {  // survivor-word column of the 48 steps at tlo
        int i = tlo < sg.warm ? 0 : (tlo - sg.warm) / step;
        if (i > sg.G - 1) i = sg.G - 1;
        const int lt = tlo - i * step;
        return uint32_t((i >> 1) * sg.seg_bytes + r0 + 256 * (lt >> 4) + 2 * (i & 1));
    };
    auto tb48 = [&](uint32_t cb, uint32_t& l4) {
        if constexpr (SOFT) return tb_body<false>(cb, l4, 0);
        else return tb_body8<false>(cb, l4, 0);
    };
    uint8_t* ob = smem;  // decoded bytes (wave 0's table ring is free now), index t / 8
    const int nb48 = Tpad / kChunk;
    const int tbp = (nb48 + 63) / 64 * kChunk;
    const bool active = lane * tbp < Tpad;
    const int start_full = (lane + 1) * tbp + kTbWarm;
    const int start = min(start_full, Tpad);
    const bool known = start >= T;
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
        const uint32_t sf = __shfl_down(fin, 1);
        const bool okb = fixed || loc_top == sf;
        const uint64_t bad = ~__ballot(okb);
        if (bad == 0) break;
        if (round == rounds) {
            unproven = true;
            break;
        }
        if (!okb && (bad >> (lane + 1)) == 0) {
            loc = sf;
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
    // copy out (bits past L are zero: the survivor ends in state 0)
    const int nbytes = (L + 7) >> 3;
    uint8_t* o = out + size_t(blockIdx.x) * out_stride;
    if (((nbytes | size_t(o)) & 3) == 0) {
        for (int i = lane; i < (nbytes >> 2); i += 64) reinterpret_cast<uint32_t*>(o)[i] = reinterpret_cast<const uint32_t*>(ob)[i];
    } else {
        for (int i = lane; i < nbytes; i += 64) o[i] = ob[i];
    }
    if (sg.done) {
        // every lane's output stores complete, then the system-scope release store (its
        // own fence writes back; no acquire needed here, so no __threadfence_system)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(sg.done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Newest steps whose survivor words the global-survivor variant keeps in LDS: as many 48-step
// chunks as leave 8 waves per CU (2 per SIMD, where the ACS saturates the VALU) their LDS;
// HBM then sees only the older steps' words.  Hard input only: its traceback reads one byte
// per 8 steps, and config C3 hard ran 1-2 % faster (0.835 vs 0.843-0.851 ms, 65,536 x 2,048
// bits); soft input reads a word per 2 steps, and a wave walks at the pace of its slowest
// lane, so the LDS lanes gained nothing while every window paid for both loads: C3 soft
// 1.16-1.17 vs 1.07 ms (profiles/r02/hybrid_survivors_ab.txt).  VTB_DEBUG bit 11
// (testing): none.
int gs_lds_steps(const Launch& a) {
    const int T = a.T;
    if (a.soft || (a.dbg & 2048)) return 0;
    const int per_wave = 160 * 1024 / 8 - region0(T);
    int s = per_wave > 0 ? per_wave / 16 / kChunk * kChunk : 0;
    return s < t_pad(T) ? s : t_pad(T);
}
// LDS of the survivor-in-global variant: table ring, decoded bytes and the newest steps' words.
size_t lds_bytes_gs(const Launch& a) { return (size_t)region0(a.T) + 16 * (size_t)gs_lds_steps(a); }
size_t ws_wave_bytes(int T) { return 16 * (size_t)t_pad(T); }
constexpr size_t kMaxWsBytes = size_t(1) << 30;  // survivor workspace cap (global variant)

template <bool GS>
size_t lds_of(const Launch& a) { return GS ? lds_bytes_gs(a) : lds_bytes(a.T); }

template <bool GS, bool LOOP = true, bool SPLIT = false>
auto kernel_of(const Launch& a) {
    return a.soft ? k7_lds_kernel<true, GS, false, LOOP, SPLIT> : k7_lds_kernel<false, GS, false, LOOP, SPLIT>;
}

// Persistent grid: the frame pairs, at most what the CUs hold at once (occupancy of this
// kernel and LDS size), and for the global variant at most kMaxWsBytes of survivor slots.
template <bool GS>
size_t grid_waves(const Launch& a) {
    const size_t pairs = (a.frames + 1) / 2;
    const size_t lds = lds_of<GS>(a);
    auto kern = kernel_of<GS>(a);
    if (lds > 64 * 1024)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  int(lds));
    size_t grid = pairs;
    const int per_cu = (a.dbg & 32) ? 0  // VTB_DEBUG bit 5 (testing): one wave per pair
                                     : resident_per_cu(reinterpret_cast<const void*>(kern), lds);
    if (per_cu > 0) {
        const size_t resident = size_t(per_cu) * size_t(a.cus > 0 ? a.cus : 1);
        if (resident < grid) grid = resident;
    }
    if (GS) {
        size_t cap = kMaxWsBytes / ws_wave_bytes(a.T);
        if (cap < 1) cap = 1;
        if (cap < grid) grid = cap;
    }
    return grid;
}

template <bool GS>
hipError_t launch_k7(const Launch& a) {
    if (a.frames == 0) return hipSuccess;
    if (GS && !a.ws) return hipErrorInvalidValue;
    const size_t lds = lds_of<GS>(a);
    size_t grid = grid_waves<GS>(a);
    const bool loop = grid < (a.frames + 1) / 2;
    auto kern = loop ? kernel_of<GS, true>(a) : kernel_of<GS, false>(a);
    const char* name = GS ? (loop ? "k7_global_loop" : "k7_global") : (loop ? "k7_lds_loop" : "k7_lds");
    // Batches the CUs hold at one frame per wave (up to 2 per SIMD at L = 1024) run split
    // (one frame per wave, both halves at once: k7_pair SPLIT): twice the waves, about half
    // the dependent steps per wave.  VTB_DEBUG bit 8 (testing): never split.
    if (!GS && a.T >= 240 && split_t1(a.T) <= 32 * kChunk && !(a.dbg & 256)) {
        auto ks = kernel_of<false, false, true>(a);
        const int per_cu = resident_per_cu(reinterpret_cast<const void*>(ks), lds);
        if (per_cu > 0 && a.frames <= size_t(per_cu) * size_t(a.cus > 0 ? a.cus : 1)) {
            kern = ks;
            grid = a.frames;
            name = "k7_lds_split";
        }
    }
    note_kernel(name);
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
    }
    Launch la = a;
    la.gs_steps = GS ? t_pad(a.T) - gs_lds_steps(a) : (1 << 30);
    hipLaunchKernelGGL(kern, dim3(unsigned(grid)), dim3(64), lds, a.stream, a.in, a.in_stride, a.out, a.out_stride,
                       a.T, a.L, t_pad(a.T), tb_block(a.T), region0(a.T), a.frames, a.dbg, la,
                       static_cast<uint8_t*>(a.ws), ws_wave_bytes(a.T), StreamArgs());
    return hipGetLastError();
}

// Persistent split kernel (frames longer than the LDS variant holds at 8 waves per CU, e.g.
// config C3's 2,048 bits): one frame per wave as two halves (k7_pair SPLIT), survivors of
// t1 steps in LDS, frames in a persistent loop; frames whose halves do not converge go to a
// list that the persistent global-survivor kernel (LIST) decodes afterwards.  The warm-up is
// 96 steps when 8 waves per CU still fit, else 48.
bool split_loop_params(const Launch& a, int& warm, size_t& lds) {
    if (a.S != 6 || a.T < 240) return false;
    if (a.split_warm_force > 0) {  // $VTB_SPLIT_WARM (measurement only): a fixed warm-up, any occupancy
        warm = a.split_warm_force / kChunk * kChunk;
        lds = size_t(region0(a.T)) + 16 * size_t(split_t1(a.T, warm));
        return warm >= kChunk && split_t1(a.T, warm) <= 32 * kChunk && lds <= 160 * 1024;
    }
    for (int w : {kSplitWarm, kSplitWarm / 2}) {
        const int t1 = split_t1(a.T, w);
        if (t1 > 32 * kChunk) return false;  // traceback: at most 32 48-step blocks per half
        lds = size_t(region0(a.T)) + 16 * size_t(t1);
        if (lds <= 160 * 1024 / 8) {
            warm = w;
            return true;
        }
    }
    return false;
}
size_t split_list_bytes(size_t frames) { return (4 * (frames + 1) + 255) / 256 * 256; }
// waves of the list kernel: what the global variant holds at once for the batch's frame pairs
size_t list_grid(const Launch& a) { return grid_waves<true>(a); }

}  // namespace

bool k7_split_loop_supported(const Launch& a) {
    int warm;
    size_t lds;
    return split_loop_params(a, warm, lds) && k7_global_supported(a);
}

size_t k7_split_loop_workspace_bytes(const Launch& a) {
    return split_list_bytes(a.frames) + list_grid(a) * ws_wave_bytes(a.T);
}

hipError_t launch_k7_split_loop(const Launch& a) {
    if (a.frames == 0) return hipSuccess;
    int warm;
    size_t lds;
    if (!a.ws || !split_loop_params(a, warm, lds)) return hipErrorInvalidValue;
    uint32_t* list = static_cast<uint32_t*>(a.ws);
    hipError_t e = hipMemsetAsync(list, 0, 4, a.stream);
    if (e != hipSuccess) return e;
    Launch la = a;
    la.split_warm = warm;
    la.fail_list = list;
    auto kern = a.soft ? k7_lds_kernel<true, false, false, true, true> : k7_lds_kernel<false, false, false, true, true>;
    const int per_cu = resident_per_cu(reinterpret_cast<const void*>(kern), lds);
    size_t grid = size_t(per_cu > 0 ? per_cu : 8) * size_t(a.cus > 0 ? a.cus : 1);
    if (grid > a.frames) grid = a.frames;
    note_kernel("k7_split_loop");
    hipLaunchKernelGGL(kern, dim3(unsigned(grid)), dim3(64), lds, a.stream, a.in, a.in_stride, a.out, a.out_stride, a.T,
                       a.L, t_pad(a.T), tb_block(a.T), region0(a.T), a.frames, a.dbg, la, nullptr, size_t(0),
                       StreamArgs());
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // the frames that did not split: the persistent global-survivor kernel over the list (it
    // reads the count on the device; with an empty list every wave exits at once)
    auto lk = a.soft ? k7_lds_kernel<true, true, false, true, false, true> : k7_lds_kernel<false, true, false, true, false, true>;
    const size_t llds = lds_bytes_gs(a);
    if (llds > 64 * 1024) {
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(lk), hipFuncAttributeMaxDynamicSharedMemorySize, int(llds));
        if (e != hipSuccess) return e;
    }
    la.gs_steps = t_pad(a.T) - gs_lds_steps(a);
    hipLaunchKernelGGL(lk, dim3(unsigned(list_grid(a))), dim3(64), llds, a.stream, a.in, a.in_stride, a.out, a.out_stride,
                       a.T, a.L, t_pad(a.T), tb_block(a.T), region0(a.T), size_t(0), a.dbg, la,
                       static_cast<uint8_t*>(a.ws) + split_list_bytes(a.frames), ws_wave_bytes(a.T), StreamArgs());
    return hipGetLastError();
}

bool k7_lds_supported(const Launch& a) { return a.S == 6 && a.T > a.S && lds_bytes(a.T) <= 160 * 1024; }

size_t k7_lds_bytes(const Launch& a) { return lds_bytes(a.T); }

hipError_t launch_k7_lds(const Launch& a) { return launch_k7<false>(a); }

// Rate 1/3 (k = 1, n = 3), hard input: the LDS pair kernel with a 16-column branch-metric ring
// (k7_pair NB = 3), one round or persistent over the frame pairs.  a.symm holds the 3-bit labels.
bool k7_n3_supported(const Launch& a) { return a.S == 6 && !a.soft && a.T > a.S && lds_bytes(a.T, 3) <= 160 * 1024; }

hipError_t launch_k7_lds_n3(const Launch& a) {
    if (a.frames == 0) return hipSuccess;
    if (!k7_n3_supported(a)) return hipErrorInvalidValue;
    const size_t lds = lds_bytes(a.T, 3), pairs = (a.frames + 1) / 2;
    auto once = k7_lds_kernel<false, false, false, false, false, false, 3>;
    auto loop = k7_lds_kernel<false, false, false, true, false, false, 3>;
    for (auto k : {once, loop}) {
        if (lds > 64 * 1024) {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
            if (e != hipSuccess) return e;
        }
    }
    const int per_cu = resident_per_cu(reinterpret_cast<const void*>(loop), lds);
    size_t grid = pairs;
    if (per_cu > 0 && size_t(per_cu) * size_t(a.cus > 0 ? a.cus : 1) < grid) grid = size_t(per_cu) * size_t(a.cus > 0 ? a.cus : 1);
    const bool lp = grid < pairs;
    note_kernel(lp ? "k7_lds_n3_loop" : "k7_lds_n3");
    hipLaunchKernelGGL(lp ? loop : once, dim3(unsigned(grid)), dim3(64), lds, a.stream, a.in, a.in_stride, a.out,
                       a.out_stride, a.T, a.L, t_pad(a.T), tb_block(a.T), region0(a.T, 3), a.frames, a.dbg, a,
                       static_cast<uint8_t*>(nullptr), size_t(0), StreamArgs());
    return hipGetLastError();
}

bool k7_global_supported(const Launch& a) { return a.S == 6 && a.T > a.S && lds_bytes_gs(a) <= 160 * 1024; }

size_t k7_global_workspace_bytes(const Launch& a) { return grid_waves<true>(a) * ws_wave_bytes(a.T); }

hipError_t launch_k7_global(const Launch& a) { return launch_k7<true>(a); }

// SEG geometry for a frame of T steps on W waves (warm-up `warm`): n = the ACS steps per
// segment (multiple of 48) with 2W segments covering T, G = the segments whose exact region
// [s_i, s_i+1) starts before T.
bool k7_seg_geometry(int T, int W, int warm, SegArgs& sg) {
    if (W < 1 || W > 8 || warm < 48 || warm % 48) return false;
    const int G2 = 2 * W;
    int n = (T + (G2 - 1) * warm + G2 - 1) / G2;
    n = (n + kChunk - 1) / kChunk * kChunk;
    if (n < warm + kChunk) n = warm + kChunk;
    int G = 1;
    while (G < G2 && G * (n - warm) + warm < T) G++;
    if ((G - 1) * (n - warm) + n < T) return false;
    sg.n = n, sg.warm = warm, sg.G = G;
    return true;
}

bool k7_seg_supported(const Launch& a, int waves, int warm) {
    SegArgs sg;
    if (a.S != 6 || a.T < 240 || !k7_seg_geometry(a.T, waves, warm, sg)) return false;
    const int W = (sg.G + 1) / 2, nin = (a.soft ? 2 : 1) * a.T;
    const int r0 = (kRingBytes + 255) / 256 * 256;
    const size_t lds = size_t(W) * (r0 + 16 * sg.n) + (nin + 15) / 16 * 16 + 4 * (2 * 64 * W + W);
    return nin <= 16 * kSegLoads * 64 * W && lds <= 160 * 1024 && t_pad(a.T) / 8 + 8 <= r0;
}

hipError_t launch_k7_seg(const Launch& a, int waves, int warm, uint32_t* done) {
    SegArgs sg;
    if (!k7_seg_geometry(a.T, waves, warm, sg)) return hipErrorInvalidValue;
    const int W = (sg.G + 1) / 2;  // waves in use
    const int r0 = (kRingBytes + 255) / 256 * 256;
    sg.seg_bytes = r0 + 16 * sg.n;
    const int Tpad = t_pad(a.T);
    const int nin = (a.soft ? 2 : 1) * a.T;  // staged bytes (the staging loads clamp to T - 1)
    if (nin > 16 * kSegLoads * 64 * W) return hipErrorInvalidValue;
    sg.in_lds = W * sg.seg_bytes;
    sg.x_lds = sg.in_lds + (nin + 15) / 16 * 16;
    sg.done = done;
    const size_t lds = size_t(sg.x_lds) + 4 * (2 * 64 * W + W);
    auto kern = a.soft ? k7_seg_kernel<true> : k7_seg_kernel<false>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                           int(lds));
        if (e != hipSuccess) return e;
    }
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    note_kernel("k7_seg");
    hipLaunchKernelGGL(kern, dim3(unsigned(a.frames)), dim3(64 * W), lds, a.stream, a.in, a.in_stride, a.out,
                       a.out_stride, a.T, a.L, Tpad, r0, a.dbg, a, sg);
    return hipGetLastError();
}

// One streaming call: every wave (two streams) continues its trellis over [s.t_begin,
// s.t_end) and emits the final bits (stream_traceback).  LDS: the table ring only.
hipError_t launch_k7_stream(const Launch& a, const StreamArgs& s) {
    if (a.frames == 0) return hipSuccess;
    if (!a.ws || !s.state || !s.out_bits || s.ring < 48 || s.ring % 48 || s.t_begin % 48 || s.t_end % 48)
        return hipErrorInvalidValue;
    // This call's survivor words in LDS (16 B per step) while 8 waves per CU still fit (calls
    // up to ~1,000 segments): the merge test and the emission then walk LDS except for the
    // steps carried over from earlier calls; longer calls keep every word in the ring.
    const size_t r0 = (kRingBytes + 255) / 256 * 256;
    const size_t lds_l = r0 + 16 * size_t(s.t_end - s.t_begin);
    const bool in_lds = lds_l <= (160 * 1024) / 8 && !(a.dbg & 64);  // VTB_DEBUG bit 6: ring only
    auto kern = in_lds ? (a.soft ? k7_lds_kernel<true, false, true, false> : k7_lds_kernel<false, false, true, false>)
                       : (a.soft ? k7_lds_kernel<true, true, true, false> : k7_lds_kernel<false, true, true, false>);
    const size_t lds = in_lds ? lds_l : r0;
    const size_t waves = (a.frames + 1) / 2;
    note_kernel("k7_stream");
    hipLaunchKernelGGL(kern, dim3(unsigned(waves)), dim3(64), lds, a.stream, a.in, a.in_stride, a.out, a.out_stride,
                       a.T, a.L, s.t_end, 0, int(r0), a.frames, a.dbg, a, static_cast<uint8_t*>(a.ws), 16 * size_t(s.ring),
                       s);
    return hipGetLastError();
}

}  // namespace vtb
