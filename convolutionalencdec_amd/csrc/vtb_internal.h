// Internal interface between the C-ABI layer (vtb_api.hip) and the kernel TUs.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "viterbi_amd.h"

namespace vtb {

constexpr int kMaxS = 8;  // K <= 9

// Wave-uniform description of one batch launch.  symm[] is the trellis table of
// viterbiInitButterflyk1 (reference viterbiDecoderButterflyk1.c:24-29).
struct Launch {
    int S = 0;         // state bits, K-1
    int soft = 0;      // 0: hard byte-per-segment input, 1: 8-bit soft pairs
    int T = 0;         // trellis steps per frame = L + S
    int L = 0;         // information bits per frame
    const uint8_t* in = nullptr;
    size_t in_stride = 0;
    uint8_t* out = nullptr;
    size_t out_stride = 0;
    size_t frames = 0;
    hipStream_t stream = nullptr;
    void* ws = nullptr;  // device workspace of at least *_workspace_bytes() (plan-owned)
    int cus = 256;       // compute units of the device (persistent grids)
    // Measurement only (tools/tstamp.py, vtb_debug_set_tstamp): when set, the K=7 kernel's
    // waves write 8 u64 per wave -- realtime (100 MHz) at entry, after the ACS, after the
    // traceback and at exit, shader-clock at entry and exit, HW_ID and XCC_ID.  Null in
    // production (one uniform branch per stamp).
    unsigned long long* tstamp = nullptr;
    // K=7 global-survivor variant: steps [0, gs_steps) keep their survivor words in the global
    // workspace, the newest steps [gs_steps, Tpad) in LDS (set by the launcher; all global when
    // >= Tpad)
    int gs_steps = 1 << 30;
    // K=7 split frames (one frame per wave, two halves): warm-up steps of the second half (a
    // multiple of 48), and for the persistent split kernel the list of frames whose halves did
    // not converge ([0] = count, then frame indices; decoded again by the list kernel)
    int split_warm = 96;
    uint32_t* fail_list = nullptr;
    // the plan's knobs (Knobs above): VTB_DEBUG bits, a fixed split warm-up, the K=9 SEG grid stride
    int dbg = 0;
    int split_warm_force = 0;
    int seg9_xcd = -1;
    // Testing only (vtb_debug_set_guard_counter): a device word every traceback completeness
    // guard that fires adds 1 to (the frame then takes its exact slow path).  Null in production.
    uint32_t* guard_hits = nullptr;
    uint8_t symm[1 << (kMaxS - 1)] = {};
};

// Which kernel instance the calling thread's last decode launch used (a static name such as
// "k7_lds" or "k7_lds_loop"; vtb_debug_last_kernel).  Testing only: lets the parity tests prove
// they ran the instance bench.py times.
void note_kernel(const char* name);
const char* last_kernel();

// The debug timestamp buffer of the next launches (nullptr: off).  Measurement only.
unsigned long long* debug_tstamp();
void set_debug_tstamp(unsigned long long* p);

// Testing and measurement knobs, read from the environment once -- when a plan or a stream
// object is created (vtb_plan_create, vtb_stream_create; per call only for the plan-less
// vtb_genk_decode_device) -- and carried from there into every launch (Launch::dbg ...), never
// parsed per launch.  The reference is configured at compile time only
// (/root/reference/src/viterbiDecoder.h:17-39); production sets none of these.
//
// $VTB_DEBUG bits.  Exact (output unchanged; kernel choice and forced slow paths for the tests):
//   5 one wave per frame pair instead of the persistent grid, 6 streaming survivors in the global
//   ring only, 8 never split frames across the halves of a wave, 10 no single-frame SEG kernel,
//   11 global-survivor variant without its LDS part, 12 never the persistent split kernel,
//   13 full last chunk, 14 no in-wave split fix-up, 15 fix-up on every split frame, 16 fix-up
//   checkpoints never match, 17 forced completeness guards (every traceback chain with a block not
//   known from the frame end skips its checks and re-walks and takes the guard's exact slow
//   path), 18 K=9 frames on the pair kernel (two frames per wave) where one frame per wave (k9s)
//   would run, 19 the generic kernel's global-survivor variant (vtb_lds_path.hip GS) for every
//   frame length (its production choice since round 6's register-resident trellis), 20 the
//   generic kernel's LDS variant wherever its LDS fits one CU.
// Output-corrupting (phase timing only): 0 skip the traceback, 1 skip the ACS, 2 skip the
//   traceback verification, 3 warm-up walk only, 4 return at entry.  Only a -DVTB_MEASURE
//   build (tools/build_variants.sh) honours them; the shipped library masks them off.
constexpr int kDbgUnsafe = 0x1F;
constexpr int kDbgTbCap = 1 << 17;
constexpr int kDbgGenericGs = 1 << 19;
constexpr int kDbgGenericLds = 1 << 20;
#ifdef VTB_MEASURE
constexpr int kDbgHonoured = ~0;
#else
constexpr int kDbgHonoured = ~kDbgUnsafe;
#endif

// $VTB_KERNEL: force one kernel family (testing and A/B measurement).
enum class Force { Any, K7, Gws, K9, Lds, Seg, K7s, Genk, Unknown };

// Each numeric knob: unset, empty or not above its "off" value means the library's own choice
// (the value production runs with); knobs only ever select exact alternatives or measurement
// setups.  (Round 5 moved every variable here; the older per-launch readers gave VTB_SEG9_XCD < 0,
// VTB_SEG_WARM=0 and VTB_SPLIT_WARM=0 other meanings -- those are gone, listed per knob.)
struct Knobs {
    int dbg = 0;              // $VTB_DEBUG & kDbgHonoured
    Force force = Force::Any;
    int split_warm = 0;       // $VTB_SPLIT_WARM > 0: fixed split warm-up (rounded down to 48); else chosen by
                              //   occupancy (0 no longer turns the split kernel off: VTB_DEBUG bit 12 does)
    int genk_warm = -1;       // $VTB_GENK_WARM >= 0: general-k traceback warm-up; else 96
    int seg_waves = 0;        // $VTB_SEG_WAVES > 0: SEG kernel waves; else 8, or 4 where 8 do not fit
    int seg_warm = 0;         // $VTB_SEG_WARM > 0: fixed SEG warm-up and no adaptive short warm-up; else
                              //   kSegWarm with the adaptive short warm-up (VTB_SEG_ADAPT=0 turns that off)
    bool seg_adapt = true;    // $VTB_SEG_ADAPT != "0"
    int seg9_wgs = 0;         // $VTB_SEG9_WGS > 0: K=9 SEG workgroups; else kSeg9Wgs
    int segg_wgs = 0;         // $VTB_SEGG_WGS > 0: generic SEG workgroups; else kSegGenWgs for K = 6, 8, 1 below
    int seg9_waves = 0;       // $VTB_SEG9_WAVES > 0: K=9 SEG waves per workgroup; else kSeg9Waves
    int seg9_xcd = -1;        // $VTB_SEG9_XCD == 0: K=9 SEG grid stride 1 (workgroups spread over the
                              //   XCDs); any other value or unset: stride 8 (one XCD, one L2)
};
Knobs read_knobs();

// A completeness guard fired (testing counter, Launch::guard_hits; one lane calls it).
__device__ __forceinline__ void note_guard(uint32_t* hits) {
    if (hits) atomicAdd(hits, 1u);
}

// The guard counter of the next launches (nullptr: off).  Testing only.
uint32_t* debug_guard_hits();
void set_debug_guard_hits(uint32_t* p);

// Resident blocks per CU of a 64-thread kernel with `lds` bytes of dynamic LDS
// (hipOccupancyMaxActiveBlocksPerMultiprocessor, cached: the query costs host time on every
// launch otherwise).  0 if unknown.
int resident_per_cu(const void* kernel, size_t lds);

// Compute units of the calling thread's current device (cached per device; 256 if unknown).
int current_device_cus();

// Kernel families.  Each returns hipSuccess or the launch error; VTB_ERR_UNSUPPORTED-style
// shape limits are reported through *_supported() beforehand.
//
// The generic kernel (vtb_lds_path.hip), every K and every frame up to VTB_MAX_FRAME_BITS:
// survivors in LDS while a wave's survivors and input fit one CU's LDS, else (lds_path_global)
// in a workspace of lds_path_workspace_bytes(a) bytes at Launch::ws (0 when the LDS variant runs).
bool lds_path_supported(const Launch& a);
bool lds_path_global(const Launch& a);
size_t lds_path_workspace_bytes(const Launch& a);
hipError_t launch_lds_path(const Launch& a);
// The single-frame path of the generic kernel (gen_seg_kernel, K = 3..6 and 8): one frame
// (Launch::frames = 1) from host-mapped memory as segments over `waves` waves of each of `nwg`
// workgroups, warm-up `warm` steps, *done as for K=7's SEG kernel (1 decoded, 2 not converged:
// nothing written).
constexpr int kSegGenWgs = 4;
bool gen_seg_supported(const Launch& a, int waves, int nwg, int warm);
// several workgroups (nwg > 1): the workspace (arrival counter zeroed once, in stream order,
// metrics, rows); 0 for the single-workgroup form
size_t gen_seg_workspace_bytes(const Launch& a, int waves, int nwg, int warm);
hipError_t launch_gen_seg(const Launch& a, int waves, int nwg, int warm, uint32_t* done);

// K=7, survivors in LDS (vtb_k7_lds.hip): the fast path.
bool k7_lds_supported(const Launch& a);
size_t k7_lds_bytes(const Launch& a);
hipError_t launch_k7_lds(const Launch& a);
// k = 1 rate-1/3 codes, hard input (a.symm: 3-bit butterfly labels), the K=7 LDS pair kernel
bool k7_n3_supported(const Launch& a);
hipError_t launch_k7_lds_n3(const Launch& a);

// K=7, the same kernel with survivor words in a global workspace (vtb_k7_lds.hip): long
// frames, and frames whose LDS survivors would cut the occupancy.
bool k7_global_supported(const Launch& a);
size_t k7_global_workspace_bytes(const Launch& a);
hipError_t launch_k7_global(const Launch& a);

// K=7 persistent split kernel (vtb_k7_lds.hip): frames too long for the LDS variant at 8 waves
// per CU decoded one per wave as two halves with LDS survivors, frames whose halves do not
// converge re-decoded by the global-survivor kernel from a list; workspace = the list plus the
// list kernel's survivor slots.
bool k7_split_loop_supported(const Launch& a);
size_t k7_split_loop_workspace_bytes(const Launch& a);
hipError_t launch_k7_split_loop(const Launch& a);

// K=7 single-frame latency path (k7_seg_kernel): one workgroup of up to 4 waves per frame,
// the frame cut into up to 8 segments decoded at once (warm-up `warm` steps, a multiple of
// 48), input staged through LDS (so it may sit in host-mapped memory), output written
// directly, then *done (host-mapped, may be null) = 1, or 2 if a segment's metrics had not
// converged (nothing written: decode the frame again with launch_k7_lds / _global).
constexpr int kSegWarm = 96;
bool k7_seg_supported(const Launch& a, int waves, int warm);
hipError_t launch_k7_seg(const Launch& a, int waves, int warm, uint32_t* done);

// K=7 streaming decode (vtb_stream_*, include/viterbi_amd.h): the global-survivor variant of
// the K=7 kernel continued across launches.  All streams of one stream object advance in
// lockstep, so the step counters are host-side; what depends on the data (how far each
// stream has emitted) lives in the per-wave state.  Launch::T is the steps received so far
// (t_begin + carry_len + new segments), Launch::in the call's new rows, Launch::ws the
// survivor ring.
constexpr int kStreamStateWords = 68;   // per wave: M[64] (packed metric pairs), e[2], flags, pad
constexpr int kStreamCarryStride = 96;  // per stream: up to 47 held-back segments (2 B soft)
struct StreamArgs {
    uint32_t* state = nullptr;       // waves x kStreamStateWords
    const uint8_t* carry = nullptr;  // streams x kStreamCarryStride
    int carry_len = 0;               // rows in the carry at the call (< 48)
    int t_begin = 0;                 // steps decoded by earlier calls (multiple of 48)
    int t_end = 0;                   // steps decoded after this call (multiple of 48)
    int last = 0;                    // terminate: traceback from state 0 at step T
    int ring = 0;                    // survivor ring per wave in steps (multiple of 48)
    int32_t* out_bits = nullptr;     // per stream: bits emitted by this call, -1 = window overflow
};
hipError_t launch_k7_stream(const Launch& a, const StreamArgs& s);
// K = 9 (vtb_k9.hip): the same protocol, 4 metric registers per lane, 64 B of survivor words
// per step and wave in the ring.
constexpr int kStreamStateWords9 = 260;  // per wave: M[4][64], e[2], flags, pad
hipError_t launch_k9_stream(const Launch& a, const StreamArgs& s);

// Streaming decode for every K (vtb_stream_gen.hip): the generic trellis layout of the LDS
// path (F = 64 / min(2^S, 64) streams per wave), survivor ring Launch::ws of
// gen_stream_ring_bytes_per_step(S) bytes per step and wave, per-wave state StreamArgs::state
// of gen_stream_state_words(S) int32 words (metrics [R][64], emitted step [64 R + f], lost flag
// [64 R + 32 + f]).  No carry: each call runs all its segments.
__host__ __device__ constexpr int gen_stream_state_words(int S) { return 64 * ((1 << S) < 64 ? 1 : (1 << S) / 64) + 64; }
size_t gen_stream_waves(int S, size_t streams);
size_t gen_stream_ring_bytes_per_step(int S);
hipError_t launch_gen_stream(const Launch& a, const StreamArgs& s);

// K=9 single-frame latency path (k9_seg_kernel): the frame as segments over `wgs` workgroups
// of `waves` waves, input staged through LDS, survivors and metrics in a workspace (whose
// first word, an arrival counter, must be zero before the first launch), *done as for K=7.
constexpr int kSeg9Waves = 4, kSeg9Wgs = 4, kSeg9Warm = 96;
constexpr int kSegWarmShort = 48;  // single-frame paths: the short warm-up tried first
bool k9_seg_supported(const Launch& a, int waves, int wgs, int warm);
size_t k9_seg_workspace_bytes(const Launch& a, int waves, int wgs, int warm);
hipError_t launch_k9_seg(const Launch& a, int waves, int wgs, int warm, uint32_t* done);

// K=9, survivors in a global workspace (vtb_k9.hip).
bool k9_supported(const Launch& a);
size_t k9_workspace_bytes(const Launch& a);
hipError_t launch_k9(const Launch& a);
// k = 1 rate-1/3 codes, hard input (a.symm: 3-bit butterfly labels), the K=9 frame kernel
bool k9_n3_supported(const Launch& a);
size_t k9_n3_workspace_bytes(const Launch& a);
hipError_t launch_k9_n3(const Launch& a);

// True if device `dev` is a gfx950 (answered once per device: the property query costs ~1 ms).
bool device_is_gfx950(int dev);

// Stream-ordered scratch memory from a per-device pool that keeps its memory (no release
// back to the driver between launches), so a per-launch workspace costs no hipMalloc.
hipError_t workspace_alloc(void** p, size_t bytes, hipStream_t stream);
hipError_t workspace_free(void* p, hipStream_t stream);

}  // namespace vtb
