// C-ABI implementation of include/viterbi_amd.h: code tables, plans, kernel choice,
// host/device entry points and the multi-GPU shard driver.
//
// Host-side only; the trellis work happens in the kernels of vtb_k7_lds.hip (K=7, the fast
// path, survivors in LDS or, for long frames, in a global workspace), vtb_k9.hip (K=9) and
// vtb_lds_path.hip (every K).

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "viterbi_amd.h"
#include "vtb_internal.h"

#define VTB_VERSION_STRING "viterbi_amd 0.1 (gfx950)"

struct vtb_plan {
    vtb_code_t code;
    vtb_input_t input;
    int32_t L;
    int32_t T;
    int device;
    uint8_t symm[1 << (vtb::kMaxS - 1)];
    vtb::Knobs knobs;  // read from the environment once, at creation (vtb_internal.h)
    // host-path staging (grown on demand)
    uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;
    size_t cap_frames = 0;
    hipStream_t stream = nullptr;
    hipStream_t copy_stream = nullptr;  // host path: copies of one chunk overlap the next's decode
    std::vector<hipEvent_t> events;     // host path: per chunk, H2D done and decode done
    // kernel workspace (survivor words), stream-ordered pool memory, grown on demand
    void* ws = nullptr;
    size_t ws_bytes = 0;
    int cus = 256;  // compute units of the device (kernel choice)
    // synchronous single-frame path (vtb_decode_frame_sync): coherent host-mapped buffers the
    // kernel reads and writes directly, and its completion word
    uint8_t* lat_in = nullptr;
    uint8_t* lat_out = nullptr;
    uint32_t* lat_done = nullptr;
    uint8_t* lat_d_in = nullptr;  // their device addresses (looked up once)
    uint8_t* lat_d_out = nullptr;
    uint32_t* lat_d_done = nullptr;
    int seg_waves = 0;  // SEG kernel waves (0: not usable for this plan)
    int seg_warm = 0;
    int seg9_wgs = 0;            // K = 9 SEG kernel workgroups (0: not usable for this plan)
    int seg9_waves = 0;          // and waves per workgroup
    int segg_waves = 0;          // generic SEG kernel (K = 3..6, 8) waves (0: not usable for this plan)
    int segg_wgs = 0;            // and workgroups (> 1: its workspace in seg9_ws)
    // adaptive SEG warm-up (vtb_decode_frame_sync): the short warm-up while frames converge
    // with it; after a miss, the plan's warm-up for `seg_backoff` calls (doubling per miss)
    bool seg_short = false;
    int seg_backoff = 0, seg_skip = 0;
    void* seg9_ws = nullptr;     // the K=9 (or several-workgroup generic) SEG kernel's workspace
                                 // (arrival counter, metrics, survivor words)
};

// Streaming decoder (include/viterbi_amd.h "Streaming decode"): all streams advance in
// lockstep, so the step counters live here; per-stream emission state is on the device.
struct vtb_stream {
    vtb_code_t code;
    vtb_input_t input;
    size_t streams = 0;
    int ring = 0;  // survivor ring per wave, steps (multiple of 48)
    int device = 0;
    uint8_t symm[1 << (vtb::kMaxS - 1)];
    uint32_t* d_state = nullptr;  // waves x kStreamStateWords
    uint8_t* d_carry = nullptr;   // streams x kStreamCarryStride
    void* d_ring = nullptr;       // waves x 16 * ring bytes
    int t_begin = 0;              // steps decoded in the current frame (multiple of 48)
    int carry_len = 0;            // segments received but not yet decoded (< 48)
    bool gen = false;             // generic kernel (vtb_stream_gen.hip): K other than 7, 9; no carry
    vtb::Knobs knobs;             // read once, at creation
};

namespace {

int parity(uint64_t x) { return __builtin_popcountll(x) & 1; }

// src/convEncode.c:163-174: reverse the K low bits.
uint64_t reverse_bits(uint64_t v, int bits) {
    uint64_t r = 0;
    for (int i = 0; i < bits; i++) {
        r = (r << 1) | (v & 1u);
        v >>= 1;
    }
    return r;
}

int check_code(const vtb_code_t* c) {
    if (!c) return VTB_ERR_INVALID;
    if (c->coded_bits != 2) return VTB_ERR_UNSUPPORTED;
    if (c->constraint_length < VTB_MIN_K || c->constraint_length > VTB_MAX_K) return VTB_ERR_UNSUPPORTED;
    for (int i = 0; i < 2; i++) {
        if (c->generators[i] >> c->constraint_length) return VTB_ERR_INVALID;  // taps beyond the constraint length
        // viterbiDecoder.c:17-25: the symmetric butterfly needs both end taps.
        if (!((c->generators[i] >> (c->constraint_length - 1)) & 1u) || !(c->generators[i] & 1u)) return VTB_ERR_CODE;
    }
    return VTB_OK;
}

void edge_table(const vtb_code_t* c, uint8_t* symm) {
    uint64_t p0 = reverse_bits(c->generators[0], c->constraint_length), p1 = reverse_bits(c->generators[1], c->constraint_length);
    int half = 1 << (c->constraint_length - 2);
    for (int i = 0; i < half; i++) {
        uint64_t tapped = uint64_t(i) << 1;  // tappedDelay = i, shift in input 0
        symm[i] = uint8_t(parity(tapped & p0) | (parity(tapped & p1) << 1));
    }
}

size_t in_bytes(const vtb_code_t* c, vtb_input_t in, int32_t L) {
    size_t T = size_t(L) + size_t(c->constraint_length - 1);
    return in == VTB_INPUT_SOFT8 ? 2 * T : T;
}

size_t out_bytes(int32_t L) { return (size_t(L) + 7) / 8; }

// Which kernel family a plan uses (see below).  VTB_KERNEL=k7|gws|k9|lds forces one (testing
// and A/B measurement, read into the plan's knobs at creation); a forced kernel that does not
// support the shape is an error.  (VTB_KERNEL=seg leaves the choice here free: the single-frame
// path's SEG kernel is chosen in vtb_decode_frame_sync, and any other forced family turns it off
// there.)
int launch(vtb_plan* p, const uint8_t* d_in, size_t in_stride, uint8_t* d_out, size_t out_stride,
           size_t frames, hipStream_t stream) {
    vtb::Launch a;
    a.S = p->code.constraint_length - 1;
    a.soft = p->input == VTB_INPUT_SOFT8;
    a.T = p->T;
    a.L = p->L;
    a.in = d_in;
    a.in_stride = in_stride;
    a.out = d_out;
    a.out_stride = out_stride;
    a.frames = frames;
    a.stream = stream;
    a.cus = p->cus;
    a.tstamp = vtb::debug_tstamp();
    a.guard_hits = vtb::debug_guard_hits();
    a.dbg = p->knobs.dbg;
    a.split_warm_force = p->knobs.split_warm;
    a.seg9_xcd = p->knobs.seg9_xcd;
    std::memcpy(a.symm, p->symm, sizeof(a.symm));
    using vtb::Force;
    const Force force = p->knobs.force;
    const bool k7s = force == Force::K7s;  // prefer the persistent split kernel (below)
    const bool any = force == Force::Any || force == Force::Seg || k7s;  // (seg: vtb_decode_frame_sync)
    const bool want_k7 = any || force == Force::K7;
    const bool want_gws = any || force == Force::Gws;
    const bool want_lds = any || force == Force::Lds;
    const bool want_k9 = any || force == Force::K9;
    hipError_t e;
    // K=7: survivors in LDS while that LDS leaves the CU as many waves (2 frames each) as
    // the batch can give it, up to 2 per SIMD (the ACS is VALU-bound there: more waves do
    // not help); else survivors in a global workspace (3 KB LDS per wave, traceback from
    // L2/HBM).  Measured (PERF_LOG.md §4.2): 4096 x 1024 soft, LDS 36.4 us vs global 46.3 us;
    // 65536 x 2048, LDS (1 wave per SIMD) 1.56 ms vs global 0.94 ms.  Other K: the generic
    // LDS-path kernel.
    bool k7_in_lds = false;
    if (want_k7 && vtb::k7_lds_supported(a)) {
        const size_t waves_per_cu = ((frames + 1) / 2 + p->cus - 1) / p->cus;
        const size_t want = waves_per_cu < 8 ? waves_per_cu : 8;
        const size_t fit = (160 * 1024) / vtb::k7_lds_bytes(a);
        k7_in_lds = !any || fit >= want || !vtb::k7_global_supported(a);
    }
    // plan-owned workspace (survivor words), grown on demand
    auto workspace = [&](size_t need) -> bool {
        if (need > p->ws_bytes) {
            if (p->ws) (void)vtb::workspace_free(p->ws, stream);
            p->ws = nullptr;
            p->ws_bytes = 0;
            if (vtb::workspace_alloc(&p->ws, need, stream) != hipSuccess) {
                p->ws = nullptr;
                return false;
            }
            p->ws_bytes = need;
        }
        a.ws = p->ws;
        return true;
    };
    // Longer K=7 frames (the LDS variant would hold the CU below 8 waves, e.g. config C3): one
    // frame per wave as two halves with LDS survivors, persistent (launch_k7_split_loop), when
    // the halves fit 8 waves per CU.  Halves whose metrics disagree at the seam are fixed up in
    // the wave (k7_pair); only frames the fix-up cannot settle go to the list kernel.  Measured
    // on C3 shapes (round 3, PERF_LOG.md §4.2b, 65,536 x 2,048 bits): soft -5 dB 1.019 ms, no
    // frame to the list (without the fix-up 1.065 ms, 1,528 frames listed); hard p = 0.056
    // 0.808 ms against 0.805 for the global-survivor variant, whose survivor words leave the CU
    // (7.5x the algorithmic HBM bytes).  VTB_KERNEL=k7s forces it wherever it applies;
    // VTB_DEBUG bit 12 (testing): never.
    const bool want_split = k7s || (any && !k7_in_lds);
    if (want_split && !(a.dbg & 4096) && vtb::k7_split_loop_supported(a)) {
        if (!workspace(vtb::k7_split_loop_workspace_bytes(a))) return VTB_ERR_NOMEM;
        e = vtb::launch_k7_split_loop(a);
        if (e == hipErrorOutOfMemory) return VTB_ERR_NOMEM;
        return e == hipSuccess ? VTB_OK : VTB_ERR_DEVICE;
    }
    if (k7_in_lds) {
        e = vtb::launch_k7_lds(a);
    } else if (want_gws && vtb::k7_global_supported(a)) {
        if (!workspace(vtb::k7_global_workspace_bytes(a))) return VTB_ERR_NOMEM;
        e = vtb::launch_k7_global(a);
    } else if (want_k9 && vtb::k9_supported(a)) {
        if (!workspace(vtb::k9_workspace_bytes(a))) return VTB_ERR_NOMEM;
        e = vtb::launch_k9(a);
    } else if (want_lds && vtb::lds_path_supported(a)) {
        if (vtb::lds_path_global(a) && !workspace(vtb::lds_path_workspace_bytes(a))) return VTB_ERR_NOMEM;
        e = vtb::launch_lds_path(a);
    } else {
        return VTB_ERR_UNSUPPORTED;
    }
    if (e == hipErrorOutOfMemory) return VTB_ERR_NOMEM;
    return e == hipSuccess ? VTB_OK : VTB_ERR_DEVICE;
}

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    // Switches only when the calling thread is on another device (per-launch host cost).
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev == dev) {
            prev = -1;
            ok = true;
            return;
        }
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace

// hipGetDeviceProperties costs ~1 ms: answered once per device.
bool vtb::device_is_gfx950(int dev) {
    static std::mutex mu;
    static int known[64] = {};  // 0 unknown, 1 gfx950, 2 other / failed
    if (dev < 0) return false;
    if (dev < 64) {
        std::lock_guard<std::mutex> lk(mu);
        if (known[dev]) return known[dev] == 1;
    }
    hipDeviceProp_t prop;
    const bool ok = hipGetDeviceProperties(&prop, dev) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
    if (dev < 64) {
        std::lock_guard<std::mutex> lk(mu);
        known[dev] = ok ? 1 : 2;
    }
    return ok;
}

namespace {
using vtb::device_is_gfx950;

// vtb_decode_host_multi's plans, one per (code, input, frame length, device), kept for the
// process (plan creation, its allocations and the first launch's setup cost milliseconds,
// against ~0.3 ms for a 4096-frame host batch); vtb_release_cached_plans frees them.
struct CachedPlan {
    vtb_code_t code;
    vtb_input_t input;
    int32_t L;
    int device;
    vtb_plan_t* plan;
    std::unique_ptr<std::mutex> busy;  // one host thread at a time per plan
};
std::mutex g_plan_cache_mu;
std::vector<CachedPlan> g_plan_cache;

bool same_code(const vtb_code_t& a, const vtb_code_t& b) {
    if (a.constraint_length != b.constraint_length || a.coded_bits != b.coded_bits) return false;
    for (int i = 0; i < a.coded_bits && i < 2; i++)
        if (a.generators[i] != b.generators[i]) return false;
    return true;
}

}  // namespace

namespace vtb {

namespace {
std::mutex g_pool_mutex;
unsigned long long* g_tstamp = nullptr;
hipMemPool_t g_pools[64] = {};
}  // namespace

hipError_t workspace_alloc(void** p, size_t bytes, hipStream_t stream) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    hipMemPool_t pool;
    {
        std::lock_guard<std::mutex> lk(g_pool_mutex);
        if (!g_pools[dev]) {
            hipMemPoolProps props = {};
            props.allocType = hipMemAllocationTypePinned;
            props.handleTypes = hipMemHandleTypeNone;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = dev;
            e = hipMemPoolCreate(&g_pools[dev], &props);
            if (e != hipSuccess) {
                g_pools[dev] = nullptr;
                return e;
            }
            uint64_t keep = UINT64_MAX;
            (void)hipMemPoolSetAttribute(g_pools[dev], hipMemPoolAttrReleaseThreshold, &keep);
        }
        pool = g_pools[dev];
    }
    return hipMallocFromPoolAsync(p, bytes, pool, stream);
}

int current_device_cus() {
    static std::mutex mu;
    static int cache[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    std::lock_guard<std::mutex> lk(mu);
    if (cache[dev] == 0) {
        int cus = 0;
        cache[dev] = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0 ? cus : 256;
    }
    return cache[dev];
}

int resident_per_cu(const void* kernel, size_t lds) {
    struct Entry {
        const void* k;
        size_t lds;
        int dev, n;
    };
    static std::mutex mu;
    static std::vector<Entry> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    {
        std::lock_guard<std::mutex> lk(mu);
        for (const Entry& e : cache)
            if (e.k == kernel && e.lds == lds && e.dev == dev) return e.n;
    }
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, 64, lds) != hipSuccess || n < 0) n = 0;
    std::lock_guard<std::mutex> lk(mu);
    cache.push_back({kernel, lds, dev, n});
    return n;
}

hipError_t workspace_free(void* p, hipStream_t stream) { return hipFreeAsync(p, stream); }

namespace {
thread_local const char* t_last_kernel = "";
}  // namespace
void note_kernel(const char* name) { t_last_kernel = name; }
const char* last_kernel() { return t_last_kernel; }

unsigned long long* debug_tstamp() { return g_tstamp; }
void set_debug_tstamp(unsigned long long* p) { g_tstamp = p; }

namespace {
std::atomic<uint32_t*> g_guard_hits{nullptr};
}  // namespace
uint32_t* debug_guard_hits() { return g_guard_hits.load(std::memory_order_relaxed); }
void set_debug_guard_hits(uint32_t* p) { g_guard_hits.store(p, std::memory_order_relaxed); }

Knobs read_knobs() {
    auto num = [](const char* name, int dflt) {
        const char* v = std::getenv(name);
        return v && *v ? std::atoi(v) : dflt;
    };
    Knobs k;
    k.dbg = num("VTB_DEBUG", 0) & kDbgHonoured;
    if (const char* v = std::getenv("VTB_KERNEL"); v && *v) {
        static const struct {
            const char* name;
            Force f;
        } names[] = {{"k7", Force::K7}, {"gws", Force::Gws}, {"k9", Force::K9}, {"lds", Force::Lds},
                     {"seg", Force::Seg}, {"k7s", Force::K7s}, {"genk", Force::Genk}};
        k.force = Force::Unknown;  // (an unknown name forces no family that exists: unsupported)
        for (const auto& n : names)
            if (std::strcmp(v, n.name) == 0) k.force = n.f;
    }
    k.split_warm = num("VTB_SPLIT_WARM", 0);
    k.genk_warm = num("VTB_GENK_WARM", -1);
    k.seg_waves = num("VTB_SEG_WAVES", 0);
    k.seg_warm = num("VTB_SEG_WARM", 0);
    k.seg_adapt = num("VTB_SEG_ADAPT", 1) != 0;
    k.seg9_wgs = num("VTB_SEG9_WGS", 0);
    k.segg_wgs = num("VTB_SEGG_WGS", 0);
    k.seg9_waves = num("VTB_SEG9_WAVES", 0);
    k.seg9_xcd = num("VTB_SEG9_XCD", -1);
    return k;
}

}  // namespace vtb

extern "C" {

const char* vtb_version(void) { return VTB_VERSION_STRING; }

// Testing only (not in include/viterbi_amd.h): the kernel instance of the calling thread's last
// decode launch ("k7_lds", "k7_lds_loop", "k7_lds_split", "k7_global", "k7_global_loop",
// "k7_split_loop", "k9", "k9_loop", "k9s", "lds_path", "k7_seg", "k9_seg", "k7_stream", "k9_stream"),
// "" before the first.
const char* vtb_debug_last_kernel(void) { return vtb::last_kernel(); }

// Measurement only (not in include/viterbi_amd.h): device buffer of 8 u64 per wave that the
// next K=7 frame launches fill with phase timestamps (tools/tstamp.py); nullptr turns it off.
void vtb_debug_set_tstamp(unsigned long long* d_buf) { vtb::set_debug_tstamp(d_buf); }

// Testing only (not in include/viterbi_amd.h): a device word (uint32) to which every traceback
// completeness guard that fires in later launches adds 1 -- a verified block-parallel chain left
// unproven after its round cap, its frame sent to the exact slow path (vtb_internal.h
// kDbgTbCap); nullptr turns it off.
void vtb_debug_set_guard_counter(uint32_t* d_word) { vtb::set_debug_guard_hits(d_word); }

// Testing only: the VTB_DEBUG bits a plan created now would carry.  The shipped library drops
// the output-corrupting bits 0-4 (vtb_internal.h kDbgUnsafe); a -DVTB_MEASURE build keeps them.
int vtb_debug_effective_flags(void) { return vtb::read_knobs().dbg; }
int vtb_debug_measure_build(void) { return vtb::kDbgHonoured == ~0 ? 1 : 0; }

// Measurement only (not in include/viterbi_amd.h): frames of the plan's last persistent split
// launch that did not converge split (re-decoded by the list kernel); synchronises the device.
long long vtb_debug_split_failures(vtb_plan_t* plan) {
    if (!plan || !plan->ws) return -1;
    DeviceGuard g(plan->device);
    uint32_t n = 0;
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&n, plan->ws, 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return n;
}

// Testing only (not in include/viterbi_amd.h): how vtb_decode_frame_sync calls ended, SEG
// kernel decoded / SEG not converged (re-decoded) / no SEG kernel for the plan.
static std::atomic<unsigned long long> g_seg_stats[3];
// adaptive single-frame warm-up: after a miss of the short warm-up, the plan's own for 64 calls,
// doubling per consecutive miss up to 4,096
constexpr int kSegBackoff0 = 64, kSegBackoffMax = 4096;
void vtb_debug_seg_stats(unsigned long long* out3) {
    for (int i = 0; i < 3; i++) out3[i] = g_seg_stats[i].load();
}

const char* vtb_strerror(int err) {
    switch (err) {
        case VTB_OK: return "ok";
        case VTB_ERR_INVALID: return "invalid argument";
        case VTB_ERR_CODE: return "generator does not tap both the newest and the oldest input (no butterfly symmetry)";
        case VTB_ERR_UNSUPPORTED: return "unsupported code or frame length";
        case VTB_ERR_DEVICE: return "no usable gfx950 device or HIP runtime error";
        case VTB_ERR_NOMEM: return "out of memory";
        default: return "unknown error";
    }
}

int vtb_code_check(const vtb_code_t* code) { return check_code(code); }

int vtb_edge_table(const vtb_code_t* code, uint8_t* symm) {
    int e = check_code(code);
    if (e == VTB_ERR_CODE) e = VTB_OK;  // the table itself exists for any code
    if (e != VTB_OK) return e;
    if (!symm) return VTB_ERR_INVALID;
    edge_table(code, symm);
    return VTB_OK;
}

size_t vtb_input_bytes_per_frame(const vtb_code_t* code, vtb_input_t input, int32_t frame_bits) {
    if (!code || frame_bits < 1 || code->constraint_length < VTB_MIN_K || code->constraint_length > VTB_MAX_K) return 0;
    return in_bytes(code, input, frame_bits);
}

size_t vtb_output_bytes_per_frame(int32_t frame_bits) { return frame_bits < 1 ? 0 : out_bytes(frame_bits); }

int vtb_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int good = 0;
    for (int d = 0; d < n; d++) good += device_is_gfx950(d) ? 1 : 0;
    return good;
}

int vtb_plan_create(vtb_plan_t** plan, const vtb_code_t* code, vtb_input_t input, int32_t frame_bits, int device) {
    if (!plan) return VTB_ERR_INVALID;
    *plan = nullptr;
    int e = check_code(code);
    if (e != VTB_OK) return e;
    if (input != VTB_INPUT_HARD && input != VTB_INPUT_SOFT8) return VTB_ERR_INVALID;
    if (frame_bits < 1) return VTB_ERR_INVALID;
    if (frame_bits > VTB_MAX_FRAME_BITS) return VTB_ERR_UNSUPPORTED;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return VTB_ERR_DEVICE;
    if (!device_is_gfx950(device)) return VTB_ERR_DEVICE;
    vtb_plan* p = new (std::nothrow) vtb_plan();
    if (!p) return VTB_ERR_NOMEM;
    p->code = *code;
    p->input = input;
    p->L = frame_bits;
    p->T = frame_bits + code->constraint_length - 1;
    p->device = device;
    p->knobs = vtb::read_knobs();
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            p->cus = cus;
    }
    edge_table(code, p->symm);
    // Shape check up front so a plan that exists can always launch.
    vtb::Launch a;
    a.S = code->constraint_length - 1;
    a.soft = input == VTB_INPUT_SOFT8;
    a.T = p->T;
    a.L = p->L;
    if (!vtb::k7_lds_supported(a) && !vtb::k7_global_supported(a) && !vtb::k9_supported(a) &&
        !vtb::lds_path_supported(a)) {
        delete p;
        return VTB_ERR_UNSUPPORTED;
    }
    *plan = p;
    return VTB_OK;
}

void vtb_plan_destroy(vtb_plan_t* plan) {
    if (!plan) return;
    DeviceGuard g(plan->device);
    if (plan->d_in) (void)hipFree(plan->d_in);
    if (plan->d_out) (void)hipFree(plan->d_out);
    if (plan->lat_in || plan->lat_out || plan->lat_done) {
        if (plan->stream) (void)hipStreamSynchronize(plan->stream);
        if (plan->lat_in) (void)hipHostFree(plan->lat_in);
        if (plan->lat_out) (void)hipHostFree(plan->lat_out);
        if (plan->lat_done) (void)hipHostFree(plan->lat_done);
    }
    if (plan->seg9_ws) (void)hipFree(plan->seg9_ws);
    if (plan->ws) {
        (void)hipDeviceSynchronize();  // launches on any stream may still use it
        (void)vtb::workspace_free(plan->ws, nullptr);
        (void)hipStreamSynchronize(nullptr);
    }
    for (hipEvent_t e : plan->events) (void)hipEventDestroy(e);
    if (plan->copy_stream) (void)hipStreamDestroy(plan->copy_stream);
    if (plan->stream) (void)hipStreamDestroy(plan->stream);
    delete plan;
}

int vtb_decode_device(vtb_plan_t* plan, const uint8_t* d_in, size_t in_stride, uint8_t* d_out, size_t out_stride,
                      size_t frames, void* stream) {
    if (!plan) return VTB_ERR_INVALID;
    if (frames == 0) return VTB_OK;
    if (!d_in || !d_out) return VTB_ERR_INVALID;
    if (in_stride < in_bytes(&plan->code, plan->input, plan->L) || out_stride < out_bytes(plan->L))
        return VTB_ERR_INVALID;
    DeviceGuard g(plan->device);
    if (!g.ok) return VTB_ERR_DEVICE;
    return launch(plan, d_in, in_stride, d_out, out_stride, frames, static_cast<hipStream_t>(stream));
}

int vtb_decode_host(vtb_plan_t* plan, const uint8_t* h_in, uint8_t* h_out, size_t frames) {
    if (!plan) return VTB_ERR_INVALID;
    if (frames == 0) return VTB_OK;
    if (!h_in || !h_out) return VTB_ERR_INVALID;
    DeviceGuard g(plan->device);
    if (!g.ok) return VTB_ERR_DEVICE;
    const size_t ib = in_bytes(&plan->code, plan->input, plan->L), ob = out_bytes(plan->L);
    if (!plan->stream && hipStreamCreateWithFlags(&plan->stream, hipStreamNonBlocking) != hipSuccess)
        return VTB_ERR_DEVICE;
    if (frames > plan->cap_frames) {
        if (plan->d_in) (void)hipFree(plan->d_in);
        if (plan->d_out) (void)hipFree(plan->d_out);
        plan->d_in = plan->d_out = nullptr;
        plan->cap_frames = 0;
        if (hipMalloc(&plan->d_in, frames * ib) != hipSuccess) return VTB_ERR_NOMEM;
        if (hipMalloc(&plan->d_out, frames * ob) != hipSuccess) return VTB_ERR_NOMEM;
        plan->cap_frames = frames;
    }
    // After the first asynchronous operation every error exit drains both streams first:
    // queued copies still read h_in / write h_out, which the caller may free on error.
    auto fail = [&](int e) {
        if (plan->copy_stream) (void)hipStreamSynchronize(plan->copy_stream);
        (void)hipStreamSynchronize(plan->stream);
        return e;
    };
    // Large batches in chunks: the H2D copy of chunk i + 1 (copy stream) overlaps the decode of
    // chunk i (plan stream); every output copy follows its chunk's decode.  Small batches (one
    // launch round) in one piece.
    const size_t kChunkFrames = 16384;
    const size_t nch = frames <= 2 * kChunkFrames ? 1 : (frames + kChunkFrames - 1) / kChunkFrames;
    if (nch == 1) {
        if (hipMemcpyAsync(plan->d_in, h_in, frames * ib, hipMemcpyHostToDevice, plan->stream) != hipSuccess)
            return fail(VTB_ERR_DEVICE);
        int e = launch(plan, plan->d_in, ib, plan->d_out, ob, frames, plan->stream);
        if (e != VTB_OK) return fail(e);
        if (hipMemcpyAsync(h_out, plan->d_out, frames * ob, hipMemcpyDeviceToHost, plan->stream) != hipSuccess)
            return fail(VTB_ERR_DEVICE);
        return hipStreamSynchronize(plan->stream) == hipSuccess ? VTB_OK : VTB_ERR_DEVICE;
    }
    if (!plan->copy_stream && hipStreamCreateWithFlags(&plan->copy_stream, hipStreamNonBlocking) != hipSuccess)
        return VTB_ERR_DEVICE;
    while (plan->events.size() < 2 * nch) {
        hipEvent_t ev;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return VTB_ERR_DEVICE;
        plan->events.push_back(ev);
    }
    for (size_t i = 0; i < nch; i++) {
        const size_t lo = i * kChunkFrames, n = frames - lo < kChunkFrames ? frames - lo : kChunkFrames;
        hipEvent_t copied = plan->events[2 * i], decoded = plan->events[2 * i + 1];
        if (hipMemcpyAsync(plan->d_in + lo * ib, h_in + lo * ib, n * ib, hipMemcpyHostToDevice, plan->copy_stream) !=
                hipSuccess ||
            hipEventRecord(copied, plan->copy_stream) != hipSuccess ||
            hipStreamWaitEvent(plan->stream, copied, 0) != hipSuccess)
            return fail(VTB_ERR_DEVICE);
        int e = launch(plan, plan->d_in + lo * ib, ib, plan->d_out + lo * ob, ob, n, plan->stream);
        if (e != VTB_OK) return fail(e);
        if (hipEventRecord(decoded, plan->stream) != hipSuccess) return fail(VTB_ERR_DEVICE);
    }
    for (size_t i = 0; i < nch; i++) {
        const size_t lo = i * kChunkFrames, n = frames - lo < kChunkFrames ? frames - lo : kChunkFrames;
        if (hipStreamWaitEvent(plan->copy_stream, plan->events[2 * i + 1], 0) != hipSuccess ||
            hipMemcpyAsync(h_out + lo * ob, plan->d_out + lo * ob, n * ob, hipMemcpyDeviceToHost,
                           plan->copy_stream) != hipSuccess)
            return fail(VTB_ERR_DEVICE);
    }
    const bool ok_copy = hipStreamSynchronize(plan->copy_stream) == hipSuccess;
    const bool ok_dec = hipStreamSynchronize(plan->stream) == hipSuccess;
    return ok_copy && ok_dec ? VTB_OK : VTB_ERR_DEVICE;
}

int vtb_decode_host_multi(const vtb_code_t* code, vtb_input_t input, int32_t frame_bits, const uint8_t* h_in,
                          uint8_t* h_out, size_t frames, uint32_t device_mask) {
    int e = check_code(code);
    if (e != VTB_OK) return e;
    if (frame_bits < 1) return VTB_ERR_INVALID;
    if (frames == 0) return VTB_OK;
    if (!h_in || !h_out) return VTB_ERR_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return VTB_ERR_DEVICE;
    std::vector<int> devs;
    for (int d = 0; d < ndev && d < 32; d++)
        if ((device_mask == 0 || ((device_mask >> d) & 1u)) && device_is_gfx950(d)) devs.push_back(d);
    if (devs.empty()) return VTB_ERR_DEVICE;
    const size_t ib = in_bytes(code, input, frame_bits), ob = out_bytes(frame_bits);
    const size_t G = devs.size();
    std::vector<int> rc(G, VTB_OK);
    std::vector<std::thread> th;
    for (size_t i = 0; i < G; i++) {
        // Contiguous shard [i*F/G, (i+1)*F/G): frames are independent, no collective.
        size_t lo = 0, hi = 0;
        (void)vtb_shard_range(frames, G, i, &lo, &hi);
        th.emplace_back([&, i, lo, hi]() {
            if (hi <= lo) return;
            vtb_plan_t* p = nullptr;
            std::mutex* busy = nullptr;
            {
                std::lock_guard<std::mutex> lk(g_plan_cache_mu);
                for (CachedPlan& c : g_plan_cache)
                    if (c.device == devs[i] && c.input == input && c.L == frame_bits && same_code(c.code, *code)) {
                        p = c.plan;
                        busy = c.busy.get();
                        break;
                    }
                if (!p) {
                    int r = vtb_plan_create(&p, code, input, frame_bits, devs[i]);
                    if (r != VTB_OK) {
                        rc[i] = r;
                        return;
                    }
                    g_plan_cache.push_back({*code, input, frame_bits, devs[i], p, std::make_unique<std::mutex>()});
                    busy = g_plan_cache.back().busy.get();
                }
            }
            std::lock_guard<std::mutex> use(*busy);
            rc[i] = vtb_decode_host(p, h_in + lo * ib, h_out + lo * ob, hi - lo);
        });
    }
    for (auto& t : th) t.join();
    for (int r : rc)
        if (r != VTB_OK) return r;
    return VTB_OK;
}

int vtb_shard_range(size_t frames, size_t shards, size_t index, size_t* lo, size_t* hi) {
    if (!lo || !hi || shards == 0 || index >= shards) return VTB_ERR_INVALID;
    // floor(F i / G) without overflowing F i (F < 2^64, G small): quotient and remainder parts
    auto bound = [&](size_t i) { return (frames / shards) * i + (frames % shards) * i / shards; };
    *lo = bound(index);
    *hi = bound(index + 1);
    return VTB_OK;
}

// vtb_decode_peer_multi's per-shard context: a stream and buffers on the shard's device, its
// own plan (shards on one device run concurrently, and a plan's workspace belongs to one
// stream), keyed by (device, occurrence of that device in the call's list).
namespace {
struct PeerCtx {
    int device = -1, slot = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    uint8_t* in = nullptr;
    uint8_t* out = nullptr;
    size_t cap_in = 0, cap_out = 0;
    vtb_plan_t* plan = nullptr;
};
std::mutex g_peer_mu;  // one vtb_decode_peer_multi call at a time (contexts are shared)
std::vector<std::unique_ptr<PeerCtx>> g_peer;
hipEvent_t g_peer_ready[64] = {};  // per source device: the caller's stream reached the call

PeerCtx* peer_ctx(int dev, int slot) {
    for (auto& c : g_peer)
        if (c->device == dev && c->slot == slot) return c.get();
    auto c = std::make_unique<PeerCtx>();
    c->device = dev, c->slot = slot;
    DeviceGuard g(dev);
    if (!g.ok || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return nullptr;
    if (hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) {
        (void)hipStreamDestroy(c->stream);
        return nullptr;
    }
    g_peer.push_back(std::move(c));
    return g_peer.back().get();
}

bool grow(uint8_t*& p, size_t& cap, size_t need) {
    if (need <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, need) != hipSuccess) return false;
    cap = need;
    return true;
}
}  // namespace

int vtb_decode_peer_multi(const vtb_code_t* code, vtb_input_t input, int32_t frame_bits, int src_device,
                          const uint8_t* d_in, uint8_t* d_out, size_t frames, const int* devices, int ndev,
                          uint32_t flags, void* stream) {
    int e = check_code(code);
    if (e != VTB_OK) return e;
    if (input != VTB_INPUT_HARD && input != VTB_INPUT_SOFT8) return VTB_ERR_INVALID;
    if (frame_bits < 1 || !devices || ndev < 1 || ndev > 64 || (flags & ~uint32_t(VTB_PEER_STAGE_ALL)))
        return VTB_ERR_INVALID;
    if (frames == 0) return VTB_OK;
    if (!d_in || !d_out) return VTB_ERR_INVALID;
    if (frame_bits > VTB_MAX_FRAME_BITS) return VTB_ERR_UNSUPPORTED;
    int nvis = 0;
    if (hipGetDeviceCount(&nvis) != hipSuccess || src_device < 0 || src_device >= nvis || src_device >= 64 ||
        !device_is_gfx950(src_device))
        return VTB_ERR_DEVICE;
    for (int i = 0; i < ndev; i++) {
        const int d = devices[i];
        if (d < 0 || d >= nvis || !device_is_gfx950(d)) return VTB_ERR_DEVICE;
        if (d != src_device) {
            // the shard crosses xGMI both ways: peer access in both directions or nothing
            int a = 0, b = 0;
            if (hipDeviceCanAccessPeer(&a, d, src_device) != hipSuccess ||
                hipDeviceCanAccessPeer(&b, src_device, d) != hipSuccess || !a || !b)
                return VTB_ERR_UNSUPPORTED;
        }
    }
    const size_t ib = in_bytes(code, input, frame_bits), ob = out_bytes(frame_bits);
    std::lock_guard<std::mutex> lk(g_peer_mu);
    hipStream_t cs = static_cast<hipStream_t>(stream);
    {
        DeviceGuard g(src_device);
        if (!g.ok) return VTB_ERR_DEVICE;
        if (!g_peer_ready[src_device] &&
            hipEventCreateWithFlags(&g_peer_ready[src_device], hipEventDisableTiming) != hipSuccess) {
            g_peer_ready[src_device] = nullptr;
            return VTB_ERR_DEVICE;
        }
        if (hipEventRecord(g_peer_ready[src_device], cs) != hipSuccess) return VTB_ERR_DEVICE;
    }
    std::vector<PeerCtx*> used;
    int rc = VTB_OK;
    for (int i = 0; i < ndev && rc == VTB_OK; i++) {
        const int d = devices[i];
        int slot = 0;
        for (int j = 0; j < i; j++) slot += devices[j] == d ? 1 : 0;
        size_t lo = 0, hi = 0;
        (void)vtb_shard_range(frames, size_t(ndev), size_t(i), &lo, &hi);
        if (hi <= lo) continue;
        const size_t n = hi - lo;
        PeerCtx* c = peer_ctx(d, slot);
        if (!c) {
            rc = VTB_ERR_DEVICE;
            break;
        }
        DeviceGuard g(d);
        if (!g.ok) {
            rc = VTB_ERR_DEVICE;
            break;
        }
        if (d != src_device) {
            // enable both directions once (already-enabled is not an error)
            hipError_t pe = hipDeviceEnablePeerAccess(src_device, 0);
            if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) {
                rc = VTB_ERR_DEVICE;
                break;
            }
            (void)hipGetLastError();
            DeviceGuard gs(src_device);
            pe = hipDeviceEnablePeerAccess(d, 0);
            if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) {
                rc = VTB_ERR_DEVICE;
                break;
            }
            (void)hipGetLastError();
        }
        if (!c->plan || c->plan->L != frame_bits || c->plan->input != input || !same_code(c->plan->code, *code)) {
            vtb_plan_destroy(c->plan);
            c->plan = nullptr;
            if ((rc = vtb_plan_create(&c->plan, code, input, frame_bits, d)) != VTB_OK) {
                c->plan = nullptr;
                break;
            }
        }
        if (hipStreamWaitEvent(c->stream, g_peer_ready[src_device], 0) != hipSuccess) {
            rc = VTB_ERR_DEVICE;
            break;
        }
        used.push_back(c);
        if (d == src_device && !(flags & VTB_PEER_STAGE_ALL)) {
            rc = launch(c->plan, d_in + lo * ib, ib, d_out + lo * ob, ob, n, c->stream);  // in place
        } else {
            if (!grow(c->in, c->cap_in, n * ib) || !grow(c->out, c->cap_out, n * ob)) {
                rc = VTB_ERR_NOMEM;
            } else if (hipMemcpyPeerAsync(c->in, d, d_in + lo * ib, src_device, n * ib, c->stream) != hipSuccess) {
                rc = VTB_ERR_DEVICE;  // scatter (xGMI)
            } else if ((rc = launch(c->plan, c->in, ib, c->out, ob, n, c->stream)) == VTB_OK &&
                       hipMemcpyPeerAsync(d_out + lo * ob, src_device, c->out, d, n * ob, c->stream) != hipSuccess) {
                rc = VTB_ERR_DEVICE;  // gather of the decoded bytes (xGMI)
            }
        }
        if (hipEventRecord(c->done, c->stream) != hipSuccess && rc == VTB_OK) rc = VTB_ERR_DEVICE;
    }
    // the caller's stream waits for every shard (also after an error: queued copies still
    // touch the caller's buffers)
    DeviceGuard g(src_device);
    for (PeerCtx* c : used)
        if (hipStreamWaitEvent(cs, c->done, 0) != hipSuccess && rc == VTB_OK) rc = VTB_ERR_DEVICE;
    if (rc != VTB_OK)
        for (PeerCtx* c : used) (void)hipStreamSynchronize(c->stream);
    return rc;
}

void vtb_release_cached_plans(void) {
    std::lock_guard<std::mutex> lk(g_plan_cache_mu);
    for (CachedPlan& c : g_plan_cache) {
        std::lock_guard<std::mutex> use(*c.busy);
        vtb_plan_destroy(c.plan);
    }
    g_plan_cache.clear();
    std::lock_guard<std::mutex> pk(g_peer_mu);
    for (auto& c : g_peer) {
        DeviceGuard g(c->device);
        if (c->stream) (void)hipStreamSynchronize(c->stream);
        vtb_plan_destroy(c->plan);
        if (c->in) (void)hipFree(c->in);
        if (c->out) (void)hipFree(c->out);
        if (c->done) (void)hipEventDestroy(c->done);
        if (c->stream) (void)hipStreamDestroy(c->stream);
    }
    g_peer.clear();
}

int vtb_stream_create(vtb_stream_t** sp, const vtb_code_t* code, vtb_input_t input, size_t streams,
                      int32_t window_steps, int device) {
    if (!sp) return VTB_ERR_INVALID;
    *sp = nullptr;
    int e = check_code(code);
    if (e != VTB_OK) return e;
    const int K = code->constraint_length;
    // K = 7 and K = 9: their own kernels (survivor words packed per 48-step chunk, a carry of
    // < 48 segments between calls); every other K (and K = 7 / 9 with VTB_KERNEL=lds, for
    // testing): the generic stream kernel, all segments of a call at once
    const vtb::Knobs knobs = vtb::read_knobs();
    const bool gen = (K != 7 && K != 9) || knobs.force == vtb::Force::Lds;
    const bool k9 = K == 9 && !gen;
    if (input != VTB_INPUT_HARD && input != VTB_INPUT_SOFT8) return VTB_ERR_INVALID;
    if (streams == 0 || streams > (size_t(1) << 31)) return VTB_ERR_INVALID;
    // default window: 49,152 steps (K = 7, 768 KB per wave) / 12,288 (K = 9, 64 B per step:
    // the same 768 KB; K = 9 survivor paths merge within a few hundred steps at useful SNR);
    // generic: 16,416 steps (8 B per step and wave for up to 64 states, 16 B at K = 8, 9)
    const int64_t win = window_steps <= 0 ? (gen ? 16416 : k9 ? 12288 : 49152) : (int64_t(window_steps) + 47) / 48 * 48;
    if (win < 96 || win > (int64_t(1) << (k9 ? 25 : 27))) return VTB_ERR_INVALID;  // 32-bit ring offsets
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return VTB_ERR_DEVICE;
    if (!device_is_gfx950(device)) return VTB_ERR_DEVICE;
    DeviceGuard g(device);
    if (!g.ok) return VTB_ERR_DEVICE;
    vtb_stream* s = new (std::nothrow) vtb_stream();
    if (!s) return VTB_ERR_NOMEM;
    s->code = *code;
    s->input = input;
    s->streams = streams;
    s->ring = int(win);
    s->device = device;
    s->gen = gen;
    s->knobs = knobs;
    edge_table(code, s->symm);
    if (gen) {
        const int S = K - 1;
        const size_t gw = vtb::gen_stream_waves(S, streams);
        const size_t sw = size_t(vtb::gen_stream_state_words(S));
        if (hipMalloc(&s->d_state, gw * sw * 4) != hipSuccess ||
            hipMalloc(&s->d_ring, gw * vtb::gen_stream_ring_bytes_per_step(S) * size_t(s->ring)) != hipSuccess) {
            vtb_stream_destroy(s);
            return VTB_ERR_NOMEM;
        }
        if (hipMemset(s->d_state, 0, gw * sw * 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            vtb_stream_destroy(s);
            return VTB_ERR_DEVICE;
        }
        *sp = s;
        return VTB_OK;
    }
    const size_t waves = (streams + 1) / 2;
    const size_t sw = k9 ? vtb::kStreamStateWords9 : vtb::kStreamStateWords, step_bytes = k9 ? 64 : 16;
    if (hipMalloc(&s->d_state, waves * sw * 4) != hipSuccess ||
        hipMalloc(&s->d_carry, streams * vtb::kStreamCarryStride) != hipSuccess ||
        hipMalloc(&s->d_ring, waves * step_bytes * size_t(s->ring)) != hipSuccess) {
        vtb_stream_destroy(s);
        return VTB_ERR_NOMEM;
    }
    // completed before returning: the calls run on the caller's streams, which a null-stream
    // memset does not order when they are non-blocking
    if (hipMemset(s->d_state, 0, waves * sw * 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        vtb_stream_destroy(s);
        return VTB_ERR_DEVICE;
    }
    *sp = s;
    return VTB_OK;
}

void vtb_stream_destroy(vtb_stream_t* s) {
    if (!s) return;
    DeviceGuard g(s->device);
    (void)hipDeviceSynchronize();  // calls on any stream may still use the buffers
    if (s->d_state) (void)hipFree(s->d_state);
    if (s->d_carry) (void)hipFree(s->d_carry);
    if (s->d_ring) (void)hipFree(s->d_ring);
    delete s;
}

size_t vtb_stream_out_bytes(const vtb_stream_t* s) { return s ? size_t(s->ring) / 8 + 8 : 0; }

int vtb_stream_decode(vtb_stream_t* s, const uint8_t* d_in, size_t in_stride, int32_t segments, int last,
                      uint8_t* d_out, size_t out_stride, int32_t* d_out_bits, void* stream) {
    if (!s || segments < 0 || !d_out || !d_out_bits || (segments > 0 && !d_in)) return VTB_ERR_INVALID;
    const int sb = s->input == VTB_INPUT_SOFT8 ? 2 : 1;
    if (segments > 0 && in_stride < size_t(segments) * sb) return VTB_ERR_INVALID;
    if (out_stride < vtb_stream_out_bytes(s)) return VTB_ERR_INVALID;
    if (segments > s->ring - 48) return VTB_ERR_INVALID;
    if (s->gen) {
        // generic kernel: every segment of the call at once, no carry
        const int64_t T = int64_t(s->t_begin) + segments;
        if (T > int64_t(1) << 30) return VTB_ERR_UNSUPPORTED;
        if (last && T < s->code.constraint_length) return VTB_ERR_INVALID;  // a frame needs L >= 1
        DeviceGuard g(s->device);
        if (!g.ok) return VTB_ERR_DEVICE;
        hipStream_t hs = static_cast<hipStream_t>(stream);
        if (!last && segments == 0) {
            if (hipMemsetAsync(d_out_bits, 0, s->streams * sizeof(int32_t), hs) != hipSuccess) return VTB_ERR_DEVICE;
            return VTB_OK;
        }
        vtb::Launch a;
        a.S = s->code.constraint_length - 1;
        a.soft = sb == 2;
        a.T = int(T);
        a.L = int(T) - a.S;
        a.in = d_in;
        a.in_stride = in_stride;
        a.out = d_out;
        a.out_stride = out_stride;
        a.frames = s->streams;
        a.stream = hs;
        a.ws = s->d_ring;
        a.dbg = s->knobs.dbg;
        a.guard_hits = vtb::debug_guard_hits();
        std::memcpy(a.symm, s->symm, sizeof(a.symm));
        vtb::StreamArgs sa;
        sa.state = s->d_state;
        sa.t_begin = s->t_begin;
        sa.t_end = int(T);
        sa.last = last ? 1 : 0;
        sa.ring = s->ring;
        sa.out_bits = d_out_bits;
        if (vtb::launch_gen_stream(a, sa) != hipSuccess) return VTB_ERR_DEVICE;
        s->t_begin = last ? 0 : int(T);
        return VTB_OK;
    }
    const int rows = s->carry_len + segments;  // < ring
    const int64_t T = int64_t(s->t_begin) + rows;
    if (T > int64_t(1) << 30) return VTB_ERR_UNSUPPORTED;
    if (last && T < s->code.constraint_length) return VTB_ERR_INVALID;  // a frame needs L >= 1
    const int nproc = last ? (rows + 47) / 48 * 48 : rows / 48 * 48;
    const int t_end = s->t_begin + nproc;
    DeviceGuard g(s->device);
    if (!g.ok) return VTB_ERR_DEVICE;
    hipStream_t hs = static_cast<hipStream_t>(stream);
    if (!last && nproc == 0) {
        // nothing to decode yet: no bits this call
        if (hipMemsetAsync(d_out_bits, 0, s->streams * sizeof(int32_t), hs) != hipSuccess) return VTB_ERR_DEVICE;
    } else {
        vtb::Launch a;
        a.S = s->code.constraint_length - 1;
        a.soft = sb == 2;
        a.T = int(T);
        a.L = int(T) - a.S;
        a.in = d_in;
        a.in_stride = in_stride;
        a.out = d_out;
        a.out_stride = out_stride;
        a.frames = s->streams;
        a.stream = hs;
        a.ws = s->d_ring;
        a.dbg = s->knobs.dbg;
        a.guard_hits = vtb::debug_guard_hits();
        std::memcpy(a.symm, s->symm, sizeof(a.symm));
        vtb::StreamArgs sa;
        sa.state = s->d_state;
        sa.carry = s->d_carry;
        sa.carry_len = s->carry_len;
        sa.t_begin = s->t_begin;
        sa.t_end = t_end;
        sa.last = last ? 1 : 0;
        sa.ring = s->ring;
        sa.out_bits = d_out_bits;
        if ((a.S == 8 ? vtb::launch_k9_stream(a, sa) : vtb::launch_k7_stream(a, sa)) != hipSuccess) return VTB_ERR_DEVICE;
    }
    // rows received past the last whole 48-step chunk wait in the carry for the next call
    const int leftover = last ? 0 : rows - nproc;
    if (leftover > 0) {
        const int first = rows - leftover;  // first leftover row: in the carry only if nothing was decoded
        const uint8_t* src = nproc == 0 ? d_in : d_in + size_t(first - s->carry_len) * sb;
        uint8_t* dst = s->d_carry + size_t(nproc == 0 ? s->carry_len : 0) * sb;
        const int width = (nproc == 0 ? segments : leftover) * sb;
        if (width > 0 && hipMemcpy2DAsync(dst, vtb::kStreamCarryStride, src, in_stride, size_t(width), s->streams,
                                          hipMemcpyDeviceToDevice, hs) != hipSuccess)
            return VTB_ERR_DEVICE;
    }
    if (last) {
        s->t_begin = 0;
        s->carry_len = 0;
    } else {
        s->t_begin = t_end;
        s->carry_len = leftover;
    }
    return VTB_OK;
}

// A failed first call leaves no half-built single-frame state: the next call starts over.
static int lat_undo(vtb_plan_t* plan, int err) {
    if (plan->seg9_ws) (void)hipFree(plan->seg9_ws);
    if (plan->lat_in) (void)hipHostFree(plan->lat_in);
    if (plan->lat_out) (void)hipHostFree(plan->lat_out);
    if (plan->lat_done) (void)hipHostFree(plan->lat_done);
    plan->seg9_ws = nullptr;
    plan->seg9_wgs = plan->seg9_waves = 0;
    plan->segg_waves = plan->segg_wgs = 0;
    plan->lat_in = plan->lat_out = nullptr;
    plan->lat_done = nullptr;
    plan->lat_d_in = plan->lat_d_out = nullptr;
    plan->lat_d_done = nullptr;
    return err;
}

int vtb_decode_frame_sync(vtb_plan_t* plan, const uint8_t* h_in, uint8_t* h_out) {
    if (!plan || !h_in || !h_out) return VTB_ERR_INVALID;
    DeviceGuard g(plan->device);
    if (!g.ok) return VTB_ERR_DEVICE;
    const size_t ib = in_bytes(&plan->code, plan->input, plan->L), ob = out_bytes(plan->L);
    if (!plan->stream && hipStreamCreateWithFlags(&plan->stream, hipStreamNonBlocking) != hipSuccess)
        return VTB_ERR_DEVICE;
    if (!plan->lat_in) {
        // coherent (fine-grained) host memory: the kernel's reads see this call's bytes and its
        // writes reach the host without a cache flush; input padded to the kernel's 16-byte loads
        const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
        if (hipHostMalloc(reinterpret_cast<void**>(&plan->lat_in), (ib + 32) / 16 * 16, fl) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&plan->lat_out), ob + 16, fl) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&plan->lat_done), 64, fl) != hipSuccess) {
            if (plan->lat_in) (void)hipHostFree(plan->lat_in);
            if (plan->lat_out) (void)hipHostFree(plan->lat_out);
            if (plan->lat_done) (void)hipHostFree(plan->lat_done);
            plan->lat_in = plan->lat_out = nullptr;
            plan->lat_done = nullptr;
            return VTB_ERR_NOMEM;
        }
        std::memset(plan->lat_in, 0, (ib + 32) / 16 * 16);
        // SEG kernel geometry, once per plan ($VTB_SEG_WAVES / $VTB_SEG_WARM in the plan's knobs:
        // measurement): eight waves (two per SIMD, 16 segments: 128.5 against 120 Mbit/s for four
        // in the reference's speedDecode); four where eight waves' survivor words
        // do not fit the CU's LDS (frames past about 12,000 bits)
        const vtb::Knobs& kn = plan->knobs;
        int waves = kn.seg_waves > 0 ? kn.seg_waves : 8, warm = kn.seg_warm > 0 ? kn.seg_warm : vtb::kSegWarm;
        vtb::Launch a;
        a.S = plan->code.constraint_length - 1;
        a.soft = plan->input == VTB_INPUT_SOFT8;
        a.T = plan->T;
        a.L = plan->L;
        const bool any = kn.force == vtb::Force::Any || kn.force == vtb::Force::Seg;
        if (kn.seg_waves <= 0 && !vtb::k7_seg_supported(a, waves, warm)) waves = 4;
        plan->seg_waves = any && !(kn.dbg & 1024) && vtb::k7_seg_supported(a, waves, warm) ? waves : 0;
        plan->seg_warm = warm;
        // $VTB_SEG_ADAPT=0: the plan's warm-up only (measurement)
        const bool short_ok = kn.seg_warm <= 0 && kn.seg_adapt;
        plan->seg_short = short_ok && plan->seg_waves > 0 && vtb::k7_seg_supported(a, waves, vtb::kSegWarmShort);
        plan->seg_backoff = kSegBackoff0;
        // K = 9: the frame over several workgroups ($VTB_SEG9_WGS / _WAVES: measurement)
        const int wgs = kn.seg9_wgs > 0 ? kn.seg9_wgs : vtb::kSeg9Wgs, w9 = kn.seg9_waves > 0 ? kn.seg9_waves : vtb::kSeg9Waves;
        if (any && !(kn.dbg & 1024) && vtb::k9_seg_supported(a, w9, wgs, vtb::kSeg9Warm)) {
            const bool s9 = short_ok && vtb::k9_seg_supported(a, w9, wgs, vtb::kSegWarmShort);
            const size_t wsb = std::max(vtb::k9_seg_workspace_bytes(a, w9, wgs, vtb::kSeg9Warm),
                                        s9 ? vtb::k9_seg_workspace_bytes(a, w9, wgs, vtb::kSegWarmShort) : size_t(0));
            plan->seg_short = s9;
            if (hipMalloc(&plan->seg9_ws, wsb) != hipSuccess) {
                plan->seg9_ws = nullptr;
                return lat_undo(plan, VTB_ERR_NOMEM);
            }
            // the arrival counter, zeroed in stream order before the first SEG launch (a plain
            // hipMemset runs on the null stream, which does not order the non-blocking plan
            // stream: a launch could add to the counter before the zero landed, so that no
            // workgroup is elected and the completion word is never written)
            if (hipMemsetAsync(plan->seg9_ws, 0, 256, plan->stream) != hipSuccess) return lat_undo(plan, VTB_ERR_DEVICE);
            plan->seg9_wgs = wgs;
            plan->seg9_waves = w9;
        }
        // every other K (3..6, 8): the generic kernel's segments, eight waves ($VTB_SEG_WAVES:
        // measurement), the short warm-up first as above; K = 6, 8 over kSegGenWgs workgroups
        // (one workgroup's slots give 16 / 8 segments; $VTB_SEGG_WGS: measurement)
        if (any && !(kn.dbg & 1024) && plan->seg_waves == 0 && plan->seg9_wgs == 0) {
            const int wg = kn.seg_waves > 0 ? kn.seg_waves : 8;
            int nwg = kn.segg_wgs > 0 ? kn.segg_wgs : (a.S >= 5 ? vtb::kSegGenWgs : 1);
            if (nwg > 1 && !vtb::gen_seg_supported(a, wg, nwg, warm)) nwg = 1;
            if (vtb::gen_seg_supported(a, wg, nwg, warm)) {
                const bool sg_short = short_ok && vtb::gen_seg_supported(a, wg, nwg, vtb::kSegWarmShort);
                if (nwg > 1) {
                    const size_t wsb = std::max(vtb::gen_seg_workspace_bytes(a, wg, nwg, warm),
                                                sg_short ? vtb::gen_seg_workspace_bytes(a, wg, nwg, vtb::kSegWarmShort)
                                                         : size_t(0));
                    if (hipMalloc(&plan->seg9_ws, wsb) != hipSuccess) {
                        plan->seg9_ws = nullptr;
                        return lat_undo(plan, VTB_ERR_NOMEM);
                    }
                    // (the arrival counter zeroed in stream order, as for K = 9 above)
                    if (hipMemsetAsync(plan->seg9_ws, 0, 256, plan->stream) != hipSuccess)
                        return lat_undo(plan, VTB_ERR_DEVICE);
                }
                plan->segg_waves = wg;
                plan->segg_wgs = nwg;
                plan->seg_short = sg_short;
            }
        }
        if (hipHostGetDevicePointer(reinterpret_cast<void**>(&plan->lat_d_in), plan->lat_in, 0) != hipSuccess ||
            hipHostGetDevicePointer(reinterpret_cast<void**>(&plan->lat_d_out), plan->lat_out, 0) != hipSuccess ||
            hipHostGetDevicePointer(reinterpret_cast<void**>(&plan->lat_d_done), plan->lat_done, 0) != hipSuccess)
            return lat_undo(plan, VTB_ERR_DEVICE);
    }
    uint8_t *d_in = plan->lat_d_in, *d_out = plan->lat_d_out;
    uint32_t* d_done = plan->lat_d_done;
    if (!d_in || !d_out || !d_done) return VTB_ERR_DEVICE;
    std::memcpy(plan->lat_in, h_in, ib);
    volatile uint32_t* done = plan->lat_done;
    uint32_t status = 0;
    // one SEG launch at warm-up `warm`, waited for on the completion word: 1 decoded, 2 a
    // segment boundary did not converge (nothing written), 0 with an error
    auto run_seg = [&](int warm, int& st) -> int {
        *done = 0;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        vtb::Launch a;
        a.S = plan->code.constraint_length - 1;
        a.soft = plan->input == VTB_INPUT_SOFT8;
        a.T = plan->T;
        a.L = plan->L;
        a.in = d_in;
        a.in_stride = ib;
        a.out = d_out;
        a.out_stride = ob;
        a.frames = 1;
        a.stream = plan->stream;
        a.cus = plan->cus;
        a.dbg = plan->knobs.dbg;
        a.seg9_xcd = plan->knobs.seg9_xcd;
        a.guard_hits = vtb::debug_guard_hits();
        a.tstamp = vtb::debug_tstamp();  // (measurement only: gen_seg's phase times)
        std::memcpy(a.symm, plan->symm, sizeof(a.symm));
        if (plan->seg_waves > 0) {
            if (vtb::launch_k7_seg(a, plan->seg_waves, warm, d_done) != hipSuccess) return VTB_ERR_DEVICE;
        } else if (plan->segg_waves > 0) {
            a.ws = plan->seg9_ws;
            if (vtb::launch_gen_seg(a, plan->segg_waves, plan->segg_wgs, warm, d_done) != hipSuccess)
                return VTB_ERR_DEVICE;
        } else {
            a.ws = plan->seg9_ws;
            if (vtb::launch_k9_seg(a, plan->seg9_waves, plan->seg9_wgs, warm, d_done) != hipSuccess)
                return VTB_ERR_DEVICE;
        }
        // wait on the completion word (the kernel's last write); a call that takes longer than
        // ~2 ms (first launch: code-object load) synchronises the stream instead
        const auto t0 = std::chrono::steady_clock::now();
        uint32_t v;
        for (uint32_t spin = 0; (v = *done) == 0; spin++) {
            if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
                if (hipStreamSynchronize(plan->stream) != hipSuccess) return VTB_ERR_DEVICE;
                v = *done;
                if (v == 0) return VTB_ERR_DEVICE;  // finished without reporting
                break;
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        st = int(v);
        g_seg_stats[v == 1 ? 0 : 1]++;
        return VTB_OK;
    };
    if (plan->seg_waves > 0 || plan->seg9_wgs > 0 || plan->segg_waves > 0) {
        const int wsafe = plan->seg_waves > 0 || plan->segg_waves > 0 ? plan->seg_warm : vtb::kSeg9Warm;
        int st = 0;
        if (plan->seg_short && plan->seg_skip == 0) {
            // the short warm-up first: any converged decode is exact, a miss costs one more launch
            if (int r = run_seg(vtb::kSegWarmShort, st); r != VTB_OK) return r;
            if (st == 1) {
                plan->seg_backoff = kSegBackoff0;
            } else {
                plan->seg_skip = plan->seg_backoff;
                plan->seg_backoff = std::min(2 * plan->seg_backoff, kSegBackoffMax);
            }
        } else {
            if (plan->seg_skip > 0) plan->seg_skip--;
        }
        if (st != 1) {
            if (int r = run_seg(wsafe, st); r != VTB_OK) return r;
        }
        status = uint32_t(st);
    } else {
        g_seg_stats[2]++;
    }
    if (status != 1) {
        // not converged (status 2) or no SEG kernel for this plan: the frame kernel, input from
        // the same host-mapped buffer through one copy, output written straight to host memory
        if (!plan->d_in && hipMalloc(&plan->d_in, ib) != hipSuccess) return VTB_ERR_NOMEM;
        if (plan->cap_frames < 1) plan->cap_frames = 1;
        if (hipMemcpyAsync(plan->d_in, plan->lat_in, ib, hipMemcpyHostToDevice, plan->stream) != hipSuccess)
            return VTB_ERR_DEVICE;
        int r = launch(plan, plan->d_in, ib, d_out, ob, 1, plan->stream);
        if (r != VTB_OK) {
            (void)hipStreamSynchronize(plan->stream);
            return r;
        }
        if (hipStreamSynchronize(plan->stream) != hipSuccess) return VTB_ERR_DEVICE;
    }
    std::memcpy(h_out, plan->lat_out, ob);
    return VTB_OK;
}

int vtb_decode_frame_legacy(const vtb_code_t* code, const uint8_t* coded, int32_t segments, uint8_t* out) {
    if (!code || !coded || !out) return VTB_ERR_INVALID;
    int e = check_code(code);
    if (e == VTB_ERR_CODE) {
        // A generator without both end taps: the reference's butterfly still decodes it (the
        // caller skipped viterbiConfigCheck) with ē = n − e whatever the taps
        // (viterbiDecoderButterflyk1.c:101-152), which is not the code's Hamming metric.  That
        // arithmetic, uint8 wrap and renormalisation included, is the general-k kernel's
        // VTB_GENK_K1_REFERENCE_U8 mode.
        vtb_genk_code_t gc;
        std::memset(&gc, 0, sizeof(gc));
        gc.input_bits = 1;
        gc.constraint_length = code->constraint_length;
        gc.coded_bits = 2;
        gc.flags = VTB_GENK_K1_REFERENCE_U8;
        gc.generators[0] = code->generators[0];
        gc.generators[1] = code->generators[1];
        return vtb_genk_decode_frame_legacy(&gc, coded, segments, out);
    }
    if (e != VTB_OK) return e;
    const int32_t L = segments - (code->constraint_length - 1);
    if (L < 1) return VTB_ERR_INVALID;
    // One cached plan per host thread (the reference API is reentrant per state struct); the
    // frame goes through the plan's synchronous single-frame path.
    struct Cache {
        vtb_plan_t* plan = nullptr;
        ~Cache() { vtb_plan_destroy(plan); }
    };
    thread_local Cache cache;
    vtb_plan_t*& p = cache.plan;
    if (!p || p->code.constraint_length != code->constraint_length || p->code.generators[0] != code->generators[0] ||
        p->code.generators[1] != code->generators[1] || p->L != L) {
        vtb_plan_destroy(p);
        p = nullptr;
        int dev = 0;
        if (const char* s = std::getenv("VTB_LEGACY_DEVICE")) dev = std::atoi(s);
        int r = vtb_plan_create(&p, code, VTB_INPUT_HARD, L, dev);
        if (r != VTB_OK) {
            p = nullptr;
            return r;
        }
    }
    int r = vtb_decode_frame_sync(p, coded, out);
    if (r != VTB_OK) {
        // no half-built state survives a failure (the next call rebuilds)
        vtb_plan_destroy(p);
        p = nullptr;
        return r;
    }
    return (L - 1) / 8 + 1;  // src/viterbiDecoderButterflyk1.c:256
}

}  // extern "C"
