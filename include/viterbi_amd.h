/*
 * viterbi_amd.h -- C ABI of the MI355X (gfx950) batch Viterbi decoder.
 *
 * This is the drop-in boundary for the reference's hot path (SURVEY.md §8 b).  Plain C
 * types only: pointers, sizes, ints; a HIP stream travels as `void*`.  Everything is
 * runtime-parameterised (constraint length, generators, frame length, hard/soft), unlike
 * the reference, which fixes the code at compile time (src/defaultParams/convCodeParams.h).
 *
 * Reference interfaces each entry point replaces:
 *   vtb_code_check          viterbiConfigCheck            src/viterbiDecoder.c:9-30
 *                           (returns an error code instead of exit(1))
 *   vtb_edge_table          viterbiInitButterflyk1        src/viterbiDecoderButterflyk1.c:8-44
 *   vtb_decode_device /     viterbiDecoderHardButterflyk1 src/viterbiDecoderButterflyk1.c:82-263
 *   vtb_decode_host /       (one terminated frame per call with last=true, batched here
 *   vtb_decode_host_multi /  over many frames; hard input is the reference byte-per-segment
 *   vtb_decode_peer_multi
 *                            layout; soft input is the build-defined 8-bit extension)
 *   vtb_decode_frame_sync   the same, one frame from host memory, synchronous, lowest latency
 *   vtb_decode_frame_legacy the same, one frame from host memory, for the legacy shim
 *                           behind include/viterbiDecoder.h (VITERBI_DECODER_HARD)
 *   vtb_legacy_metrics_k1   the metric update of a last=false call (:101-191), so the
 *                           legacy nodeMetricsCur reads as the reference's between calls
 *   vtb_legacy_metrics_genk the generic decoder's metric update   src/viterbiDecoder.c:84-131
 *   vtb_genk_decode_frame_legacy  viterbiDecoderHard, one k>1 frame  src/viterbiDecoder.c:52-234
 *   vtb_stream_*            the same function called chunk by chunk with last = false and
 *                           then last = true (:85-196 keep the state across calls), batched
 *                           over streams, with the block traceback the reference leaves TODO
 *                           (:195,199)
 *   vtb_encode_device       convEnc                       src/convEncode.c:46-130
 *                           (whole terminated frames, batched on the device)
 *   vtb_payload_device /    the harnesses' random payloads and BSC corruption
 *   vtb_channel_device      (berTestK7.c:22-43, 135-138; speedDecode.c:38-60), re-specified
 *                           with a counter-based RNG so the device generates bulk frames
 *
 * Data layout (frame-major, reference layout per frame):
 *   hard input   T = L + K - 1 bytes per frame, byte t = coded segment t, bit i = output of
 *                generator g[i] (src/convEncode.c:153-159); only the low 2 bits are read
 *   soft input   2*T bytes per frame, byte 2t+i = q in [0,255] for coded bit i of segment t
 *                (0 = confident 0, 255 = confident 1; hard slice is q >= 128)
 *   output       ceil(L/8) bytes per frame, information bits MSB-first, last byte
 *                zero-padded (src/viterbiDecoderButterflyk1.c:226-249)
 *
 * Decisions are bit-exact with the reference C decoder for hard input (strict '>'
 * tie-break toward the lower predecessor, (uint8)(N+1) initial metric, full terminated
 * traceback from state 0).  Soft decisions follow DESIGN.md "Soft-decision format"; soft
 * input restricted to q in {0,255} reproduces the hard decoder bit for bit.
 *
 * Error convention: every function returns 0 (VTB_OK) or a negative VTB_ERR_* code; no
 * function prints or exits.  Thread-safety: plans are independent; one plan may be used
 * by one host thread at a time.
 */
#ifndef VITERBI_AMD_H
#define VITERBI_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VTB_OK 0
#define VTB_ERR_INVALID (-1)     /* bad argument (null pointer, L < 1, stride too small ...) */
#define VTB_ERR_CODE (-2)        /* generator violates the symmetric-butterfly precondition */
#define VTB_ERR_UNSUPPORTED (-3) /* K, n or frame length outside what the kernels handle */
#define VTB_ERR_DEVICE (-4)      /* no usable gfx950 device, or a HIP runtime error */
#define VTB_ERR_NOMEM (-5)       /* host or device allocation failed */

#define VTB_MIN_K 3
#define VTB_MAX_K 9
#define VTB_MAX_FRAME_BITS 16384 /* MAX_PKT_LEN_UNCODED_BITS, src/viterbiDecoder.h:18 */

typedef enum { VTB_INPUT_HARD = 0, VTB_INPUT_SOFT8 = 1 } vtb_input_t;

/* A rate-1/n, k=1 convolutional code (Proakis conventions, src/defaultParams/).  Field
 * names avoid the legacy config macros K, k, n, S so this header can be included next to
 * convCodeParams.h. */
typedef struct {
    int32_t constraint_length; /* K, VTB_MIN_K..VTB_MAX_K */
    int32_t coded_bits;        /* n, coded bits per segment; must be 2 */
    uint64_t generators[2];    /* g[], Proakis octal (MSB = newest input), e.g. {0113, 0171} */
} vtb_code_t;

typedef struct vtb_plan vtb_plan_t;

/* Library version string and a message for a VTB_ERR_* code. */
const char* vtb_version(void);
const char* vtb_strerror(int err);

/* 0 if the code is decodable by the symmetric butterfly (every g has its MSB and LSB set),
 * VTB_ERR_CODE if not, VTB_ERR_UNSUPPORTED / VTB_ERR_INVALID for bad K / n. */
int vtb_code_check(const vtb_code_t* code);

/* symm[i] = coded segment on the edge state i -> state 2i, i < 2^(K-2). */
int vtb_edge_table(const vtb_code_t* code, uint8_t* symm);

/* Bytes per frame in each layout (0 for invalid arguments). */
size_t vtb_input_bytes_per_frame(const vtb_code_t* code, vtb_input_t input, int32_t frame_bits);
size_t vtb_output_bytes_per_frame(int32_t frame_bits);

/* A plan binds a code, an input format, a frame length L (information bits) and a device
 * ordinal; it owns the device-side tables and any workspace. */
int vtb_plan_create(vtb_plan_t** plan, const vtb_code_t* code, vtb_input_t input, int32_t frame_bits,
                    int device);
void vtb_plan_destroy(vtb_plan_t* plan);

/* Decode `frames` frames already resident in device memory, asynchronously on `stream`
 * (a hipStream_t; NULL = default stream).  d_in: frames * in_stride bytes; d_out: frames *
 * out_stride bytes.  Strides >= the per-frame sizes above.  The plan's survivor workspace
 * (16-64 bytes per trellis step for each wave the device holds at once, grown on demand,
 * stream-ordered) is shared by its launches: calls on one plan must use one stream, or the
 * caller orders them. */
int vtb_decode_device(vtb_plan_t* plan, const uint8_t* d_in, size_t in_stride, uint8_t* d_out,
                      size_t out_stride, size_t frames, void* stream);

/* Host buffers (packed, stride = per-frame size): copy in, decode, copy out, synchronise.
 * Uses the plan's device. */
int vtb_decode_host(vtb_plan_t* plan, const uint8_t* h_in, uint8_t* h_out, size_t frames);

/* Host buffers sharded across the GPUs in device_mask (bit d = device d; 0 = all visible
 * devices): contiguous frame ranges, one host thread and stream per device, no
 * inter-device traffic (frames are independent).  The per-device plans (and their device
 * buffers, sized to the largest shard seen) are created on first use and kept for later
 * calls with the same code, input kind and frame length. */
int vtb_decode_host_multi(const vtb_code_t* code, vtb_input_t input, int32_t frame_bits, const uint8_t* h_in,
                          uint8_t* h_out, size_t frames, uint32_t device_mask);

/* Frees the plans vtb_decode_host_multi keeps and vtb_decode_peer_multi's per-device
 * contexts.  Not concurrently with either. */
void vtb_release_cached_plans(void);

/* Shard i of `shards` over `frames` frames: [*lo, *hi) = [floor(F i / G), floor(F (i+1) / G)),
 * contiguous, tiling [0, F), sizes differing by at most one.  The split every multi-GPU entry
 * point uses. */
int vtb_shard_range(size_t frames, size_t shards, size_t index, size_t* lo, size_t* hi);

/* Device-sourced sharding over xGMI (SURVEY.md §8 e, BASELINE config C5 fed from one GPU):
 * `frames` packed frames resident on src_device (d_in, d_out are device pointers there) are
 * split into ndev contiguous shards (vtb_shard_range), shard i decoded on devices[i]: a shard
 * on another GPU is copied there peer to peer (hipMemcpyPeerAsync over xGMI), decoded, and
 * its ceil(L/8)-byte rows copied back into d_out; a shard on src_device is decoded in place
 * (flags VTB_PEER_STAGE_ALL: staged through its own buffers like a peer shard -- testing and
 * A/B on one GPU).  A device may be listed more than once (one shard per entry).
 * Asynchronous on `stream` (a hipStream_t of src_device): the shards start after the work
 * queued there and `stream` waits for all of them.  VTB_ERR_UNSUPPORTED if a listed device
 * and src_device cannot access each other as peers (peer access is enabled on first use).
 * Per-(device, entry) streams, plans and buffers are kept for later calls
 * (vtb_release_cached_plans frees them); one call at a time. */
#define VTB_PEER_STAGE_ALL 1u
int vtb_decode_peer_multi(const vtb_code_t* code, vtb_input_t input, int32_t frame_bits, int src_device,
                          const uint8_t* d_in, uint8_t* d_out, size_t frames, const int* devices, int ndev,
                          uint32_t flags, void* stream);

/* One frame from host memory to host memory, synchronously, at the lowest latency: the
 * single-frame form of vtb_decode_host for callers that decode frame by frame (the legacy
 * VITERBI_DECODER_HARD contract, one frame per call).  h_in holds one frame in the plan's
 * input layout, h_out receives ceil(L/8) bytes.  K = 7 frames (T >= 240) are cut into up to
 * 16 segments decoded at once by the waves of one workgroup, K = 9 frames into up to 32 over
 * four workgroups (each segment after the first starts 48 or 96 steps early from equal metrics
 * and is used once its metrics provably match its predecessor's; otherwise the frame is decoded
 * again with the longer warm-up, then whole), reading the frame from and writing the bytes to
 * plan-owned host-mapped memory, with completion signalled through host memory instead of a
 * stream synchronisation.  Bit-exact with vtb_decode_host.  The plan's stream, buffers and
 * warm-up state are used: one host thread per plan at a time. */
int vtb_decode_frame_sync(vtb_plan_t* plan, const uint8_t* h_in, uint8_t* h_out);

/* One hard-input frame of `segments` coded segments from host memory (the legacy
 * VITERBI_DECODER_HARD contract).  Returns the reference's byte count
 * ((segments-K)/8 + 1) on success, or a negative VTB_ERR_* code.  Uses a per-thread
 * cached plan on device 0 (or $VTB_LEGACY_DEVICE). */
int vtb_decode_frame_legacy(const vtb_code_t* code, const uint8_t* coded, int32_t segments, uint8_t* out);

/* Number of gfx950 devices visible (0 if none); negative VTB_ERR_DEVICE on runtime error. */
int vtb_device_count(void);

/* ---- Streaming decode -------------------------------------------------
 * Replaces the reference's chunked protocol -- viterbiDecoderHardButterflyk1(state, coded,
 * out, segments, last) called with last = false for each chunk and last = true for the end
 * of the frame (src/viterbiDecoderButterflyk1.c:82-263) -- for a batch of independent
 * streams that advance in lockstep on the device, and adds what the reference leaves as
 * TODO (block traceback with early output, :195,199; src/viterbiDecoder.h:22-25):
 *   - each call pushes `segments` more coded segments per stream (row i of d_in, same layout
 *     as a frame's input: 1 byte per segment hard, 2 bytes soft), any count >= 0;
 *   - bits are emitted as soon as they are final: once the survivor paths of all states
 *     have merged behind them no later input can change them, so the concatenation of a
 *     frame's outputs equals the whole-frame decode (vtb_decode_*, the reference's output)
 *     bit for bit;
 *   - last != 0 ends the frame: the traceback from state 0 emits the rest (the reference's
 *     return of (segments - K)/8 + 1 bytes, last byte zero-padded), and every stream starts
 *     a new frame with the next call.  A frame has at least K segments in total.
 * Frames are not limited to VTB_MAX_FRAME_BITS: survivors live in a per-stream ring of
 * `window_steps` trellis steps (rounded up to a multiple of 48; <= 0: the default below) in
 * device memory.  Output bits wait until the paths merge; should a stream go window_steps
 * steps without a merge (pure-noise input), its frame is lost: d_out_bits reports -1 for it
 * until the call with last != 0, after which it restarts cleanly.
 * Every K in VTB_MIN_K..VTB_MAX_K; hard or soft input as for plans.  K = 7 and K = 9 run their
 * own kernels (the ring holds 16 or 64 bytes per step per pair of streams; window_steps <= 0
 * selects 49152 and 12288 steps); every other K the generic kernel (csrc/vtb_stream_gen.hip:
 * 64 / min(2^(K-1), 64) streams per wave, 8 bytes per step and wave up to K = 7, 16 at K = 8;
 * window_steps <= 0 selects 16416 steps). */
typedef struct vtb_stream vtb_stream_t;

int vtb_stream_create(vtb_stream_t** s, const vtb_code_t* code, vtb_input_t input, size_t streams,
                      int32_t window_steps, int device);
void vtb_stream_destroy(vtb_stream_t* s);

/* Bytes one call may write per output row (out_stride must be at least this). */
size_t vtb_stream_out_bytes(const vtb_stream_t* s);

/* One call, asynchronous on `stream` (a hipStream_t; one stream per object, or the caller
 * orders the calls).  d_in: streams rows of in_stride bytes (>= the segments' bytes); it
 * must stay valid until the call's work on `stream` completes.  Row i of d_out receives the
 * call's bits for stream i, MSB-first from bit 0 of byte 0; d_out_bits[i] (device int32)
 * their count: a multiple of 8 except on the last call of a frame, or -1 (window
 * overflow).  segments must not exceed window_steps - 48. */
int vtb_stream_decode(vtb_stream_t* s, const uint8_t* d_in, size_t in_stride, int32_t segments, int last,
                      uint8_t* d_out, size_t out_stride, int32_t* d_out_bits, void* stream);

/* ---- Synthetic frames on the device -------------------------------
 * Randomness is one counter-based stream, integer-exact on any host or device:
 *   mix64(x)                 = splitmix64 finalizer (x ^= x>>30; x *= 0xBF58476D1CE4E5B9;
 *                              x ^= x>>27; x *= 0x94D049BB133111EB; x ^= x>>31)
 *   vtb_rand64(seed, f, c)   = mix64(mix64(seed + 0x9E3779B97F4A7C15*(f+1)) ^ 0xD1B54A32D192ED03*(c+1))
 * Kernels run on the calling thread's current HIP device, asynchronously on `stream`. */
uint64_t vtb_rand64(uint64_t seed, uint64_t frame, uint64_t ctr);

/* Payload: byte j of frame f = byte (j mod 8) of vtb_rand64(seed, f, j / 8) (little-endian);
 * bits past frame_bits in the last byte are cleared (MSB-first packing). */
int vtb_payload_device(uint64_t seed, int32_t frame_bits, uint8_t* d_out, size_t stride, size_t frames,
                       void* stream);

/* convEnc (src/convEncode.c:46-130) on whole terminated frames: rows of ceil(L/8) payload
 * bytes (MSB-first) -> rows of L + K - 1 coded segment bytes (bit i = generator i), the last
 * K - 1 of them the zero tail.  Payload bits past L are ignored. */
int vtb_encode_device(const vtb_code_t* code, int32_t frame_bits, const uint8_t* d_uncoded, size_t in_stride,
                      uint8_t* d_coded, size_t out_stride, size_t frames, void* stream);

/* Channel over rows of `segments` hard coded segments:
 *   VTB_INPUT_HARD   BSC, param = crossover p: coded bit i of segment t flips iff 32-bit
 *                    half i of vtb_rand64(seed, f, t) < vtb_bsc_p32(p); output hard bytes.
 *   VTB_INPUT_SOFT8  BPSK (0 -> +1) + AWGN at param = SNR dB (sigma = sqrt(1/(2 Es/N0)),
 *                    Es/N0 = SNR + 10 log10 4, as berTestK7's SNR column) + the 8-bit soft
 *                    quantiser q = round((1 - y) * 127.5) clamped to [0, 255], in fixed
 *                    point: z_fx = sum of twelve 21-bit fields (bits 0-20, 21-41, 42-62 of
 *                    vtb_rand64(seed, f, 8t + 4i + h), h = 0..3) - 6*2^21;
 *                    q = clamp(floor((b*255*2^16 - floor(vtb_awgn_kq(snr) * z_fx / 2^21)
 *                    + 2^15) / 2^16), 0, 255); output 2 bytes per segment. */
int vtb_channel_device(vtb_input_t output, double param, uint64_t seed, const uint8_t* d_coded, size_t in_stride,
                       int32_t segments, uint8_t* d_rx, size_t out_stride, size_t frames, void* stream);

/* Fixed-point channel constants used above: round(sigma(snr) * 127.5 * 2^16) and
 * floor(p * 2^32) (saturating). */
int64_t vtb_awgn_kq(double snr_db);
uint32_t vtb_bsc_p32(double p);

/* ---- General rate-k/n codes (k input bits per trellis step) ----
 * Replaces the reference's generic decoder viterbiDecoderHard (src/viterbiDecoder.c:52-234,
 * src/viterbiDecoder.h:160), whose register-exchange traceback in uint8 registers drops
 * bits for k > 1; this one is terminated maximum likelihood over the same trellis (see
 * csrc/vtb_genk.hip).  The code uses the reference encoder's conventions
 * (src/convEncode.c:19-174): k bits per segment shifted in MSB-first, generators over k*K
 * bits (MSB = newest input bit), coded bit i of a segment = generator i, S = K-1 zero
 * segments of termination. */
typedef struct {
    int32_t input_bits;        /* k, 1..4 */
    int32_t constraint_length; /* K in k-bit segments; k*(K-1) <= 8 and k*K <= 12 */
    int32_t coded_bits;        /* n, 1..8 */
    int32_t flags;             /* 0 or VTB_GENK_K1_REFERENCE_U8 (was `reserved`, 0) */
    uint64_t generators[8];    /* g[0..n-1], each nonzero and below 2^(k*K) */
} vtb_genk_code_t;

/* k = 1 only: decode with the reference k=1 decoder's own arithmetic
 * (viterbiDecoderHardButterflyk1, src/viterbiDecoderButterflyk1.c:101-183) -- the butterfly
 * identity for the upper predecessor's branch metric (n - e), uint8 metrics whose sums wrap,
 * the strict '>' select and the subtract-the-minimum renormalisation every 121 steps -- instead
 * of exact metrics.  The two agree whenever no uint8 sum wraps (n <= 3 with symmetric
 * generators); for n >= 4 this mode is what reproduces the reference.  Used by
 * the legacy drop-in for k = 1 codes with n != 2. */
#define VTB_GENK_K1_REFERENCE_U8 1

/* Hard-decision decode of `frames` rows of info_bits/k + K-1 coded segment bytes (row stride
 * in_stride) into rows of ceil(info_bits/8) bytes, MSB-first (out_stride; a partial last byte
 * is zero-padded, as viterbiDecoderButterflyk1.c:226-249); info_bits a multiple of k, at most
 * VTB_MAX_FRAME_BITS.  Device pointers, asynchronous on `stream` (a hipStream_t, 0 = default)
 * of the current device.  VTB_ERR_UNSUPPORTED when the trellis or the frame exceeds one CU's
 * LDS. */
int vtb_genk_decode_device(const vtb_genk_code_t* code, int32_t info_bits, const uint8_t* d_in, size_t in_stride,
                           uint8_t* d_out, size_t out_stride, size_t frames, void* stream);

/* ---- Legacy per-call semantics (include/viterbiDecoder.h behind VITERBI_DECODER_HARD) ----
 * Synchronous, host buffers, run on a per-host-thread context on device 0 (or
 * $VTB_LEGACY_DEVICE). */

/* The metric update a last=false call of the reference's k=1 decoder performs over `count`
 * segments (viterbiDecoderHardButterflyk1, src/viterbiDecoderButterflyk1.c:101-191), so that
 * nodeMetricsCur reads as in the reference between calls: uint8 path metrics with wrapping
 * sums, the strict '>' select and the subtract-the-minimum renormalisation when the counter
 * reaches 120 (:159-183).  metrics[2^(K-1)] (the reference's nodeMetricsA) and
 * *renorm_counter are updated in place.  Like the reference, the butterfly identity is
 * applied whatever the generators (vtb_code_check is not required). */
int vtb_legacy_metrics_k1(const vtb_code_t* code, const uint8_t* segments, int32_t count, uint8_t* metrics,
                          uint32_t* renorm_counter);

/* The same update for a k = 1 code of any n (1..8 coded bits, code->input_bits == 1): the
 * reference's butterfly with n - e as the complement (viterbiDecoderButterflyk1.c:104-107 with
 * its compile-time n), which vtb_legacy_metrics_k1's two-generator vtb_code_t cannot describe. */
int vtb_legacy_metrics_k1n(const vtb_genk_code_t* code, const uint8_t* segments, int32_t count, uint8_t* metrics,
                           uint32_t* renorm_counter);

/* The metric update of the generic decoder (viterbiDecoderHard, src/viterbiDecoder.c:84-131):
 * destination-indexed, exact metrics, first minimum over the 2^k predecessors.  metrics[2^(k(K-1))]
 * is updated in place; prev_metrics (optional) receives the metrics one step before the last
 * (the reference's nodeMetricsNext after its final swap). */
int vtb_legacy_metrics_genk(const vtb_genk_code_t* code, const uint8_t* segments, int32_t count, uint32_t* metrics,
                            uint32_t* prev_metrics);

/* One general-k hard frame of `segments` coded segments from host memory (VITERBI_DECODER_HARD
 * for k > 1, and for k = 1 codes with n != 2 with VTB_GENK_K1_REFERENCE_U8): decoded by
 * vtb_genk_decode_device, ceil((segments - K + 1) * k / 8) bytes written to out and that count
 * returned (the reference's byte count for a whole frame, :256), or a VTB_ERR_* code. */
int vtb_genk_decode_frame_legacy(const vtb_genk_code_t* code, const uint8_t* coded, int32_t segments, uint8_t* out);

#ifdef __cplusplus
}
#endif

#endif
