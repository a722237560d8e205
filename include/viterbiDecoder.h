/*
 * Legacy Viterbi decoder API of the reference (reference src/viterbiDecoder.h:1-191),
 * kept source-, layout- and link-compatible so the reference harnesses (speedDecode.c,
 * berTestK7.c, handTraced.c) compile and link against this build unchanged.
 *
 * What changes underneath: the k=1 decode entry (viterbiDecoderHardButterflyk1, the one
 * VITERBI_DECODER_HARD selects) no longer runs the trellis on the host.  The host shim
 * (convolutionalencdec_amd/csrc/legacy/viterbiDecoder.c) buffers the frame's coded
 * segments in the caller's state struct and, on last=true, hands the frame to the
 * MI355X decoder through the C-ABI in include/viterbi_amd.h.  Decoded bytes are
 * bit-identical to the reference's (tests/test_gpu_parity.py).
 *
 * The code is configured at compile time by the harness's convCodeParams.h (K, k, S, n,
 * STARTING_STATE, g[]), as in the reference.
 */
#ifndef _VITERBI_DECODER_H_
#define _VITERBI_DECODER_H_

#include <stdbool.h>

#include "convCodeParams.h"
#include "convHelpers.h"

#ifdef __cplusplus
#define VTB_LEGACY_RESTRICT __restrict__
extern "C" {
#else
#define VTB_LEGACY_RESTRICT restrict
#endif

/* ---- limits (reference :17-26) ---- */
#define MAX_PKT_LEN_UNCODED_BITS (1024 * 16) /* longest frame, in information bits */
#define TRACEBACK_LEN (5 * K)                 /* generic-decoder traceback depth */
#define TRACEBACK_BUFFER_LEN (MAX_PKT_LEN_UNCODED_BITS)

#define NUM_STATES (POW2(k * S))

/* Feature switches the reference defines (reference :30-39). */
#define FORCE_NO_POPCNT_DECODER
#define USE_POLY_SYMMETRY

#define MAX_EDGE_WEIGHT (n) /* Hamming branch metric is at most n */
#define MAX_PKT_LEN_SEGMENTS (MAX_PKT_LEN_UNCODED_BITS + S)

/* ---- element types (reference :47-85) ---- */
#if k == 1
#define METRIC_TYPE uint8_t /* k=1: 8-bit metrics with periodic renormalisation */
#define METRIC_MAX UINT8_MAX
#else
#if MAX_EDGE_WEIGHT * MAX_PKT_LEN_SEGMENTS <= POW2(8)
#define METRIC_TYPE uint8_t
#elif MAX_EDGE_WEIGHT * MAX_PKT_LEN_SEGMENTS <= POW2(16)
#define METRIC_TYPE uint16_t
#elif MAX_EDGE_WEIGHT * MAX_PKT_LEN_SEGMENTS <= POW2(32)
#define METRIC_TYPE uint32_t
#else
#define METRIC_TYPE uint64_t
#endif
#endif

#if MAX_EDGE_WEIGHT <= POW2(8)
#define EDGE_METRIC_INDEX_TYPE uint8_t
#elif MAX_EDGE_WEIGHT <= POW2(16)
#define EDGE_METRIC_INDEX_TYPE uint16_t
#elif MAX_EDGE_WEIGHT <= POW2(32)
#define EDGE_METRIC_INDEX_TYPE uint32_t
#else
#define EDGE_METRIC_INDEX_TYPE uint64_t
#endif

#define TRACEBACK_TYPE uint8_t
#define TRACEBACK_BITS 8

/* ---- entry-point selection (reference :87-95) ---- */
#if k == 1
#define VITERBI_DECODER_HARD viterbiDecoderHardButterflyk1
#define VITERBI_INIT viterbiInitButterflyk1
#define VITERBI_RESET resetViterbiDecoderHardButterflyk1
#else
#define VITERBI_DECODER_HARD viterbiDecoderHard
#define VITERBI_INIT viterbiInit
#define VITERBI_RESET resetViterbiDecoderHard
#endif

#define TRACEBACK_BYTES ((TRACEBACK_BUFFER_LEN + S * k) / TRACEBACK_BITS + 1)

/*
 * Decoder state, caller-allocated (the harnesses put it on the stack).  Field order,
 * types and alignment follow the reference struct (reference :103-146) so sizeof and
 * every offset match (tests/test_legacy_abi.py checks both).
 *
 * This build uses the fields as follows:
 *   edgeCodedBitsSymm  trellis table (coded segment on edge i -> 2i), filled by VITERBI_INIT
 *   edgeCodedBits      full per-edge table (generic viterbiInit)
 *   nodeMetricsA/B, traceBackA/B and the Cur/Next pointers   reset values, as the reference
 *   iteration          coded segments accumulated for the current frame
 *   renormCounter      the reference's renormalisation phase for those segments
 *   tracebackBufs      staging area for the frame's coded segments between last=false
 *                      calls (the GPU keeps its own survivor memory)
 */
typedef struct {
#ifdef USE_POLY_SYMMETRY
    EDGE_METRIC_INDEX_TYPE edgeCodedBitsSymm[NUM_STATES / 2];
#endif
    EDGE_METRIC_INDEX_TYPE edgeCodedBits[POW2(k)][NUM_STATES];

    METRIC_TYPE nodeMetricsA[NUM_STATES] __attribute__((aligned(64)));
    TRACEBACK_TYPE traceBackA[NUM_STATES] __attribute__((aligned(64)));
    METRIC_TYPE nodeMetricsB[NUM_STATES];
    TRACEBACK_TYPE traceBackB[NUM_STATES];

    METRIC_TYPE (*VTB_LEGACY_RESTRICT nodeMetricsCur)[NUM_STATES];
    TRACEBACK_TYPE (*VTB_LEGACY_RESTRICT traceBackCur)[NUM_STATES];
    METRIC_TYPE (*VTB_LEGACY_RESTRICT nodeMetricsNext)[NUM_STATES];
    TRACEBACK_TYPE (*VTB_LEGACY_RESTRICT traceBackNext)[NUM_STATES];

    unsigned int iteration;
    unsigned int renormCounter;
    uint8_t decodeCarryOver;
    uint8_t decodeCarryOverCount;

    TRACEBACK_TYPE tracebackBufs[(TRACEBACK_BUFFER_LEN + S * k)][NUM_STATES] __attribute__((aligned(64)));
} viterbiHardState_t;

/*
 * Hard-decision decode of segmentsIn coded segments (one n-bit segment per byte, only the
 * low n bits are read).  The frame must start in STARTING_STATE and be terminated in
 * state 0 by S zero segments.  With last=false the segments are appended to the frame and
 * 0 is returned; with last=true the whole frame is decoded, (segments-S) information bits
 * are written MSB-first to uncoded, the state is reset and the number of bytes written,
 * ceil((segments-S)/8), is returned.
 *
 * viterbiDecoderHard is the generic-k entry (reference :160); for k=1 codes it uses the
 * same GPU path as viterbiDecoderHardButterflyk1.
 */
int viterbiDecoderHard(viterbiHardState_t* VTB_LEGACY_RESTRICT state, uint8_t* VTB_LEGACY_RESTRICT codedSegments,
                       uint8_t* VTB_LEGACY_RESTRICT uncoded, int segmentsIn, bool last);

/* Swap the Cur/Next metric and traceback pointers (reference :167). */
void swapViterbiArrays(viterbiHardState_t* state);

/* Exit(1) with a message unless STARTING_STATE is 0 and every generator taps both the
 * newest and the oldest input (the symmetric-butterfly precondition). Returns 0. */
int viterbiConfigCheck();

/* Generic-decoder trellis table (edgeCodedBits). */
void viterbiInit(viterbiHardState_t* state);

/* Generic-decoder reset. */
void resetViterbiDecoderHard(viterbiHardState_t* state);

/* Number of differing bits among the low `bits` bits of a and b. */
uint8_t calcHammingDist(uint8_t a, uint8_t b, int bits);

/* Index of the smallest metric (lowest index on ties). */
int argminPathMetrics(const METRIC_TYPE (*metrics)[POW2(k)]);
int argminNodeMetrics(const METRIC_TYPE (*metrics)[NUM_STATES]);
int argmin2(const METRIC_TYPE (*metrics)[2]);
int argmin4(const METRIC_TYPE (*metrics)[4]);
int argmin8(const METRIC_TYPE (*metrics)[8]);
int argmin16(const METRIC_TYPE (*metrics)[16]);
int argmin32(const METRIC_TYPE (*metrics)[32]);
int argmin64(const METRIC_TYPE (*metrics)[64]);

#ifdef __cplusplus
}
#endif

#include "viterbiDecoderButterflyk1.h"

#endif
