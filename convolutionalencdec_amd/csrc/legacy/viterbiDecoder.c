/*
 * Legacy decoder API (include/viterbiDecoder.h, include/viterbiDecoderButterflyk1.h) on
 * top of the MI355X C ABI (include/viterbi_amd.h).  Compiled per code configuration with
 * the harness's convCodeParams.h; the trellis itself never runs here.
 *
 * VITERBI_DECODER_HARD (viterbiDecoderHardButterflyk1) contract, reference
 * src/viterbiDecoderButterflyk1.c:82-263:
 *   - segments of one frame may arrive over several calls with last=false; they are
 *     staged in the caller's state struct (tracebackBufs, which is large enough for
 *     MAX_PKT_LEN_SEGMENTS bytes) and `iteration` counts them;
 *   - last=true decodes the whole frame on the GPU (vtb_decode_frame_legacy), writes the
 *     information bytes, resets the state and returns the byte count.
 * Node metrics are not updated between last=false calls in this build (the GPU keeps
 * them); nodeMetricsCur holds the reset values.  Errors the reference leaves undefined
 * (more than MAX_PKT_LEN_SEGMENTS segments, a last=true frame of <= S segments) print a
 * message and return 0; a missing or failing GPU prints and exit(1)s, the reference's
 * convention for fatal configuration errors (src/viterbiDecoder.c:10-13).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "convEncode.h"
#include "viterbiDecoder.h"
#include "viterbi_amd.h"

static vtb_code_t legacy_code(void) {
    vtb_code_t c;
    c.constraint_length = K;
    c.coded_bits = n;
    c.generators[0] = g[0];
    c.generators[1] = (n > 1) ? g[n - 1] : 0; /* n != 2 is rejected by the C ABI */
    return c;
}

/* ---------------- generic helpers (reference src/viterbiDecoder.c) ---------------- */

int viterbiConfigCheck() {
    if (STARTING_STATE != 0) {
        printf("Currently only support starting state of 0\n");
        exit(1);
    }
#ifdef USE_POLY_SYMMETRY
    if (k == 1) {
        for (int i = 0; i < n; i++) {
            if (!((g[i] >> (K - 1)) & 1) || !(g[i] & 1)) {
                printf("Polynomial %d does not depend on the input bit and the last bit, therefore polynomial symmetry cannot be used\n", i);
                exit(1);
            }
        }
    }
#endif
    return 0;
}

uint8_t calcHammingDist(uint8_t a, uint8_t b, int bits) {
    unsigned diff = (unsigned)(a ^ b);
    if (bits < 8) diff &= (1u << bits) - 1u;
    return (uint8_t)__builtin_popcount(diff);
}

void swapViterbiArrays(viterbiHardState_t* state) {
    METRIC_TYPE(*m)[NUM_STATES] = state->nodeMetricsCur;
    state->nodeMetricsCur = state->nodeMetricsNext;
    state->nodeMetricsNext = m;
    TRACEBACK_TYPE(*t)[NUM_STATES] = state->traceBackCur;
    state->traceBackCur = state->traceBackNext;
    state->traceBackNext = t;
}

void viterbiInit(viterbiHardState_t* state) {
    convEncoderState_t enc;
    resetConvEncoder(&enc);
    initConvEncoder(&enc);
    for (unsigned edge = 0; edge < POW2(k); edge++) {
        for (unsigned s = 0; s < NUM_STATES; s++) {
            resetConvEncoder(&enc);
            enc.tappedDelay = (TAPPED_DELAY_TYPE)s;
            state->edgeCodedBits[edge][s] = (EDGE_METRIC_INDEX_TYPE)convEncOneInput(&enc, (uint8_t)edge);
        }
    }
}

static void reset_common(viterbiHardState_t* state) {
    state->nodeMetricsCur = &state->nodeMetricsA;
    state->nodeMetricsNext = &state->nodeMetricsB;
    state->traceBackCur = &state->traceBackA;
    state->traceBackNext = &state->traceBackB;
    for (unsigned s = 0; s < NUM_STATES; s++) {
        state->nodeMetricsA[s] = (s == STARTING_STATE) ? 0 : (METRIC_TYPE)(NUM_STATES + 1);
        state->traceBackA[s] = 0;
    }
    state->iteration = 0;
    state->renormCounter = 0;
    state->decodeCarryOver = 0;
    state->decodeCarryOverCount = 0;
}

void resetViterbiDecoderHard(viterbiHardState_t* state) { reset_common(state); }

#define DEFINE_ARGMIN(NAME, LEN)                                          \
    int NAME(const METRIC_TYPE (*metrics)[LEN]) {                         \
        int best = 0;                                                     \
        for (int i = 1; i < (int)(LEN); i++)                              \
            if ((*metrics)[i] < (*metrics)[best]) best = i;               \
        return best;                                                      \
    }
DEFINE_ARGMIN(argminPathMetrics, POW2(k))
DEFINE_ARGMIN(argminNodeMetrics, NUM_STATES)
DEFINE_ARGMIN(argmin2, 2)
DEFINE_ARGMIN(argmin4, 4)
DEFINE_ARGMIN(argmin8, 8)
DEFINE_ARGMIN(argmin16, 16)
DEFINE_ARGMIN(argmin32, 32)
DEFINE_ARGMIN(argmin64, 64)

/* ---------------- k=1 entry points (reference src/viterbiDecoderButterflyk1.c) ---------------- */

void viterbiInitButterflyk1(viterbiHardState_t* state) {
    printf("Specialized Viterbi Decoder for k=1\n");
    vtb_code_t c = legacy_code();
    uint8_t symm[1 << (VTB_MAX_K - 2)];
    if (vtb_edge_table(&c, symm) == VTB_OK) {
        for (unsigned i = 0; i < NUM_STATES / 2 && i < sizeof(symm); i++) state->edgeCodedBitsSymm[i] = symm[i];
    }
}

void resetViterbiDecoderHardButterflyk1(viterbiHardState_t* state) { reset_common(state); }

/* The reference's renormalisation phase after `steps` more segments (:159-183). */
static unsigned renorm_phase_after(unsigned counter, unsigned steps) {
    for (unsigned i = 0; i < steps; i++) counter = counter >= 120 ? 0 : counter + 1;
    return counter;
}

static int decode_staged(viterbiHardState_t* VTB_LEGACY_RESTRICT state, const uint8_t* frame, int segments,
                         uint8_t* VTB_LEGACY_RESTRICT uncoded) {
    if (segments <= S) {
        printf("viterbi: frame of %d segments is not longer than the %d tail segments; nothing decoded\n", segments, S);
        return 0;
    }
    vtb_code_t c = legacy_code();
    int r = vtb_decode_frame_legacy(&c, frame, segments, uncoded);
    if (r < 0) {
        printf("viterbi: GPU decode failed: %s (%d)\n", vtb_strerror(r), r);
        exit(1);
    }
    return r;
}

int viterbiDecoderHardButterflyk1(viterbiHardState_t* VTB_LEGACY_RESTRICT state, uint8_t* VTB_LEGACY_RESTRICT codedSegments,
                                  uint8_t* VTB_LEGACY_RESTRICT uncoded, int segmentsIn, bool last) {
    uint8_t* staged = &state->tracebackBufs[0][0];
    const size_t capacity = sizeof(state->tracebackBufs);
    if (segmentsIn < 0) segmentsIn = 0;
    if ((size_t)state->iteration + (size_t)segmentsIn > (size_t)MAX_PKT_LEN_SEGMENTS || (size_t)state->iteration + (size_t)segmentsIn > capacity) {
        printf("viterbi: frame exceeds MAX_PKT_LEN_SEGMENTS (%d); dropped\n", (int)MAX_PKT_LEN_SEGMENTS);
        resetViterbiDecoderHardButterflyk1(state);
        return 0;
    }
    if (!last) {
        memcpy(staged + state->iteration, codedSegments, (size_t)segmentsIn);
        state->renormCounter = renorm_phase_after(state->renormCounter, (unsigned)segmentsIn);
        state->iteration += (unsigned)segmentsIn;
        return 0;
    }
    int r;
    if (state->iteration == 0) {
        r = decode_staged(state, codedSegments, segmentsIn, uncoded);
    } else {
        memcpy(staged + state->iteration, codedSegments, (size_t)segmentsIn);
        r = decode_staged(state, staged, (int)(state->iteration + (unsigned)segmentsIn), uncoded);
    }
    resetViterbiDecoderHardButterflyk1(state);
    return r;
}

int viterbiDecoderHard(viterbiHardState_t* VTB_LEGACY_RESTRICT state, uint8_t* VTB_LEGACY_RESTRICT codedSegments,
                       uint8_t* VTB_LEGACY_RESTRICT uncoded, int segmentsIn, bool last) {
#if k == 1
    return viterbiDecoderHardButterflyk1(state, codedSegments, uncoded, segmentsIn, last);
#else
    (void)state;
    (void)codedSegments;
    (void)uncoded;
    (void)segmentsIn;
    (void)last;
    printf("viterbi: k=%d codes are not supported by this build\n", k);
    exit(1);
#endif
}
