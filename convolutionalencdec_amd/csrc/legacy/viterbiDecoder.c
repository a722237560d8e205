/*
 * Legacy decoder API (include/viterbiDecoder.h, include/viterbiDecoderButterflyk1.h) on
 * top of the MI355X C ABI (include/viterbi_amd.h).  Compiled per code configuration with
 * the harness's convCodeParams.h; no trellis work runs on the host.
 *
 * VITERBI_DECODER_HARD contract, reference src/viterbiDecoderButterflyk1.c:82-263 (k=1) and
 * src/viterbiDecoder.c:52-234 (k>1):
 *   - segments of one frame may arrive over several calls with last=false; they are
 *     staged in the caller's state struct (tracebackBufs, which is large enough for
 *     MAX_PKT_LEN_SEGMENTS bytes) and `iteration` counts them.  Each such call also runs
 *     the reference's metric update on the GPU (vtb_legacy_metrics_k1 / _genk), so
 *     nodeMetricsCur (and, k=1, renormCounter) read exactly as in the reference between
 *     calls (handTracedTest/handTraced.c:72-111 reads them);
 *   - last=true decodes the whole frame on the GPU (vtb_decode_frame_legacy, k>1:
 *     vtb_genk_decode_frame_legacy), writes the information bytes, resets the state and
 *     returns the byte count.  For k>1 the reference would have emitted bytes during the
 *     last=false calls through its register-exchange traceback (viterbiDecoder.c:140-190,
 *     which drops bits for k*5K > 8); here every byte of the frame comes with last=true.
 * Errors the reference leaves undefined (more than MAX_PKT_LEN_SEGMENTS segments, a
 * last=true frame of <= S segments) print a message and return 0; a missing or failing GPU
 * prints and exit(1)s, the reference's convention for fatal configuration errors
 * (src/viterbiDecoder.c:10-13).
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "convEncode.h"
#include "viterbiDecoder.h"
#include "viterbi_amd.h"

static vtb_genk_code_t legacy_genk_code(void) {
    vtb_genk_code_t c;
    memset(&c, 0, sizeof(c));
    c.input_bits = k;
    c.constraint_length = K;
    c.coded_bits = n;
    for (int i = 0; i < n && i < 8; i++) c.generators[i] = g[i];
    return c;
}

/* The reference library draws nothing from rand(); the GPU runtime does (libhsa-runtime64
 * imports rand and srand).  Harnesses such as berTestK7.c build their channel from rand()
 * between decoder calls (berTestK7.c:29-43, 135-138), so every call into the GPU keeps the
 * caller's rand() stream: while any decoder call is in flight, glibc's process-wide random
 * state is switched to a private scratch state (setstate), and when the last one returns,
 * back to the caller's.  Only the public initstate / setstate contract is used: setstate
 * records the position of the state it leaves in that state's own first word and resumes
 * from it on the way back, so the caller's state array and position are untouched.
 * One process-wide mutex guards the switch and a count of calls in flight (the GPU calls
 * themselves run concurrently); the scratch state is a process-wide static, so the global
 * state never points at a thread's memory.  rand() draws other threads make while a
 * decoder call is in flight come from the scratch stream. */
static pthread_mutex_t rand_mu = PTHREAD_MUTEX_INITIALIZER;
static int32_t rand_scratch[32]; /* a TYPE_3 state of our own (128 bytes) */
static int rand_scratch_ready, rand_calls;
static char* rand_caller; /* the caller's state while calls are in flight */

static void rand_keep_begin(void) {
    pthread_mutex_lock(&rand_mu);
    if (rand_calls++ == 0) {
        if (!rand_scratch_ready) { /* seeds the scratch state (310 draws on it) and switches to it */
            rand_caller = initstate(1u, (char*)rand_scratch, sizeof(rand_scratch));
            rand_scratch_ready = 1;
        } else {
            rand_caller = setstate((char*)rand_scratch);
        }
    }
    pthread_mutex_unlock(&rand_mu);
}

static void rand_keep_end(void) {
    pthread_mutex_lock(&rand_mu);
    if (--rand_calls == 0) {
        setstate(rand_caller);
        rand_caller = NULL;
    }
    pthread_mutex_unlock(&rand_mu);
}

#define KEEP_RAND(call)        \
    ({                         \
        rand_keep_begin();     \
        int kr_r = (call);     \
        rand_keep_end();       \
        kr_r;                  \
    })

static void gpu_failed(const char* what, int r) {
    printf("viterbi: GPU %s failed: %s (%d)\n", what, vtb_strerror(r), r);
    exit(1);
}

/* k = 1 codes with n = 2 go through the rate-1/2 kernels (vtb_code_t); k = 1 codes with any
 * other n through the general-k kernel in the reference's own uint8 butterfly arithmetic
 * (VTB_GENK_K1_REFERENCE_U8), which vtb_code_t's two generators cannot describe. */
#define LEGACY_K1_RATE_HALF (k == 1 && n == 2)

static vtb_code_t legacy_code(void) {
    vtb_code_t c;
    c.constraint_length = K;
    c.coded_bits = 2;
    c.generators[0] = g[0];
    c.generators[1] = (n > 1) ? g[n > 1 ? 1 : 0] : 0; /* used only when n == 2 */
    return c;
}

static vtb_genk_code_t legacy_k1n_code(void) {
    vtb_genk_code_t c = legacy_genk_code();
    c.flags = VTB_GENK_K1_REFERENCE_U8;
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
    if (LEGACY_K1_RATE_HALF) {
        vtb_code_t c = legacy_code();
        uint8_t symm[1 << (VTB_MAX_K - 2)];
        if (vtb_edge_table(&c, symm) == VTB_OK) {
            for (unsigned i = 0; i < NUM_STATES / 2 && i < sizeof(symm); i++) state->edgeCodedBitsSymm[i] = symm[i];
        }
        return;
    }
    /* any n: the table of viterbiInitButterflyk1.c:24-29 from the drop-in's own encoder */
    convEncoderState_t enc;
    for (unsigned i = 0; i < NUM_STATES / 2; i++) {
        resetConvEncoder(&enc);
        initConvEncoder(&enc);
        enc.tappedDelay = (TAPPED_DELAY_TYPE)i;
        state->edgeCodedBitsSymm[i] = (EDGE_METRIC_INDEX_TYPE)convEncOneInput(&enc, 0);
    }
}

void resetViterbiDecoderHardButterflyk1(viterbiHardState_t* state) { reset_common(state); }

METRIC_TYPE minMetricGeneric(const METRIC_TYPE (*metrics)[NUM_STATES]) {
    METRIC_TYPE best = (*metrics)[0];
    for (unsigned i = 1; i < NUM_STATES; i++)
        if ((*metrics)[i] < best) best = (*metrics)[i];
    return best;
}

static int decode_staged(viterbiHardState_t* VTB_LEGACY_RESTRICT state, const uint8_t* frame, int segments,
                         uint8_t* VTB_LEGACY_RESTRICT uncoded) {
    if (segments <= S) {
        printf("viterbi: frame of %d segments is not longer than the %d tail segments; nothing decoded\n", segments, S);
        return 0;
    }
    int r;
    if (LEGACY_K1_RATE_HALF) {
        vtb_code_t c = legacy_code();
        r = KEEP_RAND(vtb_decode_frame_legacy(&c, frame, segments, uncoded));
    } else {
        vtb_genk_code_t c = legacy_k1n_code();
        r = KEEP_RAND(vtb_genk_decode_frame_legacy(&c, frame, segments, uncoded));
    }
    if (r < 0) gpu_failed("decode", r);
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
        if (segmentsIn > 0) {
            /* the reference's uint8 metric update and renormalisation phase (:101-191) */
            uint32_t counter = state->renormCounter;
            int r;
            if (LEGACY_K1_RATE_HALF) {
                vtb_code_t c = legacy_code();
                r = KEEP_RAND(vtb_legacy_metrics_k1(&c, codedSegments, segmentsIn, (uint8_t*)state->nodeMetricsA, &counter));
            } else {
                vtb_genk_code_t c = legacy_k1n_code();
                r = KEEP_RAND(vtb_legacy_metrics_k1n(&c, codedSegments, segmentsIn, (uint8_t*)state->nodeMetricsA, &counter));
            }
            if (r != VTB_OK) gpu_failed("metric update", r);
            state->renormCounter = counter;
        }
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
    /* General k (reference src/viterbiDecoder.c:52-234): frames staged as for k=1, decoded
     * by the GPU general-k kernel with last=true. */
    uint8_t* staged = &state->tracebackBufs[0][0];
    const size_t capacity = sizeof(state->tracebackBufs);
    if (segmentsIn < 0) segmentsIn = 0;
    if ((size_t)state->iteration + (size_t)segmentsIn > (size_t)MAX_PKT_LEN_SEGMENTS ||
        (size_t)state->iteration + (size_t)segmentsIn > capacity) {
        printf("viterbi: frame exceeds MAX_PKT_LEN_SEGMENTS (%d); dropped\n", (int)MAX_PKT_LEN_SEGMENTS);
        resetViterbiDecoderHard(state);
        return 0;
    }
    vtb_genk_code_t c = legacy_genk_code();
    if (!last) {
        memcpy(staged + state->iteration, codedSegments, (size_t)segmentsIn);
        if (segmentsIn > 0) {
            /* the reference's metric update (:84-131): every step writes Next and swaps
             * Cur/Next, so after segmentsIn steps Cur holds the newest metrics and Next the
             * ones a step before */
            uint32_t m[NUM_STATES], prev[NUM_STATES];
            for (unsigned s = 0; s < NUM_STATES; s++) m[s] = (uint32_t)(*state->nodeMetricsCur)[s];
            int r = KEEP_RAND(vtb_legacy_metrics_genk(&c, codedSegments, segmentsIn, m, prev));
            if (r != VTB_OK) gpu_failed("metric update", r);
            if (segmentsIn & 1) swapViterbiArrays(state);
            for (unsigned s = 0; s < NUM_STATES; s++) {
                (*state->nodeMetricsCur)[s] = (METRIC_TYPE)m[s];
                (*state->nodeMetricsNext)[s] = (METRIC_TYPE)prev[s];
            }
        }
        state->iteration += (unsigned)segmentsIn;
        return 0;
    }
    const uint8_t* frame = codedSegments;
    int segments = segmentsIn;
    if (state->iteration > 0) {
        memcpy(staged + state->iteration, codedSegments, (size_t)segmentsIn);
        frame = staged;
        segments = (int)(state->iteration + (unsigned)segmentsIn);
    }
    int r = 0;
    if (segments <= S || ((segments - S) * k) % 8) {
        printf("viterbi: frame of %d segments does not hold a whole number of bytes after the %d tail segments; "
               "nothing decoded\n", segments, S);
    } else {
        r = KEEP_RAND(vtb_genk_decode_frame_legacy(&c, frame, segments, uncoded));
        if (r < 0) gpu_failed("decode", r);
    }
    resetViterbiDecoderHard(state);
    return r;
#endif
}
