/*
 * Legacy convolutional encoder (include/convEncode.h), host side.
 *
 * Behaviour follows the reference encoder (src/convEncode.c:6-174): newest input bit in
 * the LSB of the shift register, bit-reversed generators, output bit j = parity of
 * generator j, generator 0 in the LSB of each segment byte, MSB-first input bytes, S
 * zero-tail segments on last=true.  Compiled per code configuration with the harness's
 * convCodeParams.h.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "convEncode.h"

static uint8_t parity_of(TAPPED_DELAY_TYPE x) { return (uint8_t)(__builtin_popcountll((unsigned long long)x) & 1); }

TAPPED_DELAY_TYPE bitReverseGenerator(TAPPED_DELAY_TYPE packed) {
    TAPPED_DELAY_TYPE out = 0;
    for (int i = 0; i < k * K; i++) out = (TAPPED_DELAY_TYPE)((out << 1) | ((packed >> i) & 1u));
    return out;
}

void resetConvEncoder(convEncoderState_t* state) {
    state->tappedDelay = STARTING_STATE;
    state->remainingUncoded = 0;
    state->remainingUncodedCount = 0;
}

void initConvEncoder(convEncoderState_t* state) {
    for (int j = 0; j < n; j++) state->polynomials[j] = bitReverseGenerator((TAPPED_DELAY_TYPE)g[j]);
}

uint8_t computeEncOutputSegment(convEncoderState_t* state) {
    uint8_t seg = 0;
    for (int j = n - 1; j >= 0; j--) seg = (uint8_t)((seg << 1) | parity_of(state->tappedDelay & state->polynomials[j]));
    return seg;
}

static void shift_in(convEncoderState_t* state, unsigned bit) {
    state->tappedDelay = (TAPPED_DELAY_TYPE)((state->tappedDelay << 1) | (bit & 1u));
}

int convEncOneInput(convEncoderState_t* state, uint8_t bitsToShiftIn) {
    for (int j = k - 1; j >= 0; j--) shift_in(state, (bitsToShiftIn >> j) & 1u); /* MSB of the k bits first */
    return computeEncOutputSegment(state);
}

#if k == 1
/* k = 1: four input bits per table lookup.  Entry (s << 4) | b holds the four output
 * segments (first in the low byte) of nibble b (MSB first) entering the encoder in state s
 * (its last K - 1 input bits); built once per library from the configuration's generators. */
#define ENC_NIB_BITS ((K - 1) + 4)
static uint32_t enc_nib[1u << ENC_NIB_BITS];
static TAPPED_DELAY_TYPE enc_poly[n];
static pthread_once_t enc_once = PTHREAD_ONCE_INIT;

static void enc_build(void) {
    for (int j = 0; j < n; j++) enc_poly[j] = bitReverseGenerator((TAPPED_DELAY_TYPE)g[j]);
    for (uint32_t idx = 0; idx < (1u << ENC_NIB_BITS); idx++) {
        unsigned long long td = idx >> 4;
        uint32_t w = 0;
        for (int i = 3; i >= 0; i--) {
            td = (td << 1) | ((idx >> i) & 1u);
            uint32_t seg = 0;
            for (int j = n - 1; j >= 0; j--) seg = (seg << 1) | (uint32_t)parity_of((TAPPED_DELAY_TYPE)(td & enc_poly[j]));
            w |= seg << (8 * (3 - i));
        }
        enc_nib[idx] = w;
    }
}

/* Whole input bytes through the nibble table (the state's polynomials must be the
 * configuration's: initConvEncoder's).  Returns the segments written (8 per byte). */
static int enc_bytes_k1(convEncoderState_t* state, const uint8_t* uncoded, uint8_t* codedSegments, int bytesIn) {
    pthread_once(&enc_once, enc_build);
    for (int j = 0; j < n; j++)
        if (state->polynomials[j] != enc_poly[j]) return -1;
    const uint32_t smask = (1u << (K - 1)) - 1u;
    TAPPED_DELAY_TYPE td = state->tappedDelay;
    uint32_t st = (uint32_t)td & smask;
    for (int b = 0; b < bytesIn; b++) {
        const uint32_t byte = uncoded[b], hi = byte >> 4, lo = byte & 15u;
        const uint32_t w0 = enc_nib[(st << 4) | hi];
        st = ((st << 4) | hi) & smask;
        const uint32_t w1 = enc_nib[(st << 4) | lo];
        st = ((st << 4) | lo) & smask;
        memcpy(codedSegments + 8 * b, &w0, 4);
        memcpy(codedSegments + 8 * b + 4, &w1, 4);
        td = (TAPPED_DELAY_TYPE)((td << 8) | byte); /* as eight single-bit shifts would leave it */
    }
    state->tappedDelay = td;
    return 8 * bytesIn;
}
#endif

int convEnc(convEncoderState_t* state, uint8_t* uncoded, uint8_t* codedSegments, int bytesIn, bool last) {
    int avail = state->remainingUncodedCount; /* bits left over from the previous call */
    uint8_t word = state->remainingUncoded;
    int total = avail + 8 * bytesIn;
    int chunks = total / k;
    int next = 0, out = 0;
#if k == 1
    if (avail == 0 && bytesIn > 0) {
        const int w = enc_bytes_k1(state, uncoded, codedSegments, bytesIn);
        if (w >= 0) {
            out = w;
            chunks = 0;
            word = uncoded[bytesIn - 1]; /* (the state's leftover word, as the bit loop leaves it) */
        }
    }
#endif
    for (int c = 0; c < chunks; c++) {
        for (int j = 0; j < k; j++) {
            if (avail == 0) {
                word = uncoded[next++];
                avail = 8;
            }
            avail--;
            shift_in(state, (word >> avail) & 1u);
        }
        codedSegments[out++] = computeEncOutputSegment(state);
    }
    if (last) {
        if (avail > 0) { /* reference src/convEncode.c:100-106 */
            printf("Recieved last flag while bits remaining to be coded are present.  Make sure the number of bits in the message is both a multiple of 8 and k\n");
            exit(1);
        }
        for (int i = 0; i < S; i++) {
            for (int j = 0; j < k; j++) shift_in(state, 0);
            codedSegments[out++] = computeEncOutputSegment(state);
        }
        resetConvEncoder(state);
    } else {
        state->remainingUncodedCount = (uint8_t)avail;
        state->remainingUncoded = word;
    }
    return out;
}
