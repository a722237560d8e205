/*
 * Legacy convolutional encoder (include/convEncode.h), host side.
 *
 * Behaviour follows the reference encoder (src/convEncode.c:6-174): newest input bit in
 * the LSB of the shift register, bit-reversed generators, output bit j = parity of
 * generator j, generator 0 in the LSB of each segment byte, MSB-first input bytes, S
 * zero-tail segments on last=true.  Compiled per code configuration with the harness's
 * convCodeParams.h.
 */
#include <stdio.h>
#include <stdlib.h>

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

int convEnc(convEncoderState_t* state, uint8_t* uncoded, uint8_t* codedSegments, int bytesIn, bool last) {
    int avail = state->remainingUncodedCount; /* bits left over from the previous call */
    uint8_t word = state->remainingUncoded;
    int total = avail + 8 * bytesIn;
    int chunks = total / k;
    int next = 0, out = 0;
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
