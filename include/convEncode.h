/*
 * Legacy convolutional-encoder API of the reference (reference src/convEncode.h:1-97),
 * kept source- and layout-compatible so the reference harnesses (speedDecode.c,
 * berTestK7.c, handTraced.c) compile against it unchanged.
 *
 * The code itself (K, k, n, S, STARTING_STATE, g[]) comes from the harness's
 * convCodeParams.h, exactly as in the reference build (speedDecode/Makefile:10-16).
 * Implementation: convolutionalencdec_amd/csrc/legacy/convEncode.c (host-side; the
 * encoder is not on the GPU hot path in this round).
 */
#ifndef _CONV_ENCODE_H_
#define _CONV_ENCODE_H_

#include <stdbool.h>

#include "convCodeParams.h"
#include "convHelpers.h"

/* Shift-register word: the narrowest unsigned type holding k*K bits (reference :8-18). */
#if k * K <= 8
#define TAPPED_DELAY_TYPE uint8_t
#elif k * K <= 16
#define TAPPED_DELAY_TYPE uint16_t
#elif k * K <= 32
#define TAPPED_DELAY_TYPE uint32_t
#elif k * K <= 64
#define TAPPED_DELAY_TYPE uint64_t
#else
#error Only constraint lengths (k*K) <=64 are currently supported
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* Encoder state (reference :29-38).  tappedDelay: newest input bit in the LSB.
 * polynomials: g[] bit-reversed to that little-endian order.  remainingUncoded /
 * remainingUncodedCount: leftover input bits between calls when 8 % k != 0. */
typedef struct {
    TAPPED_DELAY_TYPE tappedDelay;
    TAPPED_DELAY_TYPE polynomials[n];
    uint8_t remainingUncoded;
    uint8_t remainingUncodedCount;
} convEncoderState_t;

/* Reverse the k*K low bits of a Proakis (MSB = newest input) generator. */
TAPPED_DELAY_TYPE bitReverseGenerator(TAPPED_DELAY_TYPE packed);

/* Put the shift register in STARTING_STATE and drop leftover bits. */
void resetConvEncoder(convEncoderState_t* state);

/* Load the bit-reversed generators into the state. */
void initConvEncoder(convEncoderState_t* state);

/* Encode bytesIn bytes (MSB of each byte first) into k-bit-input / n-bit-output segments,
 * one segment per output byte with generator 0 in the LSB.  With last=true, S zero
 * segments terminate the trellis in state 0 and the encoder resets; leftover bits at that
 * point are a fatal error (printf + exit(1), as the reference).  Returns segments written. */
int convEnc(convEncoderState_t* state, uint8_t* uncoded, uint8_t* codedSegments, int bytesIn, bool last);

/* n-bit output for the current shift-register contents. */
uint8_t computeEncOutputSegment(convEncoderState_t* state);

/* Shift in one k-bit input (MSB first) and return the resulting coded segment. */
int convEncOneInput(convEncoderState_t* state, uint8_t bitsToShiftIn);

#ifdef __cplusplus
}
#endif

#endif
