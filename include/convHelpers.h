/*
 * Legacy helper macros of the reference C API (reference src/convHelpers.h).
 *
 * Harness-visible surface only: POW2 (used by every array size in the legacy headers,
 * reference convHelpers.h:6), the ROTATE_* index helpers (:115-116) and the two unpack
 * helpers (:8-9, reference convHelpers.c:3-14).  The ARGMIN_* tree macros (:11-102) are
 * private to the reference's generic (k>1) decoder and are not part of this API.
 */
#ifndef _CONV_HELPERS_H_
#define _CONV_HELPERS_H_

#include <stdint.h>

/* 2^X as unsigned long (the legacy headers print NUM_STATES with %lu). */
#define POW2(X) (1ul << (X))

/* Rotate the low BITS bits of VAL by SHIFT_AMT. */
#define ROTATE_RIGHT(VAL, SHIFT_AMT, BITS) \
    (((VAL) >> (SHIFT_AMT)) | (((VAL) & (POW2(SHIFT_AMT) - 1)) << ((BITS) - (SHIFT_AMT))))
#define ROTATE_LEFT(VAL, SHIFT_AMT, BITS) \
    ((((VAL) & (POW2((BITS) - (SHIFT_AMT)) - 1)) << (SHIFT_AMT)) | ((VAL) >> ((BITS) - (SHIFT_AMT))))

#ifdef __cplusplus
extern "C" {
#endif

/* Write the unpackArrayLen low bits of packed, one bit per byte: MSB-first order for the
 * BigToLittle form, LSB-first for the LittleToLittle form. */
void unpackBigToLittleEndian(uint8_t* unpackArray, int unpackArrayLen, uint64_t packed);
void unpackLittleToLittleEndian(uint8_t* unpackArray, int unpackArrayLen, uint64_t packed);

#ifdef __cplusplus
}
#endif

#endif
