/* TEST INFRASTRUCTURE ONLY: exposes the reference encoder (convEncode.c, compiled in place
 * from /root/reference/src with one general-k code configuration) to the tests, to pin
 * oracle_genk_encode for k > 1.  Built by oracle/Makefile into oracle/_ref/librefenc_*.so. */
#include "convEncode.h"
int refenc_k(void) { return k; }
int refenc_K(void) { return K; }
int refenc_n(void) { return n; }
int refenc_encode(uint8_t* unc, int nbytes, uint8_t* coded) {
    convEncoderState_t st;
    initConvEncoder(&st);
    resetConvEncoder(&st);
    return convEnc(&st, unc, coded, nbytes, true);
}
