#include "convCodeParams.h"

/* K=7 rate-1/3 generators (octal, Proakis MSB-newest convention): a k = 1 code with n != 2
 * for the legacy drop-in (the reference decoder is generic in n,
 * viterbiDecoderButterflyk1.c:104-107). */
const uint64_t g[n] = {0133, 0171, 0165};
