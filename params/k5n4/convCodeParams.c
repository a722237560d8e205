#include "convCodeParams.h"

/* K=5 rate-1/4 generators (octal, Proakis MSB-newest convention): a k = 1 code with n != 2
 * for the legacy drop-in (the reference decoder is generic in n,
 * viterbiDecoderButterflyk1.c:104-107). */
const uint64_t g[n] = {023, 035, 027, 033};
