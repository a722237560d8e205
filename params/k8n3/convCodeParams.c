#include "convCodeParams.h"

/* K=8 rate-1/3 generators (octal, Proakis MSB-newest convention): the 128-state k = 1 code
 * with n != 2 for the legacy drop-in (the general-k kernel's N = 128 layout). */
const uint64_t g[n] = {0225, 0331, 0367};
