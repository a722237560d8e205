#include "convCodeParams.h"

/* K=8 rate-1/2 generators (octal Proakis convention, MSB = newest input); both generators tap both ends. */
const uint64_t g[n] = {0247, 0371};
