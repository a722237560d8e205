#include "convCodeParams.h"

/* K=3 rate-1/2 generators (octal Proakis convention, MSB = newest input); the symmetric K=3 code (both generators tap both ends). */
const uint64_t g[n] = {07, 05};
