#include "convCodeParams.h"

/* K=4 rate-1/2 generators (octal Proakis convention, MSB = newest input); both generators tap both ends. */
const uint64_t g[n] = {015, 017};
