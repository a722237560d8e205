#include "convCodeParams.h"

/* Rate 3/4, K = 3 (k*K = 9 generator bits). */
const uint64_t g[n] = {0x1ED, 0x15B, 0x0B7, 0x1A7};
