#include "convCodeParams.h"

/* Rate 2/3, K = 4 (k*K = 8 generator bits). */
const uint64_t g[n] = {0xB5, 0x6B, 0xD9};
