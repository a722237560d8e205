#include "convCodeParams.h"

/* K=7 rate-1/2 generators (octal / binary literal, Proakis MSB-newest convention). */
const uint64_t g[n] = {0113, 0171};
