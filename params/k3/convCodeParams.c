#include "convCodeParams.h"

/* K=3 rate-1/2 generators (octal / binary literal, Proakis MSB-newest convention). */
const uint64_t g[n] = {0b111, 0b110};
