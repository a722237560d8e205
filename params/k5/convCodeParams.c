#include "convCodeParams.h"

/* K=5 rate-1/2 generators (octal / binary literal, Proakis MSB-newest convention). */
const uint64_t g[n] = {023, 035};
