#include "convCodeParams.h"

/* K=9 rate-1/2 generators (octal / binary literal, Proakis MSB-newest convention). */
const uint64_t g[n] = {0561, 0753};
