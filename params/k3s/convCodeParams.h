/* Code configuration consumed by the legacy headers (include/viterbiDecoder.h,
 * include/convEncode.h).  Same macro names as the reference's per-harness config
 * directory (reference src/defaultParams/convCodeParams.h:8-17), so harnesses built
 * with -I<this dir> see the code they expect.  Proakis naming: K constraint length,
 * k input bits per step, S = K-1 state chunks, n coded bits, Rc rate. */
#ifndef _CONV_CODE_PARAMS_H_
#define _CONV_CODE_PARAMS_H_

#include <stdint.h>

#define K (3)
#define k (1)
#define S ((K)-1)
#define n (2)
#define Rc ((double) k/n)
#define STARTING_STATE (0)

/* Generators, octal Proakis convention (MSB = newest input); defined in convCodeParams.c. */
extern const uint64_t g[n];

#endif
