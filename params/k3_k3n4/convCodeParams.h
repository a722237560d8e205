/* General-k code configuration (k = 3 input bits per step), same macro names as the
 * reference's config directory (src/defaultParams/convCodeParams.h:8-17).  Used to compile
 * the reference's own encoder for k > 1 (oracle/Makefile, test infrastructure) and by the
 * general-k decoder's tests. */
#ifndef _CONV_CODE_PARAMS_H_
#define _CONV_CODE_PARAMS_H_

#include <stdint.h>

#define K (3)
#define k (3)
#define S ((K)-1)
#define n (4)
#define Rc ((double) k/n)
#define STARTING_STATE (0)

/* Generators over k*K bits (MSB = newest input bit), defined in convCodeParams.c. */
extern const uint64_t g[n];

#endif
