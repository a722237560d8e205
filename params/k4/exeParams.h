/* Block-size knobs the reference harness configs carry (reference
 * src/defaultParams/exeParams.h:4-6); unused by the decode path. */
#ifndef _EXE_PARAMS_H_
#define _EXE_PARAMS_H_

#define ENCODE_BLOCK_SIZE 64
#define DECODE_BLOCK_SIZE 64

#endif
