/*
 * k=1 specialised decoder entry points (reference src/viterbiDecoderButterflyk1.h:6-10),
 * the functions VITERBI_INIT / VITERBI_RESET / VITERBI_DECODER_HARD resolve to when k==1.
 */
#ifndef _VITERBI_DECODER_BUTTERFLY_K1_H_
#define _VITERBI_DECODER_BUTTERFLY_K1_H_

#include "viterbiDecoder.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fill edgeCodedBitsSymm (prints "Specialized Viterbi Decoder for k=1", as the reference). */
void viterbiInitButterflyk1(viterbiHardState_t* state);

/* Start a new frame: state 0 metric 0, every other state (METRIC_TYPE)(NUM_STATES+1). */
void resetViterbiDecoderHardButterflyk1(viterbiHardState_t* state);

/* See viterbiDecoderHard in viterbiDecoder.h; decoded on the MI355X. */
int viterbiDecoderHardButterflyk1(viterbiHardState_t* VTB_LEGACY_RESTRICT state,
                                  uint8_t* VTB_LEGACY_RESTRICT codedSegments,
                                  uint8_t* VTB_LEGACY_RESTRICT uncoded, int segmentsIn, bool last);

/* Smallest of the NUM_STATES metrics (reference :19, defined at :375-391). */
METRIC_TYPE minMetricGeneric(const METRIC_TYPE (*metrics)[NUM_STATES]);

#ifdef __cplusplus
}
#endif

#endif
