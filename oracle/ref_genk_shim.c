/* TEST INFRASTRUCTURE ONLY: the reference's generic decoder (viterbiDecoderHard,
 * src/viterbiDecoder.c, compiled in place from /root/reference/src with one general-k code
 * configuration) driven chunk by chunk with last=false, recording nodeMetricsCur after every
 * chunk.  Its metric update (:84-131) is well defined; its register-exchange output is not
 * used.  Pins oracle_genk_metrics and the legacy drop-in's k>1 node
 * metrics (tests/golden/genk_metrics.npz).  Built by oracle/Makefile into
 * oracle/_ref/librefgenk_*.so. */
#include <stdlib.h>
#include <string.h>

#include "convEncode.h"
#include "viterbiDecoder.h"

int refgenk_num_states(void) { return (int)NUM_STATES; }
int refgenk_metric_bytes(void) { return (int)sizeof(METRIC_TYPE); }

int refgenk_metrics(uint8_t* coded, int count, int chunk, uint32_t* metrics_out) {
    viterbiHardState_t* st = NULL;
    if (posix_memalign((void**)&st, 64, sizeof(viterbiHardState_t)) != 0) return -1;
    memset(st, 0, sizeof(*st));
    VITERBI_RESET(st);
    VITERBI_INIT(st);
    uint8_t* scratch = (uint8_t*)calloc((size_t)count + 64, 1); /* register-exchange output, unused */
    int c = 0, done = 0;
    while (done < count) {
        int len = count - done < chunk ? count - done : chunk;
        VITERBI_DECODER_HARD(st, coded + done, scratch, len, false);
        for (unsigned s = 0; s < NUM_STATES; s++) metrics_out[(size_t)c * NUM_STATES + s] = (uint32_t)(*st->nodeMetricsCur)[s];
        done += len;
        c++;
    }
    free(scratch);
    free(st);
    return c;
}
