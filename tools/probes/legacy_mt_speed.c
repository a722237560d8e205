/* Measurement only: the speedDecode protocol (speedDecode.c:37-116: 16 packets from
 * srand(314), VITERBI_DECODER_HARD with last=true in a loop, one decoder state per thread)
 * on N host threads at once, through the legacy drop-in (libviterbi_legacy_k7 ->
 * vtb_decode_frame_sync on the GPU).  Prints the aggregate Mbit/s per thread count.
 *   legacy_mt_speed <seconds> <threads...> */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "convEncode.h"
#include "viterbiDecoder.h"

enum { PKTS = 16, PKT_BYTES = 256 };
#define T_SEGS (8 * PKT_BYTES / k + S)

static uint8_t coded[PKTS][T_SEGS];

typedef struct {
    double seconds, elapsed;
    long frames;
} job_t;

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static void* worker(void* p) {
    job_t* j = (job_t*)p;
    viterbiHardState_t st;
    VITERBI_RESET(&st);
    VITERBI_INIT(&st);
    uint8_t out[PKT_BYTES];
    VITERBI_DECODER_HARD(&st, coded[0], out, T_SEGS, true); /* warm the thread's plan */
    const double t0 = now();
    long cnt = 0;
    int cur = 0;
    while (1) {
        VITERBI_DECODER_HARD(&st, coded[cur], out, T_SEGS, true);
        cur = (cur + 1) % PKTS;
        cnt++;
        if ((cnt & 63) == 0 && now() - t0 >= j->seconds) break;
    }
    j->elapsed = now() - t0;
    j->frames = cnt;
    return NULL;
}

int main(int argc, char** argv) {
    const double secs = argc > 1 ? atof(argv[1]) : 2.0;
    uint8_t unc[PKTS][PKT_BYTES];
    srand(314);
    for (int i = 0; i < PKTS; i++)
        for (int b = 0; b < PKT_BYTES; b++) unc[i][b] = (uint8_t)rand();
    convEncoderState_t enc;
    resetConvEncoder(&enc);
    initConvEncoder(&enc);
    for (int i = 0; i < PKTS; i++) convEnc(&enc, unc[i], coded[i], PKT_BYTES, true);
    for (int a = 2; a < argc; a++) {
        const int nt = atoi(argv[a]);
        pthread_t th[256];
        job_t jobs[256];
        for (int i = 0; i < nt; i++) {
            jobs[i].seconds = secs;
            pthread_create(&th[i], NULL, worker, &jobs[i]);
        }
        double mbps = 0;
        for (int i = 0; i < nt; i++) {
            pthread_join(th[i], NULL);
            mbps += jobs[i].frames * 8.0 * PKT_BYTES / jobs[i].elapsed / 1e6;
        }
        printf("threads %d: %.1f Mbit/s aggregate\n", nt, mbps);
        fflush(stdout);
    }
    return 0;
}
