/*
 * TEST INFRASTRUCTURE ONLY -- a thin C wrapper that is compiled together with the
 * reference's own sources (/root/reference/src/{convEncode,convHelpers,viterbiDecoder}.c,
 * plus one code-parameter directory) into oracle/_ref/libref_k<K>.so by oracle/Makefile.
 * No reference source is copied into this repository; the build reads it in place.
 *
 * Purpose: (1) generate the golden vectors in tests/golden/ (make_golden.py),
 * (2) cross-check the CPU restatement (viterbi_oracle.c), (3) time the reference
 * speedDecode protocol on the GPU box's host cores for bench.py's cpu_baseline leg.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "convEncode.h"
#include "viterbiDecoder.h"

int ref_K(void) { return K; }
int ref_num_states(void) { return (int)NUM_STATES; }
unsigned long ref_generator(int i) { return (unsigned long)g[i]; }
unsigned long ref_state_size(void) { return (unsigned long)sizeof(viterbiHardState_t); }
int ref_max_segments(void) { return MAX_PKT_LEN_SEGMENTS; }

static viterbiHardState_t* new_state(void) {
    /* The struct is 64-byte aligned (viterbiDecoder.h:121,145) and the vectorised decoder
     * uses aligned AVX stores, so calloc's 16-byte alignment is not enough. */
    viterbiHardState_t* st = NULL;
    if (posix_memalign((void**)&st, 64, sizeof(viterbiHardState_t)) != 0) return NULL;
    memset(st, 0, sizeof(*st));
    VITERBI_RESET(st); /* speedDecode.c:63-66 order: reset, init (, check) */
    VITERBI_INIT(st);
    /* viterbiConfigCheck() is not called here: it exit(1)s on non-symmetric codes such as
     * the K=3 handTraced config, which would kill the calling test process. */
    return st;
}

void ref_edge_table(uint8_t* out) {
    viterbiHardState_t* st = new_state();
    for (unsigned i = 0; i < NUM_STATES / 2; i++) out[i] = st->edgeCodedBitsSymm[i];
    free(st);
}

int ref_encode(uint8_t* uncoded, int nbytes, uint8_t* coded) {
    convEncoderState_t enc;
    resetConvEncoder(&enc);
    initConvEncoder(&enc);
    return convEnc(&enc, uncoded, coded, nbytes, true);
}

/* Decode nframes frame-major frames of T segments; one state reused (it resets itself
 * after every last=true call, viterbiDecoderButterflyk1.c:259). */
int ref_decode_frames(uint8_t* coded, int T, uint8_t* out, int out_stride, int nframes) {
    if (T <= S || T > MAX_PKT_LEN_SEGMENTS) return -1;
    viterbiHardState_t* st = new_state();
    if (!st) return -1;
    int r = 0;
    for (int f = 0; f < nframes; f++)
        r = VITERBI_DECODER_HARD(st, coded + (size_t)f * T, out + (size_t)f * out_stride, T, true);
    free(st);
    return r;
}

/* Streaming: decode `coded` in chunks of chunk_len segments with last=false, then a final
 * last=true call; after every chunk copy nodeMetricsCur into metrics (N bytes per chunk). */
int ref_decode_stream(uint8_t* coded, int T, int chunk_len, uint8_t* out, uint8_t* metrics) {
    viterbiHardState_t* st = new_state();
    if (!st) return -1;
    int done = 0, chunk = 0, r = 0;
    while (done < T) {
        int len = T - done < chunk_len ? T - done : chunk_len;
        int last = (done + len == T);
        if (metrics && !last) {
            r = VITERBI_DECODER_HARD(st, coded + done, out, len, false);
            memcpy(metrics + (size_t)chunk * NUM_STATES, *st->nodeMetricsCur, NUM_STATES);
        } else {
            r = VITERBI_DECODER_HARD(st, coded + done, out, len, last);
        }
        done += len;
        chunk++;
    }
    free(st);
    return r;
}

/* ---- speedDecode protocol (speedDecode.c:37-116) on nthreads host threads ---- */
typedef struct {
    uint8_t* coded;
    int T, pkts, pkt_bytes;
    double seconds;
    long long frames;
    double elapsed;
} speed_job_t;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void* speed_worker(void* arg) {
    speed_job_t* j = (speed_job_t*)arg;
    viterbiHardState_t* st = new_state();
    uint8_t* out = (uint8_t*)malloc((size_t)j->pkt_bytes);
    long long frames = 0;
    int pkt = 0;
    double t0 = now_s(), t1 = t0;
    while (1) {
        for (int i = 0; i < 100; i++) { /* PRINT_CHECK_INTERVAL */
            VITERBI_DECODER_HARD(st, j->coded + (size_t)pkt * j->T, out, j->T, true);
            pkt = (pkt + 1) % j->pkts;
            frames++;
            __asm__ volatile("" : : "r"(out) : "memory");
        }
        t1 = now_s();
        if (t1 - t0 >= j->seconds) break;
    }
    j->frames = frames;
    j->elapsed = t1 - t0;
    free(out);
    free(st);
    return NULL;
}

/* Returns aggregate decoded Mbit/s over nthreads independent decoder states. */
double ref_speed(double seconds, int nthreads, int pkt_bytes) {
    enum { PKTS = 16 };
    int T = 8 * pkt_bytes / k + S;
    uint8_t* unc = (uint8_t*)malloc((size_t)PKTS * pkt_bytes);
    uint8_t* coded = (uint8_t*)malloc((size_t)PKTS * T);
    srand(314); /* speedDecode.c:38 */
    for (int i = 0; i < PKTS * pkt_bytes; i++) unc[i] = (uint8_t)rand();
    for (int i = 0; i < PKTS; i++) ref_encode(unc + (size_t)i * pkt_bytes, pkt_bytes, coded + (size_t)i * T);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    speed_job_t* jobs = (speed_job_t*)calloc((size_t)nthreads, sizeof(speed_job_t));
    for (int i = 0; i < nthreads; i++) {
        jobs[i] = (speed_job_t){coded, T, PKTS, pkt_bytes, seconds, 0, 0.0};
        pthread_create(&th[i], NULL, speed_worker, &jobs[i]);
    }
    double mbps = 0.0;
    for (int i = 0; i < nthreads; i++) {
        pthread_join(th[i], NULL);
        if (jobs[i].elapsed > 0) mbps += (double)jobs[i].frames * 8.0 * pkt_bytes / jobs[i].elapsed / 1e6;
    }
    free(th);
    free(jobs);
    free(unc);
    free(coded);
    return mbps;
}
