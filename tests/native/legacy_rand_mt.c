/* GPU test program (tests/test_gpu_legacy.py::test_rand_stream_kept_across_threads): the
 * legacy drop-in keeps the caller's glibc rand() stream across decoder calls made from many
 * threads at once (csrc/legacy/viterbiDecoder.c, KEEP_RAND).
 *
 *   1. srand(42); the first N draws are the expected stream.
 *   2. srand(42); draw 5; then T threads decode frames through VITERBI_DECODER_HARD at once
 *      (the GPU runtime draws from rand() inside those calls), main thread waiting;
 *   3. the next N - 5 draws must continue the expected stream, and the process's random
 *      state must be the one it was before the threads (not a worker's or the library's).
 * Frames come from an xorshift generator, never from rand().  Prints "OK" and exits 0, or
 * the first mismatch and exits 1.
 *   legacy_rand_mt <threads> <frames per thread> */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "convEncode.h"
#include "viterbiDecoder.h"

enum { PKT_BYTES = 256, NDRAW = 200 };
#define T_SEGS (8 * PKT_BYTES / k + S)

typedef struct {
    int id, frames, bad;
} job_t;

static uint64_t xs(uint64_t* s) {
    *s ^= *s << 13;
    *s ^= *s >> 7;
    *s ^= *s << 17;
    return *s;
}

static void* worker(void* p) {
    job_t* j = (job_t*)p;
    viterbiHardState_t* st = (viterbiHardState_t*)malloc(sizeof(viterbiHardState_t));
    convEncoderState_t enc;
    uint8_t unc[PKT_BYTES], out[PKT_BYTES + 1], coded[T_SEGS];
    uint64_t seed = 0x9E3779B97F4A7C15ull * (uint64_t)(j->id + 1);
    VITERBI_RESET(st);
    VITERBI_INIT(st);
    for (int f = 0; f < j->frames; f++) {
        for (int b = 0; b < PKT_BYTES; b++) unc[b] = (uint8_t)xs(&seed);
        resetConvEncoder(&enc);
        initConvEncoder(&enc);
        convEnc(&enc, unc, coded, PKT_BYTES, true);
        int r = VITERBI_DECODER_HARD(st, coded, out, T_SEGS, true);
        if (r != PKT_BYTES || memcmp(out, unc, PKT_BYTES) != 0) j->bad++;
    }
    free(st);
    return NULL;
}

static char* current_state(void) {
    static int32_t probe[32];
    static int ready;
    if (!ready) {
        /* a valid TYPE_3 state to switch to and straight back from */
        char* was = initstate(7u, (char*)probe, sizeof(probe));
        setstate(was);
        ready = 1;
    }
    char* was = setstate((char*)probe);
    setstate(was);
    return was;
}

int main(int argc, char** argv) {
    const int nthreads = argc > 1 ? atoi(argv[1]) : 8;
    const int frames = argc > 2 ? atoi(argv[2]) : 20;
    int expect[NDRAW];
    srand(42);
    for (int i = 0; i < NDRAW; i++) expect[i] = rand();
    (void)current_state();  /* set the probe up before the reference point */
    srand(42);
    char* before = current_state();
    int got[NDRAW];
    for (int i = 0; i < 5; i++) got[i] = rand();
    pthread_t th[64];
    job_t jobs[64];
    int nt = nthreads < 64 ? nthreads : 64;
    for (int t = 0; t < nt; t++) {
        jobs[t].id = t, jobs[t].frames = frames, jobs[t].bad = 0;
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    int bad = 0;
    for (int t = 0; t < nt; t++) {
        pthread_join(th[t], NULL);
        bad += jobs[t].bad;
    }
    char* after = current_state();
    for (int i = 5; i < NDRAW; i++) got[i] = rand();
    if (bad) {
        printf("FAIL: %d frames decoded wrong\n", bad);
        return 1;
    }
    if (after != before) {
        printf("FAIL: random state moved from %p to %p\n", (void*)before, (void*)after);
        return 1;
    }
    for (int i = 0; i < NDRAW; i++) {
        if (got[i] != expect[i]) {
            printf("FAIL: draw %d is %d, expected %d\n", i, got[i], expect[i]);
            return 1;
        }
    }
    printf("OK %d threads x %d frames, rand() stream and state kept\n", nt, frames);
    return 0;
}
