/*
 * TEST INFRASTRUCTURE ONLY -- NOT PART OF THE PRODUCT.  See viterbi_oracle.h.
 *
 * Plain-C restatement of the reference algorithm, written from its behaviour (each
 * function cites the reference file:line it follows).  Kept deliberately simple and
 * scalar: it is the checker, not the thing measured.
 */
#include "viterbi_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_MAX_S 12

static int parity64(uint64_t x) { return __builtin_popcountll(x) & 1; }

/* convEncode.c:163-174 -- reverse the K low bits (Proakis MSB = newest input -> LSB). */
static uint64_t reverse_bits(uint64_t v, int bits) {
    uint64_t r = 0;
    for (int i = 0; i < bits; i++) {
        r = (r << 1) | (v & 1u);
        v >>= 1;
    }
    return r;
}

/* convEncode.c:132-161 -- output bit j = parity(tappedDelay & rev(g[j])), g[0] in the LSB. */
static uint8_t enc_output(uint64_t tapped, const uint64_t polys[2]) {
    return (uint8_t)(parity64(tapped & polys[0]) | (parity64(tapped & polys[1]) << 1));
}

int oracle_config_check(int K, const uint64_t g[2]) {
    for (int i = 0; i < 2; i++) {
        if (!((g[i] >> (K - 1)) & 1u) || !(g[i] & 1u)) return i + 1; /* viterbiDecoder.c:20-23 */
    }
    return 0;
}

void oracle_edge_table(int K, const uint64_t g[2], uint8_t* symm) {
    uint64_t polys[2] = {reverse_bits(g[0], K), reverse_bits(g[1], K)};
    int half = 1 << (K - 2);
    for (int i = 0; i < half; i++) {
        /* tappedDelay = i, then convEncOneInput shifts in a 0 (convEncode.c:19-44). */
        symm[i] = enc_output(((uint64_t)i) << 1, polys);
    }
}

int oracle_encode(int K, const uint64_t g[2], const uint8_t* uncoded, int nbytes, uint8_t* coded) {
    uint64_t polys[2] = {reverse_bits(g[0], K), reverse_bits(g[1], K)};
    uint64_t mask = (K >= 64) ? ~0ull : ((1ull << K) - 1);
    uint64_t reg = 0; /* STARTING_STATE (convEncode.c:6-11) */
    int out = 0;
    for (int b = 0; b < nbytes; b++) {
        for (int i = 7; i >= 0; i--) { /* MSB first (convEncode.c:76-89) */
            reg = ((reg << 1) | ((uncoded[b] >> i) & 1u)) & mask;
            coded[out++] = enc_output(reg, polys);
        }
    }
    for (int i = 0; i < K - 1; i++) { /* S zero-tail segments (convEncode.c:100-115) */
        reg = (reg << 1) & mask;
        coded[out++] = enc_output(reg, polys);
    }
    return out;
}

/* viterbiDecoderButterflyk1.c:200-256 -- terminated traceback from state 0, skip S tail
 * decisions, pack the info bits MSB-first. dec is T rows of N bytes. */
static int traceback(int S, const uint8_t* dec, int T, uint8_t* out) {
    int N = 1 << S;
    if (T <= S) return -1;
    unsigned s = 0;
    for (int i = 0; i < S; i++) {
        int t = T - 1 - i;
        s = (s >> 1) | ((unsigned)dec[(size_t)t * N + s] << (S - 1));
    }
    int L = T - S;
    out[(L - 1) / 8] = 0; /* :226-227 */
    for (int t = L - 1; t >= 0; t--) {
        out[t / 8] = (uint8_t)((out[t / 8] >> 1) | ((s & 1u) << 7));
        s = (s >> 1) | ((unsigned)dec[(size_t)t * N + s] << (S - 1));
    }
    return (L - 1) / 8 + 1; /* :256 */
}

int oracle_decode_hard(int K, const uint64_t g[2], const uint8_t* coded, int T, uint8_t* out) {
    int S = K - 1, N = 1 << S, half = N / 2;
    if (S < 1 || S > ORACLE_MAX_S || T <= S) return -1;
    uint8_t symm[1 << ORACLE_MAX_S];
    oracle_edge_table(K, g, symm);
    uint8_t m[1 << ORACLE_MAX_S], nm[1 << ORACLE_MAX_S];
    uint8_t* dec = (uint8_t*)malloc((size_t)T * N);
    if (!dec) return -1;
    m[0] = 0; /* viterbiDecoderButterflyk1.c:59 */
    for (int i = 1; i < N; i++) m[i] = (uint8_t)(N + 1); /* :62-67, deliberately truncated */
    unsigned renorm = 0;
    for (int t = 0; t < T; t++) {
        uint8_t c = coded[t] & 3u; /* calcHammingDist reads the low n bits (viterbiDecoder.c:278-281) */
        uint8_t* d = dec + (size_t)t * N;
        for (int b = 0; b < half; b++) {
            uint8_t e = (uint8_t)__builtin_popcount((symm[b] ^ c) & 3u); /* :104 */
            uint8_t ec = (uint8_t)(2 - e);                              /* :107 */
            uint8_t a0 = (uint8_t)(m[b] + e), a1 = (uint8_t)(m[half + b] + ec);
            uint8_t b0 = (uint8_t)(m[b] + ec), b1 = (uint8_t)(m[half + b] + e);
            uint8_t ad = a0 > a1, bd = b0 > b1; /* strict '>' (:129-130) */
            nm[2 * b] = ad ? a1 : a0;
            nm[2 * b + 1] = bd ? b1 : b0;
            d[2 * b] = ad;
            d[2 * b + 1] = bd;
        }
        if (renorm >= 120) { /* :159-183 */
            uint8_t mn = nm[0];
            for (int i = 1; i < N; i++)
                if (nm[i] < mn) mn = nm[i];
            for (int i = 0; i < N; i++) nm[i] = (uint8_t)(nm[i] - mn);
            renorm = 0;
        } else {
            renorm++;
        }
        memcpy(m, nm, (size_t)N);
    }
    int r = traceback(S, dec, T, out);
    free(dec);
    return r;
}

int oracle_decode_soft(int K, const uint64_t g[2], const uint8_t* q, int T, uint8_t* out) {
    int S = K - 1, N = 1 << S, half = N / 2;
    if (S < 1 || S > ORACLE_MAX_S || T <= S) return -1;
    uint8_t symm[1 << ORACLE_MAX_S];
    oracle_edge_table(K, g, symm);
    int32_t m[1 << ORACLE_MAX_S], nm[1 << ORACLE_MAX_S];
    uint8_t* dec = (uint8_t*)malloc((size_t)T * N);
    if (!dec) return -1;
    m[0] = 0;
    for (int i = 1; i < N; i++) m[i] = (int32_t)(uint8_t)(N + 1) * 255;
    for (int t = 0; t < T; t++) {
        int q0 = q[2 * t], q1 = q[2 * t + 1];
        uint8_t* d = dec + (size_t)t * N;
        for (int b = 0; b < half; b++) {
            int e = ((symm[b] & 1u) ? 255 - q0 : q0) + ((symm[b] & 2u) ? 255 - q1 : q1);
            int ec = 510 - e;
            int32_t a0 = m[b] + e, a1 = m[half + b] + ec;
            int32_t b0 = m[b] + ec, b1 = m[half + b] + e;
            uint8_t ad = a0 > a1, bd = b0 > b1;
            nm[2 * b] = ad ? a1 : a0;
            nm[2 * b + 1] = bd ? b1 : b0;
            d[2 * b] = ad;
            d[2 * b + 1] = bd;
        }
        memcpy(m, nm, sizeof(int32_t) * (size_t)N);
    }
    int r = traceback(S, dec, T, out);
    free(dec);
    return r;
}

typedef struct {
    int K, soft, T;
    const uint64_t* g;
    const uint8_t* in;
    size_t in_stride;
    uint8_t* out;
    size_t out_stride;
    size_t lo, hi;
    int err;
} batch_job_t;

static void* batch_worker(void* arg) {
    batch_job_t* j = (batch_job_t*)arg;
    for (size_t f = j->lo; f < j->hi; f++) {
        const uint8_t* in = j->in + f * j->in_stride;
        uint8_t* out = j->out + f * j->out_stride;
        int r = j->soft ? oracle_decode_soft(j->K, j->g, in, j->T, out)
                        : oracle_decode_hard(j->K, j->g, in, j->T, out);
        if (r < 0) j->err = 1;
    }
    return NULL;
}

int oracle_decode_batch(int K, const uint64_t g[2], int soft, const uint8_t* in, size_t in_stride,
                        int T, uint8_t* out, size_t out_stride, size_t frames, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    batch_job_t jobs[64];
    size_t per = (frames + (size_t)nthreads - 1) / (size_t)nthreads;
    int started = 0;
    for (int i = 0; i < nthreads; i++) {
        size_t lo = (size_t)i * per, hi = lo + per;
        if (lo >= frames) break;
        if (hi > frames) hi = frames;
        jobs[i] = (batch_job_t){K, soft, T, g, in, in_stride, out, out_stride, lo, hi, 0};
        if (pthread_create(&th[i], NULL, batch_worker, &jobs[i]) != 0) {
            batch_worker(&jobs[i]);
            th[i] = 0;
        }
        started++;
    }
    int err = 0;
    for (int i = 0; i < started; i++) {
        if (th[i]) pthread_join(th[i], NULL);
        err |= jobs[i].err;
    }
    return err ? -1 : 0;
}

/* ---- streaming (reference state machine, viterbiHardState_t viterbiDecoder.h:103-146) ---- */
#define ORACLE_MAX_SEGMENTS (16384 + ORACLE_MAX_S)

struct oracle_stream {
    int K, S, N;
    uint8_t symm[1 << ORACLE_MAX_S];
    uint8_t m[1 << ORACLE_MAX_S];
    unsigned iteration, renorm;
    uint8_t* dec;
};

oracle_stream_t* oracle_stream_create(int K, const uint64_t g[2]) {
    if (K < 2 || K - 1 > ORACLE_MAX_S) return NULL;
    oracle_stream_t* st = (oracle_stream_t*)calloc(1, sizeof(*st));
    if (!st) return NULL;
    st->K = K;
    st->S = K - 1;
    st->N = 1 << st->S;
    st->dec = (uint8_t*)malloc((size_t)ORACLE_MAX_SEGMENTS * st->N);
    if (!st->dec) {
        free(st);
        return NULL;
    }
    oracle_edge_table(K, g, st->symm);
    oracle_stream_reset(st);
    return st;
}

void oracle_stream_destroy(oracle_stream_t* st) {
    if (!st) return;
    free(st->dec);
    free(st);
}

void oracle_stream_reset(oracle_stream_t* st) { /* viterbiDecoderButterflyk1.c:46-80 */
    st->m[0] = 0;
    for (int i = 1; i < st->N; i++) st->m[i] = (uint8_t)(st->N + 1);
    st->iteration = 0;
    st->renorm = 0;
}

int oracle_stream_decode(oracle_stream_t* st, const uint8_t* coded, int segments, uint8_t* out,
                         int last, uint8_t* metrics_after) {
    int N = st->N, half = N / 2, S = st->S;
    uint8_t nm[1 << ORACLE_MAX_S];
    for (int i = 0; i < segments; i++) {
        if (st->iteration >= ORACLE_MAX_SEGMENTS) return -1;
        uint8_t c = coded[i] & 3u;
        uint8_t* d = st->dec + (size_t)st->iteration * N;
        for (int b = 0; b < half; b++) {
            uint8_t e = (uint8_t)__builtin_popcount((st->symm[b] ^ c) & 3u);
            uint8_t ec = (uint8_t)(2 - e);
            uint8_t a0 = (uint8_t)(st->m[b] + e), a1 = (uint8_t)(st->m[half + b] + ec);
            uint8_t b0 = (uint8_t)(st->m[b] + ec), b1 = (uint8_t)(st->m[half + b] + e);
            uint8_t ad = a0 > a1, bd = b0 > b1;
            nm[2 * b] = ad ? a1 : a0;
            nm[2 * b + 1] = bd ? b1 : b0;
            d[2 * b] = ad;
            d[2 * b + 1] = bd;
        }
        if (st->renorm >= 120) {
            uint8_t mn = nm[0];
            for (int j = 1; j < N; j++)
                if (nm[j] < mn) mn = nm[j];
            for (int j = 0; j < N; j++) nm[j] = (uint8_t)(nm[j] - mn);
            st->renorm = 0;
        } else {
            st->renorm++;
        }
        memcpy(st->m, nm, (size_t)N);
        st->iteration++;
    }
    if (metrics_after) memcpy(metrics_after, st->m, (size_t)N);
    int r = 0;
    if (last) {
        r = traceback(S, st->dec, (int)st->iteration, out);
        oracle_stream_reset(st);
    }
    return r;
}

long oracle_bertest_stream(int K, const uint64_t g[2], unsigned seed, int nconfigs, const double* p,
                           int npkts, int pkt_bytes, uint8_t* uncoded, uint8_t* corrupted) {
    int T = 8 * pkt_bytes + K - 1;
    uint8_t* coded = (uint8_t*)malloc((size_t)T);
    if (!coded) return -1;
    long flips = 0;
    srand(seed); /* berTestK7.c:66 */
    for (int c = 0; c < nconfigs; c++) {
        for (int k = 0; k < npkts; k++) {
            uint8_t* u = uncoded + ((size_t)c * npkts + k) * pkt_bytes;
            uint8_t* x = corrupted + ((size_t)c * npkts + k) * T;
            for (int j = 0; j < pkt_bytes; j++) u[j] = (uint8_t)rand(); /* :135-138 */
            oracle_encode(K, g, u, pkt_bytes, coded);                  /* :142 */
            for (int i = 0; i < T; i++) {                               /* :29-43 */
                uint8_t corrupt = 0;
                for (int j = 0; j < 2; j++) {
                    double fr = (double)rand() / RAND_MAX;
                    uint8_t flip = fr > p[c] ? 0 : 1;
                    corrupt = (uint8_t)((corrupt << 1) | flip);
                    flips += flip;
                }
                x[i] = coded[i] ^ corrupt;
            }
        }
    }
    free(coded);
    return flips;
}

long oracle_bit_errors(const uint8_t* a, const uint8_t* b, size_t len) {
    long e = 0;
    for (size_t i = 0; i < len; i++) e += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return e;
}

/* ---- device frame generator checker (specification: include/viterbi_amd.h) ---- */

static uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

uint64_t oracle_rand64(uint64_t seed, uint64_t frame, uint64_t ctr) {
    return mix64(mix64(seed + 0x9E3779B97F4A7C15ull * (frame + 1)) ^ (0xD1B54A32D192ED03ull * (ctr + 1)));
}

void oracle_gen_payload(uint64_t seed, int bits, uint8_t* out, size_t stride, size_t frames) {
    const int nbytes = (bits + 7) / 8;
    for (size_t f = 0; f < frames; f++)
        for (int j = 0; j < nbytes; j++) {
            unsigned v = (unsigned)(oracle_rand64(seed, f, (uint64_t)(j / 8)) >> (8 * (j % 8))) & 0xFFu;
            if (j == nbytes - 1 && (bits % 8)) v &= (0xFFu << (8 - bits % 8)) & 0xFFu;
            out[f * stride + j] = (uint8_t)v;
        }
}

/* Bit-serial restatement of convEnc: shift each information bit (MSB-first) into the
 * tapped delay line's LSB and emit parity(delay & reverse_K(g_j)) as bit j
 * (convEncode.c:63-97, 132-161); then K-1 zero shifts (:100-122). */
void oracle_gen_encode(int K, const uint64_t g[2], int bits, const uint8_t* unc, size_t in_stride, uint8_t* coded,
                       size_t out_stride, size_t frames) {
    uint64_t rg[2] = {0, 0};
    for (int j = 0; j < 2; j++)
        for (int i = 0; i < K; i++) rg[j] |= ((g[j] >> i) & 1u) << (K - 1 - i);
    const uint64_t mask = (1ull << K) - 1;
    for (size_t f = 0; f < frames; f++) {
        uint64_t delay = 0;
        for (int t = 0; t < bits + K - 1; t++) {
            const unsigned b = t < bits ? (unc[f * in_stride + t / 8] >> (7 - t % 8)) & 1u : 0u;
            delay = ((delay << 1) | b) & mask;
            coded[f * out_stride + t] =
                (uint8_t)((__builtin_popcountll(delay & rg[0]) & 1) | ((__builtin_popcountll(delay & rg[1]) & 1) << 1));
        }
    }
}

void oracle_gen_bsc(uint64_t seed, uint32_t p32, int T, const uint8_t* coded, size_t in_stride, uint8_t* rx,
                    size_t out_stride, size_t frames) {
    for (size_t f = 0; f < frames; f++)
        for (int t = 0; t < T; t++) {
            const uint64_t r = oracle_rand64(seed, f, (uint64_t)t);
            unsigned c = coded[f * in_stride + t] & 3u;
            if ((uint32_t)r < p32) c ^= 1u;
            if ((uint32_t)(r >> 32) < p32) c ^= 2u;
            rx[f * out_stride + t] = (uint8_t)c;
        }
}

void oracle_gen_awgn8(uint64_t seed, int64_t kq, int T, const uint8_t* coded, size_t in_stride, uint8_t* rx,
                      size_t out_stride, size_t frames) {
    for (size_t f = 0; f < frames; f++)
        for (int t = 0; t < T; t++)
            for (int i = 0; i < 2; i++) {
                int64_t z = -(6ll << 21);
                for (int h = 0; h < 4; h++) {
                    const uint64_t r = oracle_rand64(seed, f, 8ull * (uint64_t)t + 4u * (unsigned)i + (unsigned)h);
                    z += (int64_t)(r & 0x1FFFFF) + (int64_t)((r >> 21) & 0x1FFFFF) + (int64_t)((r >> 42) & 0x1FFFFF);
                }
                const int64_t prod = kq * z;
                const int64_t v = prod >= 0 ? prod / (1 << 21) : -((-prod + (1 << 21) - 1) / (1 << 21)); /* floor */
                const int b = (coded[f * in_stride + t] >> i) & 1;
                const int64_t qf = (b ? (255ll << 16) : 0) - v + 32768;
                int64_t q = qf >= 0 ? qf / 65536 : -((-qf + 65535) / 65536); /* floor */
                q = q < 0 ? 0 : (q > 255 ? 255 : q);
                rx[f * out_stride + 2 * (size_t)t + i] = (uint8_t)q;
            }
}

int64_t oracle_awgn_kq(double snr_db) {
    const double esn0 = pow(10.0, (snr_db + 10.0 * log10(4.0)) / 10.0);
    return (int64_t)llround(sqrt(1.0 / (2.0 * esn0)) * 127.5 * 65536.0);
}

uint32_t oracle_bsc_p32(double p) {
    if (!(p > 0.0)) return 0u;
    if (p >= 1.0) return 0xFFFFFFFFu;
    return (uint32_t)floor(p * 4294967296.0);
}

/* ---- general rate-k/n codes (header: oracle_genk_*) ---- */

static uint64_t genk_rev(uint64_t g, int bits) { /* convEncode.c:163-174 */
    uint64_t r = 0;
    for (int i = 0; i < bits; i++) r = (r << 1) | ((g >> i) & 1u);
    return r;
}

static uint8_t genk_out(int n, const uint64_t* rg, uint64_t delay) { /* convEncode.c:132-161 */
    uint8_t o = 0;
    for (int i = 0; i < n; i++) o |= (uint8_t)(parity64(delay & rg[i]) << i);
    return o;
}

int oracle_genk_encode(int k, int K, int n, const uint64_t* g, const uint8_t* uncoded, int nbytes, uint8_t* coded) {
    if (k < 1 || K < 2 || n < 1 || n > 8 || k * K > 64 || (nbytes * 8) % k) return -1;
    uint64_t rg[8];
    for (int i = 0; i < n; i++) rg[i] = genk_rev(g[i], k * K);
    uint64_t delay = 0;
    int seg = 0, pos = 0;
    for (int c = 0; c < nbytes * 8 / k; c++) { /* convEncode.c:55-97 */
        for (int j = 0; j < k; j++, pos++) delay = (delay << 1) | ((uncoded[pos >> 3] >> (7 - (pos & 7))) & 1u);
        coded[seg++] = genk_out(n, rg, delay);
    }
    for (int i = 0; i < K - 1; i++) { /* :99-122, termination */
        delay <<= k;
        coded[seg++] = genk_out(n, rg, delay);
    }
    return seg;
}

int oracle_genk_decode(int k, int K, int n, const uint64_t* g, const uint8_t* coded, int info_bits, uint8_t* out) {
    const int S = K - 1, kS = k * S;
    if (k < 1 || K < 2 || n < 1 || n > 8 || kS > 16 || info_bits < 1 || info_bits % k) return -1;
    const int N = 1 << kS, E = 1 << k, T = info_bits / k + S;
    uint64_t rg[8];
    for (int i = 0; i < n; i++) rg[i] = genk_rev(g[i], k * K);
    int32_t* m = malloc(sizeof(int32_t) * 2 * (size_t)N);
    uint8_t* dec = malloc((size_t)T * N);
    if (!m || !dec) {
        free(m);
        free(dec);
        return -1;
    }
    int32_t *cur = m, *nxt = m + N;
    for (int s = 0; s < N; s++) cur[s] = s == 0 ? 0 : (int32_t)(uint8_t)(N + 1);
    for (int t = 0; t < T; t++) {
        const uint8_t rx = coded[t];
        for (int d = 0; d < N; d++) {
            const int bits = d & (E - 1);
            int32_t best = 0;
            int be = 0;
            for (int e = 0; e < E; e++) {
                const int src = (d >> k) | (e << (kS - k));
                const uint64_t delay = ((uint64_t)src << k) | (uint64_t)bits;
                const int32_t pm = cur[src] + __builtin_popcount((unsigned)(genk_out(n, rg, delay) ^ rx) & ((1u << n) - 1));
                if (e == 0 || pm < best) best = pm, be = e; /* first minimum */
            }
            nxt[d] = best;
            dec[(size_t)t * N + d] = (uint8_t)be;
        }
        int32_t* x = cur;
        cur = nxt;
        nxt = x;
    }
    const int nb = (info_bits + 7) / 8;
    memset(out, 0, (size_t)nb);
    int s = 0;
    for (int t = T - 1; t >= 0; t--) {
        if (t < T - S) {
            const int seg = s & (E - 1);
            for (int j = 0; j < k; j++) {
                const int pos = t * k + j;
                if ((seg >> (k - 1 - j)) & 1) out[pos >> 3] |= (uint8_t)(0x80u >> (pos & 7));
            }
        }
        s = (s >> k) | ((int)dec[(size_t)t * N + s] << (kS - k));
    }
    free(m);
    free(dec);
    return nb;
}

/* The generic decoder's metric update over `count` segments (reference
 * src/viterbiDecoder.c:84-131: destination-indexed, predecessors src = d/2^k + e*2^((S-1)k),
 * path metric = source metric + Hamming distance of the edge label, first minimum), from
 * the metrics in m[N] (updated in place); prev[N] (optional) receives the metrics one step
 * before the last.  Exact uint32 sums: the reference's METRIC_TYPE is wide enough for
 * MAX_PKT_LEN_SEGMENTS steps at k > 1 (viterbiDecoder.h:51-60). */
int oracle_genk_metrics(int k, int K, int n, const uint64_t* g, const uint8_t* coded, int count, uint32_t* m,
                        uint32_t* prev) {
    const int S = K - 1, kS = k * S;
    if (k < 1 || K < 2 || n < 1 || n > 8 || kS > 16 || count < 0) return -1;
    const int N = 1 << kS, E = 1 << k;
    uint64_t rg[8];
    for (int i = 0; i < n; i++) rg[i] = genk_rev(g[i], k * K);
    uint32_t* buf = malloc(sizeof(uint32_t) * 2 * (size_t)N);
    if (!buf) return -1;
    uint32_t *cur = buf, *nxt = buf + N;
    memcpy(cur, m, sizeof(uint32_t) * (size_t)N);
    memcpy(nxt, m, sizeof(uint32_t) * (size_t)N);
    for (int t = 0; t < count; t++) {
        const uint8_t rx = coded[t];
        for (int d = 0; d < N; d++) {
            const int bits = d & (E - 1);
            uint32_t best = 0;
            for (int e = 0; e < E; e++) {
                const int src = (d >> k) | (e << (kS - k));
                const uint64_t delay = ((uint64_t)src << k) | (uint64_t)bits;
                const uint32_t pm = cur[src] + (uint32_t)__builtin_popcount((unsigned)(genk_out(n, rg, delay) ^ rx) & ((1u << n) - 1));
                if (e == 0 || pm < best) best = pm;
            }
            nxt[d] = best;
        }
        uint32_t* x = cur;
        cur = nxt;
        nxt = x;
    }
    memcpy(m, cur, sizeof(uint32_t) * (size_t)N);
    if (prev) memcpy(prev, nxt, sizeof(uint32_t) * (size_t)N);
    free(buf);
    return 0;
}

/* The reference's k = 1 decoder for any n (viterbiDecoderButterflyk1.c:82-256 with its
 * compile-time n): symmetric edge table symm[j] = label of delay (j << 1) | 0 (:24-29), branch
 * metric e = Hamming distance over the low n bits and its complement n - e for the upper
 * predecessor (:104-107), uint8 sums, strict '>' select (:129-130), subtract-the-minimum
 * renormalisation when the counter reaches 120 (:159-183), traceback from state 0 after S
 * padding steps, MSB-first packing with the last byte zero-padded (:200-256).  Returns the
 * reference's byte count (L - 1) / 8 + 1. */
int oracle_k1n_decode(int K, int n, const uint64_t* g, const uint8_t* coded, int info_bits, uint8_t* out) {
    const int S = K - 1;
    if (K < 3 || K > 9 || n < 1 || n > 8 || info_bits < 1) return -1;
    const int N = 1 << S, T = info_bits + S;
    uint64_t rg[8];
    for (int i = 0; i < n; i++) rg[i] = genk_rev(g[i], K);
    uint8_t symm[128];
    for (int j = 0; j < N / 2; j++) symm[j] = genk_out(n, rg, (uint64_t)j << 1);
    uint8_t m[256], nm[256];
    uint8_t* dec = malloc((size_t)T * N);
    if (!dec) return -1;
    for (int st = 0; st < N; st++) m[st] = st == 0 ? 0 : (uint8_t)(N + 1);
    unsigned counter = 0;
    const unsigned nmask = (1u << n) - 1u;
    for (int t = 0; t < T; t++) {
        for (int j = 0; j < N / 2; j++) {
            const uint8_t em = (uint8_t)__builtin_popcount((unsigned)(symm[j] ^ coded[t]) & nmask);
            const uint8_t ec = (uint8_t)(n - em);
            const uint8_t a0 = (uint8_t)(m[j] + em), a1 = (uint8_t)(m[N / 2 + j] + ec);
            const uint8_t b0 = (uint8_t)(m[j] + ec), b1 = (uint8_t)(m[N / 2 + j] + em);
            nm[2 * j] = a0 > a1 ? a1 : a0;
            nm[2 * j + 1] = b0 > b1 ? b1 : b0;
            dec[(size_t)t * N + 2 * j] = a0 > a1;
            dec[(size_t)t * N + 2 * j + 1] = b0 > b1;
        }
        if (counter >= 120) {
            uint8_t mn = nm[0];
            for (int st = 1; st < N; st++) mn = nm[st] < mn ? nm[st] : mn;
            for (int st = 0; st < N; st++) nm[st] = (uint8_t)(nm[st] - mn);
            counter = 0;
        } else {
            counter++;
        }
        memcpy(m, nm, (size_t)N);
    }
    const int nb = (info_bits - 1) / 8 + 1;
    memset(out, 0, (size_t)nb);
    unsigned st = 0;
    for (int t = T - 1; t >= 0; t--) {
        if (t < T - S && ((st & 1u) != 0)) out[t >> 3] |= (uint8_t)(0x80u >> (t & 7));
        st = (st >> 1) | ((unsigned)dec[(size_t)t * N + st] << (S - 1));
    }
    free(dec);
    return nb;
}
