/*
 * oracle/rans_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker).
 *
 * A plain-C restatement of the reference's native rANS coder
 *   /root/reference/rans/rans.pyx (Cython source) and the exact types of its
 *   generated code /root/reference/rans/rans.cpp.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product path (HIP kernels behind include/idf_codec.h)
 * never links or calls it.
 *
 * Parity pinning: checked bit-for-bit against (a) the reference's compiled
 * Cython coder (oracle/_ref, built by oracle/Makefile from rans.cpp) and
 * (b) the committed golden vectors in tests/golden/ (KAT1 of SURVEY App. C,
 * rans/test.py-style random streams, per-(image,level) flow streams, edges).
 *
 * Arithmetic follows the generated C++ exactly:
 *   - libm expf / round / roundf (the reference links these from libm),
 *   - the float/double mix of each expression,
 *   - compiled with -ffp-contract=off so no FMA is introduced.
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_OK 0
#define ORACLE_ERR_SCALE_ZERO 1   /* ZeroDivisionError("float division")             rans.cpp:1435-1438 */
#define ORACLE_ERR_FREQ_ZERO 2    /* ZeroDivisionError("integer division or modulo") rans.cpp:1825-1834 */
#define ORACLE_ERR_NEG_CDF 3      /* OverflowError: negative CDF -> unsigned long long (decode)  */
#define ORACLE_ERR_UNDERFLOW 4    /* decode read past the word buffer (UB in the reference)      */

/* rans.pyx:13-22 */
static const uint64_t RANS_L = 0x100000000ull;
static const uint64_t RANS_MASK = 0xffffffffull;
static const uint64_t RANS_M = 0x1000000ull;

/* rans.pyx:25-26 logistic(x: float) = 1.0 / (1.0 + exp(-x)); exp(float) -> expf. */
static double logistic(float x) { return 1.0 / (1.0 + (double)expf(-x)); }

/* rans.pyx:31-35, rans.cpp:1395-1484.
 * part2 = int(round((x - lower) * 256)) + 1      (f32 subtraction, f64 multiply, libm round)
 * part1 = int(round(logistic((x + 0.5/256 - mean) / scale) * (M - 2048)))
 *         (f64 chain -> f32 argument -> expf; double * 16775168 -> f32 -> roundf) */
int oracle_cdf(float x, float mean, float scale, float lower, int *err) {
    float d = x - lower;
    int part2 = (int)round((double)d * 256.0) + 1;
    double t = ((double)x + (0.5 / 256.0)) - (double)mean;
    if (scale == 0.0f) {
        if (err) *err = ORACLE_ERR_SCALE_ZERO;
        return 0;
    }
    float u = (float)(t / (double)scale);
    float p = (float)(logistic(u) * (double)(RANS_M - 2048));
    int part1 = (int)roundf(p);
    return part1 + part2;
}

/* rans.pyx:51 lower = int(round(mean*256 - 1024)) / 256.   (as float) */
static float enc_lower(float mean) {
    double r = round((double)mean * 256.0 - 1024.0);
    return (float)(r / 256.0);
}

/* Pass 1 of encode (rans.pyx:50-56): per-symbol start (cdf) and freq. */
int oracle_cdf_freq(int64_t n, const float *x, const float *mean, const float *scale,
                    int32_t *start_out, int32_t *freq_out) {
    int err = 0;
    for (int64_t i = 0; i < n; ++i) {
        float lower = enc_lower(mean[i]);
        float xm = (float)((double)x[i] - 1.0 / 256.0);
        int start = oracle_cdf(xm, mean[i], scale[i], lower, &err);
        if (err) return err;
        int end = oracle_cdf(x[i], mean[i], scale[i], lower, &err);
        if (err) return err;
        start_out[i] = start;
        freq_out[i] = end - start;
    }
    return ORACLE_OK;
}

/* rans.pyx:37-67.  words are written in push order; *nwords is the count. */
int oracle_rans_encode(uint64_t *state_io, int64_t n, const float *x, const float *mean,
                       const float *scale, uint32_t *words, int64_t *nwords) {
    uint64_t state = *state_io;
    int64_t nw = 0;
    /* pass 1 (rans.pyx:50-56): vector<ull> cdf, freq */
    int32_t *st = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int32_t *fr = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    if (!st || !fr) { free(st); free(fr); return -1; }
    int err = oracle_cdf_freq(n, x, mean, scale, st, fr);
    if (err) { free(st); free(fr); return err; }
    /* pass 2 (rans.pyx:61-66) */
    for (int64_t i = 0; i < n; ++i) {
        uint64_t cdf = (uint64_t)(int64_t)st[i];       /* vector<ull>.push_back(int) */
        uint64_t freq = (uint64_t)(int64_t)fr[i];
        if (state >= (freq << 40)) {
            words[nw++] = (uint32_t)(state & RANS_MASK);
            state >>= 32;
        }
        if (freq == 0) { free(st); free(fr); return ORACLE_ERR_FREQ_ZERO; }
        state = ((state / freq) << 24) + (state % freq) + cdf;
    }
    free(st);
    free(fr);
    *state_io = state;
    *nwords = nw;
    return ORACLE_OK;
}

/* rans.pyx:69-110.  The reference receives buffer, mean and scale REVERSED and
 * returns the symbols reversed.  Here: words in push order (read from the end),
 * mean/scale/out in natural order, symbol i = n-1 decoded first.  This is the
 * same computation with the reversal folded into indexing. */
int oracle_rans_decode(uint64_t *state_io, const uint32_t *words, int64_t nwords, int64_t n,
                       const float *mean, const float *scale, float *out) {
    uint64_t state = *state_io;
    int64_t pos = nwords;  /* next word to read is words[pos-1] */
    int err = 0;
    for (int64_t j = 0; j < n; ++j) {
        int64_t i = n - 1 - j;
        if (state < RANS_L) {
            if (pos <= 0) return ORACLE_ERR_UNDERFLOW;
            state = (state << 32) | (uint64_t)words[--pos];
        }
        uint64_t mod = state & 0xffffff;
        int lower = (int)round((double)mean[i] * 256.0 - 1024.0);
        int upper = lower + 0x7FF;
        float lower_f = (float)(lower / 256.);
        while (lower <= upper) {
            int s = (lower + upper) >> 1;
            int c = oracle_cdf((float)(s / 256.), mean[i], scale[i], lower_f, &err);
            if (err) return err;
            if (c < 0) return ORACLE_ERR_NEG_CDF;
            if ((uint64_t)c > mod) upper = s - 1;
            else lower = s + 1;
        }
        int s = lower;
        out[i] = (float)(s / 256.);
        int c0 = oracle_cdf((float)((s - 1) / 256.), mean[i], scale[i], lower_f, &err);
        if (err) return err;
        if (c0 < 0) return ORACLE_ERR_NEG_CDF;
        int c1 = oracle_cdf((float)(s / 256.), mean[i], scale[i], lower_f, &err);
        if (c1 - c0 < 0) return ORACLE_ERR_NEG_CDF;
        uint64_t cdf_s = (uint64_t)c0;
        uint64_t freq_s = (uint64_t)(c1 - c0);
        state = (state >> 24) * freq_s + (state & 0xffffff) - cdf_s;
    }
    *state_io = state;
    (void)pos;
    return ORACLE_OK;
}

/* Consumed-word count of the last decode is implied: every word is read once. */

/* Batched helpers over independent streams (stream k = symbols
 * [sym_off[k], sym_off[k+1]) coded from init_state[k]).  Words of stream k land
 * at words + sym_off[k] (capacity = its symbol count; at most one word per
 * symbol is possible, rans.pyx:62-64).  Optional OpenMP over streams for the
 * CPU baseline; results do not depend on the thread count. */
int oracle_encode_streams(int64_t nstreams, const int64_t *sym_off, const float *x,
                          const float *mean, const float *scale, const uint64_t *init_state,
                          uint64_t *final_state, uint32_t *words, int64_t *nwords,
                          int32_t *status) {
    int any = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(| : any)
    for (int64_t k = 0; k < nstreams; ++k) {
        uint64_t st = init_state[k];
        int64_t nw = 0;
        int64_t b = sym_off[k], n = sym_off[k + 1] - sym_off[k];
        int e = oracle_rans_encode(&st, n, x + b, mean + b, scale + b, words + b, &nw);
        final_state[k] = st;
        nwords[k] = nw;
        status[k] = e;
        any |= (e != 0);
    }
    return any;
}

int oracle_decode_streams(int64_t nstreams, const int64_t *sym_off, const int64_t *word_off,
                          const int64_t *nwords, const uint32_t *words, const float *mean,
                          const float *scale, const uint64_t *init_state, uint64_t *final_state,
                          float *out, int32_t *status) {
    int any = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(| : any)
    for (int64_t k = 0; k < nstreams; ++k) {
        uint64_t st = init_state[k];
        int64_t b = sym_off[k], n = sym_off[k + 1] - sym_off[k];
        int e = oracle_rans_decode(&st, words + word_off[k], nwords[k], n, mean + b, scale + b,
                                   out + b);
        final_state[k] = st;
        status[k] = e;
        any |= (e != 0);
    }
    return any;
}

/* Host libm expf, exposed so tests can compare the device restatement of
 * glibc's expf against the exact function the reference calls. */
void oracle_expf_many(int64_t n, const float *in, float *out) {
    for (int64_t i = 0; i < n; ++i) out[i] = expf(in[i]);
}

int oracle_omp_threads(void) {
#ifdef _OPENMP
    extern int omp_get_max_threads(void);
    return omp_get_max_threads();
#else
    return 1;
#endif
}
