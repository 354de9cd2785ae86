/*
 * gdbf_oracle.c -- CPU ORACLE of the reference's GDBF / NGDBF bit-flipping
 * decoders (test infrastructure only; see ldpc_oracle.h).
 *
 * Restates ereiss123/LDPCsimulation C_implementations/src/decodeGDBF.cpp in
 * its parallel-flip mode (mu = 1, :284-289) with the compile-time switches of
 * the Makefile targets decodeMNGDBF / decodeSMNGDBF / decodeATGDBF /
 * decodeSATGDBF / decodeSMGDBF (Makefile:33-53) as runtime flags:
 *   addNoise            E += perturbation, a fresh noiseSigma*rann() per bit
 *                       and iteration (:318-333, :559-561)
 *   thresholdAdaptation theta_i *= lambda when bit i did not flip (:612-617)
 *   weightSyndromes     syndrome weight w = alpha instead of 1 (:548-551)
 *   outputSmoothing     d = sgn(sum of d over the last iterations) when the
 *                       checks are not satisfied (:348-367, :371-375)
 *   saturateSamples     |yq| > Ymax -> yq *= Ymax/|yq| (:255-258)
 *   quantizeSamples     quantize() with NQ levels (:265-267, :488-493)
 * and the flip schedules of the other three targets:
 *   sequentialmode      mu = 0: only the first bit of minimal energy flips
 *                       (E < Emin from +inf in index order, :573-580, :619-620)
 *   modeswitching       mu = 1 until, after Tswitch, the objective
 *                       f = sum d*yq + sum s (:623-632, s as checked) before
 *                       the bit update is >= the one after it; then mu = 0
 *                       (:309-311, :338-345)
 *   quantizeProbabilities  flip with probability pcdf = normalCDF((theta - E) /
 *                       noiseSigma) rounded to the nearest of 8 levels, by
 *                       ranu() < level (:562-597); the ranu() draws are the
 *                       caller's pert rows
 * (decodeSGDBF = sequentialmode, decodeMGDBF = modeswitching,
 * decodeStochasticNGDBF = quantizeSamples|quantizeProbabilities|weightSyndromes|
 * saturateSamples, Makefile:24-31).
 * Build: oracle/Makefile (plain IEEE, -ffp-contract=off).
 */
#include "ldpc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* quantize() :488-493 (its own sgn: y > 0 ? 1 : -1, :495-501) */
static double gdbf_quantize(double x, double ymax, int nq)
{
    const double qmax = pow(2, (nq - 1));
    const double lmax = ymax / 2.0;
    const double s = x > 0 ? 1.0 : -1.0;
    return s * floor((fabs(x) * qmax) / (2 * lmax) + 0.5) * (2.0 * lmax / qmax);
}

double orc_gdbf_front(double y, const orc_gdbf_cfg *cfg, int *r)
{
    double yq = y;                                             /* :254 */
    if (cfg->flags & ORC_GDBF_SATURATE)
        if (fabs(yq) > cfg->ymax) yq *= cfg->ymax / fabs(yq);   /* :255-258 */
    *r = yq > 0 ? 1 : -1;                                      /* :259-264 */
    if (cfg->flags & ORC_GDBF_QUANTIZE) yq = gdbf_quantize(yq, cfg->ymax, cfg->nq);   /* :265-267 */
    return yq;
}

float orc_gdbf_front_f32(float y, const orc_gdbf_cfg *cfg, int *r)
{
    float yq = y;
    const float ymax = (float)cfg->ymax;
    if (cfg->flags & ORC_GDBF_SATURATE)
        if (fabsf(yq) > ymax) yq *= ymax / fabsf(yq);
    *r = yq > 0 ? 1 : -1;
    if (cfg->flags & ORC_GDBF_QUANTIZE) {
        const float qmax = (float)pow(2, (cfg->nq - 1));
        const float lmax = ymax / 2.0f;
        const float s = yq > 0 ? 1.0f : -1.0f;
        yq = s * floorf((fabsf(yq) * qmax) / (2 * lmax) + 0.5f) * (2.0f * lmax / qmax);
    }
    return yq;
}

/* One frame of the iteration loop :298-367 from its front-end output:
 * d (in: r, out: decisions), pert [T][N] (may be NULL without addNoise; row
 * `it` is used by iteration it), returns the iterations run (`it` after the
 * loop, :399) and sets *satisfied (:300-306). */
/* The 8 flipping probabilities of quantizeProbabilities (:564-573) and the nearest
 * one to pcdf by squared distance, first minimum (:574-585). */
static const double kPrLevels[8] = {0, 0.0625, 0.125, 0.25, 0.34375, 0.4106, 0.68359, 1};
static double nearest_level(double pcdf)
{
    double min_dist = 1;
    int min_idx = 0;
    for (int j = 0; j < 8; j++) {
        double t = kPrLevels[j] - pcdf;
        t = t * t;
        if (t < min_dist) {
            min_dist = t;
            min_idx = j;
        }
    }
    return kPrLevels[min_idx];
}
static float nearest_level_f32(float pcdf)
{
    float min_dist = 1;
    int min_idx = 0;
    for (int j = 0; j < 8; j++) {
        float t = (float)kPrLevels[j] - pcdf;
        t = t * t;
        if (t < min_dist) {
            min_dist = t;
            min_idx = j;
        }
    }
    return (float)kPrLevels[min_idx];
}
/* normalCDF (:66-69): 0.5 * erfc(-x * M_SQRT1_2) */
static double ncdf_f64(double x) { return 0.5 * erfc(-x * 0.70710678118654752440); }
static float ncdf_f32(float x) { return 0.5f * erfcf(-x * 0.70710678118654752440f); }

#define ORC_DEFINE_GDBF(FT, SUFFIX)                                                     \
int orc_gdbf_decode_##SUFFIX(const orc_alist *H, const FT *yq, const FT *pert,         \
                             const orc_gdbf_cfg *cfg, int8_t *d, int *satisfied)        \
{                                                                                       \
    const int N = H->N, M = H->M, T = cfg->T;                                           \
    int *s = (int *)malloc(sizeof(int) * (M + 1));                                      \
    int *dsum = (int *)calloc((size_t)N + 1, sizeof(int));                              \
    FT *theta = (FT *)malloc(sizeof(FT) * (N + 1));                                     \
    const FT w = (cfg->flags & ORC_GDBF_WEIGHT) ? (FT)cfg->alpha : (FT)1;   /* :541-551 */ \
    const FT lambda = (FT)cfg->lambda;                                                  \
    for (int i = 0; i < N; ++i) theta[i] = (FT)cfg->theta;                 /* :291-294 */ \
    int it, sat = 0;                                                                    \
    int mu = (cfg->flags & ORC_GDBF_SEQUENTIAL) ? 0 : 1;                   /* :284-289 */ \
    const int modesw = (cfg->flags & ORC_GDBF_MODESWITCH) != 0;                         \
    const FT qsig = (FT)cfg->qsigma;                                                    \
    for (it = 0; it < T; ++it) {                                                        \
        sat = 1;                                                                        \
        for (int j = 0; j < M; ++j) {                          /* :517-534 */           \
            int prod = 1;                                                               \
            for (int k = 0; k < H->deg_m[j]; ++k) prod *= d[H->mlist[(long)j * H->maxdc + k] - 1]; \
            if (prod < 0) sat = 0;                                                      \
            s[j] = prod;                                                                \
        }                                                                               \
        if (sat) break;                                        /* :305-306 */           \
        FT f1 = 0;                                                                      \
        if (modesw && it > cfg->tswitch) {                     /* :309-311, :623-632 */ \
            for (int i = 0; i < N; ++i) f1 += (FT)d[i] * yq[i];                         \
            for (int j = 0; j < M; ++j) f1 += (FT)s[j];                                 \
        }                                                                               \
        FT Emin = (FT)INFINITY;                                                         \
        int mindx = -1;                                                                 \
        for (int i = 0; i < N; ++i) {                          /* :536-621 */           \
            int flip = 0;                                                               \
            FT E = (FT)d[i] * yq[i];                                                    \
            for (int k = 0; k < H->deg_n[i]; ++k)                                       \
                E += w * (FT)s[H->nlist[(long)i * H->maxdv + k] - 1];                   \
            if (cfg->flags & ORC_GDBF_NOISE) E += pert[(long)it * N + i];               \
            if (cfg->flags & ORC_GDBF_QPROB) {                 /* :562-597 */           \
                const FT lev = ORC_GDBF_LEVEL_##SUFFIX(ORC_GDBF_NCDF_##SUFFIX((-E + theta[i]) / qsig)); \
                if (pert[(long)it * N + i] < lev) {                                     \
                    flip = 1;                                                           \
                    d[i] = (int8_t)-d[i];                                               \
                }                                                                       \
            } else {                                                                    \
                if (mu == 1 && E < theta[i]) {                 /* :598-603 */           \
                    flip = 1;                                                           \
                    d[i] = (int8_t)-d[i];                                               \
                }                                                                       \
                if (mu == 0 && E < Emin) {                     /* :604-610 */           \
                    flip = 1;                                                           \
                    Emin = E;                                                           \
                    mindx = i;                                                          \
                }                                                                       \
            }                                                                           \
            if ((cfg->flags & ORC_GDBF_ADAPT) && !flip) theta[i] *= lambda;             \
        }                                                                               \
        if (mu == 0 && mindx >= 0) d[mindx] = (int8_t)-d[mindx];   /* :619-620 */       \
        if (modesw && it > cfg->tswitch) {                     /* :338-345 */           \
            FT f2 = 0;                                                                  \
            for (int i = 0; i < N; ++i) f2 += (FT)d[i] * yq[i];                         \
            for (int j = 0; j < M; ++j) f2 += (FT)s[j];                                 \
            if (f1 >= f2) mu = 0;                                                       \
        }                                                                               \
        if ((cfg->flags & ORC_GDBF_SMOOTH) && it > T - cfg->windowsize)  /* :348-354 */ \
            for (int i = 0; i < N; ++i) dsum[i] += d[i];                                \
    }                                                                                   \
    if ((cfg->flags & ORC_GDBF_SMOOTH) && !sat)                /* :358-367 */           \
        for (int i = 0; i < N; ++i) d[i] = dsum[i] > 0 ? 1 : -1;                        \
    free(s); free(dsum); free(theta);                                                   \
    *satisfied = sat;                                                                   \
    return it;                                                                          \
}

#define ORC_GDBF_LEVEL_f64 nearest_level
#define ORC_GDBF_LEVEL_f32 nearest_level_f32
#define ORC_GDBF_NCDF_f64 ncdf_f64
#define ORC_GDBF_NCDF_f32 ncdf_f32
ORC_DEFINE_GDBF(double, f64)
ORC_DEFINE_GDBF(float, f32)

/* main() frame loop :224-413 (parallel mode). */
int64_t orc_gdbf_run(const orc_alist *H, double R, double snr, const orc_gdbf_cfg *cfg, uint32_t seed,
                     const char *const *cw_lines, int ncw, int64_t max_frames,
                     int32_t *frame_w, int32_t *frame_it, int64_t cap, orc_stats *out, int64_t *smoothing_used)
{
    const int N = H->N, T = cfg->T;
    const double N0 = pow(10.0, -snr / 10.0) / R;             /* :175-176 */
    const double sigma = sqrt(N0 / 2.0);
    const double noise_sigma = sigma * cfg->noise_scale;      /* :296 */
    int min_word_errors = 20;                                  /* :221-223 */
    if (N > 10000) min_word_errors = 10;
    if (N > 50000) min_word_errors = 5;
    orc_rng g;
    orc_srandom(&g, seed);                                     /* :224 */
    int *c = (int *)malloc(sizeof(int) * N);
    double *yq = (double *)malloc(sizeof(double) * N);
    double *pert = (double *)malloc(sizeof(double) * (size_t)N * (T > 0 ? T : 1));
    int8_t *d = (int8_t *)malloc((size_t)N);
    memset(out, 0, sizeof(*out));
    *smoothing_used = 0;
    int64_t frames = 0, cwi = 0;
    for (int i = 0; i < N; ++i) c[i] = 1;
    while (max_frames >= 0 ? frames < max_frames
                           : (out->errors < 200 || out->word_errors < min_word_errors)) {
        if (cw_lines && ncw > 0) {                             /* :230-249 */
            const char *s = cw_lines[cwi++ % ncw];
            for (int i = 0; i < N; ++i) c[i] = s[i] == '1' ? -1 : +1;
        }
        for (int i = 0; i < N; ++i) {                          /* :251-274 */
            const double y = c[i] * (1.0 + sigma * orc_rann(&g));
            int r;
            yq[i] = orc_gdbf_front(y, cfg, &r);
            if (r * c[i] < 0) out->uncoded++;
            d[i] = (int8_t)r;
        }
        /* The loop of :298-356 draws N perturbations for each iteration that
         * passes its syndrome check: draw all T rows from a copy of the
         * generator, decode, then advance the real one by the `it` rows used. */
        int it, sat = 0;
        orc_rng g2 = g;
        orc_gdbf_cfg c2 = *cfg;
        c2.qsigma = noise_sigma;                               /* symNodeUpdates' sigma (:296, :353) */
        if (cfg->flags & ORC_GDBF_NOISE)
            for (long k = 0; k < (long)N * T; ++k) pert[k] = noise_sigma * orc_rann(&g2);
        if (cfg->flags & ORC_GDBF_QPROB)                       /* one ranu() per bit and iteration (:588) */
            for (long k = 0; k < (long)N * T; ++k) pert[k] = orc_ranu(&g2);
        it = orc_gdbf_decode_f64(H, yq, pert, &c2, d, &sat);
        if (cfg->flags & ORC_GDBF_NOISE)
            for (long k = 0; k < (long)N * it; ++k) (void)orc_rann(&g);
        if (cfg->flags & ORC_GDBF_QPROB)
            for (long k = 0; k < (long)N * it; ++k) (void)orc_ranu(&g);
        if ((cfg->flags & ORC_GDBF_SMOOTH) && it > T - cfg->windowsize) ++*smoothing_used;   /* :371-375 */
        int w = 0;
        for (int i = 0; i < N; ++i) w += d[i] != c[i];         /* :378 */
        if (w > 0) {
            out->errors += w;
            out->word_errors++;
        }
        if (frame_w && frames < cap) frame_w[frames] = w;
        if (frame_it && frames < cap) frame_it[frames] = it;
        out->words++;
        out->bits += N;
        out->iters += it;                                      /* :399 */
        ++frames;
    }
    free(c); free(yq); free(pert); free(d);
    return frames;
}
