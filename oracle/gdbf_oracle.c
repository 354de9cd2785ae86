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
 * Not restated: modeswitching / sequentialmode (single-bit flips, mu = 0) and
 * quantizeProbabilities (decodeStochasticNGDBF) -- no product counterpart.
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
    for (it = 0; it < T; ++it) {                                                        \
        sat = 1;                                                                        \
        for (int j = 0; j < M; ++j) {                          /* :517-534 */           \
            int prod = 1;                                                               \
            for (int k = 0; k < H->deg_m[j]; ++k) prod *= d[H->mlist[(long)j * H->maxdc + k] - 1]; \
            if (prod < 0) sat = 0;                                                      \
            s[j] = prod;                                                                \
        }                                                                               \
        if (sat) break;                                        /* :305-306 */           \
        for (int i = 0; i < N; ++i) {                          /* :536-621, mu = 1 */   \
            FT E = (FT)d[i] * yq[i];                                                    \
            for (int k = 0; k < H->deg_n[i]; ++k)                                       \
                E += w * (FT)s[H->nlist[(long)i * H->maxdv + k] - 1];                   \
            if (cfg->flags & ORC_GDBF_NOISE) E += pert[(long)it * N + i];               \
            const int flip = E < theta[i];                                              \
            if (flip) d[i] = (int8_t)-d[i];                                             \
            if ((cfg->flags & ORC_GDBF_ADAPT) && !flip) theta[i] *= lambda;             \
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
        if (cfg->flags & ORC_GDBF_NOISE)
            for (long k = 0; k < (long)N * T; ++k) pert[k] = noise_sigma * orc_rann(&g2);
        it = orc_gdbf_decode_f64(H, yq, pert, cfg, d, &sat);
        if (cfg->flags & ORC_GDBF_NOISE)
            for (long k = 0; k < (long)N * it; ++k) (void)orc_rann(&g);
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
