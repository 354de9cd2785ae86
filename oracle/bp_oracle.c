/*
 * bp_oracle.c -- CPU ORACLE of the reference's belief-propagation decoder
 * (test infrastructure only; see ldpc_oracle.h).
 *
 * Restates ereiss123/LDPCsimulation C_implementations/src/decodeBP.cpp:
 *   front-end   yq = 4*y/N0, |yq| <= MAXLLR = 20 (:58, :184-197)
 *   init        v2c = yq (initializeSymMessages :307-313)
 *   check node  c2v_j = log((1+p)/(1-p)), p = prod_{k != j} tanh(v2c_k/2),
 *               the product in mlist order skipping j (:353-377)
 *   bit node    sum = yq + sum_j c2v (nlist order); v2c = sum - c2v clipped
 *               to +-MAXLLR; d = sum > 0 ? +1 : -1 (:379-409)
 *   T fixed iterations, no early stop (:206-213).
 * Build: oracle/Makefile (plain IEEE, -ffp-contract=off, glibc libm).
 */
#include "ldpc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

static double bp_sgn(double x) { return x >= 0.0 ? 1.0 : -1.0; }   /* :412-417 */

double orc_bp_front(double y, double N0, double maxllr, int *r)
{
    double yq = 4.0 * y / N0;                                    /* :188 */
    if (fabs(yq) > maxllr) yq = bp_sgn(yq) * maxllr;             /* :190-191 */
    *r = (int)bp_sgn(yq);                                        /* :193 */
    return yq;
}

/* CLIP_C2V: fp32 only. |c2v| <= min_k |v2c_k| <= MAXLLR in exact arithmetic,
 * and in fp64 tanh(MAXLLR/2) < 1 keeps 1 - prod > 0 (c2v stays below ~20);
 * in fp32 tanhf(10) rounds to 1, so (1+p)/(1-p) becomes 2/0 and c2v = +-inf,
 * then app = inf and v2c = inf - inf = NaN. The fp32 decoder therefore clips
 * c2v to +-MAXLLR, which is a no-op wherever the float result is finite and
 * within range. The fp64 path (the reference's precision) is unclipped. */
#define ORC_DEFINE_BP(FT, SUFFIX, TANH, LOG, FABS, CLIP_C2V)                                \
void orc_bp_decode_##SUFFIX(const orc_alist *H, const FT *yq, int T, double maxllr_d,       \
                            int8_t *d, FT *c2v_out)                                         \
{                                                                                           \
    const int N = H->N, M = H->M, dcs = H->maxdc > 0 ? H->maxdc : 1;                        \
    const FT maxllr = (FT)maxllr_d;                                                         \
    FT *v2c = (FT *)malloc(sizeof(FT) * ((size_t)M * dcs + 1));  /* by check edge */        \
    FT *c2v = (FT *)calloc((size_t)M * dcs + 1, sizeof(FT));                                \
    FT *th = (FT *)malloc(sizeof(FT) * (dcs + 1));                                          \
    /* edge (j,k) of bit i: the LAST k with mlist[j][k] == i+1, as find() */                \
    int *eidx = (int *)malloc(sizeof(int) * ((size_t)N * (H->maxdv > 0 ? H->maxdv : 1) + 1)); \
    for (int i = 0; i < N; ++i)                                                             \
        for (int e = 0; e < H->deg_n[i]; ++e) {                                             \
            const int j = H->nlist[(long)i * H->maxdv + e] - 1;                             \
            int kk = -1;                                                                    \
            for (int k = 0; k < H->deg_m[j]; ++k)                                           \
                if (H->mlist[(long)j * H->maxdc + k] - 1 == i) kk = k;                       \
            eidx[(long)i * H->maxdv + e] = j * dcs + kk;                                    \
            v2c[j * dcs + kk] = yq[i];                           /* :307-313 */             \
        }                                                                                   \
    for (int i = 0; i < N; ++i) d[i] = yq[i] >= 0 ? 1 : -1;      /* d = r (:193-194) */     \
    for (int it = 0; it < T; ++it) {                                                        \
        for (int j = 0; j < M; ++j) {                            /* :353-377 */             \
            const int dg = H->deg_m[j];                                                     \
            for (int k = 0; k < dg; ++k) th[k] = TANH(v2c[j * dcs + k] / (FT)2.0);          \
            for (int jj = 0; jj < dg; ++jj) {                                               \
                FT prod = 1.0;                                                              \
                for (int k = 0; k < dg; ++k)                                                \
                    if (k != jj) prod *= th[k];                                             \
                FT o = LOG(((FT)1.0 + prod) / ((FT)1.0 - prod));                            \
                if (CLIP_C2V && FABS(o) > maxllr) o = o >= 0 ? maxllr : -maxllr;            \
                c2v[j * dcs + jj] = o;                                                      \
            }                                                                               \
        }                                                                                   \
        for (int i = 0; i < N; ++i) {                            /* :379-409 */             \
            FT sum = yq[i];                                                                 \
            for (int e = 0; e < H->deg_n[i]; ++e) sum += c2v[eidx[(long)i * H->maxdv + e]]; \
            for (int e = 0; e < H->deg_n[i]; ++e) {                                         \
                const int x = eidx[(long)i * H->maxdv + e];                                 \
                FT out = sum - c2v[x];                                                      \
                if (FABS(out) > maxllr) out = maxllr * (out >= 0 ? (FT)1.0 : (FT)-1.0);    \
                v2c[x] = out;                                                               \
            }                                                                               \
            d[i] = sum > 0 ? 1 : -1;                                                        \
        }                                                                                   \
    }                                                                                       \
    if (c2v_out) memcpy(c2v_out, c2v, sizeof(FT) * (size_t)M * dcs);                         \
    free(v2c); free(c2v); free(th); free(eidx);                                             \
}

ORC_DEFINE_BP(double, f64, tanh, log, fabs, 0)
ORC_DEFINE_BP(float, f32, tanhf, logf, fabsf, 1)

/* main() frame loop :145-252. */
int64_t orc_bp_run(const orc_alist *H, double R, double snr, int T, uint32_t seed,
                   const char *const *cw_lines, int ncw, int64_t max_frames,
                   int32_t *frame_w, int64_t cap, orc_stats *out)
{
    const int N = H->N;
    const double N0 = pow(10.0, -snr / 10.0) / R;               /* :104-105 */
    const double sigma = sqrt(N0 / 2.0);
    int min_word_errors = 20;                                    /* :145-147 */
    if (N > 10000) min_word_errors = 10;
    if (N > 50000) min_word_errors = 5;
    orc_rng g;
    orc_srandom(&g, seed);                                       /* :148 */
    int *c = (int *)malloc(sizeof(int) * N);
    double *yq = (double *)malloc(sizeof(double) * N);
    int8_t *d = (int8_t *)malloc((size_t)N);
    memset(out, 0, sizeof(*out));
    int64_t frames = 0, cwi = 0;
    for (int i = 0; i < N; ++i) c[i] = 1;
    while (max_frames >= 0 ? frames < max_frames
                           : (out->errors < 200 || out->word_errors < min_word_errors)) {
        if (cw_lines && ncw > 0) {                               /* :154-173 */
            const char *s = cw_lines[cwi++ % ncw];
            for (int i = 0; i < N; ++i) c[i] = s[i] == '1' ? -1 : +1;
        }
        for (int i = 0; i < N; ++i) {                            /* :175-197 */
            const double y = c[i] * (1.0 + sigma * orc_rann(&g));
            int r;
            yq[i] = orc_bp_front(y, N0, 20.0, &r);
            if (r * c[i] < 0) out->uncoded++;
        }
        orc_bp_decode_f64(H, yq, T, 20.0, d, NULL);
        int w = 0;
        for (int i = 0; i < N; ++i) w += d[i] != c[i];          /* :220 */
        if (w > 0) {
            out->errors += w;
            out->word_errors++;
        }
        if (frame_w && frames < cap) frame_w[frames] = w;
        out->words++;
        out->bits += N;
        out->iters += T;                                         /* :239, it == T */
        ++frames;
    }
    free(c); free(yq); free(d);
    return frames;
}
