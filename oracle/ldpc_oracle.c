/*
 * ldpc_oracle.c -- CPU ORACLE (test infrastructure only; see ldpc_oracle.h).
 *
 * Restates, in plain C, the reference's min-sum path so the HIP product can
 * be checked against it. Each routine cites the reference file:line it
 * follows (paths relative to ereiss123/LDPCsimulation/C_implementations/).
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off, no -ffast-math:
 * the arithmetic must be plain IEEE as in the reference's g++ build).
 */
#include "ldpc_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ===================================================================== */
/* glibc random(): TYPE_3 additive feedback generator, r = 31, sep = 3.   */
/* The reference calls srandom() through ran_seed (inc/rand.h:6) and      */
/* random() through ranf (inc/rand.h:10-11).                               */
/* ===================================================================== */
void orc_srandom(orc_rng *g, uint32_t seed)
{
    int32_t word = (int32_t)(seed == 0 ? 1u : seed);
    g->tbl[0] = word;
    for (int i = 1; i < 31; ++i) {
        /* 16807 * word mod (2^31 - 1), by Schrage's factorisation */
        int32_t hi = word / 127773, lo = word % 127773;
        word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        g->tbl[i] = word;
    }
    g->front = 3;     /* the "front" tap runs SEP = 3 ahead of the "rear" tap */
    g->rear = 0;
    for (int i = 0; i < 310; ++i) (void)orc_random(g);   /* 10 * degree discards */
}

int32_t orc_random(orc_rng *g)
{
    uint32_t v = (uint32_t)g->tbl[g->front] + (uint32_t)g->tbl[g->rear];
    g->tbl[g->front] = (int32_t)v;
    if (++g->front == 31) g->front = 0;
    if (++g->rear == 31) g->rear = 0;
    return (int32_t)(v >> 1);
}

/* ranf(): uniform [0,1) = random() / 2^31 (rand.h:10-11) */
double orc_ranf(orc_rng *g)
{
    return (double)orc_random(g) / (1.0 + (double)0x7fffffff);
}

double orc_ranu(orc_rng *g)
{
    return (1.0 + (double)orc_random(g)) / (2.0 + (double)0x7fffffff);
}

/* rann(): cos(2*3.141592654*ranf()) * sqrt(-2*log(1-ranf())) (rand.h:19-20).
 * g++ evaluates the cos operand's ranf() first (verified against the
 * reference binary: tests/test_oracle.py::test_rann_kat). */
double orc_rann(orc_rng *g)
{
    double u_angle = orc_ranf(g);
    double u_rad = orc_ranf(g);
    return cos(2.0 * 3.141592654 * u_angle) * sqrt(-2.0 * log(1.0 - u_rad));
}

/* n draws of scale * rann() in order (the perturbation rows of
 * decodeGDBF.cpp:318-333: noiseSigma * rann() per bit and iteration). */
void orc_rann_fill(orc_rng *g, long n, double scale, double *out)
{
    for (long i = 0; i < n; ++i) out[i] = scale * orc_rann(g);
}

/* ===================================================================== */
/* alist reader: loadFile (src/alist.cpp:70-93): "N M", "maxdv maxdc",     */
/* N column weights, M row weights, then N lines of maxdv and M lines of   */
/* maxdc 1-based indices zero padded (fread_imatrix, src/r.cpp:277-300).    */
/* ===================================================================== */
static int read_ints(FILE *f, int *dst, long n)
{
    for (long i = 0; i < n; ++i)
        if (fscanf(f, "%d ", &dst[i]) != 1) return -1;
    return 0;
}

int orc_alist_load(const char *path, orc_alist *H)
{
    memset(H, 0, sizeof(*H));
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    int hdr[4];
    if (read_ints(f, hdr, 4)) { fclose(f); return -1; }
    H->N = hdr[0]; H->M = hdr[1]; H->maxdv = hdr[2]; H->maxdc = hdr[3];
    H->deg_n = (int *)calloc((size_t)H->N, sizeof(int));
    H->deg_m = (int *)calloc((size_t)H->M, sizeof(int));
    H->nlist = (int *)calloc((size_t)H->N * H->maxdv, sizeof(int));
    H->mlist = (int *)calloc((size_t)H->M * H->maxdc, sizeof(int));
    int rc = read_ints(f, H->deg_n, H->N) || read_ints(f, H->deg_m, H->M) ||
             read_ints(f, H->nlist, (long)H->N * H->maxdv) ||
             read_ints(f, H->mlist, (long)H->M * H->maxdc);
    fclose(f);
    if (rc) { orc_alist_free(H); return -1; }
    return 0;
}

void orc_alist_free(orc_alist *H)
{
    free(H->deg_n); free(H->deg_m); free(H->nlist); free(H->mlist);
    memset(H, 0, sizeof(*H));
}

/* ===================================================================== */
/* Channel front-end.                                                    */
/* ===================================================================== */
/* quantize() (decodeMinSum.cpp:480-489) */
static double sgn_d(double x) { return x >= 0.0 ? 1.0 : -1.0; }   /* :518-523 */
static float  sgn_f(float x)  { return x >= 0.0f ? 1.0f : -1.0f; }

double orc_quantize(double x, double ymax, double nq)
{
    if (fabs(x) > ymax) return sgn_d(x) * ymax;
    double q = sgn_d(x) * (floor(fabs(x) * (nq - 1) / (2.0 * ymax)) + 0.0) * (2 * ymax / (nq - 1));
    if (q == 0.0) q = sgn_d(x) * 2.0 * ymax / (nq - 1);
    return q;
}

float orc_quantize_f32(float x, float ymax, float nq)
{
    if (fabsf(x) > ymax) return sgn_f(x) * ymax;
    float q = sgn_f(x) * (floorf(fabsf(x) * (nq - 1) / (2.0f * ymax)) + 0.0f) * (2 * ymax / (nq - 1));
    if (q == 0.0f) q = sgn_f(x) * 2.0f * ymax / (nq - 1);
    return q;
}

/* AWGN: y = x * (1 + sigma * rann()) (decodeMinSum.cpp:214-216) */
void orc_channel(orc_rng *g, int N, double sigma, const int *c, double *y)
{
    for (int i = 0; i < N; ++i) y[i] = (double)c[i] * (1.0 + sigma * orc_rann(g));
}

/* ===================================================================== */
/* Flooding min-sum iteration, written once per precision via a macro.   */
/* Message memories are ragged per node as in setupSymMessages /         */
/* setupCheckMessages (:345-361): v2c[i][0..deg_n[i]) and                */
/* c2v[j][0..deg_m[j]); edges are located with the reference's linear    */
/* find() (:527-536), which keeps the LAST match.                        */
/* ===================================================================== */
static int find_last(const int *list, int len, int target0)
{
    int hit = -1;
    for (int i = 0; i < len; ++i)
        if (list[i] - 1 == target0) hit = i;
    return hit;
}

typedef struct { int *off_n, *off_m; } ragged;
static void ragged_init(const orc_alist *H, ragged *r)
{
    r->off_n = (int *)malloc(sizeof(int) * (H->N + 1));
    r->off_m = (int *)malloc(sizeof(int) * (H->M + 1));
    r->off_n[0] = 0;
    for (int i = 0; i < H->N; ++i) r->off_n[i + 1] = r->off_n[i] + H->deg_n[i];
    r->off_m[0] = 0;
    for (int j = 0; j < H->M; ++j) r->off_m[j + 1] = r->off_m[j] + H->deg_m[j];
}
static void ragged_free(ragged *r) { free(r->off_n); free(r->off_m); }

#define ORC_DEFINE_DECODER(FT, SUFFIX, SGN, FABS)                                  \
static void decode_##SUFFIX(const orc_alist *H, const ragged *R, const FT *yq,   \
                            int T, const orc_cfg *cfg, int8_t *d,                \
                            FT *v2c, FT *c2v, int snap_it, FT *c2v_snap,          \
                            FT *app_snap)                                         \
{                                                                                 \
    const int N = H->N, M = H->M;                                                 \
    const FT alpha = (FT)cfg->alpha, delta = (FT)cfg->delta;                      \
    /* initializeSymMessages (:364-370) and d = r (:231-235) */                   \
    for (int i = 0; i < N; ++i) {                                                 \
        for (int k = 0; k < H->deg_n[i]; ++k) v2c[R->off_n[i] + k] = yq[i];        \
        d[i] = yq[i] > 0 ? 1 : -1;                                                \
    }                                                                             \
    for (int it = 0; it < T; ++it) {                                              \
        /* checkNodeUpdates (:410-450) */                                         \
        for (int j = 0; j < M; ++j) {                                             \
            const int *row = H->mlist + (long)j * H->maxdc;                       \
            FT mn1 = (FT)INFINITY, mn2 = (FT)INFINITY, prod = 1;                  \
            int amin = -1;                                                        \
            for (int k = 0; k < H->deg_m[j]; ++k) {                               \
                int s = row[k] - 1;                                               \
                int p = find_last(H->nlist + (long)s * H->maxdv, H->deg_n[s], j);  \
                FT msg = v2c[R->off_n[s] + p];                                    \
                prod *= SGN(msg);                                                 \
                if (FABS(msg) <= mn1) { mn2 = mn1; mn1 = FABS(msg); amin = k; }   \
                else if (FABS(msg) < mn2) mn2 = FABS(msg);                        \
            }                                                                     \
            for (int k = 0; k < H->deg_m[j]; ++k) {                               \
                int s = row[k] - 1;                                               \
                int p = find_last(H->nlist + (long)s * H->maxdv, H->deg_n[s], j);  \
                FT msg = v2c[R->off_n[s] + p];                                    \
                c2v[R->off_m[j] + k] = (k == amin ? prod * mn2 : prod * mn1) * SGN(msg); \
            }                                                                     \
        }                                                                         \
        /* applyNormalization (:494-499) / applyOffset (:503-515) */              \
        if (cfg->variant == ORC_NMS) {                                            \
            for (int e = 0; e < R->off_m[M]; ++e) c2v[e] /= alpha;                \
        } else if (cfg->variant == ORC_OMS) {                                     \
            for (int e = 0; e < R->off_m[M]; ++e) {                               \
                FT mag = FABS(c2v[e]) - delta;                                    \
                c2v[e] = mag > 0 ? SGN(c2v[e]) * mag : 0;                         \
            }                                                                     \
        }                                                                         \
        /* symNodeUpdates (:452-476) */                                           \
        for (int i = 0; i < N; ++i) {                                             \
            const int *col = H->nlist + (long)i * H->maxdv;                       \
            FT sum = yq[i];                                                       \
            for (int k = 0; k < H->deg_n[i]; ++k) {                               \
                int c = col[k] - 1;                                               \
                int p = find_last(H->mlist + (long)c * H->maxdc, H->deg_m[c], i);  \
                sum += c2v[R->off_m[c] + p];                                      \
            }                                                                     \
            for (int k = 0; k < H->deg_n[i]; ++k) {                               \
                int c = col[k] - 1;                                               \
                int p = find_last(H->mlist + (long)c * H->maxdc, H->deg_m[c], i);  \
                v2c[R->off_n[i] + k] = sum - c2v[R->off_m[c] + p];                \
            }                                                                     \
            d[i] = sum > 0 ? 1 : -1;                                              \
            if (app_snap && it == snap_it) app_snap[i] = sum;                     \
        }                                                                         \
        if (c2v_snap && it == snap_it)                                            \
            memcpy(c2v_snap, c2v, sizeof(FT) * (size_t)R->off_m[M]);              \
    }                                                                             \
}

ORC_DEFINE_DECODER(double, f64, sgn_d, fabs)
ORC_DEFINE_DECODER(float, f32, sgn_f, fabsf)

void orc_decode_f64_snap(const orc_alist *H, const double *yq, int T,
                         const orc_cfg *cfg, int8_t *d,
                         int snap_it, double *c2v_out, double *app_out)
{
    ragged R; ragged_init(H, &R);
    double *v2c = (double *)malloc(sizeof(double) * (R.off_n[H->N] + 1));
    double *c2v = (double *)malloc(sizeof(double) * (R.off_m[H->M] + 1));
    decode_f64(H, &R, yq, T, cfg, d, v2c, c2v, snap_it, c2v_out, app_out);
    free(v2c); free(c2v); ragged_free(&R);
}

void orc_decode_f64(const orc_alist *H, const double *yq, int T,
                    const orc_cfg *cfg, int8_t *d)
{
    orc_decode_f64_snap(H, yq, T, cfg, d, -1, NULL, NULL);
}

void orc_decode_f32(const orc_alist *H, const float *yq, int T,
                    const orc_cfg *cfg, int8_t *d)
{
    ragged R; ragged_init(H, &R);
    float *v2c = (float *)malloc(sizeof(float) * (R.off_n[H->N] + 1));
    float *c2v = (float *)malloc(sizeof(float) * (R.off_m[H->M] + 1));
    decode_f32(H, &R, yq, T, cfg, d, v2c, c2v, -1, NULL, NULL);
    free(v2c); free(c2v); ragged_free(&R);
}

/* ===================================================================== */
/* Layered (row-serial) normalized/offset min-sum -- SURVEY §8(f) row 2,  */
/* BASELINE config 3. The reference has no layered schedule; this is the  */
/* standard row-serial restatement of its check-node rule, so parity for  */
/* layered-specific results is against this oracle only ("parity          */
/* unpinned" w.r.t. the reference; its flooding results stay pinned).     */
/*   app[i] = yq[i];  c2v[j][k] = 0                                        */
/*   for each iteration, for each row j in `order` (serially):             */
/*     x_k  = app[b_k] - c2v[j][k]                 (v2c, as :469)          */
/*     c_k  = (k == amin ? prod*mn2 : prod*mn1) * sgn(x_k)  (:426-447)     */
/*     c_k /= alpha (NMS, :498) | offset (OMS, :509-513)                   */
/*     c2v[j][k] = c_k;  app[b_k] = x_k + c_k                              */
/*   d[i] = app[i] > 0 ? +1 : -1                    (:471-474)             */
/* Rows that share no bit commute exactly, so any grouping of consecutive  */
/* bit-disjoint rows of `order` into parallel layers gives these results.  */
/* ===================================================================== */
#define ORC_DEFINE_LAYERED(FT, SUFFIX, SGN, FABS)                                  \
void orc_decode_layered_##SUFFIX(const orc_alist *H, const FT *yq, int T,         \
                                 const orc_cfg *cfg, const int32_t *order,        \
                                 int8_t *d)                                       \
{                                                                                 \
    const int N = H->N, M = H->M, dc = H->maxdc > 0 ? H->maxdc : 1;               \
    const FT alpha = (FT)cfg->alpha, delta = (FT)cfg->delta;                      \
    FT *app = (FT *)malloc(sizeof(FT) * (N + 1));                                 \
    FT *c2v = (FT *)calloc((size_t)M * dc + 1, sizeof(FT));                       \
    FT *x = (FT *)malloc(sizeof(FT) * (dc + 1));                                  \
    for (int i = 0; i < N; ++i) app[i] = yq[i];                                   \
    for (int it = 0; it < T; ++it) {                                              \
        for (int r = 0; r < M; ++r) {                                             \
            const int j = order ? order[r] : r;                                   \
            const int *row = H->mlist + (long)j * H->maxdc;                       \
            FT *cj = c2v + (long)j * dc;                                          \
            FT mn1 = (FT)INFINITY, mn2 = (FT)INFINITY, prod = 1;                  \
            int amin = -1;                                                        \
            for (int k = 0; k < H->deg_m[j]; ++k) {                               \
                x[k] = app[row[k] - 1] - cj[k];                                   \
                prod *= SGN(x[k]);                                                \
                if (FABS(x[k]) <= mn1) { mn2 = mn1; mn1 = FABS(x[k]); amin = k; } \
                else if (FABS(x[k]) < mn2) mn2 = FABS(x[k]);                      \
            }                                                                     \
            for (int k = 0; k < H->deg_m[j]; ++k) {                               \
                FT c = (k == amin ? prod * mn2 : prod * mn1) * SGN(x[k]);         \
                if (cfg->variant == ORC_NMS) c /= alpha;                          \
                else if (cfg->variant == ORC_OMS) {                               \
                    FT mag = FABS(c) - delta;                                     \
                    c = mag > 0 ? SGN(c) * mag : 0;                               \
                }                                                                 \
                cj[k] = c;                                                        \
                app[row[k] - 1] = x[k] + c;                                       \
            }                                                                     \
        }                                                                         \
    }                                                                             \
    for (int i = 0; i < N; ++i) d[i] = app[i] > 0 ? 1 : -1;                       \
    free(app); free(c2v); free(x);                                                \
}

ORC_DEFINE_LAYERED(double, f64, sgn_d, fabs)
ORC_DEFINE_LAYERED(float, f32, sgn_f, fabsf)

/* ===================================================================== */
/* The Monte-Carlo frame loop of main() (decodeMinSum.cpp:146-311).      */
/* ===================================================================== */
int64_t orc_minsum_run(const orc_alist *H, double R, double snr, int T,
                       const orc_cfg *cfg, uint32_t seed,
                       const char *const *cw_lines, int ncw,
                       int64_t max_frames, int32_t *frame_w, int64_t cap,
                       orc_stats *out)
{
    const int N = H->N;
    const double N0 = pow(10.0, -snr / 10.0) / R;          /* :146 */
    const double sigma = sqrt(N0 / 2.0);                   /* :147 */
    const double nq = pow(2.0, cfg->qbits);                /* :121 */
    ragged Rg; ragged_init(H, &Rg);
    double *v2c = (double *)malloc(sizeof(double) * (Rg.off_n[N] + 1));
    double *c2v = (double *)malloc(sizeof(double) * (Rg.off_m[H->M] + 1));
    double *y = (double *)malloc(sizeof(double) * N);
    double *yq = (double *)malloc(sizeof(double) * N);
    int *c = (int *)malloc(sizeof(int) * N);
    int8_t *d = (int8_t *)malloc((size_t)N);
    for (int i = 0; i < N; ++i) c[i] = 1;
    orc_stats st; memset(&st, 0, sizeof(st));
    orc_rng g; orc_srandom(&g, seed);                      /* :187 */
    int64_t frames = 0;
    for (;;) {
        if (max_frames < 0) { if (!(st.errors < 200 || st.word_errors < 40)) break; }  /* :189 */
        else if (frames >= max_frames) break;
        if (cw_lines && ncw > 0) {                         /* :193-212 */
            const char *s = cw_lines[frames % ncw];
            for (int i = 0; i < N; ++i) {
                if (s[i] == '1') c[i] = -1;
                else if (s[i] == '0') c[i] = +1;
            }
        }
        orc_channel(&g, N, sigma, c, y);                   /* :214-216 */
        for (int i = 0; i < N; ++i) {                      /* :218-238 */
            double q = y[i];
            if (cfg->quantize) q = orc_quantize(y[i], cfg->ymax, nq);
            if (cfg->saturate) { if (q > cfg->ymax) q = cfg->ymax; if (q < -cfg->ymax) q = -cfg->ymax; }
            yq[i] = q;
            int r = q > 0 ? 1 : -1;
            if (r * c[i] < 0) st.uncoded++;
        }
        decode_f64(H, &Rg, yq, T, cfg, d, v2c, c2v, -1, NULL, NULL);   /* :240-263 */
        int w = 0;                                         /* :270, :382-393 */
        for (int i = 0; i < N; ++i) w += (d[i] != c[i]);
        if (w > 0) { st.errors += w; st.word_errors++; }  /* :272-283 */
        if (frame_w && frames < cap) frame_w[frames] = w;
        st.words++; st.bits += N; st.iters += T;          /* :286-288 */
        frames++;
    }
    if (out) *out = st;
    free(v2c); free(c2v); free(y); free(yq); free(c); free(d); ragged_free(&Rg);
    return frames;
}

/* ===================================================================== */
/* Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11; Random123 1.09).     */
/* ===================================================================== */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4])
{
    uint32_t x0 = ctr[0], x1 = ctr[1], x2 = ctr[2], x3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * x0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * x2;
        uint32_t y0 = (uint32_t)(p1 >> 32) ^ x1 ^ k0;
        uint32_t y1 = (uint32_t)p1;
        uint32_t y2 = (uint32_t)(p0 >> 32) ^ x3 ^ k1;
        uint32_t y3 = (uint32_t)p0;
        x0 = y0; x1 = y1; x2 = y2; x3 = y3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = x0; out[1] = x1; out[2] = x2; out[3] = x3;
}

/* ---------------------------------------------------------------------------
 * Test helper, not a restatement of the reference: the fp64 fast kernel
 * (ldpcsimulation_amd/csrc/rows_fast.hip) divides the check-node minima by
 * alpha as q = x*r, q = fma(fma(-q, alpha, x), r, q) with r = RN(1/alpha),
 * claimed equal to IEEE x/alpha (the reference's `/= alpha`,
 * decodeMinSum.cpp:494-499) for alpha = P*2^E, odd P < 2^20, and
 * 2^-960 <= x < 2^1000. Counts the x of a sample for which that fails: n
 * splitmix64 draws (uniform significand, exponent uniform in [-960, 999]),
 * plus for every exponent in that range the significands 1, 2 - ulp and the
 * multiples k*alpha' (alpha' = alpha's significand) nearest to binade points.
 * ------------------------------------------------------------------------- */
static uint64_t splitmix64(uint64_t *s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int markstein_bad(double x, double alpha, double r)
{
    const double q = x * r;
    const double m = fma(fma(-q, alpha, x), r, q);
    const double d = x / alpha;
    return memcmp(&m, &d, sizeof m) != 0;
}

long orc_markstein_mismatch(double alpha, long n, uint64_t seed)
{
    const double r = 1.0 / alpha;
    long bad = 0;
    uint64_t s = seed;
    for (long i = 0; i < n; ++i) {
        const uint64_t u = splitmix64(&s);
        const int e = (int)(splitmix64(&s) % 1960u) - 960;
        const double x = ldexp(1.0 + (double)(u >> 12) * 0x1p-52, e);
        bad += markstein_bad(x, alpha, r);
    }
    int ea;
    const double am = frexp(alpha, &ea) * 2.0;   /* alpha's significand in [1, 2) */
    for (int e = -960; e < 1000; ++e) {
        const double edge[2] = {1.0, 2.0 - 0x1p-52};
        for (int k = 0; k < 2; ++k) bad += markstein_bad(ldexp(edge[k], e), alpha, r);
        for (int k = 1; k <= 64; ++k) {   /* x near k * alpha': quotients near small integers */
            double x = ldexp(am * k, e), lo = nextafter(x, 0.0), hi = nextafter(x, INFINITY);
            bad += markstein_bad(x, alpha, r) + markstein_bad(lo, alpha, r) + markstein_bad(hi, alpha, r);
        }
    }
    return bad;
}
