/*
 * ldpc_oracle.h -- CPU ORACLE for the LDPC min-sum hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library. The product path
 * (libldpc_hip.so, the CLI front-ends, ldpcsimulation_amd/) never links or
 * calls it; it is the checker, never the thing measured or shipped.
 *
 * It is a plain-C restatement of the reference algorithm
 * (ereiss123/LDPCsimulation, C_implementations/):
 *   - glibc random()/srandom() TYPE_3 generator and the Neal rand.h macros
 *     ranf()/rann() (inc/rand.h:6-20);
 *   - the MacKay alist reader (src/alist.cpp:70-93, src/r.cpp:277-300,448-464);
 *   - decodeMinSum main() frame loop (src/decodeMinSum.cpp:146-311), with the
 *     -D normalizedMS / offsetMS / quantizeSamples / saturateSamples variants;
 *   - checkNodeUpdates / symNodeUpdates / applyNormalization / applyOffset /
 *     quantize / sgn / find (src/decodeMinSum.cpp:410-536).
 * Plus Philox4x32-10 (Salmon et al., SC'11, Random123) used by the product's
 * on-device AWGN, restated for integer known-answer checks.
 *
 * Parity pins (tests/test_oracle.py): oracle/_ref binaries compiled from the
 * unmodified reference sources (oracle/Makefile.ref) and the golden fixtures
 * under tests/golden/ generated from them (tests/golden/make_golden.py).
 */
#ifndef LDPC_ORACLE_H
#define LDPC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- glibc random() TYPE_3 (degree 31, separation 3) ---- */
typedef struct { int32_t tbl[31]; int front, rear; } orc_rng;
void    orc_srandom(orc_rng *g, uint32_t seed);
int32_t orc_random(orc_rng *g);
double  orc_ranf(orc_rng *g);            /* rand.h:10-11 */
double  orc_rann(orc_rng *g);            /* rand.h:19-20, cos operand drawn first */
void    orc_rann_fill(orc_rng *g, long n, double scale, double *out);   /* out[i] = scale * rann() */

/* ---- alist (reference loader semantics: fixed-width padded lines) ---- */
typedef struct {
    int N, M, maxdv, maxdc;
    int *deg_n;      /* [N] column weights (num_nlist)          */
    int *deg_m;      /* [M] row weights    (num_mlist)          */
    int *nlist;      /* [N*maxdv] 1-based check indices, 0 pads */
    int *mlist;      /* [M*maxdc] 1-based bit   indices, 0 pads */
} orc_alist;
int  orc_alist_load(const char *path, orc_alist *H);   /* 0 ok, -1 io */
void orc_alist_free(orc_alist *H);

/* ---- decoder configuration (the reference's compile-time -D switches) ---- */
enum { ORC_MS = 0, ORC_NMS = 1, ORC_OMS = 2 };
typedef struct {
    int    variant;      /* ORC_MS / ORC_NMS (-D normalizedMS) / ORC_OMS (-D offsetMS) */
    double alpha;        /* NMS divisor (decodeMinSum.cpp:498)                        */
    double delta;        /* OMS offset  (decodeMinSum.cpp:509)                         */
    int    quantize;     /* -D quantizeSamples: Ymax, Q                               */
    int    saturate;     /* -D saturateSamples: Ymax                                  */
    double ymax;
    int    qbits;
} orc_cfg;

typedef struct {
    int64_t errors, uncoded, bits, words, word_errors, iters;
} orc_stats;

/* Frame loop of decodeMinSum main() (decodeMinSum.cpp:146-311).
 * seed: the value ran_seed() receives (time(0) in the reference).
 * cw_lines/ncw: optional codeword file lines ('0'/'1' chars, N each), cycled
 * in order as :193-212 does; NULL = all-zero codeword.
 * max_frames < 0: run until errors>=200 && word_errors>=40 (:189); else run
 * exactly max_frames frames. frame_w (optional, capacity cap) receives the
 * per-frame error weight. Returns number of frames run. */
int64_t orc_minsum_run(const orc_alist *H, double R, double snr, int T,
                       const orc_cfg *cfg, uint32_t seed,
                       const char *const *cw_lines, int ncw,
                       int64_t max_frames, int32_t *frame_w, int64_t cap,
                       orc_stats *out);

/* Channel of one frame exactly as :214-238 (fp64). x = bipolar codeword. */
void orc_channel(orc_rng *g, int N, double sigma, const int *c, double *y);
double orc_quantize(double x, double ymax, double nq);          /* :480-489 */
float  orc_quantize_f32(float x, float ymax, float nq);         /* same, in float */

/* Decode ONE frame from channel samples y (already quantized/saturated if
 * the caller wants that front-end), T flooding iterations, reference
 * arithmetic (checkNodeUpdates :410-450, normalisation :494-499, offset
 * :503-515, symNodeUpdates :452-476). d receives +1/-1 decisions.
 * f64: the reference's own precision; f32: the same arithmetic in float
 * (the product's fast-path precision) for bit-exact decision parity. */
void orc_decode_f64(const orc_alist *H, const double *yq, int T,
                    const orc_cfg *cfg, int8_t *d);
void orc_decode_f32(const orc_alist *H, const float *yq, int T,
                    const orc_cfg *cfg, int8_t *d);
/* Same, also exports c2v messages after iteration `snap_it` (flattened in
 * mlist row order) for message-level fixtures. */
void orc_decode_f64_snap(const orc_alist *H, const double *yq, int T,
                         const orc_cfg *cfg, int8_t *d,
                         int snap_it, double *c2v_out, double *app_out);

/* Layered (row-serial) min-sum in the row order `order` [M] (NULL = 0..M-1);
 * same check-node rule, normalisation and offset as above, app updated in
 * place (see ldpc_oracle.c). No reference counterpart: own restatement. */
void orc_decode_layered_f64(const orc_alist *H, const double *yq, int T,
                            const orc_cfg *cfg, const int32_t *order, int8_t *d);
void orc_decode_layered_f32(const orc_alist *H, const float *yq, int T,
                            const orc_cfg *cfg, const int32_t *order, int8_t *d);

/* ---- GDBF / NGDBF bit flipping (src/decodeGDBF.cpp, parallel mode) ---- */
enum {
    ORC_GDBF_NOISE = 1,      /* -D addNoise            */
    ORC_GDBF_ADAPT = 2,      /* -D thresholdAdaptation */
    ORC_GDBF_WEIGHT = 4,     /* -D weightSyndromes     */
    ORC_GDBF_SMOOTH = 8,     /* -D outputSmoothing     */
    ORC_GDBF_SATURATE = 16,  /* -D saturateSamples     */
    ORC_GDBF_QUANTIZE = 32,  /* -D quantizeSamples     */
    ORC_GDBF_SEQUENTIAL = 64,   /* -D sequentialmode: mu = 0 from the start          */
    ORC_GDBF_MODESWITCH = 128,  /* -D modeswitching: mu -> 0 once f1 >= f2 (:309-345) */
    ORC_GDBF_QPROB = 256        /* -D quantizeProbabilities: stochastic flips (:562-597);
                                   pert[it][i] then holds the ranu() draws           */
};
typedef struct {
    int    flags, T, windowsize, nq;
    double theta, lambda, alpha, noise_scale, ymax;
    int    tswitch;      /* Tswitch (:51, 0 in the reference)                       */
    double qsigma;       /* quantizeProbabilities: the sigma of normalCDF (noiseSigma) */
} orc_gdbf_cfg;
/* ranu() (rand.h:13-14): (1 + random()) / (2 + 0x7fffffff) */
double orc_ranu(orc_rng *g);
/* channel front-end of one sample (:254-267): returns yq, *r = hard decision */
double orc_gdbf_front(double y, const orc_gdbf_cfg *cfg, int *r);
float  orc_gdbf_front_f32(float y, const orc_gdbf_cfg *cfg, int *r);
/* One frame (:298-367): d = r on entry, decisions on exit; pert [T][N]
 * (iteration it uses row it; NULL without ORC_GDBF_NOISE). Returns the
 * iterations run; *satisfied = all checks satisfied (early stop). */
int orc_gdbf_decode_f64(const orc_alist *H, const double *yq, const double *pert,
                        const orc_gdbf_cfg *cfg, int8_t *d, int *satisfied);
int orc_gdbf_decode_f32(const orc_alist *H, const float *yq, const float *pert,
                        const orc_gdbf_cfg *cfg, int8_t *d, int *satisfied);
/* main() frame loop (:224-413): stop rule errors >= 200 && wordErrors >=
 * 20/10/5 (N > 10000 / 50000) unless max_frames >= 0. */
int64_t orc_gdbf_run(const orc_alist *H, double R, double snr, const orc_gdbf_cfg *cfg, uint32_t seed,
                     const char *const *cw_lines, int ncw, int64_t max_frames,
                     int32_t *frame_w, int32_t *frame_it, int64_t cap, orc_stats *out,
                     int64_t *smoothing_used);

/* ---- belief propagation (src/decodeBP.cpp) ---- */
/* front-end of one sample (:184-197): yq = 4y/N0 clipped to +-maxllr; *r = sgn(yq) */
double orc_bp_front(double y, double N0, double maxllr, int *r);
/* T flooding BP iterations on the front-end output yq (:199-213, :353-409);
 * c2v_out (optional) receives the last c2v messages by (row, mlist position). */
void orc_bp_decode_f64(const orc_alist *H, const double *yq, int T, double maxllr, int8_t *d, double *c2v_out);
void orc_bp_decode_f32(const orc_alist *H, const float *yq, int T, double maxllr, int8_t *d, float *c2v_out);
/* main() frame loop (:145-252), MAXLLR = 20, stop rule 200 / 20|10|5. */
int64_t orc_bp_run(const orc_alist *H, double R, double snr, int T, uint32_t seed,
                   const char *const *cw_lines, int ncw, int64_t max_frames,
                   int32_t *frame_w, int64_t cap, orc_stats *out);

/* ---- non-binary GF(q) EMS (ems_oracle.c; parity unpinned, see there) ---- */
int  orc_gf_poly(int q);
int  orc_gf_mul(int q, int a, int b);
void orc_nb_front(const float *y, int n, float n0, float *lam);
int  orc_ems_decode(int N, int M, int q, const int *row_ptr, const int *row_col, const int *row_h,
                    const int *col_ptr, const int *col_slot, const float *lam, int T, int nm, float offset,
                    int early_stop, uint8_t *d, int *synd_fail);

/* Philox4x32-10 (Random123 reference constants). */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* test helper: x in a sample where x*r + one fma correction != IEEE x/alpha (fp64) */
long orc_markstein_mismatch(double alpha, long n, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif
