/*
 * ldpc_hip.h -- C ABI of the MI355X-native LDPC min-sum decoder
 * (libldpc_hip.so, built from ldpcsimulation_amd/csrc/).
 *
 * Drop-in boundary for the hot path of ereiss123/LDPCsimulation
 * (paths relative to C_implementations/):
 *   - ldpc_graph_create / ldpc_graph_load_alist replace the H-matrix loader
 *     loadFile() (src/alist.cpp:22-95, inc/alist.h:21-41) and the message
 *     memory setup setupSymMessages/setupCheckMessages (src/decodeMinSum.cpp
 *     :345-361). ldpc_graph_create takes exactly the arrays of an
 *     alist_struct (N, M, num_nlist, nlist, num_mlist, mlist; 1-based,
 *     zero padded), so an existing loadFile() result passes straight through.
 *   - ldpc_decode_batch replaces the per-frame decode loop
 *     initializeSymMessages + T x {checkNodeUpdates, applyNormalization |
 *     applyOffset, symNodeUpdates} + countDecisionErrors
 *     (src/decodeMinSum.cpp:240-270, functions at :364-370, :410-515,
 *     :382-393) for a batch of frames whose channel samples y are given
 *     (the reference's `y`/`yq` vectors, :214-238).
 *   - ldpc_sim_launch / ldpc_sim_batch replace the body of the Monte-Carlo
 *     frame loop (src/decodeMinSum.cpp:189-289: AWGN, quantise/saturate,
 *     decode, error accounting) with one fused device pass per batch; the
 *     stop rule (:189) stays with the caller, which reads ldpc_counts.
 *   The compile-time variants of the reference (-D normalizedMS, offsetMS,
 *   quantizeSamples, saturateSamples; src/decodeMinSum.cpp:26-32,
 *   Makefile:58-65) are runtime fields of ldpc_decoder_cfg.
 *   The belief-propagation decoder (src/decodeBP.cpp) is variant LDPC_BP.
 *   - ldpc_gdbf_decode_batch / ldpc_gdbf_sim_* replace the frame body of the
 *     GDBF / NGDBF bit-flipping decoders (src/decodeGDBF.cpp:250-399,
 *     checkNodeUpdates :517-534, symNodeUpdates :536-621), whose -D switches
 *     (Makefile:33-53) are the flags of ldpc_gdbf_cfg.
 *   - ldpc_nb_* / ldpc_ems_* (ABI 5): non-binary GF(16) codes (BASELINE
 *     config 5). ldpc_nb_graph_create / _load_alist replace the NB-LDPC
 *     model's loadFile() (SystemC/NB-LDPC/src/alist.cpp:23-56,
 *     inc/alist.h:25-43: (index, GF value) pairs); the decode replaces its
 *     symbol/check node iteration (inc/nodes.h:82-166, :240-293; a q^dc-LUT
 *     BP there, which does not compile) with the Extended Min-Sum.
 *
 * Conventions: every function returns LDPC_OK (0) or a negative
 * ldpc_status; ldpc_last_error() gives a thread-local message. No C++
 * exception crosses the ABI. Buffers may be host or device pointers (the
 * library checks with hipPointerGetAttributes); the caller owns them and the
 * library never frees caller memory. A context is not thread-safe: one host
 * thread (or process) per GPU. Graphs are immutable after creation and may
 * be shared read-only between contexts.
 */
#ifndef LDPC_HIP_H
#define LDPC_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDPC_ABI_VERSION 11

typedef enum {
    LDPC_OK = 0,
    LDPC_ERR_INVALID = -1,     /* bad argument                         */
    LDPC_ERR_NOMEM = -2,       /* host or device allocation failed     */
    LDPC_ERR_DEVICE = -3,      /* HIP runtime / kernel error           */
    LDPC_ERR_UNSUPPORTED = -4, /* shape or option not supported        */
    LDPC_ERR_IO = -5,          /* file could not be read               */
    LDPC_ERR_GRAPH = -6        /* inconsistent / malformed H matrix    */
} ldpc_status;

/* Check-node rule: MS = decodeMinSum, NMS = -D normalizedMS (c2v /= alpha,
 * src/decodeMinSum.cpp:494-499), OMS = -D offsetMS (:503-515), BP = the
 * tanh rule of src/decodeBP.cpp (:353-409) with its LLR front-end
 * yq = 4*y/n0 clipped to +-max_llr (:184-197; quantize/saturate ignored,
 * flooding only). */
typedef enum { LDPC_MS = 0, LDPC_NMS = 1, LDPC_OMS = 2, LDPC_BP = 3 } ldpc_variant;

/* Message arithmetic. F64 is the reference's own precision and reproduces
 * its decisions bit-for-bit for identical y; F32 is the throughput path. */
typedef enum { LDPC_F32 = 0, LDPC_F64 = 1 } ldpc_precision;

/* Message-passing schedule. FLOODING is the reference's (all check nodes,
 * then all bit nodes: src/decodeMinSum.cpp:247-263). LAYERED is the
 * row-serial schedule of SURVEY §8(f) row 2 (BASELINE config 3; no
 * reference counterpart): rows in the order ldpc_graph_layers() returns,
 * each row updating the posteriors of its bits in place, bit-disjoint rows
 * of a layer in parallel. */
typedef enum { LDPC_FLOODING = 0, LDPC_LAYERED = 1 } ldpc_schedule;

typedef struct ldpc_graph ldpc_graph;
typedef struct ldpc_ctx ldpc_ctx;

/* Error accounting of src/decodeMinSum.cpp:167-172,270-288, int64 as the
 * reference's `long` counters, plus a syndrome check (H*d != 0). */
typedef struct {
    int64_t bit_err;         /* errors          */
    int64_t frame_err;       /* wordErrors      */
    int64_t uncoded_bit_err; /* uncodedErrors   */
    int64_t frames;          /* totalWords      */
    int64_t iters;           /* totalIterations */
    int64_t syndrome_fail;   /* frames whose hard decision is not a codeword */
} ldpc_counts;

/* Per-frame outcome (optional output), in frame order. */
typedef struct {
    int32_t bit_err;          /* newErrors of :270 (0 = frame decoded)  */
    int32_t uncoded_bit_err;  /* hard-decision errors before decoding    */
    int32_t syndrome_fail;    /* 1 if H*d != 0                          */
    int32_t iters;            /* GDBF: iterations run (`it`, decodeGDBF.cpp:399); min-sum: 0 */
} ldpc_frame_result;

typedef struct {
    int32_t variant;    /* ldpc_variant                                     */
    int32_t precision;  /* ldpc_precision                                   */
    int32_t T;          /* iterations (num_iterations), fixed, no early stop */
    int32_t quantize;   /* -D quantizeSamples: quantize(y, ymax, 2^qbits)   */
    int32_t saturate;   /* -D saturateSamples: clip at +-ymax               */
    int32_t qbits;      /* Q                                                */
    double  ymax;       /* Ymax                                             */
    double  alpha;      /* NMS divisor                                      */
    double  delta;      /* OMS offset                                       */
    int32_t schedule;   /* ldpc_schedule (ABI 2)                            */
    int32_t reserved;   /* 0                                                */
    double  n0;         /* BP: noise density N0 of the LLR front-end 4*y/N0 (ABI 4);
                         * ldpc_decode_batch needs it > 0, the sim entry points
                         * compute it from Eb/N0 and R (:104)               */
    double  max_llr;    /* BP: MAXLLR message clip, 0 = the reference's 20 (:58) */
} ldpc_decoder_cfg;

int         ldpc_abi_version(void);
const char *ldpc_last_error(void);
/* (ABI 9) 1 when the fp64 NMS division m / alpha (applyNormalization,
 * decodeMinSum.cpp:494-499) runs as Markstein's q = m*r, q += fma(-q, alpha, m)*r
 * with r = RN(1/alpha) -- exact for alpha = P * 2^E, odd P < 2^20, 2^-900 < alpha
 * <= 2^60 -- else 0 (IEEE division). No device call. */
int         ldpc_f64_nms_fast_division(double alpha);
/* (ABI 11) The fp64 BP check node's transcendentals as the device computes
 * them (bp_math.h: tanh for th_k = tanh(v2c/2) and log for c2v = log((1+p)/(1-p)),
 * decodeBP.cpp:353-377), evaluated on device `device` for n host values x:
 * tanh_out[i] = tanh(x[i]), log_out[i] = log(x[i]) (either output may be NULL).
 * Verification only (tests/test_bp.py measures their ulp distance to glibc). */
int         ldpc_bp_math_probe(int device, const double *x, int n, double *tanh_out, double *log_out);
/* (ABI 11) The device bounds checks of the checked build (`make checked`,
 * ldpcsimulation_amd/lib/checked/libldpc_hip_checked.so; check.h): launches one
 * kernel that indexes past a bound on purpose and returns what every launch of
 * that build returns on a violation -- LDPC_ERR_DEVICE, ldpc_last_error() naming
 * the site, index and bound. The product library compiles no checks and returns
 * LDPC_ERR_UNSUPPORTED. */
int         ldpc_check_selftest(int device);

/* ---- graph (H matrix) ------------------------------------------------ */
/* Arrays exactly as alist_struct (inc/alist.h:21-36): nlist[i] has
 * num_nlist[i] 1-based check indices of bit i, mlist[j] has num_mlist[j]
 * 1-based bit indices of check j (entries beyond the weight are ignored).
 * Validates that both views describe the same edge set. */
int  ldpc_graph_create(int N, int M, const int *num_nlist, const int *const *nlist,
                       const int *num_mlist, const int *const *mlist, ldpc_graph **out);
/* MacKay alist file with the reference loader's fixed-width semantics
 * (src/alist.cpp:70-93). */
int  ldpc_graph_load_alist(const char *path, ldpc_graph **out);
int  ldpc_graph_info(const ldpc_graph *g, int *N, int *M, int *E, int *maxdv, int *maxdc);
void ldpc_graph_destroy(ldpc_graph *g);
/* Row order and layer partition of the LAYERED schedule: row_order[M] lists
 * the rows in serial order, layer_ptr[nlayers+1] delimits the layers (runs
 * of rows that share no bit). Either array may be NULL (query nlayers
 * first). No reference counterpart. */
int  ldpc_graph_layers(const ldpc_graph *g, int32_t *row_order, int32_t *layer_ptr, int *nlayers);

/* ---- device context --------------------------------------------------- */
int  ldpc_device_count(int *n);
/* One per device: uploads the graph, owns a HIP stream, counters, scratch.
 * max_batch bounds the frames of one decode/sim call. */
int  ldpc_ctx_create(int device, const ldpc_graph *g, int max_batch, ldpc_ctx **out);
/* Launch on an external hipStream_t (e.g. torch.cuda.current_stream()); NULL
 * restores the context's own stream. A context's launches share its counters and
 * buffers, so a stream change is ordered after the work already queued on the
 * previous stream (an event): one context's launches never overlap. Use one
 * context per stream for concurrent launches. */
int  ldpc_ctx_set_stream(ldpc_ctx *ctx, void *hip_stream);
int  ldpc_ctx_synchronize(ldpc_ctx *ctx);
void ldpc_ctx_destroy(ldpc_ctx *ctx);

/* Decode `batch` frames of given channel samples y[batch][N] (float for
 * LDPC_F32, double for LDPC_F64; host or device). The cfg front-end
 * (quantize / saturate) is applied to y first, as :218-229 does.
 * c: transmitted bipolar codewords [batch][N] (+1/-1, int8) or NULL for the
 *    all-zero codeword (c = +1, :159).
 * d_out [batch][N] int8 +1/-1 decisions and frames [batch] per-frame
 * results: optional (NULL). counts: optional, ACCUMULATED (+=). Synchronous. */
int  ldpc_decode_batch(ldpc_ctx *ctx, const void *y, int batch, const ldpc_decoder_cfg *cfg,
                       const int8_t *c, int8_t *d_out, ldpc_frame_result *frames,
                       ldpc_counts *counts);

/* Codeword-file mode (:136-143, :193-212): rows of 0/1 bits [rows][N];
 * frame with global index f transmits row f % rows. rows = 0 restores the
 * all-zero codeword. */
int  ldpc_sim_set_codewords(ldpc_ctx *ctx, const uint8_t *bits, int rows);

/* Fused on-device Monte-Carlo of one SNR point: BPSK, AWGN with
 * sigma = sqrt(10^(-ebn0/10)/R/2) (:146-147) from counter-based
 * Philox4x32-10 keyed by (seed, stream_id, global frame index, bit index)
 * and a Box-Muller transform in fp32 on the SIMD's transcendental instructions
 * (v_log/v_sqrt/v_sin/v_cos_f32; the normals widened to double for the fp64
 * decoders), front-end, T iterations, error accounting into the context's device
 * counters. Frames first_cw .. first_cw+batch-1; the result does not depend
 * on how frames are split across calls or devices. Asynchronous.
 * frames_dev: optional DEVICE pointer [batch] of per-frame results. */
int  ldpc_sim_launch(ldpc_ctx *ctx, double ebn0_db, double R, const ldpc_decoder_cfg *cfg,
                     uint64_t seed, uint32_t stream_id, uint64_t first_cw, int batch,
                     ldpc_frame_result *frames_dev);
/* Synchronising read of the accumulated device counters (reset != 0 zeroes them). */
int  ldpc_ctx_read_counts(ldpc_ctx *ctx, ldpc_counts *out, int reset);
/* Error-weight histogram (error_weight_hist, :173,:280): out[w-1] = frames
 * with w bit errors, N entries. */
int  ldpc_ctx_read_histogram(ldpc_ctx *ctx, int64_t *out, int reset);
/* ldpc_sim_launch + the batch's counts accumulated into *accum; frames
 * (optional) may be host or device. Synchronous. */
int  ldpc_sim_batch(ldpc_ctx *ctx, double ebn0_db, double R, const ldpc_decoder_cfg *cfg,
                    uint64_t seed, uint32_t stream_id, uint64_t first_cw, int batch,
                    ldpc_frame_result *frames, ldpc_counts *accum);

/* ldpc_sim_batch that also returns what the fused kernel generated: the
 * channel samples y_out [batch][N] (float for F32, double for F64, before
 * the front-end) and the decisions d_out [batch][N] (+1/-1). Either may be
 * NULL; host or device. For verification of the on-device channel. */
int  ldpc_sim_trace(ldpc_ctx *ctx, double ebn0_db, double R, const ldpc_decoder_cfg *cfg,
                    uint64_t seed, uint32_t stream_id, uint64_t first_cw, int batch,
                    void *y_out, int8_t *d_out, ldpc_frame_result *frames, ldpc_counts *accum);

/* Device time (ms) of the last decode kernel, from HIP events recorded on
 * the launch stream around it. Synchronises that stream. */
int  ldpc_ctx_last_kernel_ms(ldpc_ctx *ctx, float *ms);
/* Kernel chosen for a cfg ("rows_pp", "rows_fast", "rows", "lds", "flood",
 * "global", "layered_*", "bp_*") and its per-codeword LDS bytes. */
int  ldpc_ctx_kernel_info(ldpc_ctx *ctx, const ldpc_decoder_cfg *cfg, char *name, int name_len,
                          int *lds_bytes, int *blocks_per_cu);
/* Codewords of the last min-sum launch that the fast row kernel (fp64,
 * "rows_fast") handed to the exact path because its premise failed (huge or
 * non-finite values, minima below 2^-960; 0 for any launch that did not use
 * the fast kernel). Diagnostic of the fast/exact split; synchronises the
 * stream. No reference counterpart (the reference has one exact path). */
int  ldpc_ctx_redo_count(ldpc_ctx *ctx, int64_t *n);
/* Shape of the row kernel ("rows"/"rows_fast"/"rows_pp") that decodes cfg, for the
 * on-chip (LDS) roofline model of bench.py: info[10] = {threads per block,
 * rows per thread, bit slots per thread, padded row degree, padded edge slots
 * e_pad, codewords per block, LDS bytes per block, blocks per CU, the low row
 * degree of rows_pp's degree-aware slots (0: every slot runs the padded degree),
 * check-node edge slots issued per codeword-iteration} (ABI 10: 10 entries).
 * LDPC_ERR_UNSUPPORTED when another kernel decodes cfg. Host-only, no device
 * call. No reference counterpart (diagnostic of decodeMinSum.cpp:247-263's
 * replacement). */
int  ldpc_ctx_row_sched_info(ldpc_ctx *ctx, const ldpc_decoder_cfg *cfg, int32_t *info);

/* ---- kernel-selection options (ABI 10) ------------------------------- */
/* The library picks the kernel for a cfg by itself (the reference fixes its
 * algorithm per binary at build time, C_implementations/Makefile:58-65). These
 * per-context options override that choice for tests and A/B measurements;
 * every alternative decodes bit-identically to the default (the GPU tests pin
 * that). 0 is the library's own choice for every option; the library never
 * reads them from the environment. Options take effect at the next launch. */
typedef enum {
    LDPC_OPT_ROWS64 = 1,           /* fp64 row graphs: 0 ping-pong (rows_pp), 1 rows_fast, 2 the row kernel   */
    LDPC_OPT_ROWS32 = 2,           /* fp32 MS / NMS row graphs: 0 rows_pp pairs, 1 rows_fast pairs, 2 the row kernel */
    LDPC_OPT_PP_SLOTS = 3,         /* rows_pp row slots: 0 degree-aware (when the code admits them), 1 plain  */
    LDPC_OPT_KERNEL = 4,           /* generic kernel: 0 auto, 1 lds, 2 flood (persistent), 3 global           */
    LDPC_OPT_FLOOD_MODE = 5,       /* codes beyond LDS: 0 one launch per phase, 1 the persistent kernel       */
    LDPC_OPT_FLOOD_MSG = 6,        /* phase flooding messages: 0 packed row state, 1 the c2v array            */
    LDPC_OPT_FLOOD_SPS_CHECK = 7,  /* phase flooding: resident slots per check-kernel step (0 = default)      */
    LDPC_OPT_FLOOD_SPS_BIT = 8,    /* phase flooding: resident slots per bit-kernel step (0 = default)        */
    LDPC_OPT_FLOOD_RESIDENT = 9,   /* phase flooding: resident codewords (0 = sized to the Infinity Cache)    */
    LDPC_OPT_FLOOD_STREAMS = 10,   /* phase flooding: 2 = the resident set in two halves on two streams       */
    LDPC_OPT_FLOOD_BPC = 11,       /* persistent flooding kernel: blocks per CU cap (0 = occupancy)           */
    LDPC_OPT_LAYERED_BPC = 12,     /* global layered kernel: blocks per CU (0 = 1, capped by the 208 MiB      */
                                   /* resident-state budget; set: that many per CU, no cap)                  */
    LDPC_OPT_LAYERED_LDS_POS = 13, /* global layered kernel: positions kept in LDS + 1 (0 = as many as fit)   */
    LDPC_OPT_LAYERED_ROWS64 = 14,  /* 512-thread global layered kernel, fp64 rows per pass: 1 or 2 (0 = 2)    */
    LDPC_OPT_LAYERED_THREADS = 15, /* global layered kernel threads: 512 or 1024 (0 = 1024)                   */
    LDPC_OPT_ROWS_BPC = 16,        /* row kernel (k_decode_rows): blocks per CU cap (0 = occupancy)           */
    LDPC_OPT_FAST_BPC = 17,        /* rows_fast: blocks per CU cap (0 = occupancy)                            */
    LDPC_OPT_BP_KERNEL = 18,       /* belief propagation: 0 bp_rows when the code fits, 1 the generic kernel  */
    LDPC_OPT_GDBF_KERNEL = 19,     /* GDBF: 0 gdbf_rows when the code and flags fit, 1 the generic kernel     */
    LDPC_OPT_EMS_THREADS = 20,     /* EMS (nb context), row degree 4: 0 = 1024 threads, 512                   */
    LDPC_OPT_EMS_SWIZZLE = 21      /* EMS (nb context): 0 swizzled message slots, 1 the plain layout          */
} ldpc_option;
#define LDPC_OPT_COUNT 22
/* LDPC_ERR_INVALID for an unknown option, a value outside its range, or an
 * EMS option (LDPC_OPT_EMS_*: the nb context's, ldpc_nb_ctx_set_option). */
int  ldpc_ctx_set_option(ldpc_ctx *ctx, int option, int value);
int  ldpc_ctx_get_option(const ldpc_ctx *ctx, int option, int *value);

/* ---- GDBF / NGDBF bit flipping (BASELINE config 4) --------------------- */
/* src/decodeGDBF.cpp in its parallel-flip mode (mu = 1): syndrome check
 * nodes with early stop (:298-306, :517-534), energy E = d*yq + w*sum(s)
 * [+ perturbation] and flip when E < theta (:536-621). The compile-time
 * switches of C_implementations/Makefile:33-53 are runtime flags:
 * decodeMNGDBF = NOISE|ADAPT|WEIGHT|SATURATE, decodeSMNGDBF = the same|SMOOTH,
 * decodeATGDBF = ADAPT, decodeSATGDBF = ADAPT|SMOOTH, decodeSMGDBF = SMOOTH,
 * and (ABI 8, Makefile:24-31) decodeSGDBF = SEQUENTIAL, decodeMGDBF =
 * MODESWITCH, decodeStochasticNGDBF = QUANTIZE|QPROB|WEIGHT|SATURATE.
 * ADAPT with SEQUENTIAL/MODESWITCH and NOISE with QPROB are not supported
 * (no reference target combines them). */
typedef enum {
    LDPC_GDBF_NOISE = 1,      /* -D addNoise: E += noiseScale*sigma*n per bit and iteration */
    LDPC_GDBF_ADAPT = 2,      /* -D thresholdAdaptation: theta *= lambda when not flipped   */
    LDPC_GDBF_WEIGHT = 4,     /* -D weightSyndromes: syndrome weight alpha (else 1)         */
    LDPC_GDBF_SMOOTH = 8,     /* -D outputSmoothing: majority of the last windowsize d's    */
    LDPC_GDBF_SATURATE = 16,  /* -D saturateSamples: |yq| <= Ymax                           */
    LDPC_GDBF_QUANTIZE = 32,  /* -D quantizeSamples: quantize(yq) with NQ levels            */
    LDPC_GDBF_SEQUENTIAL = 64,   /* -D sequentialmode: flip only the first bit of least energy
                                    per iteration (mu = 0, :573-580, :619-620)              */
    LDPC_GDBF_MODESWITCH = 128,  /* -D modeswitching: parallel flips until, after Tswitch,
                                    the objective sum(d*yq)+sum(s) does not grow (:309-345);
                                    then sequential                                         */
    LDPC_GDBF_QPROB = 256        /* -D quantizeProbabilities: flip with probability
                                    normalCDF((theta-E)/qsigma) rounded to 8 levels (:562-597) */
} ldpc_gdbf_flag;

typedef struct {
    int32_t flags;        /* OR of ldpc_gdbf_flag                         */
    int32_t precision;    /* ldpc_precision                               */
    int32_t T;            /* num_iterations (maximum; early stop)         */
    int32_t windowsize;   /* outputSmoothing window                       */
    int32_t nq;           /* quantizeSamples NQ                           */
    int32_t tswitch;      /* MODESWITCH: Tswitch (0 in the reference, :51) */
    double  theta;        /* initial flip threshold                       */
    double  lambda;       /* threshold adaptation factor                  */
    double  alpha;        /* syndrome weight (weightSyndromes)            */
    double  noise_scale;  /* perturbation sigma = noise_scale * channel sigma */
    double  ymax;         /* saturation / quantizer range                 */
    double  qsigma;       /* QPROB, ldpc_gdbf_decode_batch only: the normalCDF sigma
                           * (noiseSigma = noise_scale * channel sigma, :296); the sim
                           * entry points compute it from Eb/N0 and R (ABI 8) */
} ldpc_gdbf_cfg;

/* Decode `batch` frames of given RAW channel samples y[batch][N] (float for
 * F32, double for F64; host or device): front-end (:254-267), then the
 * iterations with the caller's perturbations pert[batch][T][N] (iteration it
 * of frame b adds pert[b][it][i] to E_i; required with LDPC_GDBF_NOISE; with
 * LDPC_GDBF_QPROB pert[b][it][i] is instead the uniform draw ranu() of bit i
 * in iteration it (:588); else ignored). c, d_out, frames, counts as ldpc_decode_batch; frames[].iters and
 * counts->iters report the iterations run. Synchronous. Replaces the frame
 * body of decodeGDBF.cpp main() (:250-399). */
int  ldpc_gdbf_decode_batch(ldpc_ctx *ctx, const void *y, const void *pert, int batch, const ldpc_gdbf_cfg *cfg,
                            const int8_t *c, int8_t *d_out, ldpc_frame_result *frames, ldpc_counts *counts);
/* Fused on-device Monte-Carlo of one SNR point (as ldpc_sim_launch: the
 * channel of frame f is the same as the min-sum path's); perturbations from
 * Philox4x32-10 keyed by (seed; bit/4, frame, stream_id | (it+1) << 20).
 * stream_id < 2^20. Asynchronous; counts accumulate in the context. */
int  ldpc_gdbf_sim_launch(ldpc_ctx *ctx, double ebn0_db, double R, const ldpc_gdbf_cfg *cfg, uint64_t seed,
                          uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames_dev);
/* ldpc_gdbf_sim_launch + counts accumulated into *accum; frames host or device. Synchronous. */
int  ldpc_gdbf_sim_batch(ldpc_ctx *ctx, double ebn0_db, double R, const ldpc_gdbf_cfg *cfg, uint64_t seed,
                         uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames,
                         ldpc_counts *accum);
/* Kernel chosen for a GDBF cfg ("gdbf_lds" / "gdbf_global") and its LDS bytes. */
int  ldpc_gdbf_kernel_info(ldpc_ctx *ctx, const ldpc_gdbf_cfg *cfg, char *name, int name_len, int *lds_bytes);

/* ---- non-binary GF(q) codes, Extended Min-Sum (BASELINE config 5) ------ */
/* Messages are reliabilities over GF(q) (0 = most likely symbol); check
 * nodes are the forward-backward EMS with messages truncated to the nm most
 * likely symbols and absent symbols filled with (largest kept value +
 * offset); symbol nodes add the channel reliabilities and the incoming
 * messages. Channel: each symbol is m = log2(q) BPSK bits (bit i of the
 * symbol's integer value, 0 -> +1), y = x(1 + sigma n), bit LLR 4y/N0.
 * Exact definition: DESIGN.md §11 and oracle/ems_oracle.c. No reference
 * counterpart computes this (parity unpinned); q = 2 reduces to min-sum. */
typedef struct ldpc_nb_graph ldpc_nb_graph;
typedef struct ldpc_nb_ctx ldpc_nb_ctx;

typedef struct {
    int32_t T;          /* maximum iterations                                */
    int32_t nm;         /* message truncation (>= q: full vectors)           */
    int32_t early_stop; /* stop when H*d = 0 (checked before each iteration)  */
    int32_t reserved;   /* 0                                                 */
    double  offset;     /* fill offset for truncated (absent) symbols        */
} ldpc_ems_cfg;

/* ldpc_counts + symbol errors; bit_err counts bits of the decided symbols. */
typedef struct {
    int64_t bit_err, frame_err, uncoded_bit_err, frames, iters, syndrome_fail, symbol_err;
} ldpc_nb_counts;

/* Arrays as the NB alist_struct (SystemC/NB-LDPC/inc/alist.h:25-43): nlist /
 * nvals per column (1-based check, GF value), mlist / mvals per row. q a
 * power of two (2..64), coefficients 1..q-1, check degree >= 2; both views
 * must describe the same edges and coefficients (else LDPC_ERR_GRAPH). */
int  ldpc_nb_graph_create(int N, int M, int q, const int *num_nlist, const int *const *nlist,
                          const int *const *nvals, const int *num_mlist, const int *const *mlist,
                          const int *const *mvals, ldpc_nb_graph **out);
int  ldpc_nb_graph_load_alist(const char *path, ldpc_nb_graph **out);
int  ldpc_nb_graph_info(const ldpc_nb_graph *g, int *N, int *M, int *q, int *E, int *maxdv, int *maxdc);
void ldpc_nb_graph_destroy(ldpc_nb_graph *g);

/* Device context (GF(16), row degree <= 8). */
int  ldpc_nb_ctx_create(int device, const ldpc_nb_graph *g, int max_batch, ldpc_nb_ctx **out);
int  ldpc_nb_ctx_set_stream(ldpc_nb_ctx *ctx, void *hip_stream);
void ldpc_nb_ctx_destroy(ldpc_nb_ctx *ctx);
int  ldpc_nb_ctx_read_counts(ldpc_nb_ctx *ctx, ldpc_nb_counts *out, int reset);
int  ldpc_nb_ctx_last_kernel_ms(ldpc_nb_ctx *ctx, float *ms);
/* "ems_lds" (messages in LDS) or "ems_global" (a global slot per workgroup). */
int  ldpc_ems_kernel_info(ldpc_nb_ctx *ctx, char *name, int name_len, int *lds_bytes);
/* (ABI 10) The EMS options of ldpc_option (LDPC_OPT_EMS_*); the others are refused. */
int  ldpc_nb_ctx_set_option(ldpc_nb_ctx *ctx, int option, int value);

/* Decode given channel samples y[batch][N*m] (float, host or device) with
 * bit LLRs 4y/n0. c: transmitted symbols [batch][N] or NULL (all-zero).
 * d_out [batch][N] symbols, frames[].iters = iterations run. Synchronous. */
int  ldpc_ems_decode_batch(ldpc_nb_ctx *ctx, const float *y, int batch, double n0, const ldpc_ems_cfg *cfg,
                           const uint8_t *c, uint8_t *d_out, ldpc_frame_result *frames, ldpc_nb_counts *counts);
/* Fused Monte-Carlo of the all-zero codeword: Philox4x32-10 keyed by
 * (seed; symbol, frame, stream_id), sigma = sqrt(10^(-ebn0/10)/R/2).
 * Asynchronous; counts accumulate in the context. */
int  ldpc_ems_sim_launch(ldpc_nb_ctx *ctx, double ebn0_db, double R, const ldpc_ems_cfg *cfg, uint64_t seed,
                         uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames_dev);
int  ldpc_ems_sim_batch(ldpc_nb_ctx *ctx, double ebn0_db, double R, const ldpc_ems_cfg *cfg, uint64_t seed,
                        uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames,
                        ldpc_nb_counts *accum);
/* ldpc_ems_sim_batch that also returns the generated samples y_out [batch][N*m]
 * and decisions d_out [batch][N] (host or device; either may be NULL). */
int  ldpc_ems_sim_trace(ldpc_nb_ctx *ctx, double ebn0_db, double R, const ldpc_ems_cfg *cfg, uint64_t seed,
                        uint32_t stream_id, uint64_t first_cw, int batch, float *y_out, uint8_t *d_out,
                        ldpc_frame_result *frames, ldpc_nb_counts *accum);

#ifdef __cplusplus
}
#endif
#endif /* LDPC_HIP_H */
