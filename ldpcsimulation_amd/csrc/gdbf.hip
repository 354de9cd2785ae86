// gdbf.hip -- CDNA4 (gfx950) kernels of the GDBF / NGDBF bit-flipping
// decoders (BASELINE config 4).
//
// Restates src/decodeGDBF.cpp with the Makefile's compile-time switches as
// runtime flags (gdbf.h): the parallel-flip mode (mu = 1, :284-289), the
// sequential one (mu = 0: one flip per iteration, a block argmin), mode
// switching (the objective of :623-632 summed by one lane in the reference's
// order) and quantized flipping probabilities (:562-597);
//   check nodes  s_j = prod_k d_k over mlist[j]; early stop when every
//                s_j = +1 (checkNodeUpdates :517-534, :300-306)
//   bit nodes    E_i = d_i*yq_i + sum_j w*s_j (nlist order) [+ perturbation]
//                flip d_i when E_i < theta_i; theta_i *= lambda when it did
//                not flip (symNodeUpdates :536-621)
//   smoothing    over the last `windowsize` iterations, d = sgn(sum d) when
//                the checks were never all satisfied (:348-367)
// One workgroup per codeword; its per-bit state (yq, theta, dsum, d) and
// the syndromes live in LDS (or in a global slot for codes beyond LDS).
// The perturbation of bit i in iteration `it` is the NGDBF noise
// noiseSigma*n with n from Philox4x32-10 keyed by (seed; bit/4, frame,
// stream_id | (it+1) << 20) -- the channel uses the same counters with
// it = -1, so GDBF and min-sum see identical channel samples -- or, for
// verification, given by the caller as pert[frame][it][bit].
// Compiled with -ffp-contract=off: E is accumulated with the reference's
// operation order, so fp64 decisions equal the reference's for the same noise.
#include "gdbf.h"
#include "device_common.h"
#include "minsum_common.h"

#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstring>

namespace ldpc {

template <typename F> __device__ __forceinline__ F gabs(F x) { return x < F(0) ? -x : x; }
__device__ __forceinline__ float gfloor(float x) { return __builtin_floorf(x); }
__device__ __forceinline__ double gfloor(double x) { return __builtin_floor(x); }

// Front-end of one sample (:254-267): saturation, hard decision r, quantize()
// (:488-493, whose sgn is y > 0 ? 1 : -1).
template <typename F>
__device__ __forceinline__ F gdbf_front(F y, const GdbfArgs &a, int &r)
{
    F yq = y;
    const F ymax = (F)a.ymax;
    if (a.flags & GDBF_SATURATE)
        if (gabs(yq) > ymax) yq *= ymax / gabs(yq);
    r = yq > F(0) ? 1 : -1;
    if (a.flags & GDBF_QUANTIZE) {
        const F qmax = (F)a.qmax, lmax = ymax / F(2);
        const F s = yq > F(0) ? F(1) : F(-1);
        yq = s * gfloor((gabs(yq) * qmax) / (F(2) * lmax) + F(0.5)) * (F(2) * lmax / qmax);
    }
    return yq;
}

// normalCDF (:66-69) and the nearest of quantizeProbabilities' 8 flipping
// probabilities by squared distance, first minimum (:564-585).
__device__ __forceinline__ double gncdf(double x) { return 0.5 * erfc(-x * 0.70710678118654752440); }
__device__ __forceinline__ float gncdf(float x) { return 0.5f * erfcf(-x * 0.70710678118654752440f); }
template <typename F>
__device__ __forceinline__ F gdbf_level(F pcdf)
{
    constexpr double lv[8] = {0, 0.0625, 0.125, 0.25, 0.34375, 0.4106, 0.68359, 1};
    F min_dist = F(1), best = F(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        F t = (F)lv[j] - pcdf;
        t = t * t;
        if (t < min_dist) {
            min_dist = t;
            best = (F)lv[j];
        }
    }
    return best;
}

// (E, i) pair order of the sequential flip (:604-610): E < Emin scanning i
// upwards keeps the first index of the least energy; +inf and NaN never win.
template <typename F>
__device__ __forceinline__ bool gdbf_before(F e1, int i1, F e2, int i2)
{
    return e1 < e2 || (e1 == e2 && i1 < i2);
}

// The objective of modeswitching (evaluateObjectiveFunction, :623-632): one
// lane, the reference's summation order.
template <typename F>
__device__ __forceinline__ F gdbf_objective(const DevGraph &g, const int8_t *d, const F *yq, const int8_t *s)
{
    F f = F(0);
    for (int i = 0; i < g.N; ++i) f += (F)d[i] * yq[i];
    for (int j = 0; j < g.M; ++j) f += (F)s[j];
    return f;
}

// NGDBF perturbation normals (the noise of :318-333, which the reference draws
// from glibc random() by Box-Muller, rand.h:19-20): Box-Muller on the hardware
// transcendentals -- v_log_f32 (log2), v_sqrt_f32, v_sin_f32 / v_cos_f32 (which
// take revolutions, so 2*pi*a needs no multiply) -- instead of OCML's correctly
// rounded logf / sqrtf / sincospif: a few ulp of error in a random perturbation
// leaves its distribution unchanged, and it is ~10x fewer instructions (the
// accurate form was ~80 % of the parallel-flip iteration). Both GDBF kernels use
// it, so they decode identical perturbations; parity with the reference's own
// perturbation draws goes through the caller-given path (SRC_GIVEN).
__device__ __forceinline__ void pert_normals(uint32_t ua, uint32_t ur, float &n0, float &n1)
{
    const float a = (float)ua * 2.3283064365386963e-10f + 1.1641532182693481e-10f;   // (0, 1]
    const float r = (float)ur * 2.3283064365386963e-10f + 1.1641532182693481e-10f;
    const float rad = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(r));   // sqrt(-2 ln r)
    n0 = rad * __builtin_amdgcn_cosf(a);
    n1 = rad * __builtin_amdgcn_sinf(a);
}

template <typename F, int SRC>
__device__ __forceinline__ void gdbf_codeword(const GdbfArgs &a, const DevGraph &g, int b, F *yq, F *theta,
                                              int16_t *dsum, int8_t *d, int8_t *s, int *red, F *redE, int *redI,
                                              F *fobj)
{
    const int tid = threadIdx.x, nt = blockDim.x;
    const int N = g.N, M = g.M, T = a.T;
    const uint64_t cw = a.first_cw + (uint64_t)b;
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
    const int8_t *cvec = nullptr;
    if (SRC == SRC_GIVEN) {
        if (a.c) cvec = a.c + (size_t)b * N;
    } else if (a.cw_table) {
        cvec = a.cw_table + (size_t)(cw % (uint64_t)a.cw_rows) * N;
    }
    const bool smooth = (a.flags & GDBF_SMOOTH) != 0;
    // ---- channel + front-end (:251-274) ----
    int unc = 0;
    for (int g4 = tid; g4 * 4 < N; g4 += nt) {
        F yv[4];
        if (SRC == SRC_GIVEN) {
            const F *y = reinterpret_cast<const F *>(a.y) + (size_t)b * N;
#pragma unroll
            for (int q = 0; q < 4; ++q) yv[q] = (g4 * 4 + q < N) ? y[g4 * 4 + q] : F(1);
        } else {
            uint32_t u[4];
            philox4x32_10<true>((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, k0, k1, u);
            F n[4];
            box_muller(u[0], u[1], n[0], n[1]);
            box_muller(u[2], u[3], n[2], n[3]);
            const F sigma = (F)a.sigma;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int v = g4 * 4 + q;
                yv[q] = (F)(v < N && cvec ? cvec[v] : 1) * (F(1) + sigma * n[q]);
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int v = g4 * 4 + q;
            if (v < N) {
                int r;
                yq[v] = gdbf_front<F>(yv[q], a, r);
                const int cv = cvec ? cvec[v] : 1;
                unc += (r * cv < 0);
                d[v] = (int8_t)r;
                theta[v] = (F)a.theta0;   // :291-294 (and :211 without adaptation)
                dsum[v] = 0;
            }
        }
    }
    __syncthreads();

    const F w = (F)a.w, lambda = (F)a.lambda, nsig = (F)a.noise_sigma, qsig = (F)a.qsigma;
    const bool qprob = (a.flags & GDBF_QPROB) != 0, modesw = (a.flags & GDBF_MODESWITCH) != 0;
    int mu = (a.flags & GDBF_SEQUENTIAL) ? 0 : 1;   // :284-289 (uniform over the workgroup)
    int it;
    bool sat = false;
    for (it = 0; it < T; ++it) {
        // ---- check nodes (:517-534) ----
        int fail = 0;
        for (int j = tid; j < M; j += nt) {
            const int deg = g.row_deg[j];
            const int32_t *rc = g.row_cols + (size_t)j * g.dcs;
            int p = 0;
            for (int k = 0; k < deg; ++k) p ^= d[rc[k]] < 0;
            s[j] = p ? -1 : 1;
            fail |= p;
        }
        sat = !__syncthreads_or(fail);
        if (sat) break;   // :305-306, uniform over the workgroup
        const bool eval = modesw && it > a.tswitch;   // :309-311
        if (eval) {
            if (tid == 0) fobj[0] = gdbf_objective<F>(g, d, yq, s);
            __syncthreads();
        }
        // ---- bit nodes (:536-621) ----
        const bool acc_smooth = smooth && it > T - a.windowsize;   // :349
        const bool seq = mu == 0 && !qprob;
        F ebest = dinf<F>();
        int ibest = 0x7fffffff;
        for (int g4 = tid; g4 * 4 < N; g4 += nt) {
            F pv[4] = {F(0), F(0), F(0), F(0)};   // NOISE: perturbations; QPROB: the ranu() draws
            if (a.flags & (GDBF_NOISE | GDBF_QPROB)) {
                if (SRC == SRC_GIVEN) {
                    const F *pr = reinterpret_cast<const F *>(a.pert) + ((size_t)b * T + it) * N;
#pragma unroll
                    for (int q = 0; q < 4; ++q) pv[q] = (g4 * 4 + q < N) ? pr[g4 * 4 + q] : F(0);
                } else {
                    uint32_t u[4];
                    philox4x32_10<true>((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32),
                                  (a.stream_id & 0xFFFFFu) | ((uint32_t)(it + 1) << 20), k0, k1, u);
                    if (qprob) {
#pragma unroll
                        for (int q = 0; q < 4; ++q)   // in (0, 1): fp32 from the top 24 bits ((float)u rounds up to 2^32)
                            pv[q] = sizeof(F) == 8 ? ((F)u[q] + F(0.5)) * (F)0x1p-32 : ((F)(u[q] >> 8) + F(0.5)) * (F)0x1p-24;
                    } else {
                        float n[4];
                        pert_normals(u[0], u[1], n[0], n[1]);
                        pert_normals(u[2], u[3], n[2], n[3]);
#pragma unroll
                        for (int q = 0; q < 4; ++q) pv[q] = nsig * (F)n[q];
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int i = g4 * 4 + q;
                if (i >= N) break;
                const int di = d[i];
                F E = (F)di * yq[i];
                const int e1 = g.col_ptr[i + 1];
                for (int e = g.col_ptr[i]; e < e1; ++e)
                    E += w * (F)s[g.col_refs[e] >> 6];
                if (a.flags & GDBF_NOISE) E += pv[q];
                bool flip;
                if (qprob)   // :562-597
                    flip = pv[q] < gdbf_level<F>(gncdf((-E + theta[i]) / qsig));
                else if (!seq)
                    flip = E < theta[i];   // mu = 1 (:598-603)
                else {
                    flip = false;          // mu = 0: the least energy flips after the sweep (:604-610)
                    if (E < ebest) {
                        ebest = E;
                        ibest = i;
                    }
                }
                const int dn = flip ? -di : di;
                if (flip) d[i] = (int8_t)dn;
                if ((a.flags & GDBF_ADAPT) && !flip) theta[i] *= lambda;   // :612-617
                if (acc_smooth && !seq) dsum[i] = (int16_t)(dsum[i] + dn);   // :348-354
            }
        }
        if (seq) {   // block argmin of (E, i), then the one flip (:619-620)
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const F eo = __shfl_xor(ebest, o, 64);
                const int io = __shfl_xor(ibest, o, 64);
                if (gdbf_before<F>(eo, io, ebest, ibest)) {
                    ebest = eo;
                    ibest = io;
                }
            }
            const int wv = tid >> 6, nw = (nt + 63) >> 6;
            if ((tid & 63) == 0) {
                redE[wv] = ebest;
                redI[wv] = ibest;
            }
            __syncthreads();
            if (tid == 0) {
                for (int k = 1; k < nw; ++k)
                    if (gdbf_before<F>(redE[k], redI[k], ebest, ibest)) {
                        ebest = redE[k];
                        ibest = redI[k];
                    }
                if (ebest < dinf<F>()) d[ibest] = (int8_t)-d[ibest];
            }
            __syncthreads();
            if (acc_smooth)
                for (int i = tid; i < N; i += nt) dsum[i] = (int16_t)(dsum[i] + d[i]);
        }
        __syncthreads();
        if (eval) {   // :338-345
            if (tid == 0) fobj[1] = (fobj[0] >= gdbf_objective<F>(g, d, yq, s)) ? F(1) : F(0);
            __syncthreads();
            if (fobj[1] != F(0)) mu = 0;
        }
    }
    if (smooth && !sat)   // :358-367
        for (int i = tid; i < N; i += nt) d[i] = dsum[i] > 0 ? 1 : -1;
    __syncthreads();

    // ---- error weight (:378), syndrome of the output, accounting ----
    int wgt = 0, synd = 0;
    for (int v = tid; v < N; v += nt) {
        const int dv = d[v];
        const int cv = cvec ? cvec[v] : 1;
        wgt += (dv != cv);
        if (a.d_out) a.d_out[(size_t)b * N + v] = (int8_t)dv;
    }
    for (int j = tid; j < M; j += nt) {
        const int deg = g.row_deg[j];
        const int32_t *rc = g.row_cols + (size_t)j * g.dcs;
        int p = 0;
        for (int k = 0; k < deg; ++k) p ^= d[rc[k]] < 0;
        synd |= p;
    }
    int sums[3] = {wgt, unc, synd};
    block_sum_n_t0<3>(sums, red);
    if (tid == 0) {
        const int sf = sums[2] > 0;
        atomicAdd(&a.counts[0], (unsigned long long)sums[0]);
        atomicAdd(&a.counts[1], (unsigned long long)(sums[0] > 0));
        atomicAdd(&a.counts[2], (unsigned long long)sums[1]);
        atomicAdd(&a.counts[3], 1ull);
        atomicAdd(&a.counts[4], (unsigned long long)it);   // totalIterations += it (:399)
        atomicAdd(&a.counts[5], (unsigned long long)sf);
        if (sums[0] > 0 && a.hist) atomicAdd(&a.hist[sums[0] - 1], 1ull);
        if (a.frame_res) a.frame_res[b] = make_int4(sums[0], sums[1], sf, it);
    }
    __syncthreads();
}

// Byte offsets of one codeword's state: yq[N] | theta[N] | dsum[N] (int16) | d[N] | s[M].
struct GdbfLayout {
    size_t theta, dsum, d, s, total;
};
static GdbfLayout gdbf_layout(int N, int M, size_t fsz)
{
    GdbfLayout L;
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    L.theta = al(fsz * N);
    L.dsum = L.theta + al(fsz * N);
    L.d = L.dsum + al(2 * (size_t)N);
    L.s = L.d + al((size_t)N);
    L.total = L.s + al((size_t)M);
    return L;
}

template <typename F, int SRC>
__global__ __launch_bounds__(256) void k_gdbf_lds(GdbfArgs a, DevGraph g, GdbfLayout L)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int red[16 * 4];
    __shared__ F redE[16], fobj[2];
    __shared__ int redI[16];
    gdbf_codeword<F, SRC>(a, g, blockIdx.x, reinterpret_cast<F *>(smem), reinterpret_cast<F *>(smem + L.theta),
                          reinterpret_cast<int16_t *>(smem + L.dsum), reinterpret_cast<int8_t *>(smem + L.d),
                          reinterpret_cast<int8_t *>(smem + L.s), red, redE, redI, fobj);
}

template <typename F, int SRC>
__global__ __launch_bounds__(1024) void k_gdbf_global(GdbfArgs a, DevGraph g, GdbfLayout L, unsigned char *scratch)
{
    __shared__ int red[16 * 4];
    __shared__ F redE[16], fobj[2];
    __shared__ int redI[16];
    unsigned char *base = scratch + L.total * blockIdx.x;
    for (int b = blockIdx.x; b < a.batch; b += gridDim.x)
        gdbf_codeword<F, SRC>(a, g, b, reinterpret_cast<F *>(base), reinterpret_cast<F *>(base + L.theta),
                              reinterpret_cast<int16_t *>(base + L.dsum), reinterpret_cast<int8_t *>(base + L.d),
                              reinterpret_cast<int8_t *>(base + L.s), red, redE, redI, fobj);
}

// ---------------------------------------------------------------------
// gdbf_rows: the parallel-flip family (MNGDBF, SMNGDBF, ATGDBF, SATGDBF, SMGDBF
// and their quantised / saturated forms; no SEQUENTIAL, MODESWITCH or QPROB)
// for codes with N <= 4 * 1024, row degree <= 8 and column degree <= 12 --
// config 4 (802.11n N=1944). Same arithmetic, in the same order, as
// gdbf_codeword; what differs is where the state lives:
//  * thread t owns the Philox group of bits 4t..4t+3 (the counter the channel
//    and the perturbations are keyed by) and rows t and t + blockDim;
//  * the Tanner graph sits in registers, loaded once per workgroup: a row's 8
//    bit indices and a bit's <= DVM check indices in nlist order, 16 bits each;
//    padding entries point at a dummy bit (d = +1) or a dummy check whose
//    term is -0.0 (E + -0.0 == E for every E, so E is exactly the reference's sum);
//  * yq, theta, dsum and d of the thread's bits stay in registers; LDS holds
//    the d < 0 flags as bytes (one 32-bit word per thread; a row's parity is
//    the xor of its bytes) and, per check, the term w * s_j in F (the check
//    thread computes the product a bit would, so a bit adds one LDS word per
//    edge), plus a double-buffered early-stop flag, so the early stop costs one
//    barrier instead of __syncthreads_or's reduction;
//  * a bit slot's syndrome reads are issued together, up to the wave's largest
//    degree (a uniform bound), not the code's; the workgroup is persistent.
// ---------------------------------------------------------------------
struct GdbfRowsLayout {
    int np, soff, floff, total;
};
static GdbfRowsLayout gdbf_rows_layout(int N, int M, int fsz)
{
    GdbfRowsLayout L;
    L.np = ((N + 3) & ~3) + 4;                // d < 0 flags [0..N) + pad; the last word: dummy bits (0)
    L.soff = (L.np + 7) & ~7;
    L.floff = L.soff + ((M + 2 + (M >> 5)) * fsz + 7) / 8 * 8;   // w*s at sidx(j), sidx(M) = the dummy check (-0.0)
    L.total = L.floff + 16;                   // flags[2] (+ pad)
    return L;
}

// NT = 512 (N <= 2048) or 1024 threads. Measured on the way (config 4, fp32):
// 2 bits per thread in 1024-thread workgroups (each pair of lanes running the
// same Philox call) was slower (48 vs 36 ms at that stage) -- the kernel is
// VALU-bound, Philox is a large share of it, and more waves per codeword do
// not shorten a codeword's chain of LDS round trips and barriers.
// Waves per SIMD the 512-thread instances are bounded to (fp32 / fp64): 6 = three
// workgroups per CU at 80 VGPRs, measured 22.8 vs 24.5 ms at 4 (fp32, config 4)
// despite a few spilled registers.
#ifndef LDPC_GDBF_ROWS_WAVES
#define LDPC_GDBF_ROWS_WAVES 6
#endif
// 1: the perturbations are drawn between the row gathers and their use; 0 (default):
// after the check phase's barrier -- fewer live registers, measured 21.4 vs 22.8 ms
// (fp32) and 28.2 vs 28.7 ms (fp64), 2 interleaved rounds
// 1: gdbf_rows hands out codewords past the first grid by a global ticket counter.
#ifndef LDPC_GDBF_TICKETS
#define LDPC_GDBF_TICKETS 1
#endif
#ifndef LDPC_GDBF_HOIST
#define LDPC_GDBF_HOIST 0
#endif
#ifndef LDPC_GDBF_ROWS_WAVES64
#define LDPC_GDBF_ROWS_WAVES64 4
#endif
// LDS index of check j's term: one pad word per 32, so the stride-4 rows that
// the lanes of a bit slot read (bits 4t + q of a quasi-cyclic block) fall in
// distinct banks (measured 4-way conflicts with the plain index)
__device__ __forceinline__ uint32_t sidx(uint32_t j) { return j + (j >> 5); }

template <typename F, int SRC, int DVM, int NT>
__global__ __launch_bounds__(NT, NT != 512 ? 4 : sizeof(F) == 4 ? LDPC_GDBF_ROWS_WAVES : LDPC_GDBF_ROWS_WAVES64) void k_gdbf_rows(GdbfArgs a, DevGraph g, int np, int soff, int floff)
{
    constexpr int DC = 8, BPT = 4, RPT = 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int red[16 * 4 + 1];                    // block sums; [64]: the next codeword
    uint8_t *dl = smem;                                // 1 where d = -1
    F *sl = reinterpret_cast<F *>(smem + soff);        // w * s_j, the term a bit adds for check j
    volatile int *fl = reinterpret_cast<int *>(smem + floff);
    const int tid = threadIdx.x;
    const int N = g.N, M = g.M, T = a.T;
    const int dbit = np - 1;              // dummy bit index
    const int v0 = BPT * tid;             // the thread's first bit
    const int g4 = tid;                   // its Philox group
    // ---- the graph, into registers (once per workgroup) ----
    uint32_t rc[RPT][DC / 2];
    bool rvalid[RPT];
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
        const int j = tid + r * NT;
        rvalid[r] = j < M;
        const int deg = rvalid[r] ? g.row_deg[j] : 0;
#pragma unroll
        for (int k = 0; k < DC; k += 2) {
            const uint32_t c0 = k < deg ? (uint32_t)g.row_cols[(size_t)j * g.dcs + k] : (uint32_t)dbit;
            const uint32_t c1 = k + 1 < deg ? (uint32_t)g.row_cols[(size_t)j * g.dcs + k + 1] : (uint32_t)dbit;
            rc[r][k / 2] = c0 | (c1 << 16);
        }
    }
    const bool own = v0 < N;
    uint32_t bc[BPT][DVM / 2];
    int wdeg[BPT];   // wave-uniform bound of each slot's degree
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
        const int i = v0 + q;
        int e0 = 0, deg = 0;
        if (i < N) {
            e0 = g.col_ptr[i];
            deg = g.col_ptr[i + 1] - e0;
        }
#pragma unroll
        for (int k = 0; k < DVM; k += 2) {
            const uint32_t j0 = k < deg ? g.col_refs[e0 + k] >> 6 : (uint32_t)M;
            const uint32_t j1 = k + 1 < deg ? g.col_refs[e0 + k + 1] >> 6 : (uint32_t)M;
            bc[q][k / 2] = sidx(j0) | (sidx(j1) << 16);
        }
        int m = deg;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
        wdeg[q] = __builtin_amdgcn_readfirstlane(m);
    }
    if (tid == 0) {
        *reinterpret_cast<uint32_t *>(dl + np - 4) = 0u;   // dummy bits: d = +1
        sl[sidx(M)] = -F(0);                                // dummy check: E + -0.0 == E for every E
    }
    const bool smooth = (a.flags & GDBF_SMOOTH) != 0, noise = (a.flags & GDBF_NOISE) != 0;
    const bool adapt = (a.flags & GDBF_ADAPT) != 0;
    const F w = (F)a.w, lambda = (F)a.lambda, nsig = (F)a.noise_sigma;
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);

    // Codewords: blockIdx.x first, then tickets from a.ticket, so that a block whose
    // codewords stopped early takes more (the iterations per codeword run from a few to
    // T); thread 0 draws the next ticket while the current codeword decodes.
    [[maybe_unused]] unsigned nxt = 0;
    if (LDPC_GDBF_TICKETS && tid == 0) nxt = gridDim.x + atomicAdd(a.ticket, 1u);
    for (int b = blockIdx.x; b < a.batch;) {
        const uint64_t cw = a.first_cw + (uint64_t)b;
        const int8_t *cvec = nullptr;
        if (SRC == SRC_GIVEN) {
            if (a.c) cvec = a.c + (size_t)b * N;
        } else if (a.cw_table) {
            cvec = a.cw_table + (size_t)(cw % (uint64_t)a.cw_rows) * N;
        }
        // ---- channel + front-end (:251-274), as gdbf_codeword ----
        F yq[BPT], theta[BPT];
        int d[BPT], dsum[BPT];
        int unc = 0;
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            yq[q] = F(0);
            theta[q] = (F)a.theta0;
            d[q] = 1;
            dsum[q] = 0;
        }
        if (own) {
            F yv[BPT];
            if (SRC == SRC_GIVEN) {
                const F *y = reinterpret_cast<const F *>(a.y) + (size_t)b * N;
#pragma unroll
                for (int q = 0; q < BPT; ++q) yv[q] = (v0 + q < N) ? y[v0 + q] : F(1);
            } else {
                uint32_t u[4];
                philox4x32_10<true>((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, k0, k1, u);
                F n[4];
                box_muller(u[0], u[1], n[0], n[1]);
                box_muller(u[2], u[3], n[2], n[3]);
                const F sigma = (F)a.sigma;
#pragma unroll
                for (int q = 0; q < BPT; ++q) {
                    const int v = v0 + q;
                    yv[q] = (F)(v < N && cvec ? cvec[v] : 1) * (F(1) + sigma * n[q]);
                }
            }
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                const int v = v0 + q;
                if (v < N) {
                    int r;
                    yq[q] = gdbf_front<F>(yv[q], a, r);
                    const int cv = cvec ? cvec[v] : 1;
                    unc += (r * cv < 0);
                    d[q] = r;
                }
            }
        }
        auto put_d = [&]() {
            if (own)
                *reinterpret_cast<uint32_t *>(dl + v0) = (uint32_t)(d[0] < 0) | ((uint32_t)(d[1] < 0) << 8) |
                                                         ((uint32_t)(d[2] < 0) << 16) | ((uint32_t)(d[3] < 0) << 24);
        };
        put_d();
        if (tid == 0) {
            fl[0] = 0;
            fl[1] = 0;
        }
        __syncthreads();

        int it;
        bool sat = false;
        for (it = 0; it < T; ++it) {
            // the packed 16-bit schedule words are opaque per iteration: otherwise the
            // compiler hoists the unpacked indices out of the loop and spills them
#pragma unroll
            for (int r = 0; r < RPT; ++r)
#pragma unroll
                for (int k = 0; k < DC / 2; ++k) asm volatile("" : "+v"(rc[r][k]));
#pragma unroll
            for (int q = 0; q < BPT; ++q)
#pragma unroll
                for (int k = 0; k < DVM / 2; ++k) asm volatile("" : "+v"(bc[q][k]));
            // ---- check nodes (:517-534); with LDPC_GDBF_HOIST the row gathers' LDS
            // latency is covered by this iteration's perturbations (which do not depend
            // on the decoder state; one spare set on the iteration that stops) ----
            uint32_t g8[RPT][DC];
#pragma unroll
            for (int r = 0; r < RPT; ++r)
#pragma unroll
                for (int k = 0; k < DC; ++k)
                    g8[r][k] = dl[LDPC_CHK((rc[r][k / 2] >> (16 * (k & 1))) & 0xffffu, (uint32_t)np, CHK_GDBF_BIT)];
            F pv[BPT];
#pragma unroll
            for (int q = 0; q < BPT; ++q) pv[q] = F(0);
            auto draw = [&]() {
            if (noise && own) {
                if (SRC == SRC_GIVEN) {
                    const F *pr = reinterpret_cast<const F *>(a.pert) + ((size_t)b * T + it) * N;
#pragma unroll
                    for (int q = 0; q < BPT; ++q) pv[q] = (v0 + q < N) ? pr[v0 + q] : F(0);
                } else {
                    uint32_t u[4];
                    philox4x32_10<true>((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32),
                                  (a.stream_id & 0xFFFFFu) | ((uint32_t)(it + 1) << 20), k0, k1, u);
                    float n[4];
                    pert_normals(u[0], u[1], n[0], n[1]);
                    pert_normals(u[2], u[3], n[2], n[3]);
#pragma unroll
                    for (int q = 0; q < BPT; ++q) pv[q] = nsig * (F)n[q];
                }
            }
            };
            if (LDPC_GDBF_HOIST) draw();
            int fail = 0;
#pragma unroll
            for (int r = 0; r < RPT; ++r) {
                uint32_t p = 0;
#pragma unroll
                for (int k = 0; k < DC; ++k) p ^= g8[r][k];
                if (rvalid[r])
                    sl[LDPC_CHK(sidx(tid + r * NT), sidx(M) + 1, CHK_GDBF_CHECK)] = w * (p ? F(-1) : F(1));   // w * (F)s_j, as :541-551 adds it
                fail |= (int)p;
            }
            if (fail) fl[it & 1] = 1;
            __syncthreads();
            sat = fl[it & 1] == 0;   // :305-306, uniform over the workgroup
            if (sat) break;
            if (tid == 0) fl[(it + 1) & 1] = 0;   // nobody reads or sets it before the next barrier
            if (!LDPC_GDBF_HOIST) draw();
            // ---- bit nodes (:536-621), mu = 1 ----
            const bool acc_smooth = smooth && it > T - a.windowsize;   // :349
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                // all of the slot's syndrome reads first (one LDS round trip, not one per
                // edge: a read inside the guarded add could not be issued before the
                // previous add), up to the wave's largest degree; the adds keep the
                // reference's order and skip this lane's padding by a select
                // :541-551 in nlist order, padding adds -0.0: the first K0 terms (every
                // slot reads them), then, behind one uniform branch, the rest
                constexpr int K0 = DVM < 4 ? DVM : 4;
                F sv[K0];
#pragma unroll
                for (int k = 0; k < K0; ++k)
                    sv[k] = sl[LDPC_CHK((bc[q][k / 2] >> (16 * (k & 1))) & 0xffffu, sidx(M) + 1, CHK_GDBF_CHECK)];
                F E = (F)d[q] * yq[q];
#pragma unroll
                for (int k = 0; k < K0; ++k) E += sv[k];
                if (DVM > K0 && wdeg[q] > K0) {
                    F sw[DVM - K0 > 0 ? DVM - K0 : 1];
#pragma unroll
                    for (int k = K0; k < DVM; ++k)
                        sw[k - K0] = sl[LDPC_CHK((bc[q][k / 2] >> (16 * (k & 1))) & 0xffffu, sidx(M) + 1, CHK_GDBF_CHECK)];
#pragma unroll
                    for (int k = K0; k < DVM; ++k)
                        if (k < wdeg[q]) E += sw[k - K0];
                }
                if (noise) E += pv[q];
                const bool flip = E < theta[q];             // :598-603
                const int dn = flip ? -d[q] : d[q];
                if (adapt && !flip) theta[q] *= lambda;     // :612-617
                if (acc_smooth) dsum[q] += dn;              // :348-354
                d[q] = dn;
            }
#pragma unroll
            for (int q = 0; q < BPT; ++q)   // bits past N keep +1
                if (v0 + q >= N) d[q] = 1;
            put_d();
            __syncthreads();
        }
        if (smooth && !sat) {   // :358-367
#pragma unroll
            for (int q = 0; q < BPT; ++q) d[q] = (v0 + q < N) ? (dsum[q] > 0 ? 1 : -1) : 1;
            put_d();
        }
        __syncthreads();

        // ---- error weight (:378), syndrome of the output, accounting ----
        int wgt = 0, synd = 0;
        if (own)
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                const int v = v0 + q;
                if (v < N) {
                    const int cv = cvec ? cvec[v] : 1;
                    wgt += (d[q] != cv);
                    if (a.d_out) a.d_out[(size_t)b * N + v] = (int8_t)d[q];
                }
            }
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
            uint32_t p = 0;
#pragma unroll
            for (int k = 0; k < DC; ++k) p ^= dl[LDPC_CHK((rc[r][k / 2] >> (16 * (k & 1))) & 0xffffu, (uint32_t)np, CHK_GDBF_BIT)];
            synd |= (int)p;
        }
        int sums[3] = {wgt, unc, synd};
        block_sum_n_t0<3>(sums, red);
        if (tid == 0) {
            const int sf = sums[2] > 0;
            atomicAdd(&a.counts[0], (unsigned long long)sums[0]);
            atomicAdd(&a.counts[1], (unsigned long long)(sums[0] > 0));
            atomicAdd(&a.counts[2], (unsigned long long)sums[1]);
            atomicAdd(&a.counts[3], 1ull);
            atomicAdd(&a.counts[4], (unsigned long long)it);   // totalIterations += it (:399)
            atomicAdd(&a.counts[5], (unsigned long long)sf);
            if (sums[0] > 0 && a.hist) atomicAdd(&a.hist[sums[0] - 1], 1ull);
            if (a.frame_res) a.frame_res[b] = make_int4(sums[0], sums[1], sf, it);
            if (LDPC_GDBF_TICKETS) red[64] = (int)nxt;
        }
        __syncthreads();
        if (LDPC_GDBF_TICKETS) {
            b = red[64];   // rewritten only after the next codeword's barriers
            if (tid == 0 && b < a.batch) nxt = gridDim.x + atomicAdd(a.ticket, 1u);
        } else {
            b += gridDim.x;
        }
    }
}

constexpr size_t kGdbfMaxLds = 64 * 1024;
constexpr int kGdbfRowsUnsupported = GDBF_SEQUENTIAL | GDBF_MODESWITCH | GDBF_QPROB;

LDPC_CHECK_TU(gdbf)

static bool gdbf_rows_forced_off() { return opt(LDPC_OPT_GDBF_KERNEL) == 1; }

GdbfChoice gdbf_choose(const DevGraph &g, bool f64, int flags, int maxdv, int maxdc)
{
    GdbfChoice ch;
    if (!(flags & kGdbfRowsUnsupported) && g.N >= 1 && g.N <= 4 * 1024 && g.M <= 2 * 1024 && maxdc <= 8 &&
        maxdv <= 12 && !gdbf_rows_forced_off()) {
        ch.name = "gdbf_rows";
        ch.threads = g.N <= 4 * 512 && g.M <= 2 * 512 ? 512 : 1024;
        ch.dvm = maxdv <= 4 ? 4 : 12;
        ch.lds_bytes = gdbf_rows_layout(g.N, g.M, f64 ? 8 : 4).total;
        ch.slot_bytes = 0;
        return ch;
    }
    const GdbfLayout L = gdbf_layout(g.N, g.M, f64 ? 8 : 4);
    if (L.total <= kGdbfMaxLds) {
        ch.name = "gdbf_lds";
        ch.lds_bytes = (int)L.total;
        ch.threads = 256;
        ch.slot_bytes = 0;
    } else {
        ch.name = "gdbf_global";
        ch.lds_bytes = 0;
        ch.threads = 1024;
        ch.slot_bytes = L.total;
    }
    return ch;
}

template <typename F, int SRC, int DVM, int NT>
static hipError_t gdbf_rows_launch_b(const DevGraph &g, const GdbfArgs &a, int num_cus, hipStream_t s)
{
    if (LDPC_GDBF_TICKETS) {
        if (!a.ticket) return hipErrorInvalidValue;
        const hipError_t e = hipMemsetAsync(a.ticket, 0, sizeof(unsigned), s);
        if (e != hipSuccess) return e;
    }
    const GdbfRowsLayout L = gdbf_rows_layout(g.N, g.M, (int)sizeof(F));
    auto fn = k_gdbf_rows<F, SRC, DVM, NT>;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NT, L.total) != hipSuccess || per_cu < 1)
        per_cu = 1;
    int grid = per_cu * (num_cus > 0 ? num_cus : 1);
    if (grid > a.batch) grid = a.batch;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(NT), L.total, s, a, g, L.np, L.soff, L.floff);
    return hipGetLastError();
}
template <typename F, int SRC, int DVM>
static hipError_t gdbf_rows_launch(const DevGraph &g, const GdbfArgs &a, const GdbfChoice &ch, int num_cus,
                                   hipStream_t s)
{
    return ch.threads == 512 ? gdbf_rows_launch_b<F, SRC, DVM, 512>(g, a, num_cus, s)
                             : gdbf_rows_launch_b<F, SRC, DVM, 1024>(g, a, num_cus, s);
}

template <typename F, int SRC>
static hipError_t gdbf_launch_t(const DevGraph &g, const GdbfArgs &a, const GdbfChoice &ch, void *scratch,
                                int slots, int num_cus, hipStream_t s)
{
    if (ch.dvm == 4) return gdbf_rows_launch<F, SRC, 4>(g, a, ch, num_cus, s);
    if (ch.dvm == 12) return gdbf_rows_launch<F, SRC, 12>(g, a, ch, num_cus, s);
    const GdbfLayout L = gdbf_layout(g.N, g.M, sizeof(F));
    if (ch.lds_bytes > 0) {
        hipLaunchKernelGGL((k_gdbf_lds<F, SRC>), dim3(a.batch), dim3(ch.threads), ch.lds_bytes, s, a, g, L);
    } else {
        const int grid = slots < a.batch ? slots : a.batch;
        if (grid <= 0 || !scratch) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_gdbf_global<F, SRC>), dim3(grid), dim3(ch.threads), 0, s, a, g, L,
                           (unsigned char *)scratch);
    }
    return hipGetLastError();
}

hipError_t gdbf_launch(const DevGraph &g, const GdbfArgs &a, bool f64, const GdbfChoice &ch, void *scratch,
                       int slots, int num_cus, hipStream_t s)
{
    if (a.batch <= 0) return hipSuccess;
    if (f64)
        return a.src == SRC_GIVEN ? gdbf_launch_t<double, SRC_GIVEN>(g, a, ch, scratch, slots, num_cus, s)
                                  : gdbf_launch_t<double, SRC_PHILOX>(g, a, ch, scratch, slots, num_cus, s);
    return a.src == SRC_GIVEN ? gdbf_launch_t<float, SRC_GIVEN>(g, a, ch, scratch, slots, num_cus, s)
                              : gdbf_launch_t<float, SRC_PHILOX>(g, a, ch, scratch, slots, num_cus, s);
}

}  // namespace ldpc
