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
            philox4x32_10((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, k0, k1, u);
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
                    philox4x32_10((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32),
                                  (a.stream_id & 0xFFFFFu) | ((uint32_t)(it + 1) << 20), k0, k1, u);
                    if (qprob) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) pv[q] = ((F)u[q] + F(0.5)) * (F)0x1p-32;   // in (0, 1)
                    } else {
                        F n[4];
                        box_muller(u[0], u[1], n[0], n[1]);
                        box_muller(u[2], u[3], n[2], n[3]);
#pragma unroll
                        for (int q = 0; q < 4; ++q) pv[q] = nsig * n[q];
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
    block_sum_n<3>(sums, red);
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

constexpr size_t kGdbfMaxLds = 64 * 1024;

GdbfChoice gdbf_choose(const DevGraph &g, bool f64)
{
    GdbfChoice ch;
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

template <typename F, int SRC>
static hipError_t gdbf_launch_t(const DevGraph &g, const GdbfArgs &a, const GdbfChoice &ch, void *scratch,
                                int slots, hipStream_t s)
{
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
                       int slots, hipStream_t s)
{
    if (a.batch <= 0) return hipSuccess;
    if (f64)
        return a.src == SRC_GIVEN ? gdbf_launch_t<double, SRC_GIVEN>(g, a, ch, scratch, slots, s)
                                  : gdbf_launch_t<double, SRC_PHILOX>(g, a, ch, scratch, slots, s);
    return a.src == SRC_GIVEN ? gdbf_launch_t<float, SRC_GIVEN>(g, a, ch, scratch, slots, s)
                              : gdbf_launch_t<float, SRC_PHILOX>(g, a, ch, scratch, slots, s);
}

}  // namespace ldpc
