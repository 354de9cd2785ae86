// bp.hip -- CDNA4 (gfx950) kernels of the belief-propagation (tanh rule)
// decoder (reference src/decodeBP.cpp).
//
//   front-end   yq = 4*y/N0 clipped to +-MAXLLR (:184-197)
//   check node  c2v_j = log((1+p)/(1-p)), p = prod_{k != j} tanh(v2c_k/2)
//               in mlist order skipping j (checkNodeUpdates :353-377)
//   bit node    sum = yq + sum c2v in nlist order, v2c = clip(sum - c2v),
//               d = sum > 0 ? +1 : -1 (symNodeUpdates :379-409)
// One workgroup per codeword. The state is app[N] (= the bit sums), yq[N]
// and c2v[M][dcs] (by row and mlist position); v2c is not stored: the check
// node rebuilds it as clip(app - c2v_old), the same IEEE subtraction and
// clip the reference's bit node performs. State in LDS when it fits, else in
// a global slot. tanh/log are the device's (OCML), so messages agree with the
// glibc reference to a few ulp, not bit for bit: parity is by tolerance and
// by FER (tests/test_bp.py).
#include "bp.h"
#include "device_common.h"

#include <hip/hip_runtime.h>

namespace ldpc {

__device__ __forceinline__ float bp_tanh(float x) { return tanhf(x); }
__device__ __forceinline__ double bp_tanh(double x) { return tanh(x); }
__device__ __forceinline__ float bp_log(float x) { return logf(x); }
__device__ __forceinline__ double bp_log(double x) { return log(x); }
template <typename F> __device__ __forceinline__ F bp_abs(F x) { return x < F(0) ? -x : x; }

template <typename F, int SRC, int DCB>
__device__ __forceinline__ void bp_codeword(const DecodeArgs &a, const DevGraph &g, int b, F *app, F *yq, F *c2v,
                                            int *red)
{
    const int tid = threadIdx.x, nt = blockDim.x;
    const int N = g.N, M = g.M, dcs = g.dcs;
    const uint64_t cw = a.first_cw + (uint64_t)b;
    const F n0 = (F)a.n0, maxllr = (F)a.max_llr;
    const int8_t *cvec = nullptr;
    if (SRC == SRC_GIVEN) {
        if (a.c) cvec = a.c + (size_t)b * N;
    } else if (a.cw_table) {
        cvec = a.cw_table + (size_t)(cw % (uint64_t)a.cw_rows) * N;
    }
    // ---- channel + LLR front-end (:184-197) ----
    int unc = 0;
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
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
                if (v < N && a.y_out) reinterpret_cast<F *>(a.y_out)[(size_t)b * N + v] = yv[q];
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int v = g4 * 4 + q;
            if (v < N) {
                F l = F(4) * yv[q] / n0;                                   // :188
                if (bp_abs(l) > maxllr) l = (l >= F(0) ? F(1) : F(-1)) * maxllr;   // :190-191
                yq[v] = l;
                app[v] = l;
                const int cv = cvec ? cvec[v] : 1;
                unc += ((l >= F(0) ? 1 : -1) * cv < 0);                    // r = sgn(yq) (:193-196)
            }
        }
    }
    for (int e = tid; e < M * dcs; e += nt) c2v[e] = F(0);   // v2c = yq on the first pass (:307-313)
    __syncthreads();

    for (int it = 0; it < a.T; ++it) {
        // ---- check nodes (:353-377) ----
        for (int j = tid; j < M; j += nt) {
            const int deg = g.row_deg[j];
            const int32_t *rc = g.row_cols + (size_t)j * dcs;
            F *cj = c2v + (size_t)j * dcs;
            // DCB >= deg, loops unrolled so that th[] lives in registers
            F th[DCB];
#pragma unroll
            for (int k = 0; k < DCB; ++k)
                if (k < deg) {
                    F v = app[rc[k]] - cj[k];                              // v2c = sum - c2v (:399)
                    if (bp_abs(v) > maxllr) v = maxllr * (v >= F(0) ? F(1) : F(-1));   // :400-401
                    th[k] = bp_tanh(v / F(2));
                }
#pragma unroll
            for (int jj = 0; jj < DCB; ++jj)
                if (jj < deg) {
                    F prod = F(1);
#pragma unroll
                    for (int k = 0; k < DCB; ++k)
                        if (k != jj && k < deg) prod *= th[k];
                    F o = bp_log((F(1) + prod) / (F(1) - prod));
                    // fp32: tanhf(10) rounds to 1 and 1 - prod to 0; clip c2v to
                    // +-MAXLLR (a no-op in exact arithmetic, see oracle/bp_oracle.c)
                    if (sizeof(F) == 4 && bp_abs(o) > maxllr) o = o >= F(0) ? maxllr : -maxllr;
                    cj[jj] = o;
                }
        }
        __syncthreads();
        // ---- bit nodes: sum in nlist order (:384-393) ----
        for (int v = tid; v < N; v += nt) {
            F sum = yq[v];
            const int e1 = g.col_ptr[v + 1];
            for (int e = g.col_ptr[v]; e < e1; ++e) {
                const uint32_t ref = g.col_refs[e];
                sum += c2v[(size_t)(ref >> 6) * dcs + (ref & 63u)];
            }
            app[v] = sum;
        }
        __syncthreads();
    }

    // ---- decisions (:404-407; d = r when T = 0), error weight, syndrome ----
    int w = 0, synd = 0;
    for (int v = tid; v < N; v += nt) {
        const int d = a.T > 0 ? (app[v] > F(0) ? 1 : -1) : (yq[v] >= F(0) ? 1 : -1);
        const int cv = cvec ? cvec[v] : 1;
        w += (d != cv);
        if (a.d_out) a.d_out[(size_t)b * N + v] = (int8_t)d;
    }
    for (int j = tid; j < M; j += nt) {
        const int deg = g.row_deg[j];
        const int32_t *rc = g.row_cols + (size_t)j * dcs;
        int par = 0;
        for (int k = 0; k < deg; ++k) {
            const F s = app[rc[k]];
            par ^= a.T > 0 ? (s > F(0) ? 0 : 1) : (yq[rc[k]] >= F(0) ? 0 : 1);
        }
        synd |= par;
    }
    int sums[3] = {w, unc, synd};
    block_sum_n<3>(sums, red);
    if (tid == 0) {
        const int sf = sums[2] > 0;
        atomicAdd(&a.counts[0], (unsigned long long)sums[0]);
        atomicAdd(&a.counts[1], (unsigned long long)(sums[0] > 0));
        atomicAdd(&a.counts[2], (unsigned long long)sums[1]);
        atomicAdd(&a.counts[3], 1ull);
        atomicAdd(&a.counts[4], (unsigned long long)a.T);
        atomicAdd(&a.counts[5], (unsigned long long)sf);
        if (sums[0] > 0 && a.hist) atomicAdd(&a.hist[sums[0] - 1], 1ull);
        if (a.frame_res) a.frame_res[b] = make_int4(sums[0], sums[1], sf, 0);
    }
    __syncthreads();
}

static size_t bp_state_bytes(const DevGraph &g, size_t fsz)
{
    return (fsz * (2 * (size_t)g.N + (size_t)g.M * g.dcs) + 255) & ~(size_t)255;
}

template <typename F, int SRC, int DCB>
__global__ __launch_bounds__(512) void k_bp_lds(DecodeArgs a, DevGraph g)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int red[16 * 4];
    F *app = reinterpret_cast<F *>(smem);
    bp_codeword<F, SRC, DCB>(a, g, blockIdx.x, app, app + g.N, app + 2 * g.N, red);
}

template <typename F, int SRC, int DCB>
__global__ __launch_bounds__(512) void k_bp_global(DecodeArgs a, DevGraph g, unsigned char *scratch, size_t slot)
{
    __shared__ int red[16 * 4];
    F *app = reinterpret_cast<F *>(scratch + slot * blockIdx.x);
    for (int b = blockIdx.x; b < a.batch; b += gridDim.x)
        bp_codeword<F, SRC, DCB>(a, g, b, app, app + g.N, app + 2 * g.N, red);
}

constexpr size_t kBpMaxLds = 160 * 1024;

KernelChoice bp_choose(const DevGraph &g, bool f64)
{
    KernelChoice kc;
    kc.threads = 512;   // measured (N=1944 fp32): 256 -> 1.06, 512 -> 1.50, 1024 -> 0.92 Gbit/s
    kc.cw_per_block = 1;
    const size_t st = bp_state_bytes(g, f64 ? 8 : 4);
    if (st <= kBpMaxLds) {
        kc.name = "bp_lds";
        kc.lds_bytes = (int)st;
        kc.scratch_per_block = 0;
    } else {
        kc.name = "bp_global";
        kc.lds_bytes = 0;
        kc.scratch_per_block = st;
    }
    return kc;
}

template <typename F, int SRC, int DCB>
static hipError_t bp_launch_d(const DevGraph &g, const DecodeArgs &a, const KernelChoice &kc, void *gs, int gblocks,
                              hipStream_t s)
{
    if (kc.lds_bytes > 0) {
        auto fn = k_bp_lds<F, SRC, DCB>;
        if (kc.lds_bytes > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               kc.lds_bytes);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(fn, dim3(a.batch), dim3(kc.threads), kc.lds_bytes, s, a, g);
    } else {
        const int grid = gblocks < a.batch ? gblocks : a.batch;
        if (grid <= 0 || !gs) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_bp_global<F, SRC, DCB>), dim3(grid), dim3(kc.threads), 0, s, a, g, (unsigned char *)gs,
                           kc.scratch_per_block);
    }
    return hipGetLastError();
}

template <typename F, int SRC>
static hipError_t bp_launch_t(const DevGraph &g, const DecodeArgs &a, const KernelChoice &kc, void *gs, int gblocks,
                              hipStream_t s)
{
    if (g.dcs <= 8) return bp_launch_d<F, SRC, 8>(g, a, kc, gs, gblocks, s);
    if (g.dcs <= 16) return bp_launch_d<F, SRC, 16>(g, a, kc, gs, gblocks, s);
    return bp_launch_d<F, SRC, kBpMaxDc>(g, a, kc, gs, gblocks, s);
}

hipError_t bp_launch(const DevGraph &g, const DecodeArgs &a, bool f64, const KernelChoice &kc, void *gscratch,
                     int gblocks, hipStream_t s)
{
    if (a.batch <= 0) return hipSuccess;
    if (f64)
        return a.src == SRC_GIVEN ? bp_launch_t<double, SRC_GIVEN>(g, a, kc, gscratch, gblocks, s)
                                  : bp_launch_t<double, SRC_PHILOX>(g, a, kc, gscratch, gblocks, s);
    return a.src == SRC_GIVEN ? bp_launch_t<float, SRC_GIVEN>(g, a, kc, gscratch, gblocks, s)
                              : bp_launch_t<float, SRC_PHILOX>(g, a, kc, gscratch, gblocks, s);
}

}  // namespace ldpc
