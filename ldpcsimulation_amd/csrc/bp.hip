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
// a global slot. tanh/log are the device's (fp64: bp_math.h, branch-free argument
// reduction + polynomial; fp32: OCML), so messages agree with the glibc reference
// to a few ulp, not bit for bit: parity is by tolerance and by FER (tests/test_bp.py).
#include "bp.h"
#include "bp_math.h"
#include "device_common.h"

#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstring>

namespace ldpc {

__device__ __forceinline__ float bp_tanh(float x) { return tanhf(x); }
__device__ __forceinline__ double bp_tanh(double x) { return bp_tanh64(x); }   // bp_math.h
__device__ __forceinline__ float bp_log(float x) { return logf(x); }
__device__ __forceinline__ double bp_log(double x) { return bp_log64(x); }     // bp_math.h

__global__ __launch_bounds__(256) void k_bp_math_probe(const double *x, double *t, double *l, int n)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (t) t[i] = bp_tanh(x[i]);
    if (l) l[i] = bp_log(x[i]);
}

hipError_t bp_math_probe(const double *x, double *t, double *l, int n, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_bp_math_probe, dim3((n + 255) / 256), dim3(256), 0, s, x, t, l, n);
    return hipGetLastError();
}
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
    block_sum_n_t0<3>(sums, red);
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

// ---------------------------------------------------------------------
// bp_rows: the same check and bit node arithmetic, in the same order, for
// codes with N <= 4 * 1024, M <= 2 * 1024 and row degree <= 8 (802.11n
// N=1944, PEG 504x1008, 4000.2000), with the Tanner graph in registers:
//  * thread t owns bits 4t..4t+3 (the Philox group of the channel draw) and
//    rows t and t + NT; a row keeps its 8 bit indices, the bit-major slots of
//    its 8 messages and the messages it sent last iteration in registers (so
//    v2c = clip(app - c2v_old) needs no message read, :399-401), a bit keeps
//    yq, its first slot and its degree;
//  * LDS holds app[N] and the messages in bit-major order (c2v of bit i at
//    col_ptr[i] + k, nlist order): a row scatters its outputs, a bit sums its
//    slots in order (:384-393); padding edges use th = 1.0 in the product
//    (x * 1.0 == x) and a bit's padding reads a slot holding -0.0 (the exact
//    identity of +), so every message and sum is the generic kernel's;
//  * persistent workgroups, two barriers per iteration.
// LDPC_BP_KERNEL=generic keeps the one-workgroup-per-codeword kernel.
// ---------------------------------------------------------------------
struct BpRowsLayout {
    int app_off, msg_off, total, e;
};
static BpRowsLayout bp_rows_layout(int N, int E, int fsz)
{
    BpRowsLayout L;
    L.e = E;
    L.app_off = 0;                                   // app[N + 1] (app[N]: the padding gather)
    L.msg_off = ((N + 1) * fsz + 15) & ~15;          // msg[E + 1] (msg[E] = -0.0)
    L.total = L.msg_off + (((E + 1) * fsz + 15) & ~15);
    return L;
}
static bool bp_rows_fits(const DevGraph &g, int E, bool f64)
{
    if (g.N < 1 || g.N > 4 * 1024 || g.M > 2 * 1024 || g.dcs > 8 || E >= 65535) return false;
    const BpRowsLayout L = bp_rows_layout(g.N, E, f64 ? 8 : 4);
    return L.total <= 150 * 1024 && (size_t)g.M * 8 * 2 <= (size_t)(L.total - L.msg_off);   // + the prologue's slot map
}

// Progress-ordered wave priorities in the rows kernel's check phase: s_setprio 3 at the
// phase start, 2 after the first row, 0 for the bit phase (a wave behind outranks the
// ones ahead: the transcendental-heavy phase does not end on lone waves; N=1944 T=50:
// fp32 47.1 -> 41.3 ms, fp64 53.8 -> 51.2 ms). 0: none.
#ifndef LDPC_BP_PRIOBAL
#define LDPC_BP_PRIOBAL 1
#endif
#ifndef LDPC_BP_ROWS_WAVES
#define LDPC_BP_ROWS_WAVES 8   // 512-thread fp32 instance: 64 VGPRs, 4 workgroups per CU (11.9 vs 14.2 ms at 4)
#endif
template <typename F, int SRC, int NT>
__global__ __launch_bounds__(NT, NT == 512 && sizeof(F) == 4 ? LDPC_BP_ROWS_WAVES : 4) void k_bp_rows(DecodeArgs a, DevGraph g, int msg_off, int E)
{
    constexpr int DC = 8, RPT = 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int red[16 * 4];
    F *app = reinterpret_cast<F *>(smem);
    F *msg = reinterpret_cast<F *>(smem + msg_off);
    const int tid = threadIdx.x;
    const int N = g.N, M = g.M;
    const F n0 = (F)a.n0, maxllr = (F)a.max_llr;
    const int v0 = 4 * tid;
    const bool own = v0 < N;
    // ---- the graph, into registers (once per workgroup) ----
    int e0[4], deg[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        e0[q] = v0 + q < N ? g.col_ptr[v0 + q] : E;
        deg[q] = v0 + q < N ? g.col_ptr[v0 + q + 1] - e0[q] : 0;
    }
    int wdeg = max(max(deg[0], deg[1]), max(deg[2], deg[3]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wdeg = max(wdeg, __shfl_xor(wdeg, o, 64));
    wdeg = __builtin_amdgcn_readfirstlane(wdeg);
    // slot map: the bit-major slot of (row j, mlist position k), through LDS once
    uint16_t *smap = reinterpret_cast<uint16_t *>(msg);
#pragma unroll
    for (int q = 0; q < 4; ++q)
        for (int k = 0; k < deg[q]; ++k) {
            const uint32_t ref = g.col_refs[e0[q] + k];
            smap[(ref >> 6) * DC + (ref & 63u)] = (uint16_t)(e0[q] + k);
        }
    __syncthreads();
    uint32_t rc[RPT][DC / 2], rp[RPT][DC / 2];
    int rdeg[RPT], wmax[RPT];   // wmax: the wave's largest degree of row slot r (wave-uniform)
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
        const int j = tid + r * NT;
        rdeg[r] = j < M ? g.row_deg[j] : 0;
        int m = rdeg[r];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
        wmax[r] = __builtin_amdgcn_readfirstlane(m);
#pragma unroll
        for (int k = 0; k < DC; k += 2) {
            const uint32_t c0 = k < rdeg[r] ? (uint32_t)g.row_cols[(size_t)j * g.dcs + k] : (uint32_t)N;
            const uint32_t c1 = k + 1 < rdeg[r] ? (uint32_t)g.row_cols[(size_t)j * g.dcs + k + 1] : (uint32_t)N;
            rc[r][k / 2] = c0 | (c1 << 16);
            const uint32_t p0 = k < rdeg[r] ? smap[j * DC + k] : (uint32_t)E;
            const uint32_t p1 = k + 1 < rdeg[r] ? smap[j * DC + k + 1] : (uint32_t)E;
            rp[r][k / 2] = p0 | (p1 << 16);
        }
    }
    __syncthreads();
    if (tid == 0) {
        app[N] = F(0);
        msg[E] = -F(0);
#pragma unroll
        for (int q = 0; q < 3; ++q) red[q] = 0;   // block_sum_lds totals
    }
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);

    for (int b = blockIdx.x; b < a.batch; b += gridDim.x) {
        const uint64_t cw = a.first_cw + (uint64_t)b;
        const int8_t *cvec = nullptr;
        if (SRC == SRC_GIVEN) {
            if (a.c) cvec = a.c + (size_t)b * N;
        } else if (a.cw_table) {
            cvec = a.cw_table + (size_t)(cw % (uint64_t)a.cw_rows) * N;
        }
        // ---- channel + LLR front-end (:184-197), as bp_codeword ----
        int unc = 0;
        F yq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) yq[q] = F(0);
        if (own) {
            F yv[4];
            if (SRC == SRC_GIVEN) {
                const F *y = reinterpret_cast<const F *>(a.y) + (size_t)b * N;
#pragma unroll
                for (int q = 0; q < 4; ++q) yv[q] = (v0 + q < N) ? y[v0 + q] : F(1);
            } else {
                uint32_t u[4];
                philox4x32_10<true>((uint32_t)tid, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, k0, k1, u);
                F n[4];
                box_muller(u[0], u[1], n[0], n[1]);
                box_muller(u[2], u[3], n[2], n[3]);
                const F sigma = (F)a.sigma;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int v = v0 + q;
                    yv[q] = (F)(v < N && cvec ? cvec[v] : 1) * (F(1) + sigma * n[q]);
                    if (v < N && a.y_out) reinterpret_cast<F *>(a.y_out)[(size_t)b * N + v] = yv[q];
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int v = v0 + q;
                if (v < N) {
                    F l = F(4) * yv[q] / n0;                                            // :188
                    if (bp_abs(l) > maxllr) l = (l >= F(0) ? F(1) : F(-1)) * maxllr;   // :190-191
                    yq[q] = l;
                    app[v] = l;
                    const int cv = cvec ? cvec[v] : 1;
                    unc += ((l >= F(0) ? 1 : -1) * cv < 0);                             // :193-196
                }
            }
        }
        F prev[RPT][DC];   // c2v sent last iteration: 0 before the first (:307-313)
#pragma unroll
        for (int r = 0; r < RPT; ++r)
#pragma unroll
            for (int k = 0; k < DC; ++k) prev[r][k] = F(0);
        __syncthreads();

        for (int it = 0; it < a.T; ++it) {
#pragma unroll
            for (int r = 0; r < RPT; ++r)
#pragma unroll
                for (int k = 0; k < DC / 2; ++k) asm volatile("" : "+v"(rc[r][k]), "+v"(rp[r][k]));
            // ---- check nodes (:353-377) ----
            if (LDPC_BP_PRIOBAL) __builtin_amdgcn_s_setprio(3);
#pragma unroll
            for (int r = 0; r < RPT; ++r) {
                if (LDPC_BP_PRIOBAL && r > 0) __builtin_amdgcn_s_setprio(2);
                // fp64: edges and outputs past the wave's largest row degree are skipped (an
                // SGPR branch): th = 1 there, as for a padding edge of a lower-degree row (fp32
                // keeps the straight-line row: 10.3 vs 11.3 ms with the branches)
                F th[DC];
#pragma unroll
                for (int k = 0; k < DC; ++k) {
                    th[k] = F(1);
                    if (sizeof(F) == 4 || k < wmax[r]) {
                        F v = app[LDPC_CHK((rc[r][k / 2] >> (16 * (k & 1))) & 0xffffu, (uint32_t)N + 1, CHK_BP_COL)] -
                              prev[r][k];   // :399
                        if (bp_abs(v) > maxllr) v = maxllr * (v >= F(0) ? F(1) : F(-1));      // :400-401
                        th[k] = k < rdeg[r] ? bp_tanh(v / F(2)) : F(1);
                    }
                }
                // prod over k != jj in mlist order from 1 (:362-371): its first jj factors
                // are the running prefix pre[jj] -- the same roundings -- so only the
                // factors after jj are multiplied per output (35 multiplies, not 56)
                F pre[DC];
                pre[0] = F(1);
#pragma unroll
                for (int k = 0; k + 1 < DC; ++k) pre[k + 1] = pre[k] * th[k];
#pragma unroll
                for (int jj = 0; jj < DC; ++jj) {
                    if (sizeof(F) == 8 && jj >= wmax[r]) continue;
                    F prod = pre[jj];
#pragma unroll
                    for (int k = jj + 1; k < DC; ++k) prod *= th[k];
                    F o = bp_log((F(1) + prod) / (F(1) - prod));
                    if (sizeof(F) == 4 && bp_abs(o) > maxllr) o = o >= F(0) ? maxllr : -maxllr;
                    prev[r][jj] = o;
                    if (jj < rdeg[r]) msg[LDPC_CHK((rp[r][jj / 2] >> (16 * (jj & 1))) & 0xffffu, (uint32_t)E + 1, CHK_BP_MSG)] = o;
                }
            }
            if (LDPC_BP_PRIOBAL) __builtin_amdgcn_s_setprio(0);
            __syncthreads();
            // ---- bit nodes: sum in nlist order (:384-393) ----
            if (own) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    F sum = yq[q];
                    for (int k = 0; k < wdeg; ++k) sum += msg[LDPC_CHK(k < deg[q] ? e0[q] + k : E, E + 1, CHK_BP_MSG)];
                    if (v0 + q < N) app[v0 + q] = sum;
                }
            }
            __syncthreads();
        }

        // ---- decisions (:404-407; d = r when T = 0), error weight, syndrome ----
        int w = 0, synd = 0;
        if (own)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int v = v0 + q;
                if (v < N) {
                    const F s = app[v];
                    const int d = a.T > 0 ? (s > F(0) ? 1 : -1) : (s >= F(0) ? 1 : -1);
                    const int cv = cvec ? cvec[v] : 1;
                    w += (d != cv);
                    if (a.d_out) a.d_out[(size_t)b * N + v] = (int8_t)d;
                }
            }
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
            int par = 0;
#pragma unroll
            for (int k = 0; k < DC; ++k)
                if (k < rdeg[r]) {
                    const F s = app[LDPC_CHK((rc[r][k / 2] >> (16 * (k & 1))) & 0xffffu, (uint32_t)N + 1, CHK_BP_COL)];
                    par ^= a.T > 0 ? (s > F(0) ? 0 : 1) : (s >= F(0) ? 0 : 1);
                }
            synd |= par;
        }
        int sums[3] = {w, unc, synd};
        block_sum_lds<3>(sums, red);   // re-zeroed by thread 0; the step's last barrier orders it
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
}

LDPC_CHECK_TU(bp)

#ifdef LDPC_CHECK
__global__ void k_check_selftest(int *sink)
{
    // entry 7 of a 3-entry table: recorded (site CHK_BP_COL) and clamped to 0
    const int i = LDPC_CHK(threadIdx.x + 7, 3, CHK_BP_COL);
    if (sink) sink[i] = 1;
}
hipError_t check_selftest_launch(hipStream_t s)
{
    hipLaunchKernelGGL(k_check_selftest, dim3(1), dim3(1), 0, s, (int *)nullptr);
    return hipGetLastError();
}
#endif

static bool bp_rows_forced_off() { return opt(LDPC_OPT_BP_KERNEL) == 1; }

constexpr size_t kBpMaxLds = 160 * 1024;

KernelChoice bp_choose(const DevGraph &g, bool f64, int E)
{
    KernelChoice kc;
    if (bp_rows_fits(g, E, f64) && !bp_rows_forced_off()) {
        kc.name = "bp_rows";
        kc.threads = g.N <= 4 * 512 && g.M <= 2 * 512 ? 512 : 1024;
        kc.cw_per_block = 1;
        kc.lds_bytes = bp_rows_layout(g.N, E, f64 ? 8 : 4).total;
        kc.scratch_per_block = 0;
        return kc;
    }
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

template <typename F, int SRC, int NT>
static hipError_t bp_rows_launch(const DevGraph &g, const DecodeArgs &a, const KernelChoice &kc, int E, int num_cus,
                                 hipStream_t s)
{
    const BpRowsLayout L = bp_rows_layout(g.N, E, (int)sizeof(F));
    auto fn = k_bp_rows<F, SRC, NT>;
    if (L.total > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, L.total);
        if (e != hipSuccess) return e;
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NT, L.total) != hipSuccess || per_cu < 1)
        per_cu = 1;
    int grid = per_cu * (num_cus > 0 ? num_cus : 1);
    if (grid > a.batch) grid = a.batch;
    (void)kc;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(NT), L.total, s, a, g, L.msg_off, E);
    return hipGetLastError();
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
                              int E, int num_cus, hipStream_t s)
{
    if (kc.name[3] == 'r')   // "bp_rows"
        return kc.threads == 512 ? bp_rows_launch<F, SRC, 512>(g, a, kc, E, num_cus, s)
                                 : bp_rows_launch<F, SRC, 1024>(g, a, kc, E, num_cus, s);
    if (g.dcs <= 8) return bp_launch_d<F, SRC, 8>(g, a, kc, gs, gblocks, s);
    if (g.dcs <= 16) return bp_launch_d<F, SRC, 16>(g, a, kc, gs, gblocks, s);
    return bp_launch_d<F, SRC, kBpMaxDc>(g, a, kc, gs, gblocks, s);
}

hipError_t bp_launch(const DevGraph &g, const DecodeArgs &a, bool f64, const KernelChoice &kc, void *gscratch,
                     int gblocks, int E, int num_cus, hipStream_t s)
{
    if (a.batch <= 0) return hipSuccess;
    if (f64)
        return a.src == SRC_GIVEN ? bp_launch_t<double, SRC_GIVEN>(g, a, kc, gscratch, gblocks, E, num_cus, s)
                                  : bp_launch_t<double, SRC_PHILOX>(g, a, kc, gscratch, gblocks, E, num_cus, s);
    return a.src == SRC_GIVEN ? bp_launch_t<float, SRC_GIVEN>(g, a, kc, gscratch, gblocks, E, num_cus, s)
                              : bp_launch_t<float, SRC_PHILOX>(g, a, kc, gscratch, gblocks, E, num_cus, s);
}

}  // namespace ldpc
