// nb.hip -- CDNA4 (gfx950) kernels of the non-binary GF(16) Extended Min-Sum
// decoder (BASELINE config 5; no reference counterpart:
// the reference's NB model, SystemC/NB-LDPC/inc/nodes.h, is a q^dc-LUT BP
// that does not compile). The algorithm is defined by the CPU oracle
// oracle/ems_oracle.c, which this reproduces bit for bit.
//
// Mapping: a message is a 16-vector over GF(16); a group of 16 consecutive
// lanes holds one message, lane x the entry of symbol x. Everything a check
// or symbol node needs across the vector is a cross-lane move inside the
// group, done with ds_swizzle in bitmask mode (no LDS traffic):
//   broadcast of lane a   ->  and = 0x10, or = a
//   lane x reads lane x^a ->  and = 0x1F, xor = a
// so the elementary check node W(x) = min_a P(a) + Q(a ^ x) is 16 steps of
// (swizzle, swizzle, add, min) per lane. One workgroup = 1024 threads =
// 64 groups decodes one codeword at a time (persistent over the batch); the
// codeword's edge messages (E x 16 fp32, in place: c2v after the check phase,
// v2c after the symbol phase) and bit LLRs live in LDS when they fit
// (145 KB for N = 1000, E = 2000), else in a global slot per workgroup.
#include "nb.h"
#include "device_common.h"
#include "kernels.h"

#include <hip/hip_runtime.h>

namespace ldpc {

constexpr float kInf = __builtin_huge_valf();

template <int PAT>
__device__ __forceinline__ float swz(float v)
{
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), PAT));
}
template <int PAT>
__device__ __forceinline__ int swz(int v)
{
    return __builtin_amdgcn_ds_swizzle(v, PAT);
}
// lane x of a Q-lane group reads lane x ^ X / lane A of its group
template <int Q, int X> struct XorPat { static constexpr int v = (X << 10) | 0x1F; };
template <int Q, int A> struct BcastPat { static constexpr int v = (A << 5) | (0x1F & ~(Q - 1)); };

// W(x) = min over a of P(a) + Q(a ^ x)  (oracle ecn(): the same single adds, exact min)
template <int Q, int A>
struct Ecn {
    static __device__ __forceinline__ float run(float p, float qv, float w)
    {
        const float s = swz<BcastPat<Q, A>::v>(p) + swz<XorPat<Q, A>::v>(qv);
        return Ecn<Q, A + 1>::run(p, qv, fminf(w, s));
    }
};
template <int Q>
struct Ecn<Q, Q> {
    static __device__ __forceinline__ float run(float, float, float w) { return w; }
};

// number of lanes y != x with (v_y, y) < (v_x, x)
template <int Q, int X>
struct Rank {
    static __device__ __forceinline__ int run(float v, int x, int r)
    {
        const float o = swz<XorPat<Q, X>::v>(v);
        const int y = x ^ X;
        r += (o < v) | ((o == v) & (y < x));
        return Rank<Q, X + 1>::run(v, x, r);
    }
};
template <int Q>
struct Rank<Q, Q> {
    static __device__ __forceinline__ int run(float, int, int r) { return r; }
};

template <int Q>
__device__ __forceinline__ float trunc_nm(float v, int x, int nm)
{
    if (nm >= Q) return v;
    return Rank<Q, 1>::run(v, x, 0) < nm ? v : kInf;
}

template <int Q>
__device__ __forceinline__ float ecn(float p, float qv)
{
    return Ecn<Q, 0>::run(p, qv, kInf);
}

template <int Q>
__device__ __forceinline__ float group_min(float v)
{
    v = fminf(v, swz<XorPat<Q, 1>::v>(v));
    v = fminf(v, swz<XorPat<Q, 2>::v>(v));
    v = fminf(v, swz<XorPat<Q, 4>::v>(v));
    if (Q > 8) v = fminf(v, swz<XorPat<Q, 8>::v>(v));
    return v;
}
template <int Q>
__device__ __forceinline__ float group_max(float v)
{
    v = fmaxf(v, swz<XorPat<Q, 1>::v>(v));
    v = fmaxf(v, swz<XorPat<Q, 2>::v>(v));
    v = fmaxf(v, swz<XorPat<Q, 4>::v>(v));
    if (Q > 8) v = fmaxf(v, swz<XorPat<Q, 8>::v>(v));
    return v;
}
// first minimum: smallest (value, symbol)
template <int Q, int X>
__device__ __forceinline__ void argmin_step(float &bv, int &bi)
{
    const float ov = swz<XorPat<Q, X>::v>(bv);
    const int oi = swz<XorPat<Q, X>::v>(bi);
    if (ov < bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
    }
}
template <int Q>
__device__ __forceinline__ int group_argmin(float v, int x)
{
    float bv = v;
    int bi = x;
    argmin_step<Q, 1>(bv, bi);
    argmin_step<Q, 2>(bv, bi);
    argmin_step<Q, 4>(bv, bi);
    if (Q > 8) argmin_step<Q, 8>(bv, bi);
    return bi;
}

// L(x) = sum over bits i (ascending) disagreeing with the hard decision of |lam_i| (oracle symbol_llr)
template <int MB>
__device__ __forceinline__ float sym_llr(const float *lam, int x)
{
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < MB; ++i) {
        const float l = lam[i];
        const int hd = l < 0.0f;
        if (((x >> i) & 1) != hd) s += fabsf(l);
    }
    return s;
}

// The graph, re-packed into LDS once per workgroup (global loads in the
// per-iteration loops would put two dependent HBM/L2 round trips on every
// check and symbol round).
struct NbSched {
    const uint32_t *cn;      // [M]  r0 | d << 24
    const uint8_t *ehinv;    // [E]  h^-1 of each edge slot
    const uint8_t *eh;       // [E]  h
    const uint16_t *ecol;    // [E]  symbol of each edge slot
    const uint32_t *vn;      // [N]  first col entry << 8 | degree
    const uint16_t *vslot;   // [E]  edge slots of each symbol, nlist order
};

template <int Q>
__device__ __forceinline__ int syndrome_fail(const NbDevGraph &g, const NbSched &s, const uint8_t *dec,
                                             const uint8_t *gmul)
{
    int fail = 0;
    for (int j = threadIdx.x; j < g.M; j += blockDim.x) {
        const uint32_t sc = s.cn[j];
        const int r0 = sc & 0xFFFFFF, d = sc >> 24;
        int sy = 0;
        for (int e = r0; e < r0 + d; ++e) sy ^= gmul[s.eh[e] * Q + dec[s.ecol[e]]];
        fail |= sy != 0;
    }
    return __syncthreads_or(fail);
}

template <int Q, int MB, int DC, int SRC>
__device__ __forceinline__ void ems_codeword(const NbArgs &a, const NbDevGraph &g, int b, float *msg, float *lam,
                                             uint8_t *dec, const uint8_t *gmul, const NbSched &sc, int *red)
{
    const int tid = threadIdx.x, nt = blockDim.x;
    const int x = tid & (Q - 1), grp = tid / Q, ngrp = nt / Q;
    const int N = g.N, M = g.M;
    const uint64_t cw = a.first_cw + (uint64_t)b;
    const uint8_t *cvec = (SRC == SRC_GIVEN && a.c) ? a.c + (size_t)b * N : nullptr;

    // ---- channel: BPSK per bit, AWGN, bit LLRs lam = (4*y)/N0 ----
    int unc = 0;
    {
        const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
        for (int v = tid; v < N; v += nt) {
            const int cs = cvec ? cvec[v] : 0;
            float yv[MB];
            if (SRC == SRC_GIVEN) {
#pragma unroll
                for (int i = 0; i < MB; ++i) yv[i] = a.y[((size_t)b * N + v) * MB + i];
            } else {
                static_assert(MB == 4, "one Philox call per GF(16) symbol");
                uint32_t u[4];
                philox4x32_10((uint32_t)v, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, k0, k1, u);
                float n[4];
                box_muller(u[0], u[1], n[0], n[1]);
                box_muller(u[2], u[3], n[2], n[3]);
#pragma unroll
                for (int i = 0; i < MB; ++i) {
                    const float xb = ((cs >> i) & 1) ? -1.0f : 1.0f;
                    yv[i] = xb * (1.0f + a.sigma * n[i]);
                    if (a.y_out) a.y_out[((size_t)b * N + v) * MB + i] = yv[i];
                }
            }
#pragma unroll
            for (int i = 0; i < MB; ++i) {
                const float l = (4.0f * yv[i]) / a.n0;
                lam[v * MB + i] = l;
                unc += (int)(l < 0.0f) != ((cs >> i) & 1);
            }
        }
    }
    __syncthreads();
    // ---- initial messages v2c = L, decisions argmin L ----
    for (int v = grp; v < N; v += ngrp) {
        const float L = sym_llr<MB>(lam + v * MB, x);
        const uint32_t vp = sc.vn[v];
        const int e0 = vp >> 8, e1 = e0 + (vp & 255);
        for (int e = e0; e < e1; ++e) msg[(size_t)sc.vslot[e] * Q + x] = L;
        const int d = group_argmin<Q>(L, x);
        if (x == 0) dec[v] = (uint8_t)d;
    }
    __syncthreads();
    int fail = syndrome_fail<Q>(g, sc, dec, gmul);
    int it = 0;
    while (it < a.T && (!a.early_stop || fail)) {
        // ---- check nodes: forward-backward EMS ----
        for (int j = grp; j < M; j += ngrp) {
            const uint32_t cs = sc.cn[j];
            const int r0 = cs & 0xFFFFFF, d = cs >> 24;
            float U[DC], F[DC], B[DC];
            int idx[DC];
#pragma unroll
            for (int k = 0; k < DC; ++k)
                if (k < d) {
                    idx[k] = (r0 + k) * Q + gmul[sc.ehinv[r0 + k] * Q + x];   // U(x) = v2c(h^-1 x)
                    U[k] = trunc_nm<Q>(msg[idx[k]], x, a.nm);
                }
            F[0] = U[0];
#pragma unroll
            for (int k = 1; k < DC - 1; ++k)
                if (k <= d - 2) F[k] = trunc_nm<Q>(ecn<Q>(F[k - 1], U[k]), x, a.nm);
#pragma unroll
            for (int k = DC - 1; k >= 1; --k) {
                if (k == d - 1)
                    B[k] = U[k];
                else if (k < d - 1)
                    B[k] = trunc_nm<Q>(ecn<Q>(B[k + 1 < DC ? k + 1 : k], U[k]), x, a.nm);
            }
#pragma unroll
            for (int k = 0; k < DC; ++k)
                if (k < d) {
                    float w;
                    if (k == 0)
                        w = B[1];
                    else if (k == d - 1)
                        w = F[k - 1];
                    else
                        w = trunc_nm<Q>(ecn<Q>(F[k - 1], B[k + 1 < DC ? k + 1 : k]), x, a.nm);
                    const float mx = group_max<Q>(w < kInf ? w : -1.0f);
                    msg[idx[k]] = w < kInf ? w : mx + a.offset;        // c2v(a) = W(h a), a = h^-1 x
                }
        }
        __syncthreads();
        // ---- symbol nodes ----
        for (int v = grp; v < N; v += ngrp) {
            float app = sym_llr<MB>(lam + v * MB, x);
            const uint32_t vp = sc.vn[v];
            const int e0 = vp >> 8, e1 = e0 + (vp & 255);
            for (int e = e0; e < e1; ++e) app += msg[(size_t)sc.vslot[e] * Q + x];
            const int d = group_argmin<Q>(app, x);
            if (x == 0) dec[v] = (uint8_t)d;
            for (int e = e0; e < e1; ++e) {
                float *p = msg + (size_t)sc.vslot[e] * Q + x;
                const float t = app - *p;
                *p = t - group_min<Q>(t);
            }
        }
        __syncthreads();
        fail = syndrome_fail<Q>(g, sc, dec, gmul);
        ++it;
    }

    // ---- accounting ----
    int be = 0, se = 0;
    for (int v = tid; v < N; v += nt) {
        const int cs = cvec ? cvec[v] : 0, dv = dec[v];
        be += __popc((unsigned)(dv ^ cs));
        se += dv != cs;
        if (a.d_out) a.d_out[(size_t)b * N + v] = (uint8_t)dv;
    }
    int sums[3] = {be, se, unc};
    block_sum_n<3>(sums, red);
    if (tid == 0) {
        atomicAdd(&a.counts[0], (unsigned long long)sums[0]);
        atomicAdd(&a.counts[1], (unsigned long long)(sums[1] > 0));
        atomicAdd(&a.counts[2], (unsigned long long)sums[2]);
        atomicAdd(&a.counts[3], 1ull);
        atomicAdd(&a.counts[4], (unsigned long long)it);
        atomicAdd(&a.counts[5], (unsigned long long)fail);
        atomicAdd(&a.counts[6], (unsigned long long)sums[1]);
        if (a.frame_res) a.frame_res[b] = make_int4(sums[0], sums[2], fail, it);
    }
    __syncthreads();
}

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// dynamic LDS: [msg E*Q f32 (ems_lds only)] [lam N*m f32] [dec N u8] [gf_mul Q*Q u8]
//              [cn M u32] [vn N u32] [ecol E u16] [vslot E u16] [ehinv E u8] [eh E u8]
__host__ __device__ inline size_t aux_bytes(const NbDevGraph &g)
{
    return align16((size_t)g.N * g.m * 4) + align16((size_t)g.N) + align16((size_t)g.q * g.q) +
           align16((size_t)g.M * 4) + align16((size_t)g.N * 4) + 2 * align16((size_t)g.E * 2) +
           2 * align16((size_t)g.E);
}

template <int Q, int MB, int DC, int SRC, bool GSTATE>
__global__ __launch_bounds__(1024) void k_ems(NbArgs a, NbDevGraph g, float *gscratch, size_t slot_floats)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int red[16 * 3];
    unsigned char *p = smem;
    float *msg;
    if (GSTATE) {
        msg = gscratch + slot_floats * blockIdx.x;
    } else {
        msg = reinterpret_cast<float *>(p);
        p += align16((size_t)g.E * Q * 4);
    }
    float *lam = reinterpret_cast<float *>(p);
    p += align16((size_t)g.N * MB * 4);
    uint8_t *dec = p;
    p += align16((size_t)g.N);
    uint8_t *gmul = p;
    p += align16((size_t)Q * Q);
    uint32_t *cn = reinterpret_cast<uint32_t *>(p);
    p += align16((size_t)g.M * 4);
    uint32_t *vn = reinterpret_cast<uint32_t *>(p);
    p += align16((size_t)g.N * 4);
    uint16_t *ecol = reinterpret_cast<uint16_t *>(p);
    p += align16((size_t)g.E * 2);
    uint16_t *vslot = reinterpret_cast<uint16_t *>(p);
    p += align16((size_t)g.E * 2);
    uint8_t *ehinv = p;
    p += align16((size_t)g.E);
    uint8_t *eh = p;
    for (int i = threadIdx.x; i < Q * Q; i += blockDim.x) gmul[i] = g.gf_mul[i];
    for (int j = threadIdx.x; j < g.M; j += blockDim.x)
        cn[j] = (uint32_t)g.row_ptr[j] | ((uint32_t)(g.row_ptr[j + 1] - g.row_ptr[j]) << 24);
    for (int v = threadIdx.x; v < g.N; v += blockDim.x)
        vn[v] = ((uint32_t)g.col_ptr[v] << 8) | (uint32_t)(g.col_ptr[v + 1] - g.col_ptr[v]);
    for (int e = threadIdx.x; e < g.E; e += blockDim.x) {
        ecol[e] = (uint16_t)g.row_col[e];
        vslot[e] = (uint16_t)g.col_slot[e];
        eh[e] = g.row_h[e];
        ehinv[e] = g.gf_inv[g.row_h[e]];
    }
    __syncthreads();
    const NbSched sc{cn, ehinv, eh, ecol, vn, vslot};
    for (int b = blockIdx.x; b < a.batch; b += gridDim.x)
        ems_codeword<Q, MB, DC, SRC>(a, g, b, msg, lam, dec, gmul, sc, red);
}

constexpr size_t kNbMaxLds = 160 * 1024;

NbChoice nb_choose(const NbDevGraph &g, int maxdc)
{
    NbChoice ch;
    ch.threads = 1024;
    ch.dc = maxdc <= 4 ? 4 : (maxdc <= 8 ? 8 : 16);
    const size_t aux = aux_bytes(g), msgb = align16((size_t)g.E * g.q * 4);
    if (aux > kNbMaxLds || g.E > 65535 || g.N > 65535) {
        ch.name = "";   // unsupported: the schedule does not fit LDS / 16-bit indices
        return ch;
    }
    if (aux + msgb <= kNbMaxLds) {
        ch.name = "ems_lds";
        ch.lds_bytes = (int)(aux + msgb);
    } else {
        ch.name = "ems_global";
        ch.lds_bytes = (int)aux;
        ch.slot_bytes = msgb;
    }
    return ch;
}

template <int DC, int SRC, bool GS>
static hipError_t launch_t(const NbDevGraph &g, const NbArgs &a, const NbChoice &ch, void *scratch, int grid,
                           hipStream_t s)
{
    auto fn = k_ems<kNbQ, 4, DC, SRC, GS>;
    hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, ch.lds_bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(ch.threads), ch.lds_bytes, s, a, g, (float *)scratch,
                       ch.slot_bytes / 4);
    return hipGetLastError();
}

template <int DC>
static hipError_t launch_dc(const NbDevGraph &g, const NbArgs &a, const NbChoice &ch, void *scratch, int grid,
                            hipStream_t s)
{
    const bool gs = ch.slot_bytes != 0;
    if (a.src == SRC_GIVEN)
        return gs ? launch_t<DC, SRC_GIVEN, true>(g, a, ch, scratch, grid, s)
                  : launch_t<DC, SRC_GIVEN, false>(g, a, ch, scratch, grid, s);
    return gs ? launch_t<DC, SRC_PHILOX, true>(g, a, ch, scratch, grid, s)
              : launch_t<DC, SRC_PHILOX, false>(g, a, ch, scratch, grid, s);
}

hipError_t nb_launch(const NbDevGraph &g, const NbArgs &a, const NbChoice &ch, void *scratch, int slots,
                     int num_cus, hipStream_t s)
{
    if (a.batch <= 0) return hipSuccess;
    if (g.q != kNbQ || g.m != 4) return hipErrorInvalidValue;
    int grid;
    if (ch.slot_bytes) {
        if (!scratch || slots <= 0) return hipErrorInvalidValue;
        grid = slots < a.batch ? slots : a.batch;
    } else {
        const int per_cu = (int)(kNbMaxLds / (size_t)ch.lds_bytes) >= 2 ? 2 : 1;
        grid = per_cu * num_cus;
        if (grid > a.batch) grid = a.batch;
    }
    switch (ch.dc) {
    case 4: return launch_dc<4>(g, a, ch, scratch, grid, s);
    case 8: return launch_dc<8>(g, a, ch, scratch, grid, s);
    default: return launch_dc<16>(g, a, ch, scratch, grid, s);
    }
}

}  // namespace ldpc
