// kernels.hip -- CDNA4 (gfx950) kernels of the flooding min-sum decoder.
//
// One workgroup (4 waves) decodes one codeword for all T iterations with its
// whole message state on chip:
//   app[N]   posterior sums  sum = yq + sum_k c2v  (symNodeUpdates :456-463)
//   yq[N]    channel samples after the front-end (:214-229)
//   rows[M]  compressed check state {m1, m2, meta}: the two smallest |v2c|
//            after normalisation/offset, argmin position and the sign of
//            every c2v on the row (checkNodeUpdates :410-450 +
//            applyNormalization :494-499 / applyOffset :503-515).
// Every c2v message is a pure function of its row state, so the flooding
// schedule needs no E-sized message arrays: the check phase rebuilds the old
// c2v from the row state it owns and forms v2c = app - c2v_old, which is
// bit-identical to the reference's v2c = sum - c2v (:469) because both are
// the same IEEE subtraction of the same operands. The bit phase re-sums
// yq + c2v in the reference's nlist order, so app (and the hard decision
// d = sum > 0 ? +1 : -1, :471-474) is bit-identical too, in fp64 to the
// reference and in fp32 to the fp32 restatement.
//
// The translation unit is compiled with -ffp-contract=off (see Makefile):
// no FMA may fuse the channel's 1 + sigma*n or the quantiser.
#include "kernels.h"
#include "device_common.h"
// The fp32 row kernel (k_decode_rows) adds its pairs as one v_pk_add_f32: two plain
// v_add_f32 measured 10.0 vs 8.8 ms per bench launch there (the ping-pong kernel is the
// other way round: minsum_common.h padd, template parameter PK).
#include "minsum_common.h"

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace ldpc {


// ---------------------------------------------------------------------
// One codeword, all T iterations. rows/app/yq may live in LDS or in a
// per-workgroup global scratch slot; red is LDS.
// ---------------------------------------------------------------------
template <typename F, int SRC>
__device__ __forceinline__ void decode_codeword(const DecodeArgs &a, const DevGraph &g, int b,
                                                RowState<F> *rows, F *app, F *yq, int *red)
{
    const int tid = threadIdx.x, nt = blockDim.x;
    const int N = g.N, M = g.M;
    const uint64_t cw = a.first_cw + (uint64_t)b;

    // ---- channel + front-end (:214-238) ----
    const int8_t *cvec = nullptr;
    if (SRC == SRC_GIVEN) {
        if (a.c) cvec = a.c + (size_t)b * N;
    } else if (a.cw_table) {
        cvec = a.cw_table + (size_t)(cw % (uint64_t)a.cw_rows) * N;
    }
    int unc = 0;
    if (SRC == SRC_GIVEN) {
        const F *y = reinterpret_cast<const F *>(a.y) + (size_t)b * N;
        for (int v = tid; v < N; v += nt) {
            const F q = front_end<F>(y[v], a);
            yq[v] = q;
            app[v] = q;
            const int cv = cvec ? cvec[v] : 1;
            unc += ((q > F(0) ? 1 : -1) * cv < 0);
        }
    } else {
        const F sigma = (F)a.sigma;
        const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
        for (int g4 = tid; g4 * 4 < N; g4 += nt) {
            uint32_t u[4];
            philox4x32_10((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, k0, k1, u);
            F n[4];
            box_muller(u[0], u[1], n[0], n[1]);
            box_muller(u[2], u[3], n[2], n[3]);
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int v = g4 * 4 + q4;
                if (v < N) {
                    const int cv = cvec ? cvec[v] : 1;
                    const F yv = (F)cv * (F(1) + sigma * n[q4]);
                    if (a.y_out) reinterpret_cast<F *>(a.y_out)[(size_t)b * N + v] = yv;
                    const F q = front_end<F>(yv, a);
                    yq[v] = q;
                    app[v] = q;
                    unc += ((q > F(0) ? 1 : -1) * cv < 0);
                }
            }
        }
    }
    for (int j = tid; j < M; j += nt) {
        RowState<F> z;
        z.m1 = F(0); z.m2 = F(0); z.meta = 0;
        rows[j] = z;   // c2v_old = +0: v2c = yq on the first pass (:364-370)
    }
    __syncthreads();

    const F alpha = (F)a.alpha, delta = (F)a.delta;
    for (int it = 0; it < a.T; ++it) {
        // ---- check nodes ----
        for (int j = tid; j < M; j += nt) {
            RowState<F> st = rows[j];
            const int deg = g.row_deg[j];
            const int32_t *rc = g.row_cols + (size_t)j * g.dcs;
            const int oidx = (int)(st.meta & 63u);
            const uint64_t osg = st.meta >> 6;
            F mn1 = dinf<F>(), mn2 = dinf<F>();
            int amin = 63;
            uint64_t sg = 0;
            for (int k = 0; k < deg; ++k) {
                F cold = (k == oidx) ? st.m2 : st.m1;
                if ((osg >> k) & 1u) cold = -cold;
                const F x = app[rc[k]] - cold;               // v2c (:469)
                sg |= (uint64_t)(!(x >= F(0))) << k;          // sgn(v2c) < 0
                const F ax = dabs(x);
                if (ax <= mn1) { mn2 = mn1; mn1 = ax; amin = k; }   // :428-433
                else if (ax < mn2) { mn2 = ax; }                    // :434-437
            }
            const uint64_t degmask = (deg >= 64) ? ~0ull : ((1ull << deg) - 1ull);
            uint64_t eff = (__popcll(sg) & 1) ? (sg ^ degmask) : sg;   // prod * sgn(v2c_k)
            F M1 = mn1, M2 = mn2;
            if (a.variant == V_NMS) {
                M1 = mn1 / alpha;                              // :498 (IEEE division)
                M2 = mn2 / alpha;
            } else if (a.variant == V_OMS) {
                const F t1 = mn1 - delta, t2 = mn2 - delta;    // :509
                const bool p1 = t1 > F(0), p2 = t2 > F(0);
                M1 = p1 ? t1 : F(0);
                M2 = p2 ? t2 : F(0);
                // sgn(c2v) of :511 maps -0.0 to +1; a zeroed message is +0 (:513)
                const uint64_t abit = (amin < 64) ? (1ull << amin) : 0ull;
                if (!p1 || mn1 == F(0)) eff &= abit;
                if (!p2 || mn2 == F(0)) eff &= ~abit;
            }
            st.m1 = M1;
            st.m2 = M2;
            st.meta = (uint64_t)amin | (eff << 6);
            rows[j] = st;
        }
        __syncthreads();
        // ---- bit nodes: sum = yq + c2v in nlist order (:456-463) ----
        for (int v = tid; v < N; v += nt) {
            F sum = yq[v];
            const int e1 = g.col_ptr[v + 1];
            for (int e = g.col_ptr[v]; e < e1; ++e) {
                const uint32_t ref = g.col_refs[e];
                const int k = (int)(ref & 63u);
                const RowState<F> st = rows[ref >> 6];
                const F mag = (k == (int)(st.meta & 63u)) ? st.m2 : st.m1;
                sum += ((st.meta >> (6 + k)) & 1u) ? -mag : mag;
            }
            app[v] = sum;
        }
        __syncthreads();
    }

    // ---- decisions, error weight (:270, :382-393), syndrome ----
    int w = 0;
    for (int v = tid; v < N; v += nt) {
        const int d = app[v] > F(0) ? 1 : -1;                 // :471-474
        const int cv = cvec ? cvec[v] : 1;
        w += (d != cv);
        if (a.d_out) a.d_out[(size_t)b * N + v] = (int8_t)d;
    }
    int synd = 0;
    for (int j = tid; j < M; j += nt) {
        const int deg = g.row_deg[j];
        const int32_t *rc = g.row_cols + (size_t)j * g.dcs;
        int par = 0;
        for (int k = 0; k < deg; ++k) par ^= (app[rc[k]] > F(0)) ? 0 : 1;
        synd |= par;
    }
    int sums[3] = {w, unc, synd};
    block_sum_n_t0<3>(sums, red);
    if (tid == 0) {   // the block totals exist in thread 0 only
        w = sums[0];
        unc = sums[1];
        synd = sums[2];
        atomicAdd(&a.counts[0], (unsigned long long)w);
        atomicAdd(&a.counts[1], (unsigned long long)(w > 0));
        atomicAdd(&a.counts[2], (unsigned long long)unc);
        atomicAdd(&a.counts[3], 1ull);
        atomicAdd(&a.counts[4], (unsigned long long)a.T);
        atomicAdd(&a.counts[5], (unsigned long long)(synd > 0));
        if (w > 0 && a.hist) atomicAdd(&a.hist[w - 1], 1ull);
        if (a.frame_res) a.frame_res[b] = make_int4(w, unc, synd > 0 ? 1 : 0, 0);
    }
    __syncthreads();
}

// State in LDS: one codeword per workgroup, grid = batch.
template <typename F, int SRC>
__global__ __launch_bounds__(256) void k_decode_lds(DecodeArgs a, DevGraph g)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    RowState<F> *rows = reinterpret_cast<RowState<F> *>(smem);
    F *app = reinterpret_cast<F *>(smem + sizeof(RowState<F>) * (size_t)g.M);
    F *yq = app + g.N;
    int *red = reinterpret_cast<int *>(yq + g.N);
    decode_codeword<F, SRC>(a, g, blockIdx.x, rows, app, yq, red);
}

// Re-decode list of the fast row kernel (rows_fast.hip): redo[0] codewords
// whose fast-path premise failed, batch indices in redo[1..]; each is decoded
// from scratch on this exact path (state in LDS), persistent grid. With an
// empty list every block exits at once.
template <typename F, int SRC>
__global__ __launch_bounds__(256) void k_redo(DecodeArgs a, DevGraph g, const unsigned *redo)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    RowState<F> *rows = reinterpret_cast<RowState<F> *>(smem);
    F *app = reinterpret_cast<F *>(smem + sizeof(RowState<F>) * (size_t)g.M);
    F *yq = app + g.N;
    int *red = reinterpret_cast<int *>(yq + g.N);
    const unsigned n = redo[0];
    for (unsigned i = blockIdx.x; i < n; i += gridDim.x) decode_codeword<F, SRC>(a, g, (int)redo[1 + i], rows, app, yq, red);
}

// State in a global scratch slot per workgroup (codes whose state exceeds
// LDS, e.g. DVB-S2 N=64800): persistent grid, codewords strided.
template <typename F, int SRC>
__global__ __launch_bounds__(256) void k_decode_global(DecodeArgs a, DevGraph g, unsigned char *scratch,
                                                       size_t slot_bytes)
{
    __shared__ int red[16];
    unsigned char *base = scratch + slot_bytes * blockIdx.x;
    RowState<F> *rows = reinterpret_cast<RowState<F> *>(base);
    F *app = reinterpret_cast<F *>(base + sizeof(RowState<F>) * (size_t)g.M);
    F *yq = app + g.N;
    for (int b = blockIdx.x; b < a.batch; b += gridDim.x)
        decode_codeword<F, SRC>(a, g, b, rows, app, yq, red);
}

// =====================================================================
// Row-parallel kernel (the throughput path).
//
// Block = `threads` threads (>= M, multiple of 64): thread t owns check row t
// for the whole persistent launch, with its row's bit indices and c2v slot
// positions held in registers (loaded once per launch from the RowSchedule
// built on the host), and CPT bit-node slots (columns sorted by degree).
// Each thread decodes C codewords at once (independent instruction streams).
// LDS per codeword: app[N] + c2v[e_pad], c2v in wave-slot-major order so the
// bit-node phase reads 64 consecutive words per wave instruction.
// Per iteration: check phase (gather app, rebuild the old c2v from the row
// state kept in registers, v2c = app - c2v_old, min/second-min/argmin/signs,
// normalise/offset, scatter the new c2v) | barrier | bit phase (sum yq + c2v
// in nlist order, write app) | barrier.
// =====================================================================

// x / alpha for the check-node normalisation (:498). fp32 with a verified
// alpha: reciprocal + one FMA correction (3 VALU instead of ~10); otherwise,
// and for non-finite minima, the IEEE division.
template <typename F>
__device__ __forceinline__ F nms_div(F x, F alpha, const DecodeArgs &a)
{
    return x / alpha;
}
template <>
__device__ __forceinline__ float nms_div<float>(float x, float alpha, const DecodeArgs &a)
{
    if (a.nms_fast && x < __builtin_huge_valf()) {
        const float q = x * a.alpha_rcp;
        return __builtin_fmaf(__builtin_fmaf(-q, alpha, x), a.alpha_rcp, q);
    }
    return x / alpha;
}

// =====================================================================
// Global-memory flooding kernel (codes whose state exceeds LDS, DVB-S2).
//
// One workgroup per codeword (persistent), the codeword's state in a global
// scratch slot, laid out by the FloodSchedule so every access is coalesced:
//   app[NP + 1], yq[NP]     bits in storage order (NP = ngroups*64; app[NP] = +inf)
//   c2v[e_pad + 64]         edge e of position p at gbase[p/64] + 64e + p%64
//   m12[M_pad], meta[M_pad] the packed check state, rows in chain order:
//                           (min1, min2) after /alpha or the offset, and
//                           argmin | output sign bits << 5
// Check phase: thread per row (slot-major schedule: lane i reads sp[k*M_pad+i]);
// the row's last messages are rebuilt from its packed state, the new ones are
// computed with the reference's comparisons (as cn_exact) and scattered into
// c2v. Bit phase: thread per position, sum = yq + c2v in nlist order.
// =====================================================================
template <typename F> struct F2T;
template <> struct F2T<float> { using T = float2; };
template <> struct F2T<double> { using T = double2; };

template <typename F, int SRC, int DC>
__global__ __launch_bounds__(512, (sizeof(F) == 4 && DC <= 8) ? 8 : 4) void k_decode_flood(DecodeArgs a, DevGraph g, FloodSched fs, unsigned char *scratch,
                                                      size_t slot_bytes)
{
    using F2 = typename F2T<F>::T;
    __shared__ int red[32 + 16 * 8];
    __shared__ unsigned long long acc[6];   // the block's totals (thread 0)
    const int tid = threadIdx.x, nt = blockDim.x;
    const int N = g.N, NP = fs.ngroups * 64, MP = fs.M_pad;
    unsigned char *base = scratch + slot_bytes * blockIdx.x;
    F *app = reinterpret_cast<F *>(base);                       // [NP + 1]
    F *yq = app + (NP + 1);                                     // [NP]
    F *c2v = yq + NP;                                           // [e_pad + 64]
    F2 *m12 = reinterpret_cast<F2 *>(c2v + (fs.e_pad + 64 + 1) / 2 * 2);   // 16-B aligned for double2
    uint32_t *meta = reinterpret_cast<uint32_t *>(m12 + MP);
    const F alpha = (F)a.alpha, delta = (F)a.delta;

    if (tid == 0) {
        app[NP] = dinf<F>();   // sentinel position of padding slots
#pragma unroll
        for (int q = 0; q < 6; ++q) acc[q] = 0;
    }

    for (int b = blockIdx.x; b < a.batch; b += gridDim.x) {
        const uint64_t cw = a.first_cw + (uint64_t)b;
        const int8_t *cvec = nullptr;
        if (SRC == SRC_GIVEN) {
            if (a.c) cvec = a.c + (size_t)b * N;
        } else if (a.cw_table) {
            cvec = a.cw_table + (size_t)(cw % (uint64_t)a.cw_rows) * N;
        }
        // ---- channel + front-end (:214-238) into storage order ----
        int unc = 0;
        if (SRC == SRC_GIVEN) {
            const F *y = reinterpret_cast<const F *>(a.y) + (size_t)b * N;
            for (int v = tid; v < N; v += nt) {
                const F q = front_end<F>(y[v], a);
                const int p = fs.pos_of_bit[v];
                yq[p] = q;
                app[p] = q;
                const int cv = cvec ? cvec[v] : 1;
                unc += ((q > F(0) ? 1 : -1) * cv < 0);
            }
        } else {
            const F sigma = (F)a.sigma;
            const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
            for (int g4 = tid; g4 * 4 < N; g4 += nt) {
                uint32_t u[4];
                philox4x32_10((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, k0, k1, u);
                F n[4];
                box_muller(u[0], u[1], n[0], n[1]);
                box_muller(u[2], u[3], n[2], n[3]);
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    const int v = g4 * 4 + q4;
                    if (v < N) {
                        const int cv = cvec ? cvec[v] : 1;
                        const F yv = (F)cv * (F(1) + sigma * n[q4]);
                        if (a.y_out) reinterpret_cast<F *>(a.y_out)[(size_t)b * N + v] = yv;
                        const F q = front_end<F>(yv, a);
                        const int p = fs.pos_of_bit[v];
                        yq[p] = q;
                        app[p] = q;
                        unc += ((q > F(0) ? 1 : -1) * cv < 0);
                    }
                }
            }
        }
        for (int i = tid; i < MP; i += nt) {   // c2v_old = +0: v2c = yq on the first pass (:364-370)
            F2 z;
            z.x = F(0);
            z.y = F(0);
            m12[i] = z;
            meta[i] = 0;
        }
        __syncthreads();

        for (int it = 0; it < a.T; ++it) {
            // ---- check nodes (:410-450, :494-515) ----
            for (int i = tid; i < MP; i += nt) {
                const int deg = fs.rdeg[i];
                if (deg == 0) continue;
                int sp[DC];
#pragma unroll
                for (int k = 0; k < DC; ++k) sp[k] = k < deg ? fs.sp[(size_t)k * MP + i] : NP;
                F xa[DC];
#pragma unroll
                for (int k = 0; k < DC; ++k) xa[k] = app[sp[k]];
                const F2 old = m12[i];
                const uint32_t om = meta[i];
                const int oidx = (int)(om & 31u);
                F mn1 = dinf<F>(), mn2 = dinf<F>();
                int amin = 31;
                uint32_t sg = 0;
                F ax[DC];
#pragma unroll
                for (int k = 0; k < DC; ++k) {
                    if (k < deg) {
                        F cold = (k == oidx) ? old.y : old.x;
                        if ((om >> (5 + k)) & 1u) cold = -cold;
                        const F x = xa[k] - cold;                     // v2c (:469)
                        sg |= (uint32_t)(!(x >= F(0))) << k;          // sgn(v2c) < 0 (:518-523)
                        ax[k] = dabs(x);
                        if (ax[k] <= mn1) { mn2 = mn1; mn1 = ax[k]; amin = k; }   // :428-433
                        else if (ax[k] < mn2) { mn2 = ax[k]; }                    // :434-437
                    }
                }
                const uint32_t degmask = (1u << deg) - 1u;
                uint32_t eff = (__popc(sg) & 1) ? (sg ^ degmask) : sg;   // prod * sgn(v2c_k)
                F M1 = mn1, M2 = mn2;
                if (a.variant == V_NMS) {
                    M1 = nms_div<F>(mn1, alpha, a);               // :498
                    M2 = nms_div<F>(mn2, alpha, a);
                } else if (a.variant == V_OMS) {
                    const F t1 = mn1 - delta, t2 = mn2 - delta;   // :509
                    const bool p1 = t1 > F(0), p2 = t2 > F(0);
                    M1 = p1 ? t1 : F(0);
                    M2 = p2 ? t2 : F(0);
                    // sgn(c2v) of :511 maps -0.0 to +1; a zeroed message is +0 (:513)
                    const uint32_t abit = (amin < 31) ? (1u << amin) : 0u;
                    if (!p1 || mn1 == F(0)) eff &= abit;
                    if (!p2 || mn2 == F(0)) eff &= ~abit;
                }
                F2 nw;
                nw.x = M1;
                nw.y = M2;
                m12[i] = nw;
                meta[i] = (uint32_t)amin | (eff << 5);
#pragma unroll
                for (int k = 0; k < DC; ++k) {
                    if (k < deg) {
                        const F mag = (k == amin) ? M2 : M1;
                        c2v[fs.sq[(size_t)k * MP + i]] = ((eff >> k) & 1u) ? -mag : mag;
                    }
                }
            }
            __syncthreads();
            // ---- bit nodes: sum = yq + c2v in nlist order (:452-476) ----
            for (int p = tid; p < NP; p += nt) {
                const int d = fs.pdeg[p];
                if (d == 0) continue;
                const F *cp = c2v + fs.gbase[p >> 6] + (p & 63);
                F sum = yq[p];
                for (int e = 0; e < d; ++e) sum += cp[64 * e];
                app[p] = sum;
            }
            __syncthreads();
        }

        // ---- decisions, error weight (:270, :382-393), syndrome ----
        int w = 0, synd = 0;
        for (int v = tid; v < N; v += nt) {
            const int d = app[fs.pos_of_bit[v]] > F(0) ? 1 : -1;   // :471-474
            const int cv = cvec ? cvec[v] : 1;
            w += (d != cv);
            if (a.d_out) a.d_out[(size_t)b * N + v] = (int8_t)d;
        }
        for (int i = tid; i < MP; i += nt) {
            const int deg = fs.rdeg[i];
            int par = 0;
            for (int k = 0; k < deg; ++k) par ^= (app[fs.sp[(size_t)k * MP + i]] > F(0)) ? 0 : 1;
            synd |= par;
        }
        int sums[3] = {w, unc, synd};
        block_sum_n_t0<3>(sums, red + 32);
        if (tid == 0) {
            const int sf = sums[2] > 0;
            acc[0] += (unsigned long long)sums[0];
            acc[1] += (unsigned long long)(sums[0] > 0);
            acc[2] += (unsigned long long)sums[1];
            acc[3] += 1ull;
            acc[5] += (unsigned long long)sf;
            if (sums[0] > 0 && a.hist) atomicAdd(&a.hist[sums[0] - 1], 1ull);
            if (a.frame_res) a.frame_res[b] = make_int4(sums[0], sums[1], sf, 0);
        }
        __syncthreads();
    }
    if (tid == 0 && acc[3] > 0) {
        acc[4] = acc[3] * (unsigned long long)a.T;
#pragma unroll
        for (int q = 0; q < 6; ++q) atomicAdd(&a.counts[q], acc[q]);
    }
}

static size_t flood_slot_bytes(const DevGraph &g, const FloodSched &fs, bool f64)
{
    const size_t fsz = f64 ? 8 : 4, NP = (size_t)fs.ngroups * 64;
    const size_t nf = (NP + 1) + NP + ((size_t)fs.e_pad + 64 + 1) / 2 * 2;
    return (nf * fsz + (size_t)fs.M_pad * (2 * fsz + 4) + 255) & ~(size_t)255;
}

// =====================================================================
// Phase-per-launch flooding (codes beyond LDS; the default since round 2,
// LDPC_FLOOD_MODE=persistent selects k_decode_flood).
//
// The same per-codeword state slots, arithmetic and storage order as
// k_decode_flood, but the resident set is sized to stay inside the 256 MiB
// Infinity Cache (K codewords, K * slot_bytes ~ 150 MB) and every phase is
// its own launch over all K codewords: init (channel), T x {check, bit},
// finish (decisions, accounting). A launch boundary is the flooding
// barrier, so a codeword is no longer confined to one workgroup: one thread
// per row (check) or per bit position (bit) of every resident codeword, the
// whole GPU on each phase, with no spin-waits. Grid (blocks of the phase,
// K); slot r of the launch holds codeword b0 + r.
// =====================================================================
struct FloodSlot {
    template <typename F> struct View {
        F *app, *yq, *c2v;
        typename F2T<F>::T *m12;
        uint32_t *meta;
    };
    template <typename F>
    static __device__ __forceinline__ View<F> at(unsigned char *scratch, size_t slot_bytes, int r, const FloodSched &fs)
    {
        using F2 = typename F2T<F>::T;
        View<F> v;
        const int NP = fs.ngroups * 64;
        unsigned char *base = scratch + slot_bytes * (size_t)r;
        v.app = reinterpret_cast<F *>(base);
        v.yq = v.app + (NP + 1);
        v.c2v = v.yq + NP;
        v.m12 = reinterpret_cast<F2 *>(v.c2v + (fs.e_pad + 64 + 1) / 2 * 2);
        v.meta = reinterpret_cast<uint32_t *>(v.m12 + fs.M_pad);
        return v;
    }
};

template <typename F, int SRC>
__global__ __launch_bounds__(256) void k_flood_init(DecodeArgs a, DevGraph g, FloodSched fs, unsigned char *scratch,
                                                    size_t slot_bytes, int b0, int *unc_out)
{
    const int r = blockIdx.y, b = b0 + r;
    if (b >= a.batch) return;
    const auto S = FloodSlot::at<F>(scratch, slot_bytes, r, fs);
    const int N = g.N, NP = fs.ngroups * 64, MP = fs.M_pad;
    const uint64_t cw = a.first_cw + (uint64_t)b;
    const int8_t *cvec = nullptr;
    if (SRC == SRC_GIVEN) {
        if (a.c) cvec = a.c + (size_t)b * N;
    } else if (a.cw_table) {
        cvec = a.cw_table + (size_t)(cw % (uint64_t)a.cw_rows) * N;
    }
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    int unc = 0;
    if (t * 4 < N) {   // ---- channel + front-end (:214-238) into storage order ----
        F yv[4];
        if (SRC == SRC_GIVEN) {
            const F *y = reinterpret_cast<const F *>(a.y) + (size_t)b * N;
#pragma unroll
            for (int q = 0; q < 4; ++q) yv[q] = (t * 4 + q < N) ? y[t * 4 + q] : F(1);
        } else {
            uint32_t u[4];
            philox4x32_10((uint32_t)t, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, (uint32_t)a.seed,
                          (uint32_t)(a.seed >> 32), u);
            F n[4];
            box_muller(u[0], u[1], n[0], n[1]);
            box_muller(u[2], u[3], n[2], n[3]);
            const F sigma = (F)a.sigma;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int v = t * 4 + q;
                yv[q] = (F)(v < N && cvec ? cvec[v] : 1) * (F(1) + sigma * n[q]);
                if (v < N && a.y_out) reinterpret_cast<F *>(a.y_out)[(size_t)b * N + v] = yv[q];
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int v = t * 4 + q;
            if (v < N) {
                const F q2 = front_end<F>(yv[q], a);
                const int p = LDPC_CHK(fs.pos_of_bit[v], NP, CHK_FLOOD_APP);
                S.yq[p] = q2;
                S.app[p] = q2;
                const int cv = cvec ? cvec[v] : 1;
                unc += ((q2 > F(0) ? 1 : -1) * cv < 0);
            }
        }
    }
    for (int i = t; i < MP; i += gridDim.x * blockDim.x) {   // c2v_old = +0 (:364-370)
        typename F2T<F>::T z;
        z.x = F(0);
        z.y = F(0);
        S.m12[i] = z;
        S.meta[i] = 0;
    }
    if (t == 0) S.app[NP] = dinf<F>();   // sentinel position of padding slots
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) unc += __shfl_xor(unc, o, 64);
    if ((threadIdx.x & 63) == 0 && unc) atomicAdd(&unc_out[r], unc);
}

// Progress-ordered wave priorities in k_decode_rows' check phase: s_setprio 3 at the
// phase start, 2 after the first row, 0 for the bit phase (fp32 OMS on N=1944, T=50:
// 13.2 -> 11.6 ms; PEG 1008 fp32 MS T=10 +3 %). 0: none.
// A/B switches of the row kernel's per-step work: block sums with one barrier into LDS
// totals (block_sum_lds, 1) vs block_sum_n_t0 (0); Philox products by v_mad_u64_u32.
// Measured (fp32, 65 536 codewords): block_sum_lds makes PEG 1008 MS T=10 39.6 -> 42.3
// Gbit/s but N=1944 OMS T=50 11.0 -> 10.1 (the same instance; a code-layout effect, not
// the reduction's own cost), so the default stays 0; v_mad_u64_u32 is neutral and kept.
#ifndef LDPC_ROWS_ACCT
#define LDPC_ROWS_ACCT 0
#endif
#ifndef LDPC_ROWS_MAD64
#define LDPC_ROWS_MAD64 1
#endif
#ifndef LDPC_ROWS_PRIOBAL
#define LDPC_ROWS_PRIOBAL 1
#endif
#ifndef LDPC_FLOOD_CPW
#define LDPC_FLOOD_CPW 8
#endif
#ifndef LDPC_FLOOD_XCD
#define LDPC_FLOOD_XCD 1
#endif
// Codewords per thread of the phase kernels: the row's (or bit position's)
// schedule is loaded once and used for CPW resident codewords (slots
// blockIdx.y + j * gridDim.y).
//
// The check node of k_decode_flood (:410-450, :494-515) on one resident slot:
// xa = the gathered app values, (old, om) = the row's packed state.
template <typename F, int DC, bool C2V>
__device__ __forceinline__ void flood_cn(const DecodeArgs &a, const FloodSlot::View<F> &S, int i, int deg,
                                         const int (&sq)[DC], const F (&xa)[DC], typename F2T<F>::T old, uint32_t om)
{
    using F2 = typename F2T<F>::T;
    const F alpha = (F)a.alpha, delta = (F)a.delta;
    const int oidx = (int)(om & 31u);
    F mn1 = dinf<F>(), mn2 = dinf<F>();
    int amin = 31;
    uint32_t sg = 0;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k < deg) {
            F cold = (k == oidx) ? old.y : old.x;
            if ((om >> (5 + k)) & 1u) cold = -cold;
            const F x = xa[k] - cold;                     // v2c (:469)
            sg |= (uint32_t)(!(x >= F(0))) << k;          // sgn(v2c) < 0 (:518-523)
            const F ax = dabs(x);
            if (ax <= mn1) { mn2 = mn1; mn1 = ax; amin = k; }   // :428-433
            else if (ax < mn2) { mn2 = ax; }                    // :434-437
        }
    }
    const uint32_t degmask = (1u << deg) - 1u;
    uint32_t eff = (__popc(sg) & 1) ? (sg ^ degmask) : sg;   // prod * sgn(v2c_k)
    F M1 = mn1, M2 = mn2;
    if (a.variant == V_NMS) {
        M1 = nms_div<F>(mn1, alpha, a);               // :498
        M2 = nms_div<F>(mn2, alpha, a);
    } else if (a.variant == V_OMS) {
        const F t1 = mn1 - delta, t2 = mn2 - delta;   // :509
        const bool p1 = t1 > F(0), p2 = t2 > F(0);
        M1 = p1 ? t1 : F(0);
        M2 = p2 ? t2 : F(0);
        const uint32_t abit = (amin < 31) ? (1u << amin) : 0u;   // sgn(-0.0) = +1 (:511-513)
        if (!p1 || mn1 == F(0)) eff &= abit;
        if (!p2 || mn2 == F(0)) eff &= ~abit;
    }
    F2 nw;
    nw.x = M1;
    nw.y = M2;
    S.m12[i] = nw;
    S.meta[i] = (uint32_t)amin | (eff << 5);
    if constexpr (C2V) {
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (k < deg) {
                const F mag = (k == amin) ? M2 : M1;
                S.c2v[sq[k]] = ((eff >> k) & 1u) ? -mag : mag;
            }
        }
    }
}

// The c2v message of position k of a row with packed state (m, meta): exactly
// the value flood_cn stores (magnitude M2 at the argmin, M1 elsewhere, signed
// by the row's sign bit k).
template <typename F>
__device__ __forceinline__ F flood_msg(typename F2T<F>::T m, uint32_t meta, uint32_t k)
{
    const F mag = (k == (meta & 31u)) ? m.y : m.x;
    return ((meta >> (5 + k)) & 1u) ? -mag : mag;
}

// SPS resident slots per step: their gathers are issued together (one memory
// round trip for SPS slots), the check nodes then run slot by slot.
template <typename F, int DC, int SPS, bool C2V>
__global__ __launch_bounds__(256) void k_flood_check(DecodeArgs a, FloodSched fs, unsigned char *scratch,
                                                     size_t slot_bytes, int nres)
{
    using F2 = typename F2T<F>::T;
    const int MP = fs.M_pad, NP = fs.ngroups * 64;
#if LDPC_FLOOD_XCD
    // XCD-aware: blocks b and b + 8 share an XCD (round-robin placement, speed
    // only); XCD x decodes the slots x, x + 8, ... one after the other, all
    // rows of a slot at once, so the ~3.5 gathers of each app value hit its L2.
    const int i = (blockIdx.x >> 3) * blockDim.x + threadIdx.x, r0 = blockIdx.x & 7, rs = 8;
#else
    const int i = blockIdx.x * blockDim.x + threadIdx.x, r0 = blockIdx.y, rs = gridDim.y;
#endif
    if (i >= MP) return;
    const int deg = fs.rdeg[i];
    if (deg == 0) return;
    int sp[DC], sq[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        sp[k] = k < deg ? LDPC_CHK(fs.sp[(size_t)k * MP + i], NP + 1, CHK_FLOOD_APP) : NP;
        sq[k] = k < deg ? LDPC_CHK(fs.sq[(size_t)k * MP + i], fs.e_pad + 64, CHK_FLOOD_C2V) : 0;
    }
    for (int r = r0; r < nres; r += SPS * rs) {
        F xa[SPS][DC];
        F2 old[SPS];
        uint32_t om[SPS];
#pragma unroll
        for (int j = 0; j < SPS; ++j) {
            const int rr = r + j * rs < nres ? r + j * rs : r;   // past the end: a harmless re-read of slot r
            const auto S = FloodSlot::at<F>(scratch, slot_bytes, rr, fs);
#pragma unroll
            for (int k = 0; k < DC; ++k) xa[j][k] = S.app[sp[k]];
            old[j] = S.m12[i];
            om[j] = S.meta[i];
        }
#pragma unroll
        for (int j = 0; j < SPS; ++j)
            if (r + j * rs < nres)
                flood_cn<F, DC, C2V>(a, FloodSlot::at<F>(scratch, slot_bytes, r + j * rs, fs), i, deg, sq, xa[j],
                                     old[j], om[j]);
    }
}

// DV = a bound on the column degree: the d loads of a bit are issued together
// (one memory round trip per slot instead of d dependent ones; the adds stay in
// nlist order), and SPS slots are in flight per step. DV = 0: any degree, one
// load at a time.
template <typename F, int DV, int SPS>
__global__ __launch_bounds__(256) void k_flood_bit(FloodSched fs, unsigned char *scratch, size_t slot_bytes, int nres)
{
    const int NP = fs.ngroups * 64;
#if LDPC_FLOOD_XCD
    const int p = (blockIdx.x >> 3) * blockDim.x + threadIdx.x, r0 = blockIdx.x & 7, rs = 8;
#else
    const int p = blockIdx.x * blockDim.x + threadIdx.x, r0 = blockIdx.y, rs = gridDim.y;
#endif
    if (p >= NP) return;
    const int d = fs.pdeg[p];
    if (d == 0) return;
    const int off = fs.gbase[p >> 6] + (p & 63);
    [[maybe_unused]] const int ea = fs.e_pad + 64;
    if constexpr (DV == 0) {
        for (int r = r0; r < nres; r += rs) {
            const auto S = FloodSlot::at<F>(scratch, slot_bytes, r, fs);
            const F *cp = S.c2v + off;
            F sum = S.yq[p];
            for (int e = 0; e < d; ++e) sum += cp[LDPC_CHK(64 * e, ea - off, CHK_FLOOD_C2V)];   // nlist order (:452-476)
            S.app[p] = sum;
        }
    } else {
        for (int r = r0; r < nres; r += SPS * rs) {
            F v[SPS][DV], y[SPS];
#pragma unroll
            for (int j = 0; j < SPS; ++j) {
                const auto S = FloodSlot::at<F>(scratch, slot_bytes, r + j * rs < nres ? r + j * rs : r, fs);
                y[j] = S.yq[p];
#pragma unroll
                for (int e = 0; e < DV; ++e) v[j][e] = e < d ? S.c2v[LDPC_CHK(off + 64 * e, ea, CHK_FLOOD_C2V)] : F(0);
            }
#pragma unroll
            for (int j = 0; j < SPS; ++j) {
                F sum = y[j];
#pragma unroll
                for (int e = 0; e < DV; ++e)
                    if (e < d) sum += v[j][e];   // nlist order (:452-476)
                if (r + j * rs < nres) FloodSlot::at<F>(scratch, slot_bytes, r + j * rs, fs).app[p] = sum;
            }
        }
    }
}

// Bit phase without the c2v array (LDPC_FLOOD_MSG=packed, the default): each
// message is rebuilt from its row's packed state (m12, meta), gathered through
// the element -> (row, position) table eref. The check phase then writes only
// the 12 (fp32) / 20 (fp64) bytes of state per row instead of dc messages, and
// the bit phase reads each row's state once per L2 instead of a message per
// edge -- the same sums, in nlist order, of the same values.
template <typename F, int DV, int SPS>
__global__ __launch_bounds__(256) void k_flood_bit_packed(FloodSched fs, unsigned char *scratch, size_t slot_bytes,
                                                          int nres)
{
    using F2 = typename F2T<F>::T;
    const int NP = fs.ngroups * 64;
#if LDPC_FLOOD_XCD
    const int p = (blockIdx.x >> 3) * blockDim.x + threadIdx.x, r0 = blockIdx.x & 7, rs = 8;
#else
    const int p = blockIdx.x * blockDim.x + threadIdx.x, r0 = blockIdx.y, rs = gridDim.y;
#endif
    if (p >= NP) return;
    const int d = fs.pdeg[p];
    if (d == 0) return;
    const int off = fs.gbase[p >> 6] + (p & 63);
    uint32_t ref[DV];
#pragma unroll
    for (int e = 0; e < DV; ++e) {
        ref[e] = e < d ? fs.eref[LDPC_CHK(off + 64 * e, fs.e_pad + 64, CHK_FLOOD_C2V)] : 0u;
#ifdef LDPC_CHECK
        ref[e] = (LDPC_CHK(ref[e] >> 5, (uint32_t)fs.M_pad, CHK_FLOOD_ROW) << 5) | (ref[e] & 31u);
#endif
    }
    for (int r = r0; r < nres; r += SPS * rs) {
        F2 m[SPS][DV];
        uint32_t me[SPS][DV];
        F y[SPS];
#pragma unroll
        for (int j = 0; j < SPS; ++j) {
            const auto S = FloodSlot::at<F>(scratch, slot_bytes, r + j * rs < nres ? r + j * rs : r, fs);
            y[j] = S.yq[p];
#pragma unroll
            for (int e = 0; e < DV; ++e)
                if (e < d) {
                    m[j][e] = S.m12[ref[e] >> 5];
                    me[j][e] = S.meta[ref[e] >> 5];
                }
        }
#pragma unroll
        for (int j = 0; j < SPS; ++j) {
            F sum = y[j];
#pragma unroll
            for (int e = 0; e < DV; ++e)
                if (e < d) sum += flood_msg<F>(m[j][e], me[j][e], ref[e] & 31u);   // nlist order (:452-476)
            if (r + j * rs < nres) FloodSlot::at<F>(scratch, slot_bytes, r + j * rs, fs).app[p] = sum;
        }
    }
}

// Decisions, error weight (:270, :382-393) and syndrome of every resident
// codeword: one thread per bit / row, per-slot sums by atomics.
template <typename F>
__global__ __launch_bounds__(256) void k_flood_finish(DecodeArgs a, DevGraph g, FloodSched fs, unsigned char *scratch,
                                                      size_t slot_bytes, int b0, int nres, int *wsum, int *ssum)
{
    const int N = g.N, MP = fs.M_pad;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    for (int r = blockIdx.y; r < nres; r += gridDim.y) {
        const int b = b0 + r;
        const auto S = FloodSlot::at<F>(scratch, slot_bytes, r, fs);
        int w = 0, par = 0;
        if (t < N) {
            const uint64_t cw = a.first_cw + (uint64_t)b;
            const int8_t *cvec = nullptr;
            if (a.src == SRC_GIVEN) {
                if (a.c) cvec = a.c + (size_t)b * N;
            } else if (a.cw_table) {
                cvec = a.cw_table + (size_t)(cw % (uint64_t)a.cw_rows) * N;
            }
            const int d = S.app[LDPC_CHK(fs.pos_of_bit[t], fs.ngroups * 64 + 1, CHK_FLOOD_APP)] > F(0) ? 1 : -1;   // :471-474
            w = d != (cvec ? cvec[t] : 1);
            if (a.d_out) a.d_out[(size_t)b * N + t] = (int8_t)d;
        }
        if (t < MP) {
            const int deg = fs.rdeg[t];
            for (int k = 0; k < deg; ++k)
                par ^= (S.app[LDPC_CHK(fs.sp[(size_t)k * MP + t], fs.ngroups * 64 + 1, CHK_FLOOD_APP)] > F(0)) ? 0 : 1;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            w += __shfl_xor(w, o, 64);
            par += __shfl_xor(par, o, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            if (w) atomicAdd(&wsum[r], w);
            if (par) atomicAdd(&ssum[r], par);
        }
    }
}

// The frame accounting of the resident codewords (one thread per slot).
__global__ __launch_bounds__(256) void k_flood_account(DecodeArgs a, int b0, int nres, const int *unc,
                                                       const int *wsum, const int *ssum)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nres) return;
    const int b = b0 + r, w = wsum[r], uc = unc[r], sf = ssum[r] > 0;
    atomicAdd(&a.counts[0], (unsigned long long)w);
    atomicAdd(&a.counts[1], (unsigned long long)(w > 0));
    atomicAdd(&a.counts[2], (unsigned long long)uc);
    atomicAdd(&a.counts[3], 1ull);
    atomicAdd(&a.counts[4], (unsigned long long)a.T);
    atomicAdd(&a.counts[5], (unsigned long long)sf);
    if (w > 0 && a.hist) atomicAdd(&a.hist[w - 1], 1ull);
    if (a.frame_res) a.frame_res[b] = make_int4(w, uc, sf, 0);
}

// Messages between the phases: the packed row state (default) or the c2v
// array (option LDPC_OPT_FLOOD_MSG = 1). The packed bit phase is built for column degrees
// up to 32 (k_flood_bit_packed<F, 8|16|32>); a code with a heavier column takes
// the c2v array, whose bit phase has an any-degree instance (DV = 0).
constexpr int kFloodPackedMaxDv = 32;
static bool flood_packed(const FloodSched &fs)
{
    if (fs.dv > kFloodPackedMaxDv) return false;
    return opt(LDPC_OPT_FLOOD_MSG) != 1;
}

// Resident slots per step of the check (LDPC_OPT_FLOOD_SPS_CHECK) and bit
// (LDPC_OPT_FLOOD_SPS_BIT) phase kernels.
static int flood_sps(bool check, const FloodSched &fs)
{
    if (const int v = opt(check ? LDPC_OPT_FLOOD_SPS_CHECK : LDPC_OPT_FLOOD_SPS_BIT)) return v;
    return check || flood_packed(fs) ? 1 : 2;   // packed bit phase: 1 (2 204 vs 2 124 Mbit/s fp32)
}

// Resident codewords of the phase-per-launch flooding: the state the phases
// touch fits the Infinity Cache with room to spare. `touched` = bytes per slot
// the phases read and write (the packed-message phases leave the c2v array of
// the slot alone). Measured on DVB-S2 R1/2 with packed messages (4096
// codewords, T=50): fp32 K = 96/112/128/144 -> 2277/2307/2331/2310 Mbit/s,
// fp64 K = 64/80/96/128 -> 1520/1508/1487/1401 -- best near 110 MB touched.
// LDPC_OPT_FLOOD_RESIDENT overrides.
constexpr size_t kFloodPhaseExtra = 65536;   // per-slot counters after the slots (3 ints per slot)
static int flood_phase_resident(size_t slot_bytes, size_t touched, size_t gscratch_bytes)
{
    long k = (long)((112ull << 20) / touched);
    if (const int v = opt(LDPC_OPT_FLOOD_RESIDENT)) k = v;
    if (k > 4096) k = 4096;
    const long cap = (long)((gscratch_bytes - kFloodPhaseExtra) / slot_bytes);
    if (k > cap) k = cap;
    return k < 1 ? 1 : (int)k;
}

// The phase launches of resident slots [lo, lo + n) of a chunk whose first codeword
// is b0: init, T x (check, bit), finish, accounting -- issued on stream s.
template <typename F, int SRC>
struct FloodHalf {
    const DevGraph *g;
    const FloodSched *fs;
    const DecodeArgs *a;
    unsigned char *scratch;
    size_t sb;
    int *unc, *wsum, *ssum;   // per-slot counters (index = slot)
    hipStream_t s;
    int lo, n;
    hipError_t begin(int b0) const
    {
        if (n <= 0) return hipSuccess;
        hipError_t e = hipMemsetAsync(unc + lo, 0, sizeof(int) * (size_t)n, s);
        if (e == hipSuccess) e = hipMemsetAsync(wsum + lo, 0, sizeof(int) * (size_t)n, s);
        if (e == hipSuccess) e = hipMemsetAsync(ssum + lo, 0, sizeof(int) * (size_t)n, s);
        if (e != hipSuccess) return e;
        const int ib = ((g->N + 3) / 4 + 255) / 256;
        hipLaunchKernelGGL((k_flood_init<F, SRC>), dim3(ib > 1 ? ib : 1, n), dim3(256), 0, s, *a, *g, *fs,
                           scratch + sb * (size_t)lo, sb, b0 + lo, unc + lo);
        return hipSuccess;
    }
    void check() const
    {
        if (n <= 0) return;
        const int NPc = fs->M_pad;
#if LDPC_FLOOD_XCD
        const dim3 cg(8 * ((NPc + 255) / 256));
#else
        const dim3 cg((NPc + 255) / 256, (n + LDPC_FLOOD_CPW - 1) / LDPC_FLOOD_CPW);
#endif
        unsigned char *sc = scratch + sb * (size_t)lo;
        const int sps = flood_sps(true, *fs);
        const bool packed = flood_packed(*fs);
#define CHK(DC, SPS)                                                                                     \
    do {                                                                                                 \
        if (packed) hipLaunchKernelGGL((k_flood_check<F, DC, SPS, false>), cg, dim3(256), 0, s, *a, *fs, sc, sb, n); \
        else hipLaunchKernelGGL((k_flood_check<F, DC, SPS, true>), cg, dim3(256), 0, s, *a, *fs, sc, sb, n);         \
    } while (0)
        if (fs->dc <= 8) {
            if (sps >= 4) CHK(8, 4);
            else if (sps == 2) CHK(8, 2);
            else CHK(8, 1);
        } else if (fs->dc <= 16) {
            if (sps >= 2) CHK(16, 2);
            else CHK(16, 1);
        } else {
            CHK(32, 1);
        }
#undef CHK
    }
    void bit() const
    {
        if (n <= 0) return;
        const int NP = fs->ngroups * 64;
#if LDPC_FLOOD_XCD
        const dim3 bg(8 * ((NP + 255) / 256));
#else
        const dim3 bg((NP + 255) / 256, (n + LDPC_FLOOD_CPW - 1) / LDPC_FLOOD_CPW);
#endif
        unsigned char *sc = scratch + sb * (size_t)lo;
        const int sps = flood_sps(false, *fs);
        if (flood_packed(*fs)) {
            if (fs->dv <= 8) {
                if (sps >= 2) hipLaunchKernelGGL((k_flood_bit_packed<F, 8, 2>), bg, dim3(256), 0, s, *fs, sc, sb, n);
                else hipLaunchKernelGGL((k_flood_bit_packed<F, 8, 1>), bg, dim3(256), 0, s, *fs, sc, sb, n);
            } else if (fs->dv <= 16) {
                hipLaunchKernelGGL((k_flood_bit_packed<F, 16, 1>), bg, dim3(256), 0, s, *fs, sc, sb, n);
            } else {
                hipLaunchKernelGGL((k_flood_bit_packed<F, 32, 1>), bg, dim3(256), 0, s, *fs, sc, sb, n);
            }
            return;
        }
        if (fs->dv <= 8) {
            if (sps >= 4) hipLaunchKernelGGL((k_flood_bit<F, 8, 4>), bg, dim3(256), 0, s, *fs, sc, sb, n);
            else hipLaunchKernelGGL((k_flood_bit<F, 8, 2>), bg, dim3(256), 0, s, *fs, sc, sb, n);
        } else if (fs->dv <= 16) {
            if (sps >= 4) hipLaunchKernelGGL((k_flood_bit<F, 16, 4>), bg, dim3(256), 0, s, *fs, sc, sb, n);
            else hipLaunchKernelGGL((k_flood_bit<F, 16, 2>), bg, dim3(256), 0, s, *fs, sc, sb, n);
        } else {
            hipLaunchKernelGGL((k_flood_bit<F, 0, 1>), bg, dim3(256), 0, s, *fs, sc, sb, n);
        }
    }
    void end(int b0) const
    {
        if (n <= 0) return;
        const int gy = (n + LDPC_FLOOD_CPW - 1) / LDPC_FLOOD_CPW;
        const int fx = ((g->N > fs->M_pad ? g->N : fs->M_pad) + 255) / 256;
        hipLaunchKernelGGL((k_flood_finish<F>), dim3(fx, gy), dim3(256), 0, s, *a, *g, *fs, scratch + sb * (size_t)lo,
                           sb, b0 + lo, n, wsum + lo, ssum + lo);
        hipLaunchKernelGGL(k_flood_account, dim3((n + 255) / 256), dim3(256), 0, s, *a, b0 + lo, n, unc + lo, wsum + lo,
                           ssum + lo);
    }
};

// The resident set in two halves on two streams (aux): one half's launch
// boundaries and its small init / finish / accounting launches overlap the other
// half's phase kernels. The single stream is 95 % busy already
// (profiles/r03_dvbs2_flood_gaps.json).
// LDPC_OPT_FLOOD_STREAMS = 2 (opt-in): measured +6 % while the bit kernel's loads were
// serialised, 7 % slower once they are batched (1 855 vs 2 000 Mbit/s).
static bool flood_two_streams() { return opt(LDPC_OPT_FLOOD_STREAMS) == 2; }

template <typename F, int SRC>
static hipError_t launch_flood_phase_t(const DevGraph &g, const FloodSched &fs, const DecodeArgs &a,
                                       const KernelChoice &kc, void *gs, size_t gs_bytes, hipStream_t s,
                                       const AuxStream *aux)
{
    const size_t sb = kc.scratch_per_block;
    const size_t c2v_bytes = (size_t)((fs.e_pad + 64 + 1) / 2 * 2) * sizeof(F);
    const int K = flood_phase_resident(sb, flood_packed(fs) ? sb - c2v_bytes : sb, gs_bytes);
    unsigned char *scratch = (unsigned char *)gs;
    int *unc = reinterpret_cast<int *>(scratch + sb * (size_t)K);   // per-slot counters after the slots
    int *wsum = unc + K, *ssum = wsum + K;
    const bool two = aux && aux->s && flood_two_streams() && K >= 2;
    hipError_t e;
    if (two) {   // fork: the aux stream starts after everything queued on s
        if ((e = hipEventRecord(aux->fork, s)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(aux->s, aux->fork, 0)) != hipSuccess) return e;
    }
    for (int b0 = 0; b0 < a.batch; b0 += K) {
        const int nres = a.batch - b0 < K ? a.batch - b0 : K;
        const int na = two ? (nres + 1) / 2 : nres;
        const FloodHalf<F, SRC> A{&g, &fs, &a, scratch, sb, unc, wsum, ssum, s, 0, na};
        const FloodHalf<F, SRC> B{&g, &fs, &a, scratch, sb, unc, wsum, ssum, two ? aux->s : s, na, nres - na};
        if ((e = A.begin(b0)) != hipSuccess) return e;
        if ((e = B.begin(b0)) != hipSuccess) return e;
        for (int it = 0; it < a.T; ++it) {
            A.check();
            B.check();
            A.bit();
            B.bit();
        }
        A.end(b0);
        B.end(b0);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (two) {   // join: s continues after the aux stream's last launch
        if ((e = hipEventRecord(aux->join, aux->s)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(s, aux->join, 0)) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_flood_phase(const DevGraph &g, const FloodSched &fs, const DecodeArgs &a, bool f64,
                              const KernelChoice &kc, void *gscratch, size_t gscratch_bytes, hipStream_t s,
                              const AuxStream *aux)
{
    if (a.batch <= 0) return hipSuccess;
    if (f64)
        return a.src == SRC_GIVEN ? launch_flood_phase_t<double, SRC_GIVEN>(g, fs, a, kc, gscratch, gscratch_bytes, s, aux)
                                  : launch_flood_phase_t<double, SRC_PHILOX>(g, fs, a, kc, gscratch, gscratch_bytes, s, aux);
    return a.src == SRC_GIVEN ? launch_flood_phase_t<float, SRC_GIVEN>(g, fs, a, kc, gscratch, gscratch_bytes, s, aux)
                              : launch_flood_phase_t<float, SRC_PHILOX>(g, fs, a, kc, gscratch, gscratch_bytes, s, aux);
}

// =====================================================================
// Layered (row-serial) min-sum -- SURVEY §8(f) row 2, BASELINE config 3.
// The reference only floods (src/decodeMinSum.cpp:247-263); this is the
// row-serial schedule of the same check-node rule (:410-450, :494-515),
// restated in oracle/ldpc_oracle.c (orc_decode_layered_*):
//   x_k = app[b_k] - c2v_old_k;  c2v_k = rule(x);  app[b_k] = x_k + c2v_k
// row by row in the layered order. Rows that share no bit commute exactly, so
// each layer (LayerSched: bit-disjoint sets of whole row chains; DVB-S2
// N=64800: 17 layers of 275-3 044 rows) is updated by all its rows at once,
// one thread per row, with a workgroup barrier between layers. One workgroup
// per codeword (persistent over the batch). State:
//   app[NP + 1]            posteriors in layered position order (app[NP] = +inf pad)
//   m12[M_pad], meta[M_pad] the packed check state as in k_decode_flood (meta:
//                          argmin | signs << 5, 16 bits for rows of degree <= 8)
// -- in LDS when it fits (k_decode_layered_lds) or in a per-workgroup global
// slot (k_decode_layered_global: DVB-S2's 583 KB), where in fp64 positions [0, P) --
// the highest-degree bits, LayerSchedule::pos_of_bit -- stay in LDS (LayApp).
// No yq and no E-sized message array: a row's old messages are rebuilt from
// its packed state.
// =====================================================================
// Raw buffer access (32-bit byte offsets from a descriptor). The global half
// of a split posterior array goes through these: a distinct instruction, so
// the compiler cannot fold "LDS or global" into one flat load.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(void *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)bytes, 0x00020000);
}
template <typename F>
__device__ __forceinline__ F buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t off);
template <>
__device__ __forceinline__ float buf_ld<float>(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
template <>
__device__ __forceinline__ double buf_ld<double>(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    const u2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
    return __hiloint2double((int)v.y, (int)v.x);
}
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, uint32_t off, float x)
{
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), r, (int)off, 0, 0);
}
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, uint32_t off, double x)
{
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    u2 v;
    v.x = (unsigned)__double2loint(x);
    v.y = (unsigned)__double2hiint(x);
    __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)off, 0, 0);
}

// SPLIT: branch-free -- every access issues both the LDS and the buffer
// instruction; the side that does not hold p gets LDS slot P (a dummy) or an
// offset past the descriptor's range (the buffer unit drops it: no traffic).
template <typename F, bool SPLIT>
struct LayApp {
    F *lo;                       // positions [0, P): LDS (all of them unless SPLIT); SPLIT: lo[P] = dummy
    __amdgpu_buffer_rsrc_t hi;   // positions [P, NP]: the global slot, at p - P (SPLIT only)
    int P;
    static constexpr uint32_t kOut = 0x80000000u;   // beyond any slot
    __device__ __forceinline__ F ld(int p) const
    {
        if (!SPLIT) return lo[p];
        const bool in = p < P;
        const F a = lo[in ? p : P];
        const F b = buf_ld<F>(hi, in ? kOut : (uint32_t)(p - P) * (uint32_t)sizeof(F));
        return in ? a : b;
    }
    __device__ __forceinline__ void st(int p, F x) const
    {
        if (!SPLIT) {
            lo[p] = x;
            return;
        }
        const bool in = p < P;
        lo[in ? p : P] = x;
        buf_st(hi, in ? kOut : (uint32_t)(p - P) * (uint32_t)sizeof(F), x);
    }
};

template <typename F, int SRC, bool SPLIT>
__device__ __forceinline__ int channel_to_storage(const DecodeArgs &a, const DevGraph &g, const LayerSched &ls,
                                                  int b, const int8_t *cvec, const LayApp<F, SPLIT> &app,
                                                  [[maybe_unused]] int np1)
{
    const int tid = threadIdx.x, nt = blockDim.x, N = g.N;
    const uint64_t cw = a.first_cw + (uint64_t)b;
    int unc = 0;
    if (SRC == SRC_GIVEN) {
        const F *y = reinterpret_cast<const F *>(a.y) + (size_t)b * N;
        for (int v = tid; v < N; v += nt) {
            const F q = front_end<F>(y[v], a);
            app.st(LDPC_CHK(ls.pos_of_bit[v], np1, CHK_FLOOD_APP), q);
            const int cv = cvec ? cvec[v] : 1;
            unc += ((q > F(0) ? 1 : -1) * cv < 0);
        }
    } else {
        const F sigma = (F)a.sigma;
        const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
        for (int g4 = tid; g4 * 4 < N; g4 += nt) {
            uint32_t u[4];
            philox4x32_10((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, k0, k1, u);
            F n[4];
            box_muller(u[0], u[1], n[0], n[1]);
            box_muller(u[2], u[3], n[2], n[3]);
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int v = g4 * 4 + q4;
                if (v < N) {
                    const int cv = cvec ? cvec[v] : 1;
                    const F yv = (F)cv * (F(1) + sigma * n[q4]);
                    if (a.y_out) reinterpret_cast<F *>(a.y_out)[(size_t)b * N + v] = yv;
                    const F q = front_end<F>(yv, a);
                    app.st(LDPC_CHK(ls.pos_of_bit[v], np1, CHK_FLOOD_APP), q);
                    unc += ((q > F(0) ? 1 : -1) * cv < 0);
                }
            }
        }
    }
    return unc;
}

// One check row of the layered schedule: xs[k] = app of its bits on entry,
// the updated posteriors x_k + c2v_k on exit; returns the new packed meta
// (argmin | sign bits << 5) and the new minima in nw. The check-node rule is
// the reference's (checkNodeUpdates :410-450, applyNormalization :494-499,
// applyOffset :503-515), as in k_decode_flood.
template <typename F, int DC>
__device__ __forceinline__ uint32_t layered_row(const DecodeArgs &a, int deg, typename F2T<F>::T old, uint32_t om,
                                                F (&xs)[DC], F alpha, F delta, typename F2T<F>::T &nw)
{
    const int oidx = (int)(om & 31u);
    F mn1 = dinf<F>(), mn2 = dinf<F>();
    int amin = 31;
    uint32_t sg = 0;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k < deg) {
            F cold = (k == oidx) ? old.y : old.x;
            if ((om >> (5 + k)) & 1u) cold = -cold;
            xs[k] = xs[k] - cold;                           // v2c (:469)
            sg |= (uint32_t)(!(xs[k] >= F(0))) << k;        // sgn(v2c) < 0 (:518-523)
            const F ax = dabs(xs[k]);
            if (ax <= mn1) { mn2 = mn1; mn1 = ax; amin = k; }   // :428-433
            else if (ax < mn2) { mn2 = ax; }                    // :434-437
        }
    }
    const uint32_t degmask = (1u << deg) - 1u;
    uint32_t eff = (__popc(sg) & 1) ? (sg ^ degmask) : sg;   // prod * sgn(v2c_k)
    F M1 = mn1, M2 = mn2;
    if (a.variant == V_NMS) {
        M1 = nms_div<F>(mn1, alpha, a);                   // :498
        M2 = nms_div<F>(mn2, alpha, a);
    } else if (a.variant == V_OMS) {
        const F t1 = mn1 - delta, t2 = mn2 - delta;       // :509
        const bool p1 = t1 > F(0), p2 = t2 > F(0);
        M1 = p1 ? t1 : F(0);
        M2 = p2 ? t2 : F(0);
        // sgn(c2v) of :511 maps -0.0 to +1; a zeroed message is +0 (:513)
        const uint32_t abit = (amin < 31) ? (1u << amin) : 0u;
        if (!p1 || mn1 == F(0)) eff &= abit;
        if (!p2 || mn2 == F(0)) eff &= ~abit;
    }
    nw.x = M1;
    nw.y = M2;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k < deg) {
            const F mag = (k == amin) ? M2 : M1;
            xs[k] = xs[k] + (((eff >> k) & 1u) ? -mag : mag);
        }
    }
    return (uint32_t)amin | (eff << 5);
}

// Layered check state: argmin (5 bits) | signs << 5 -- 16 bits for the DC = 8 instantiation
// (fs.dc <= 8, launch_layered_dc), 32 above (2 B less state per row: DVB-S2
// 65 KB per codeword, more resident codewords inside the Infinity Cache).
template <int DC> using LayMeta = typename std::conditional<(DC <= 8), uint16_t, uint32_t>::type;
__host__ __device__ inline size_t layered_meta_bytes(const FloodSched &fs) { return fs.dc <= 8 ? 2 : 4; }

// Diagnostic builds (-DLDPC_STAMPS, `make variant`; scripts/lay_stamp_run.sh): per wave,
// s_memtime cycles of the layered kernel's phases, each closed by a wait on its memory
// operations (0 schedule loads, 1 posterior gathers + check state, 2 check rule, 6 scatter
// issue, 3 scatter drain, 4 layer barrier, 5 channel, init, decisions and accounting;
// 7 counts the passes), to a.stamps[(block*16+wave)*8 + k].
struct LayStamps {
#ifdef LDPC_STAMPS
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), acc[8] = {};
    __device__ __forceinline__ void mark(int k, bool drain = false)
    {
        if (drain) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        acc[k] += t - t0;
        t0 = t;
    }
    __device__ __forceinline__ void pass() { acc[7] += 1; }
    __device__ __forceinline__ void out(const DecodeArgs &a) const
    {
        if (a.stamps && (threadIdx.x & 63) == 0 && blockIdx.x < 256)
            for (int k = 0; k < 8; ++k) a.stamps[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 + k] = acc[k];
    }
#else
    __device__ __forceinline__ void mark(int, bool = false) {}
    __device__ __forceinline__ void pass() {}
    __device__ __forceinline__ void out(const DecodeArgs &) const {}
#endif
};

template <typename F, int SRC, int DC, int R, bool SPLIT>
__device__ __forceinline__ void decode_layered_cw(const DecodeArgs &a, const DevGraph &g, const FloodSched &fs,
                                                  const LayerSched &ls, int b, const LayApp<F, SPLIT> &app,
                                                  typename F2T<F>::T *m12, LayMeta<DC> *meta, int *red,
                                                  unsigned long long *acc, LayStamps &st)
{
    using F2 = typename F2T<F>::T;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int N = g.N, NP = fs.ngroups * 64, MP = ls.M_pad;
    const F alpha = (F)a.alpha, delta = (F)a.delta;
    const uint64_t cw = a.first_cw + (uint64_t)b;
    const int8_t *cvec = nullptr;
    if (SRC == SRC_GIVEN) {
        if (a.c) cvec = a.c + (size_t)b * N;
    } else if (a.cw_table) {
        cvec = a.cw_table + (size_t)(cw % (uint64_t)a.cw_rows) * N;
    }
    // ---- channel + front-end (:214-238): app = yq in storage order ----
    const int unc = channel_to_storage<F, SRC, SPLIT>(a, g, ls, b, cvec, app, NP + 1);
    for (int i = tid; i < MP; i += nt) {   // c2v_old = +0 (:364-370)
        F2 z;
        z.x = F(0);
        z.y = F(0);
        m12[i] = z;
        meta[i] = 0;
    }
    __syncthreads();
    st.mark(5);

    for (int it = 0; it < a.T; ++it) {
        for (int L = 0; L < ls.nlayers; ++L) {
            const int r1 = ls.lptr[L + 1];
            // R rows per thread per pass: every gather of the pass is issued
            // before the first row is computed (one memory round trip per pass)
            for (int i0 = ls.lptr[L] + tid; i0 < r1; i0 += nt * R) {
                int deg[R], sp[R][DC];
                F xs[R][DC];
                F2 old[R];
                uint32_t om[R];
#pragma unroll
                for (int r = 0; r < R; ++r) deg[r] = (i0 + r * nt < r1) ? ls.rdeg[i0 + r * nt] : 0;
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int k = 0; k < DC; ++k)
                        sp[r][k] = k < deg[r] ? LDPC_CHK(ls.sp[(size_t)k * MP + i0 + r * nt], NP + 1, CHK_FLOOD_APP) : NP;
                st.pass();
                st.mark(0, true);
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int k = 0; k < DC; ++k) xs[r][k] = app.ld(sp[r][k]);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (deg[r]) {
                        old[r] = m12[i0 + r * nt];
                        om[r] = meta[i0 + r * nt];
                    }
                }
                st.mark(1, true);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (deg[r]) {
                        F2 nw;
                        const uint32_t nm = layered_row<F, DC>(a, deg[r], old[r], om[r], xs[r], alpha, delta, nw);
                        st.mark(2);
                        m12[i0 + r * nt] = nw;
                        meta[i0 + r * nt] = (LayMeta<DC>)nm;
#pragma unroll
                        for (int k = 0; k < DC; ++k)
                            if (k < deg[r]) app.st(sp[r][k], xs[r][k]);   // posterior update
                    }
                }
                st.mark(6);
                st.mark(3, true);
            }
            __syncthreads();
            st.mark(4);
        }
    }

    // ---- decisions, error weight (:270, :382-393), syndrome ----
    int w = 0, synd = 0;
    for (int v = tid; v < N; v += nt) {
        const int d = app.ld(LDPC_CHK(ls.pos_of_bit[v], NP + 1, CHK_FLOOD_APP)) > F(0) ? 1 : -1;   // :471-474
        const int cv = cvec ? cvec[v] : 1;
        w += (d != cv);
        if (a.d_out) a.d_out[(size_t)b * N + v] = (int8_t)d;
    }
    for (int i = tid; i < MP; i += nt) {
        const int deg = ls.rdeg[i];
        int par = 0;
        for (int k = 0; k < deg; ++k) par ^= (app.ld(LDPC_CHK(ls.sp[(size_t)k * MP + i], NP + 1, CHK_FLOOD_APP)) > F(0)) ? 0 : 1;
        synd |= par;
    }
    int sums[3] = {w, unc, synd};
    block_sum_n_t0<3>(sums, red);
    if (tid == 0) {
        const int sf = sums[2] > 0;
        acc[0] += (unsigned long long)sums[0];
        acc[1] += (unsigned long long)(sums[0] > 0);
        acc[2] += (unsigned long long)sums[1];
        acc[3] += 1ull;
        acc[5] += (unsigned long long)sf;
        if (sums[0] > 0 && a.hist) atomicAdd(&a.hist[sums[0] - 1], 1ull);
        if (a.frame_res) a.frame_res[b] = make_int4(sums[0], sums[1], sf, 0);
    }
    __syncthreads();
    st.mark(5);
}

__device__ __forceinline__ void flush_acc(const DecodeArgs &a, unsigned long long *acc)
{
    if (threadIdx.x == 0 && acc[3] > 0) {
        acc[4] = acc[3] * (unsigned long long)a.T;
#pragma unroll
        for (int q = 0; q < 6; ++q) atomicAdd(&a.counts[q], acc[q]);
    }
}

// LDS offsets of the layered state: app[NP + 1] | pad | m12[M_pad] | meta[M_pad].
__host__ __device__ inline size_t layered_m12_off(const FloodSched &fs, size_t fsz)
{
    return (((size_t)fs.ngroups * 64 + 1) * fsz + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t layered_state_bytes(const FloodSched &fs, const LayerSched &ls, size_t fsz)
{
    return (layered_m12_off(fs, fsz) + (size_t)ls.M_pad * (2 * fsz + layered_meta_bytes(fs)) + 255) & ~(size_t)255;
}

template <typename F, int SRC, int DC, int R>
__global__ __launch_bounds__(512) void k_decode_layered_lds(DecodeArgs a, DevGraph g, FloodSched fs, LayerSched ls)
{
    using F2 = typename F2T<F>::T;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int red[16 * 4];
    __shared__ unsigned long long acc[6];
    F *app = reinterpret_cast<F *>(smem);
    F2 *m12 = reinterpret_cast<F2 *>(smem + layered_m12_off(fs, sizeof(F)));
    LayMeta<DC> *meta = reinterpret_cast<LayMeta<DC> *>(m12 + ls.M_pad);
    if (threadIdx.x == 0) {
        app[fs.ngroups * 64] = dinf<F>();
#pragma unroll
        for (int q = 0; q < 6; ++q) acc[q] = 0;
    }
    const LayApp<F, false> la{app, buf_rsrc(app, 0), 0};
    LayStamps st;
    for (int b = blockIdx.x; b < a.batch; b += gridDim.x)
        decode_layered_cw<F, SRC, DC, R, false>(a, g, fs, ls, b, la, m12, meta, red, acc, st);
    st.out(a);
    flush_acc(a, acc);
}
// State in a global slot; SPLIT (fp64): except the posteriors of layered
// positions [0, P) (dynamic LDS, (P + 1) * sizeof(F) bytes) -- DVB-S2 keeps
// 19 455 of its 64 800 bits there, every degree-8 bit and a third of the
// degree-3 ones, 54 % of the edge gathers and scatters.
template <typename F, int SRC, int DC, int R, bool SPLIT, int NT = 512>
__global__ __launch_bounds__(NT) void k_decode_layered_global(DecodeArgs a, DevGraph g, FloodSched fs, LayerSched ls,
                                                              unsigned char *scratch, size_t slot_bytes, int P)
{
    using F2 = typename F2T<F>::T;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int red[16 * 4];
    __shared__ unsigned long long acc[6];
    unsigned char *base = scratch + slot_bytes * blockIdx.x;
    F *app = reinterpret_cast<F *>(base);
    F2 *m12 = reinterpret_cast<F2 *>(base + layered_m12_off(fs, sizeof(F)));
    LayMeta<DC> *meta = reinterpret_cast<LayMeta<DC> *>(m12 + ls.M_pad);
    const LayApp<F, SPLIT> la{SPLIT ? reinterpret_cast<F *>(smem) : app,
                              buf_rsrc(app, (uint32_t)layered_m12_off(fs, sizeof(F))), P};
    if (threadIdx.x == 0) {
        la.st(fs.ngroups * 64, dinf<F>());
#pragma unroll
        for (int q = 0; q < 6; ++q) acc[q] = 0;
    }
    LayStamps st;
    for (int b = blockIdx.x; b < a.batch; b += gridDim.x)
        decode_layered_cw<F, SRC, DC, R, SPLIT>(a, g, fs, ls, b, la, m12, meta, red, acc, st);
    st.out(a);
    flush_acc(a, acc);
}


// Check node, exact path: the reference's comparisons for any input, incl.
// infinities and NaN (checkNodeUpdates :410-450, applyNormalization :494-499,
// applyOffset :503-515). pv[k].v[c]: in = c2v sent last iteration, out = new c2v.
template <typename F, int C, int DC, typename MT>
__device__ __forceinline__ void cn_exact(const Pack<F, C> (&xin)[DC], int c, Pack<F, C> (&pv)[DC], MT degmask,
                                         const DecodeArgs &a, F alpha, F delta)
{
    F ax[DC];
    F mn1 = dinf<F>(), mn2 = dinf<F>();
    MT sg = 0;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const F x = xin[k].v[c] - pv[k].v[c];                       // v2c (:469)
        sg |= (MT)(!(x >= F(0))) << k;                              // sgn(v2c) (:518-523)
        ax[k] = dabs(x);
        // :428-437 -- if (|x| <= m1) {m2 = m1; m1 = |x|} else if (|x| < m2) m2 = |x|
        // (NaN: no comparison holds and fmin returns the other operand).
        const bool le = ax[k] <= mn1;
        mn2 = dmin(mn2, le ? mn1 : ax[k]);
        mn1 = le ? ax[k] : mn1;
    }
    sg &= degmask;
    const MT eff = (__popcll((unsigned long long)sg) & 1) ? (sg ^ degmask) : sg;   // prod*sgn(v2c_k)
    // The argmin edge gets m2, every other edge m1 (:444-447). |x_k| == m1
    // identifies it: on a tie m2 == m1, so which tied edge is "argmin" does not matter.
    if (a.variant != V_OMS) {
        F M1 = mn1, M2 = mn2;
        if (a.variant == V_NMS) {
            M1 = nms_div<F>(mn1, alpha, a);
            M2 = nms_div<F>(mn2, alpha, a);
        }
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            const F mag = (ax[k] == mn1) ? M2 : M1;
            pv[k].v[c] = ((eff >> k) & 1u) ? -mag : mag;
        }
    } else {
        const F t1 = mn1 - delta, t2 = mn2 - delta;
        const bool p1 = t1 > F(0), p2 = t2 > F(0);
        const F M1 = p1 ? t1 : F(0), M2 = p2 ? t2 : F(0);
        // sgn(c2v) maps -0.0 to +1 and a zeroed message is +0
        const MT e1 = (!p1 || mn1 == F(0)) ? (MT)0 : eff;
        const MT e2 = (!p2 || mn2 == F(0)) ? (MT)0 : eff;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            const bool ism = ax[k] == mn1;
            const F mag = ism ? M2 : M1;
            pv[k].v[c] = (((ism ? e2 : e1) >> k) & 1u) ? -mag : mag;
        }
    }
}

template <int DC, int C, int DCA = DC, bool PK = false>
__device__ __forceinline__ bool cn_fast(const Pack<double, C> (&)[DCA], Pack<double, C> (&)[DCA], bool, float, float)
{
    return false;   // never called: fp64 always takes the exact path
}

// Block shape per rows-per-thread: RPT=1 up to 1024 threads (4 waves/SIMD);
// RPT=2 512 threads and RPT=3 384 threads, sized for two blocks per CU
// (4 resp. 3 waves per SIMD: 128 resp. 168 VGPRs).
template <int RPT> struct RowsShape;
template <> struct RowsShape<1> { static constexpr int threads = 1024, waves_per_eu = 4; };
#ifndef LDPC_RPT2_WAVES
#define LDPC_RPT2_WAVES 4
#endif
template <> struct RowsShape<2> { static constexpr int threads = 512, waves_per_eu = LDPC_RPT2_WAVES; };
template <> struct RowsShape<3> { static constexpr int threads = 384, waves_per_eu = 3; };

template <typename F, int SRC, int C, int DC, int CPT, int RPT>
__global__ __launch_bounds__(RowsShape<RPT>::threads, RowsShape<RPT>::waves_per_eu) void k_decode_rows(
    DecodeArgs a, DevGraph g, RowSched rs)
{
    using MT = typename MetaOf<DC>::T;
    using P = Pack<F, C>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, nt = blockDim.x;
    const int N = g.N, EA = rs.e_pad + 64;         // + one dummy slot per lane for padding edges
    P *app = reinterpret_cast<P *>(smem);          // [N + 1]: bit N is the +INF sentinel of padding edges
    P *c2v = app + (N + 2);                        // [EA] (N+2 keeps 16-B alignment)
    int *red = reinterpret_cast<int *>(c2v + EA);

    // ---- the thread's rows (tid + r*nt) and bit slots, in registers for the whole launch ----
    int deg[RPT];
    MT degmask[RPT];
    uint32_t colw[RPT][DC / 2], posw[RPT][DC / 2];
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
        const int j = tid + r * nt;
        deg[r] = rs.cn_deg[j];
        degmask[r] = (deg[r] >= (int)(8 * sizeof(MT))) ? ~(MT)0 : (((MT)1 << deg[r]) - 1);
#pragma unroll
        for (int q = 0; q < DC / 8; ++q) {
            const uint4 xc = reinterpret_cast<const uint4 *>(rs.cn_cols + (size_t)j * DC)[q];
            const uint4 xp = reinterpret_cast<const uint4 *>(rs.cn_pos + (size_t)j * DC)[q];
            colw[r][4 * q + 0] = xc.x; colw[r][4 * q + 1] = xc.y; colw[r][4 * q + 2] = xc.z; colw[r][4 * q + 3] = xc.w;
            posw[r][4 * q + 0] = xp.x; posw[r][4 * q + 1] = xp.y; posw[r][4 * q + 2] = xp.z; posw[r][4 * q + 3] = xp.w;
        }
    }
    // bit slots: a thread's slots have non-increasing group degree (graph.cpp)
    // Slot i of lane l: c2v edge k at vgb[i] + l + 64k (vgb and the group degree
    // vgd are wave-uniform: SGPRs); the bit it sums into is vdst (two 16-bit
    // entries per register; the spare app entry N+1 for an empty slot).
    const int lane = tid & 63;
    int vgb[CPT], vgd[CPT];
    uint32_t vdst2[(CPT + 1) / 2] = {};
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const int c = rs.vn_col[tid * CPT + i];
        vdst2[i / 2] |= (uint32_t)(c == 0xffff ? N + 1 : c) << (16 * (i & 1));
        const uint32_t info = rs.vn_info[tid * CPT + i];
        vgb[i] = __builtin_amdgcn_readfirstlane((int)(info & 0xffffu) - lane);
        vgd[i] = __builtin_amdgcn_readfirstlane((int)(info >> 24));
    }
    auto vdst = [&](int i) -> int { return (int)((vdst2[i / 2] >> (16 * (i & 1))) & 0xffffu); };
    if (tid == 0) {
        P inf;
#pragma unroll
        for (int c = 0; c < C; ++c) inf.v[c] = dinf<F>();
        app[N] = inf;
#pragma unroll
        for (int q = 0; q < 3 * C; ++q) red[32 + q] = 0;   // block_sum_lds totals
        red[31] = 0;   // the premise flag: cleared again by thread 0 at the end of each group
    }
    // Padding slots of the bit-node layout hold +0 (adding +0 leaves every sum, and hence
    // every decision, unchanged); nothing writes them after this (the channel stages into
    // app, the check rows scatter into their own slots and the per-lane dummies).
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const int dg = (int)((rs.vn_info[tid * CPT + i] >> 16) & 0xffu);
        const int base = vgb[i] + lane, gd = vgd[i];
        P z;
#pragma unroll
        for (int c = 0; c < C; ++c) z.v[c] = F(0);
        for (int k = dg; k < gd; ++k) c2v[base + k * 64] = z;
    }
    __syncthreads();   // the flag's first clear before any channel raises it

    // The second-dispatched half of the workgroup at priority 1 for the whole
    // launch (MI355X_MICROARCH "Two waves per SIMD" item 4): +0.25 % in an
    // interleaved 3-round A/B (14 549 -> 14 594 Mbit/s), no change in results.
    if ((tid >> 6) >= (nt >> 7)) __builtin_amdgcn_s_setprio(1);
    const F alpha = (F)a.alpha, delta = (F)a.delta;
    const int ngrp = (a.batch + C - 1) / C;
    unsigned long long st_chan = 0, st_cn = 0, st_vn = 0, st_acct = 0;
    (void)st_chan; (void)st_cn; (void)st_vn; (void)st_acct;
    // the block's totals (thread 0), added to a.counts once at the end
    unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
    for (int grp = blockIdx.x; grp < ngrp; grp += gridDim.x) {
        STAMP(t_start);
        // ---- channel (:214-238), staged into app as yq + 0 (never -0: v2c = app - c2v then
        // differs at most in the sign of a zero, which sgn() and |.| ignore, and the decision
        // app > 0 is the same; the fast check node relies on it); an input outside the fast
        // premise (|yq| >= 1e30, inf, NaN) raises the flag, which thread 0 cleared at the end
        // of the previous group ----
        int unc[C];
        bool ch_ok = true;
        auto put = [&](int v, int c, F q) {
            q = q + F(0);
            ch_ok &= dabs(q) < F(1e30f);
            app[v].v[c] = q;
        };
        const int8_t *cvec[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            unc[c] = 0;
            cvec[c] = nullptr;
            const int b = grp * C + c;
            if (b >= a.batch) {   // missing partner of an odd batch: benign +1 samples, never counted
                for (int v = tid; v < N; v += nt) app[v].v[c] = F(1);
                continue;
            }
            const uint64_t cw = a.first_cw + (uint64_t)b;
            if (SRC == SRC_GIVEN) {
                if (a.c) cvec[c] = a.c + (size_t)b * N;
                const F *y = reinterpret_cast<const F *>(a.y) + (size_t)b * N;
                for (int v = tid; v < N; v += nt) {
                    const F q = front_end<F>(y[v], a);
                    put(v, c, q);
                    const int cv = cvec[c] ? cvec[c][v] : 1;
                    unc[c] += ((q > F(0) ? 1 : -1) * cv < 0);
                }
            } else {
                if (a.cw_table) cvec[c] = a.cw_table + (size_t)(cw % (uint64_t)a.cw_rows) * N;
                const F sigma = (F)a.sigma;
                const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
                if (!a.cw_table && !a.y_out && !a.quantize && !a.saturate && (N & 3) == 0) {
                    // the common case in straight-line code (the all-zero codeword, no front end,
                    // no sample output): the same values as the general loop below
                    for (int g4 = tid; g4 * 4 < N; g4 += nt) {
                        uint32_t u[4];
                        philox4x32_10<LDPC_ROWS_MAD64 != 0>((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id,
                                                            k0, k1, u);
                        F n[4];
                        box_muller(u[0], u[1], n[0], n[1]);
                        box_muller(u[2], u[3], n[2], n[3]);
#pragma unroll
                        for (int q4 = 0; q4 < 4; ++q4) {
                            const F qv = (F(1) + sigma * n[q4]) + F(0);   // (F)cv * (1 + sigma n), cv = +1; yq + 0
                            unc[c] += (qv > F(0) ? 1 : -1) < 0;
                            ch_ok &= dabs(qv) < F(1e30f);
                            app[4 * g4 + q4].v[c] = qv;
                        }
                    }
                    continue;
                }
                for (int g4 = tid; g4 * 4 < N; g4 += nt) {
                    uint32_t u[4];
                    philox4x32_10<LDPC_ROWS_MAD64 != 0>((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, k0, k1, u);
                    F n[4];
                    box_muller(u[0], u[1], n[0], n[1]);
                    box_muller(u[2], u[3], n[2], n[3]);
#pragma unroll
                    for (int q4 = 0; q4 < 4; ++q4) {
                        const int v = g4 * 4 + q4;
                        if (v < N) {
                            const int cv = cvec[c] ? cvec[c][v] : 1;
                            const F yv = (F)cv * (F(1) + sigma * n[q4]);
                            if (a.y_out) reinterpret_cast<F *>(a.y_out)[(size_t)b * N + v] = yv;
                            const F q = front_end<F>(yv, a);
                            put(v, c, q);
                            unc[c] += ((q > F(0) ? 1 : -1) * cv < 0);
                        }
                    }
                }
            }
        }
        if (__builtin_amdgcn_ballot_w64(!ch_ok)) {   // rare: an input outside the fast premise
            asm volatile(";");
            if (!ch_ok) red[31] = 1;
        }
        __syncthreads();
        // yq of the thread's bit slots, read back as staged (v2c = yq on the first pass,
        // :364-370); a padding slot +0
        P yq[CPT];
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            yq[i] = app[vdst(i) < N ? vdst(i) : 0];
            if (vdst(i) >= N)
#pragma unroll
                for (int c = 0; c < C; ++c) yq[i].v[c] = F(0);
        }

        // c2v sent on each edge last iteration: +0 before the first. RPT <= 2 keeps
        // the check node's own copy in registers; larger RPT re-reads it from its
        // c2v slots (written only by this thread, read by the bit phase) to stay
        // within the register budget of two blocks per CU.
        // (Re-reading is only safe on the exact path: padding edges share per-lane
        // dummy slots, so their "old message" is whatever another row wrote there.)
        constexpr bool PREV_REG = RPT <= 2;
        P prev[PREV_REG ? RPT : 1][DC];
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
            if (PREV_REG) {
#pragma unroll
                for (int k = 0; k < DC; ++k)
#pragma unroll
                    for (int c = 0; c < C; ++c) prev[PREV_REG ? r : 0][k].v[c] = F(0);
            } else {
                P z;
#pragma unroll
                for (int c = 0; c < C; ++c) z.v[c] = F(0);
#pragma unroll
                for (int k = 0; k < DC; ++k) c2v[u16_at<DC>(posw[r], k)] = z;
            }
        }

        STAMP(t_iter0);
#ifdef LDPC_STAMPS
        st_chan += t_iter0 - t_start;
#endif
        // One iteration loop, instantiated twice: the fast check-node loop runs
        // while its premise holds (flag red[31] clear: every c2v entering the
        // iteration is below 1e30) and hands over to the exact loop, which
        // continues from the same state. Separate loops keep the two check-node
        // bodies out of each other's register allocation.
        auto iterate = [&](auto fast_tag, int it0) -> int {
            constexpr bool FAST = decltype(fast_tag)::value;
            int it = it0;
            // fast-path flag: read right after the check-node barrier of the previous
            // iteration (in flight during the bit-node phase), so no LDS round trip
            // opens the iteration; red[31] was cleared before the first iteration
            int flag = FAST ? red[31] : 0;   // set by an input outside the premise
            for (; it < a.T; ++it) {
                STAMP(t_cn0);
                if (FAST && __builtin_amdgcn_readfirstlane(flag) != 0) break;
                // ---- check nodes (:410-450, :494-515); row r+1's gathers are issued
                // before row r is computed ----
                P xin[2][DC];
                if (LDPC_ROWS_PRIOBAL) __builtin_amdgcn_s_setprio(3);
#pragma unroll
                for (int k = 0; k < DC; ++k) xin[0][k] = app[u16_at<DC>(colw[0], k)];   // padding edges read +INF
#pragma unroll
                for (int r = 0; r < RPT; ++r) {
                    if (LDPC_ROWS_PRIOBAL && r > 0) __builtin_amdgcn_s_setprio(2);
                    if (r + 1 < RPT) {
#pragma unroll
                        for (int k = 0; k < DC; ++k) xin[(r + 1) & 1][k] = app[u16_at<DC>(colw[r + 1 < RPT ? r + 1 : r], k)];
                    }
                    P (&pv)[DC] = prev[PREV_REG ? r : 0];
                    if (!PREV_REG) {
#pragma unroll
                        for (int k = 0; k < DC; ++k) pv[k] = c2v[u16_at<DC>(posw[r], k)];
                    }
                    if constexpr (FAST) {
                        const bool ok = cn_fast<DC, C, DC, true>(xin[r & 1], pv, a.variant == V_NMS, (float)alpha, a.alpha_rcp);
                        // Rows past M (degree 0) only write the never-read dummy slots.
                        if (!ok && deg[r] > 0) red[31] = 1;
                    } else {
#pragma unroll
                        for (int c = 0; c < C; ++c) cn_exact<F, C, DC>(xin[r & 1], c, pv, degmask[r], a, alpha, delta);
                    }
#pragma unroll
                    for (int k = 0; k < DC; ++k) c2v[u16_at<DC>(posw[r], k)] = pv[k];   // padding edges: the lane's dummy slot
#ifndef LDPC_NO_ROW_FENCE
                    // keep the rows' live ranges apart (register pressure: two blocks per CU)
                    if (RPT > 1) __builtin_amdgcn_sched_barrier(0);
#endif
                }
                if (LDPC_ROWS_PRIOBAL) __builtin_amdgcn_s_setprio(0);
                __syncthreads();
                if (FAST) flag = red[31];
                STAMP(t_vn0);
#ifdef LDPC_STAMPS
                st_cn += t_vn0 - t_cn0;
#endif
                // ---- bit nodes: sum = yq + c2v in nlist order (:452-476); edges past a
                // bit's own degree hold +0 ----
                {
                    P sum[CPT];
#pragma unroll
                    for (int i = 0; i < CPT; ++i) sum[i] = yq[i];
                    int k = 0;
                    vn_phases<F, C, CPT, CPT, true>(c2v + lane, vgb, vgd, k, sum);
#pragma unroll
                    for (int i = 0; i < CPT; ++i) app[vdst(i)] = sum[i];
                }
                __syncthreads();
#ifdef LDPC_STAMPS
                { STAMP(t_vn1); st_vn += t_vn1 - t_vn0; }
#endif
            }
            return it;
        };
        int it_done = 0;
        if constexpr (sizeof(F) == 4 && PREV_REG)
            if (a.variant == V_MS || (a.variant == V_NMS && a.nms_fast)) it_done = iterate(std::true_type{}, 0);
        if (it_done < a.T) iterate(std::false_type{}, it_done);
        STAMP(t_acct0);

        // ---- decisions, error weight, syndrome, accounting ----
        int sums[3 * C];   // per codeword: error weight, uncoded errors, syndrome failure
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int b = grp * C + c;
            int w = 0, synd = 0;
            if (b < a.batch) {
#pragma unroll
                for (int i = 0; i < CPT; ++i) {
                    const int v = vdst(i);
                    if (v < N) {
                        const int d = app[v].v[c] > F(0) ? 1 : -1;
                        const int cv = cvec[c] ? cvec[c][v] : 1;
                        w += (d != cv);
                        if (a.d_out) a.d_out[(size_t)b * N + v] = (int8_t)d;
                    }
                }
                // padding edges read the +inf sentinel: parity 0
#pragma unroll
                for (int r = 0; r < RPT; ++r) {
                    int par = 0;
#pragma unroll
                    for (int k = 0; k < DC; ++k) par ^= (app[u16_at<DC>(colw[r], k)].v[c] > F(0)) ? 0 : 1;
                    synd |= par;
                }
            }
            sums[3 * c] = w;
            sums[3 * c + 1] = unc[c];
            sums[3 * c + 2] = synd;
        }
        if (LDPC_ROWS_ACCT) block_sum_lds<3 * C>(sums, red + 32);   // re-zeroed by thread 0; the step's last barrier orders it
        else block_sum_n_t0<3 * C>(sums, red + 32);
        if (tid == 0) {
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int b = grp * C + c;
                if (b >= a.batch) continue;
                const int w = sums[3 * c], uc = sums[3 * c + 1], sf = sums[3 * c + 2] > 0;
                acc[0] += (unsigned long long)w;
                acc[1] += (unsigned long long)(w > 0);
                acc[2] += (unsigned long long)uc;
                acc[3] += 1ull;
                acc[5] += (unsigned long long)sf;
                if (w > 0 && a.hist) atomicAdd(&a.hist[w - 1], 1ull);
                if (a.frame_res) a.frame_res[b] = make_int4(w, uc, sf, 0);
            }
            red[31] = 0;   // the next group's premise flag (raised no earlier than its channel)
        }
        __syncthreads();
#ifdef LDPC_STAMPS
        { STAMP(t_end); st_acct += t_end - t_acct0; }
#endif
    }
    if (tid == 0 && acc[3] > 0) {
        acc[4] = acc[3] * (unsigned long long)a.T;
#pragma unroll
        for (int q = 0; q < 6; ++q) atomicAdd(&a.counts[q], acc[q]);
    }
#ifdef LDPC_STAMPS
    if (tid == 0 && a.stamps) {
        a.stamps[blockIdx.x * 4 + 0] = st_chan;
        a.stamps[blockIdx.x * 4 + 1] = st_cn;
        a.stamps[blockIdx.x * 4 + 2] = st_vn;
        a.stamps[blockIdx.x * 4 + 3] = st_acct;
    }
#endif
}

// Exhaustive check of the reciprocal division (see kernels.h).
__global__ __launch_bounds__(256) void k_verify_div(float alpha, float rcp, unsigned long long *bad)
{
    const uint32_t total = 0x7f800000u;   // all finite non-negative floats
    unsigned long long nbad = 0;
    for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < total; u += gridDim.x * blockDim.x) {
        const float x = __uint_as_float(u);
        const float q = x * rcp;
        const float f = __builtin_fmaf(__builtin_fmaf(-q, alpha, x), rcp, q);
        const float d = x / alpha;
        nbad += (__float_as_uint(f) != __float_as_uint(d));
    }
    for (int o = 32; o > 0; o >>= 1) nbad += __shfl_xor(nbad, o, 64);
    if ((threadIdx.x & 63) == 0 && nbad) atomicAdd(bad, nbad);
}

LDPC_CHECK_TU(kernels)

hipError_t verify_div_by_reciprocal(float alpha, float rcp, unsigned long long *bad, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(bad, 0, sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_verify_div, dim3(8192), dim3(256), 0, s, alpha, rcp, bad);
    return hipGetLastError();
}

static size_t state_bytes(const DevGraph &g, bool f64)
{
    const size_t rs = f64 ? sizeof(RowState<double>) : sizeof(RowState<float>);
    const size_t fs = f64 ? 8 : 4;
    return rs * (size_t)g.M + 2 * fs * (size_t)g.N;
}

constexpr int kThreads = 256;
constexpr size_t kMaxLds = 160 * 1024;

// Codewords per thread: 2 for the fp32 DC=8 kernel (no spills at 101 VGPRs),
// 1 where two would spill (fp64, wider rows).
static int rows_cw_per_block(bool f64, int dc)
{
#ifdef LDPC_C1
    (void)f64; (void)dc;
    return 1;
#else
    return (!f64 && dc == 8) ? 2 : 1;
#endif
}

static size_t rows_lds(const DevGraph &g, const RowSched &rs, bool f64, int C)
{
    const size_t fs = f64 ? 8 : 4;
    // + red: 32 ints (fast-path flag at [31]) and 16 waves x 8 sums
    return ((size_t)C * ((size_t)g.N + 2 + (size_t)rs.e_pad + 64) * fs + 4 * (32 + 16 * 8) + 15) & ~(size_t)15;
}

KernelChoice choose_kernel(const DevGraph &g, bool f64, const RowSched *rs, const char *force, const FloodSched *fs)
{
    KernelChoice kc;
    kc.threads = kThreads;
    kc.cw_per_block = 1;
    kc.scratch_per_block = 0;
    const bool want_lds = force && force[0] == 'l';
    const bool want_global = force && force[0] == 'g';
    const bool want_flood = force && force[0] == 'f';
    if (fs && fs->M_pad > 0 && fs->dc <= kPackedMaxDc && want_flood) {
        kc.name = "flood";
        kc.lds_bytes = 0;
        kc.threads = 512;
        kc.scratch_per_block = flood_slot_bytes(g, *fs, f64);
        return kc;
    }
    if (rs && rs->threads > 0 && !want_lds && !want_global && !want_flood) {
        const int C = rows_cw_per_block(f64, rs->dc);
        const size_t lds = rows_lds(g, *rs, f64, C);
        if (lds <= kMaxLds) {
            kc.name = "rows";
            kc.lds_bytes = (int)lds;
            kc.threads = rs->threads;
            kc.cw_per_block = C;
            return kc;
        }
    }
    const size_t lds = (state_bytes(g, f64) + 64 + 15) & ~(size_t)15;
    if (lds <= kMaxLds && !want_global && !want_flood) {
        kc.name = "lds";
        kc.lds_bytes = (int)lds;
    } else if (fs && fs->M_pad > 0 && fs->dc <= kPackedMaxDc && !want_global) {
        kc.name = "flood";
        kc.lds_bytes = 0;
        kc.threads = 512;
        kc.scratch_per_block = flood_slot_bytes(g, *fs, f64);
    } else {
        kc.name = "global";
        kc.lds_bytes = 0;
        kc.scratch_per_block = (state_bytes(g, f64) + 255) & ~(size_t)255;
    }
    return kc;
}

template <typename F, int SRC>
static hipError_t launch_t(const DevGraph &g, const DecodeArgs &a, const KernelChoice &kc, void *gs,
                           int gblocks, hipStream_t s)
{
    if (kc.lds_bytes > 0) {
        auto fn = k_decode_lds<F, SRC>;
        if (kc.lds_bytes > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               kc.lds_bytes);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(fn, dim3(a.batch), dim3(kc.threads), kc.lds_bytes, s, a, g);
    } else {
        const int grid = gblocks < a.batch ? gblocks : a.batch;
        hipLaunchKernelGGL((k_decode_global<F, SRC>), dim3(grid), dim3(kc.threads), 0, s, a, g,
                           (unsigned char *)gs, kc.scratch_per_block);
    }
    return hipGetLastError();
}

size_t redo_lds_bytes(const DevGraph &g, bool f64) { return (state_bytes(g, f64) + 64 + 15) & ~(size_t)15; }

hipError_t launch_redo(const DevGraph &g, const DecodeArgs &a, bool f64, const unsigned *redo, hipStream_t s,
                       int num_cus)
{
    const size_t lds = redo_lds_bytes(g, f64);
    auto go = [&](auto fn) -> hipError_t {
        if (lds > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(fn, dim3(num_cus), dim3(kThreads), lds, s, a, g, redo);
        return hipGetLastError();
    };
    if (f64) return a.src == SRC_GIVEN ? go(k_redo<double, SRC_GIVEN>) : go(k_redo<double, SRC_PHILOX>);
    return a.src == SRC_GIVEN ? go(k_redo<float, SRC_GIVEN>) : go(k_redo<float, SRC_PHILOX>);
}

// Row kernel: dispatch on (C, DC, CPT). Persistent grid of the resident blocks.
template <typename F, int SRC, int C, int DC, int CPT, int RPT>
static hipError_t launch_rows_t(const DevGraph &g, const RowSched &rs, const DecodeArgs &a, const KernelChoice &kc,
                                hipStream_t s, int num_cus)
{
    auto fn = k_decode_rows<F, SRC, C, DC, CPT, RPT>;
    hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, kc.lds_bytes);
    if (e != hipSuccess) return e;
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kc.threads, kc.lds_bytes);
    if (e != hipSuccess || per_cu < 1) per_cu = 1;
    if (const int cap = opt(LDPC_OPT_ROWS_BPC))   // diagnostic: fewer resident blocks
        if (cap < per_cu) per_cu = cap;
    const int ngrp = (a.batch + C - 1) / C;
    int grid = per_cu * num_cus;
    if (grid > ngrp) grid = ngrp;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kc.threads), kc.lds_bytes, s, a, g, rs);
    return hipGetLastError();
}

template <typename F, int SRC>
static hipError_t launch_rows_dc(const DevGraph &g, const RowSched &rs, const DecodeArgs &a, const KernelChoice &kc,
                                 hipStream_t s, int num_cus)
{
#ifdef LDPC_C1
    constexpr int C8 = 1;
#else
    constexpr int C8 = sizeof(F) == 4 ? 2 : 1;
#endif
#define LDPC_ROWS_CASE(CV, DCV, CPTV, RPTV)                                   \
    if (rs.dc == DCV && rs.cpt == CPTV && rs.rpt == RPTV)                   \
        return launch_rows_t<F, SRC, CV, DCV, CPTV, RPTV>(g, rs, a, kc, s, num_cus);
    LDPC_ROWS_CASE(C8, 8, 2, 1)
    LDPC_ROWS_CASE(C8, 8, 4, 1)
    LDPC_ROWS_CASE(C8, 8, 4, 2)
    LDPC_ROWS_CASE(1, 16, 2, 1)
    LDPC_ROWS_CASE(1, 16, 4, 1)
    LDPC_ROWS_CASE(1, 16, 4, 2)
    LDPC_ROWS_CASE(1, 32, 2, 1)
    LDPC_ROWS_CASE(1, 32, 4, 1)
    LDPC_ROWS_CASE(1, 32, 4, 2)
#undef LDPC_ROWS_CASE
    return hipErrorInvalidValue;
}

template <typename F, int SRC>
static hipError_t launch_flood_t(const DevGraph &g, const FloodSched &fs, const DecodeArgs &a,
                                 const KernelChoice &kc, void *gs, int gblocks, hipStream_t s)
{
    const int grid = gblocks < a.batch ? gblocks : a.batch;
    if (fs.dc <= 8)
        hipLaunchKernelGGL((k_decode_flood<F, SRC, 8>), dim3(grid), dim3(kc.threads), 0, s, a, g, fs,
                           (unsigned char *)gs, kc.scratch_per_block);
    else if (fs.dc <= 16)
        hipLaunchKernelGGL((k_decode_flood<F, SRC, 16>), dim3(grid), dim3(kc.threads), 0, s, a, g, fs,
                           (unsigned char *)gs, kc.scratch_per_block);
    else
        hipLaunchKernelGGL((k_decode_flood<F, SRC, 32>), dim3(grid), dim3(kc.threads), 0, s, a, g, fs,
                           (unsigned char *)gs, kc.scratch_per_block);
    return hipGetLastError();
}

hipError_t launch_decode(const DevGraph &g, const DecodeArgs &a, bool f64, const KernelChoice &kc,
                         void *gscratch, int gscratch_blocks, hipStream_t s, const RowSched *rs, int num_cus,
                         const FloodSched *fs)
{
    if (a.batch <= 0) return hipSuccess;
    if (kc.name[0] == 'f') {
        if (!fs) return hipErrorInvalidValue;
        if (f64)
            return a.src == SRC_GIVEN ? launch_flood_t<double, SRC_GIVEN>(g, *fs, a, kc, gscratch, gscratch_blocks, s)
                                      : launch_flood_t<double, SRC_PHILOX>(g, *fs, a, kc, gscratch, gscratch_blocks, s);
        return a.src == SRC_GIVEN ? launch_flood_t<float, SRC_GIVEN>(g, *fs, a, kc, gscratch, gscratch_blocks, s)
                                  : launch_flood_t<float, SRC_PHILOX>(g, *fs, a, kc, gscratch, gscratch_blocks, s);
    }
    if (kc.name[0] == 'r') {
        if (!rs) return hipErrorInvalidValue;
        if (f64)
            return a.src == SRC_GIVEN ? launch_rows_dc<double, SRC_GIVEN>(g, *rs, a, kc, s, num_cus)
                                      : launch_rows_dc<double, SRC_PHILOX>(g, *rs, a, kc, s, num_cus);
        return a.src == SRC_GIVEN ? launch_rows_dc<float, SRC_GIVEN>(g, *rs, a, kc, s, num_cus)
                                  : launch_rows_dc<float, SRC_PHILOX>(g, *rs, a, kc, s, num_cus);
    }
    if (f64) {
        return a.src == SRC_GIVEN ? launch_t<double, SRC_GIVEN>(g, a, kc, gscratch, gscratch_blocks, s)
                                  : launch_t<double, SRC_PHILOX>(g, a, kc, gscratch, gscratch_blocks, s);
    }
    return a.src == SRC_GIVEN ? launch_t<float, SRC_GIVEN>(g, a, kc, gscratch, gscratch_blocks, s)
                              : launch_t<float, SRC_PHILOX>(g, a, kc, gscratch, gscratch_blocks, s);
}

int blocks_per_cu(const DevGraph &g, bool f64, const KernelChoice &kc)
{
    int nb = 0;
    hipError_t e;
    if (kc.name[0] == 'r') {
        // the row kernels of one (C) share the LDS / thread shape
        // occupancy of a representative instantiation of the same block shape
        const void *fn = f64 ? (const void *)k_decode_rows<double, SRC_PHILOX, 1, 8, 4, 2>
                             : (kc.cw_per_block == 2 ? (const void *)k_decode_rows<float, SRC_PHILOX, 2, 8, 4, 2>
                                                     : (const void *)k_decode_rows<float, SRC_PHILOX, 1, 16, 4, 2>);
        (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kc.lds_bytes);
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kc.threads, kc.lds_bytes);
    } else if (kc.name[0] == 'f') {
        const void *fn = f64 ? (const void *)k_decode_flood<double, SRC_PHILOX, 8>
                             : (const void *)k_decode_flood<float, SRC_PHILOX, 8>;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kc.threads, 0);
    } else if (kc.lds_bytes > 0) {
        const void *fn = f64 ? (const void *)k_decode_lds<double, SRC_PHILOX> : (const void *)k_decode_lds<float, SRC_PHILOX>;
        (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kc.lds_bytes);
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kc.threads, kc.lds_bytes);
    } else {
        e = f64 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_decode_global<double, SRC_PHILOX>,
                                                               kc.threads, 0)
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_decode_global<float, SRC_PHILOX>,
                                                               kc.threads, 0);
    }
    if (e != hipSuccess) { (void)hipGetLastError(); return 0; }
    return nb;
}


// ---------------------------------------------------------------- layered
// Layered positions (of np) the global kernel keeps in LDS: as many as fit
// beside the static LDS (LDPC_OPT_LAYERED_LDS_POS = P + 1 caps it at P; 1 = all in the slot).
static int layered_lds_positions(int np, size_t fsz)
{
    long P = (long)((kMaxLds - 4096) / fsz) - 1;
    if (const int v = opt(LDPC_OPT_LAYERED_LDS_POS)) P = std::min(P, (long)(v - 1));
    return (int)std::min(P, (long)np);
}

// Rows per thread per pass: the global kernel batches R rows' gathers
// (latency of the L2/Infinity Cache), the LDS kernel does one row at a time.
// fp64: 2 (DVB-S2 1 530 vs 1 470 Mbit/s at 1 and 1 425 at 3); LDPC_OPT_LAYERED_ROWS64 = 1 for A/B.
static int layered_r64() { return opt(LDPC_OPT_LAYERED_ROWS64) == 1 ? 1 : 2; }
// Threads of the global layered kernel: 1024 (4 waves per SIMD at <= 128 VGPRs,
// R = 2 rows per thread per pass in fp32, 1 in fp64) -- DVB-S2 T=50: fp32 59.4 ->
// 42.7 ms, fp64 87.4 -> 74.2 ms per 2,048 codewords against 512 threads (2 waves
// per SIMD at ~256 VGPRs, R = 4 / 2: the same rows in flight per pass, half the
// waves to hide the L2 / Infinity Cache latency); LDPC_OPT_LAYERED_THREADS = 512
// keeps the latter.
static int layered_nt() { return opt(LDPC_OPT_LAYERED_THREADS) == 512 ? 512 : 1024; }
static int layered_rows_per_pass(bool global, bool f64)
{
    if (!global) return 1;
    if (layered_nt() == 1024) return f64 ? 1 : 2;
    return f64 ? layered_r64() : 4;
}

static int layered_threads(const LayerSched &ls, int R, int cap)
{
    int t = ((ls.max_layer + R - 1) / R + 63) / 64 * 64;
    return t < 64 ? 64 : (t > cap ? cap : t);
}

KernelChoice choose_layered(const DevGraph &g, bool f64, const FloodSched &fs, const LayerSched &ls, const char *force)
{
    (void)g;
    KernelChoice kc;
    kc.cw_per_block = 1;
    kc.scratch_per_block = 0;
    kc.lds_bytes = 0;
    const size_t st = layered_state_bytes(fs, ls, f64 ? 8 : 4);
    const bool want_global = force && force[0] == 'g';
    if (st <= kMaxLds - 2048 && !want_global) {
        kc.name = "layered_lds";
        kc.lds_bytes = (int)st;
        kc.threads = layered_threads(ls, layered_rows_per_pass(false, f64), 512);
    } else {
        kc.name = "layered_global";
        kc.scratch_per_block = st;
        kc.threads = layered_threads(ls, layered_rows_per_pass(true, f64), layered_nt());
    }
    return kc;
}

template <typename F, int SRC, int DC>
static hipError_t launch_layered_t(const DecodeArgs &a, const DevGraph &g, const KernelChoice &kc,
                                   const FloodSched &fs, const LayerSched &ls, void *gs, int gblocks, hipStream_t s)
{
    if (kc.lds_bytes > 0) {
        auto fn = k_decode_layered_lds<F, SRC, DC, 1>;
        hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, kc.lds_bytes);
        if (e != hipSuccess) return e;
        int per_cu = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kc.threads, kc.lds_bytes);
        if (e != hipSuccess || per_cu < 1) per_cu = 1;
        int grid = per_cu * gblocks;   // gblocks = number of CUs here
        if (grid > a.batch) grid = a.batch;
        hipLaunchKernelGGL(fn, dim3(grid), dim3(kc.threads), kc.lds_bytes, s, a, g, fs, ls);
    } else {
        const int grid = gblocks < a.batch ? gblocks : a.batch;
        // fp64 (R = 2, fewer rows in flight per pass: latency-bound): the posteriors of
        // the highest-degree bits in LDS (DVB-S2 1 130 -> 1 470 Mbit/s at R = 1); fp32
        // (R = 4): all in the slot -- the split's dual accesses cost it more (2 230 -> 2 010)
        constexpr bool SPLIT = sizeof(F) == 8;
        const int r = layered_rows_per_pass(true, sizeof(F) == 8);
        decltype(&k_decode_layered_global<F, SRC, DC, 1, SPLIT>) fn;
        if (kc.threads > 512) {   // LDPC_LAYERED_THREADS=1024
            if constexpr (sizeof(F) == 4) fn = k_decode_layered_global<F, SRC, DC, 2, SPLIT, 1024>;
            else fn = k_decode_layered_global<F, SRC, DC, 1, SPLIT, 1024>;
        } else if constexpr (sizeof(F) == 4) {
            fn = k_decode_layered_global<F, SRC, DC, 4, SPLIT>;
        } else {
            fn = r == 2 ? k_decode_layered_global<F, SRC, DC, 2, SPLIT> : k_decode_layered_global<F, SRC, DC, 1, SPLIT>;
        }
        const int P = SPLIT ? layered_lds_positions(fs.ngroups * 64 + 1, sizeof(F)) : 0;
        const int lds = SPLIT ? (P + 1) * (int)sizeof(F) : 0;   // + LayApp's dummy slot
        hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(fn, dim3(grid), dim3(kc.threads), lds, s, a, g, fs, ls, (unsigned char *)gs,
                           kc.scratch_per_block, P);
    }
    return hipGetLastError();
}

template <typename F, int SRC>
static hipError_t launch_layered_dc(const DecodeArgs &a, const DevGraph &g, const KernelChoice &kc,
                                    const FloodSched &fs, const LayerSched &ls, void *gs, int gblocks, hipStream_t s)
{
    if (fs.dc <= 8) return launch_layered_t<F, SRC, 8>(a, g, kc, fs, ls, gs, gblocks, s);
    if (fs.dc <= 16) return launch_layered_t<F, SRC, 16>(a, g, kc, fs, ls, gs, gblocks, s);
    if (fs.dc <= kPackedMaxDc) return launch_layered_t<F, SRC, kPackedMaxDc>(a, g, kc, fs, ls, gs, gblocks, s);
    return hipErrorInvalidValue;
}

hipError_t launch_layered(const DevGraph &g, const DecodeArgs &a, bool f64, const KernelChoice &kc,
                          const FloodSched &fs, const LayerSched &ls, void *gscratch, int gscratch_blocks,
                          hipStream_t s)
{
    if (a.batch <= 0) return hipSuccess;
    if (ls.nlayers <= 0 || !ls.lptr) return hipErrorInvalidValue;
    if (f64)
        return a.src == SRC_GIVEN ? launch_layered_dc<double, SRC_GIVEN>(a, g, kc, fs, ls, gscratch, gscratch_blocks, s)
                                  : launch_layered_dc<double, SRC_PHILOX>(a, g, kc, fs, ls, gscratch, gscratch_blocks, s);
    return a.src == SRC_GIVEN ? launch_layered_dc<float, SRC_GIVEN>(a, g, kc, fs, ls, gscratch, gscratch_blocks, s)
                              : launch_layered_dc<float, SRC_PHILOX>(a, g, kc, fs, ls, gscratch, gscratch_blocks, s);
}

// Bytes of its global slot one resident codeword of the global layered kernel touches:
// the posteriors outside LDS (fp64: positions [P, NP]; fp32: all) and the packed check
// state (min1/min2 + meta per row). DVB-S2 N=64800: 1.01 MB fp64, 0.65 MB fp32.
size_t layered_resident_bytes(const FloodSched &fs, const LayerSched &ls, bool f64)
{
    const long np1 = (long)fs.ngroups * 64 + 1;
    const size_t fsz = f64 ? 8 : 4;
    const long P = f64 ? layered_lds_positions((int)np1, 8) : 0;
    return (size_t)(np1 - P) * fsz + (size_t)ls.M_pad * (2 * fsz + layered_meta_bytes(fs));
}

int layered_blocks_per_cu(bool f64, const KernelChoice &kc)
{
    int nb = 0;
    const void *fn = kc.threads > 512
                         ? (f64 ? (const void *)k_decode_layered_global<double, SRC_PHILOX, 8, 1, true, 1024>
                                : (const void *)k_decode_layered_global<float, SRC_PHILOX, 8, 2, false, 1024>)
                         : (f64 ? (const void *)k_decode_layered_global<double, SRC_PHILOX, 8, 2, true>
                                : (const void *)k_decode_layered_global<float, SRC_PHILOX, 8, 4, false>);
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kc.threads,
        f64 ? (layered_lds_positions(1 << 30, 8) + 1) * 8 : 0);
    if (e != hipSuccess) { (void)hipGetLastError(); return 0; }
    return nb;
}

}  // namespace ldpc
