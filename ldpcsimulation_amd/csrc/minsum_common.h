// minsum_common.h -- device helpers shared by the min-sum kernels
// (kernels.hip: generic/flood/layered/row kernels; rows_fast.hip: the
// fast-path row kernel). Reference: C_implementations/src/decodeMinSum.cpp.
#pragma once
#include "kernels.h"
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ldpc {

enum { V_MS = 0, V_NMS = 1, V_OMS = 2 };


template <typename F> struct RowState;
template <> struct __attribute__((aligned(16))) RowState<float> { float m1, m2; uint64_t meta; };
template <> struct __attribute__((aligned(16))) RowState<double> { double m1, m2; uint64_t meta, pad; };

template <typename F> __device__ __forceinline__ F dinf();
template <> __device__ __forceinline__ float dinf<float>() { return __builtin_huge_valf(); }
template <> __device__ __forceinline__ double dinf<double>() { return __builtin_huge_val(); }
__device__ __forceinline__ float dabs(float x) { return __builtin_fabsf(x); }
__device__ __forceinline__ double dabs(double x) { return __builtin_fabs(x); }
__device__ __forceinline__ float dfloor(float x) { return __builtin_floorf(x); }
// IEEE minNum: a NaN operand yields the other operand.
__device__ __forceinline__ float dmin(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ double dmin(double a, double b) { return __builtin_fmin(a, b); }
__device__ __forceinline__ double dfloor(double x) { return __builtin_floor(x); }

// sgn() of the reference (:518-523): x >= 0 -> +1 (so -0.0 -> +1, NaN -> -1).
template <typename F> __device__ __forceinline__ F dsgn(F x) { return x >= F(0) ? F(1) : F(-1); }

// quantize() (:480-489), same operation order.
template <typename F>
__device__ __forceinline__ F quantize(F x, F ymax, F nq)
{
    if (dabs(x) > ymax) return dsgn(x) * ymax;
    F q = dsgn(x) * (dfloor(dabs(x) * (nq - F(1)) / (F(2) * ymax)) + F(0)) * (F(2) * ymax / (nq - F(1)));
    if (q == F(0)) q = dsgn(x) * F(2) * ymax / (nq - F(1));
    return q;
}

template <typename F>
__device__ __forceinline__ F front_end(F y, const DecodeArgs &a)
{
    F q = y;
    if (a.quantize) q = quantize<F>(y, (F)a.ymax, (F)a.nq);
    if (a.saturate) {
        const F ym = (F)a.ymax;
        if (q > ym) q = ym;
        if (q < -ym) q = -ym;
    }
    return q;
}

// Diagnostic phase timing (-DLDPC_STAMPS builds only; never in the shipped kernel).
#ifdef LDPC_STAMPS
#define STAMP(var) unsigned long long var = (threadIdx.x == 0) ? __builtin_amdgcn_s_memtime() : 0ull
#else
#define STAMP(var) [[maybe_unused]] constexpr unsigned long long var = 0ull
#endif

template <int DC> struct MetaOf { using T = uint32_t; static constexpr int SH = 5; };
template <> struct MetaOf<32> { using T = uint64_t; static constexpr int SH = 6; };

template <int DC>
__device__ __forceinline__ int u16_at(const uint32_t (&w)[DC / 2], int k)
{
    return (int)((w[k >> 1] >> ((k & 1) * 16)) & 0xffffu);
}

// The C codewords of a block are interleaved in LDS: one Pack = the same
// element of all C codewords, so every gather/scatter moves C values
// (ds_read_b64 / ds_write_b64 for two fp32 codewords or one fp64).
template <typename F, int C> struct __attribute__((aligned(sizeof(F) * C))) Pack { F v[C]; };

// Plain IEEE fp32 add / subtract as one v_add_f32 / v_sub_f32 each. On gfx950 the
// packed v_pk_add_f32 that -O3's SLP vectoriser forms from two adjacent adds issues
// far slower than the two plain adds (MI355X_MICROARCH constants table; the fp32
// ping-pong bit role measured 2 971 vs 2 097 cycles per interval for fp64's
// v_add_f64 at the same instruction count), so the two codewords of an fp32 pair
// are added separately. Same rounding (RNE), same values.
__device__ __forceinline__ float fadd32(float a, float b)
{
    float r;
    asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float fsub32(float a, float b)
{
    float r;
    asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// s += r for every codeword of a pack. PK (fp32 pairs only): one packed v_pk_add_f32
// -- the fp32 row kernel (kernels.hip k_decode_rows) keeps it, 8.8 vs 10.0 ms per bench
// launch for two plain adds there -- else two v_add_f32 (the ping-pong and rows_fast
// kernels: a packed add issues slower than the two plain ones on gfx950). The choice
// is a template parameter, so one inline function never means two things in two
// translation units. Same values either way.
template <bool PK = false, typename F, int C>
__device__ __forceinline__ void padd(Pack<F, C> &s, const Pack<F, C> &r)
{
    if constexpr (sizeof(F) == 4 && C == 2) {
        if constexpr (PK) {
            using V = float __attribute__((ext_vector_type(2)));
            V a, b;
            __builtin_memcpy(&a, &s, sizeof(V));
            __builtin_memcpy(&b, &r, sizeof(V));
            a += b;
            __builtin_memcpy(&s, &a, sizeof(V));
        } else {
            s.v[0] = fadd32(s.v[0], r.v[0]);
            s.v[1] = fadd32(s.v[1], r.v[1]);
        }
    } else {
#pragma unroll
        for (int c = 0; c < C; ++c) s.v[c] += r.v[c];
    }
}

// Bit nodes, edges k in [k, kend) of the first NACT slots (every one of them has
// group degree >= kend): sum_i += c2v[base_i + k*64] (c2v already offset by the
// lane, base_i wave-uniform), in edge order per slot, U edges of every slot in
// flight per step. (Steps sized exactly to the remainder were measured slower:
// the extra unrolled variants cost more in instruction fetch than they save.)
#ifndef LDPC_VN_U3
#define LDPC_VN_U3 2
#endif
#ifndef LDPC_VN_U1
#define LDPC_VN_U1 4
#endif
#ifndef LDPC_VN_PIPE
#define LDPC_VN_PIPE 0
#endif
// lim / site: the bound of the slot index base[i] + k*64 relative to c2v and the check
// site, for LDPC_CHECK builds (check.h); unused otherwise.
template <typename F, int C, int NACT, int U, int CPT>
__device__ __forceinline__ void vn_load(const Pack<F, C> *c2v, const int (&base)[CPT], int k, Pack<F, C> (&r)[NACT][U],
                                        int lim, unsigned site)
{
    (void)lim;
    (void)site;
#pragma unroll
    for (int i = 0; i < NACT; ++i)
#pragma unroll
        for (int u = 0; u < U; ++u) r[i][u] = c2v[LDPC_CHK(base[i] + (k + u) * 64, lim, site)];
}
template <typename F, int C, int NACT, int U, int CPT, bool PK = false>
__device__ __forceinline__ void vn_add(const Pack<F, C> (&r)[NACT][U], Pack<F, C> (&sum)[CPT])
{
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < NACT; ++i) padd<PK>(sum[i], r[i][u]);
}
template <typename F, int C, int NACT, int CPT, bool PK = false>
__device__ __forceinline__ void vn_phase(const Pack<F, C> *c2v, const int (&base)[CPT], int &k, int kend,
                                         Pack<F, C> (&sum)[CPT], int lim, unsigned site)
{
    (void)lim;
    (void)site;
    constexpr int U = NACT >= 3 ? LDPC_VN_U3 : LDPC_VN_U1;   // packs in flight per step: U * NACT
    if constexpr (LDPC_VN_PIPE) {
        // two steps in flight: step s+1's reads are issued before step s is added
        int n = (kend - k) / U;   // wave-uniform
        if (n > 0) {
            Pack<F, C> ra[NACT][U], rb[NACT][U];
            vn_load<F, C, NACT, U, CPT>(c2v, base, k, ra, lim, site);
            for (;;) {
                if (n >= 2) vn_load<F, C, NACT, U, CPT>(c2v, base, k + U, rb, lim, site);
                vn_add<F, C, NACT, U, CPT, PK>(ra, sum);
                k += U;
                if (--n == 0) break;
                if (n >= 2) vn_load<F, C, NACT, U, CPT>(c2v, base, k + U, ra, lim, site);
                vn_add<F, C, NACT, U, CPT, PK>(rb, sum);
                k += U;
                if (--n == 0) break;
            }
        }
    }
    for (; k + U <= kend; k += U) {
        Pack<F, C> r[NACT][U];
#pragma unroll
        for (int i = 0; i < NACT; ++i)
#pragma unroll
            for (int u = 0; u < U; ++u) r[i][u] = c2v[LDPC_CHK(base[i] + (k + u) * 64, lim, site)];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int i = 0; i < NACT; ++i) padd<PK>(sum[i], r[i][u]);
    }
    for (; k < kend; ++k) {
        Pack<F, C> r[NACT];
#pragma unroll
        for (int i = 0; i < NACT; ++i) r[i] = c2v[LDPC_CHK(base[i] + k * 64, lim, site)];
#pragma unroll
        for (int i = 0; i < NACT; ++i) padd<PK>(sum[i], r[i]);
    }
}
template <typename F, int C, int NACT, int CPT, bool PK = false>
__device__ __forceinline__ void vn_phases(const Pack<F, C> *c2v, const int (&base)[CPT], const int (&gd)[CPT], int &k,
                                          Pack<F, C> (&sum)[CPT], int lim = 0x7fffffff, unsigned site = 0)
{
    vn_phase<F, C, NACT, CPT, PK>(c2v, base, k, gd[NACT - 1], sum, lim, site);
    if constexpr (NACT > 1) vn_phases<F, C, NACT - 1, CPT, PK>(c2v, base, gd, k, sum, lim, site);
}

// Check node, fast fp32 path (MS, and NMS with a verified reciprocal). Exact
// whenever every c2v magnitude entering the iteration is below 1e30: then
// every app and v2c is finite (|app| <= |yq| + 255*1e30 < FLT_MAX), no NaN
// occurs, and
//   m2' = med3(m1, |x|, m2), m1' = min(m1, |x|)
// is exactly the reference's update (m1 <= m2 always). app is never -0 (yq is
// canonicalised, see the kernel), so v2c = app - c2v is never -0 either and
// its sign bit is the reference's sgn(v2c) (:518-523): the row parity is the
// xor of the v2c bit patterns, and c2v_k = (m1|m2) with sign bit
// parity ^ sign(v2c_k) (a zero magnitude keeps that sign, as prod*min*sgn
// does). Padding edges read +inf: sign +, never below m2. The new messages
// are always committed; the return value is false when one of them reaches
// 1e30 (or is inf), and the caller hands the block to the exact path before
// the next iteration (keeping the premise true).
// Edges [0, DC) of arrays of extent DCA >= DC (the entries past DC are not touched).
// PK: the v2c of a pair as one v_pk_add_f32 (see padd).
template <int DC, int C, int DCA = DC, bool PK = false>
__device__ __forceinline__ bool cn_fast(const Pack<float, C> (&xin)[DCA], Pack<float, C> (&pv)[DCA], bool nms,
                                        float alpha, float rcp)
{
    static_assert(DC >= 1 && DC <= DCA, "cn_fast degree");
    constexpr uint32_t SIGN = 0x80000000u;
    using V = float __attribute__((ext_vector_type(C)));
    V x[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if constexpr (PK) {
            V xi, pi;
            __builtin_memcpy(&xi, &xin[k], sizeof(V));
            __builtin_memcpy(&pi, &pv[k], sizeof(V));
            x[k] = xi - pi;                                                         // v2c (:469)
        } else {
#pragma unroll
            for (int c = 0; c < C; ++c) x[k][c] = fsub32(xin[k].v[c], pv[k].v[c]);   // v2c (:469), one v_sub_f32 each
        }
    }
    bool ok = true;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        // (m1, m2) = the two smallest |v2c| of the row, by groups of three
        // (lo, sec) = (min3, med3), merged with sec' = med3(lo, lo_g, min(sec, sec_g))
        // (or, for three groups, min(med3(lo_1..3), min3(sec_1..3))).
        constexpr int G = (DC + 2) / 3;
        float lo[G], sec[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int k0 = 3 * g, n = DC - k0 < 3 ? DC - k0 : 3;
            const float a0 = __builtin_fabsf(x[k0][c]);
            if (n == 3) {
                const float a1 = __builtin_fabsf(x[k0 + 1][c]), a2 = __builtin_fabsf(x[k0 + 2][c]);
                lo[g] = __builtin_fminf(__builtin_fminf(a0, a1), a2);
                sec[g] = __builtin_amdgcn_fmed3f(a0, a1, a2);
            } else if (n == 2) {
                const float a1 = __builtin_fabsf(x[k0 + 1][c]);
                lo[g] = __builtin_fminf(a0, a1);
                sec[g] = __builtin_fmaxf(a0, a1);
            } else {
                lo[g] = a0;
                sec[g] = __builtin_huge_valf();
            }
        }
        float mn1, mn2;
        if constexpr (G == 3) {
            mn1 = __builtin_fminf(__builtin_fminf(lo[0], lo[1]), lo[2]);
            mn2 = __builtin_fminf(__builtin_amdgcn_fmed3f(lo[0], lo[1], lo[2]),
                                  __builtin_fminf(__builtin_fminf(sec[0], sec[1]), sec[2]));
        } else {
            mn1 = lo[0];
            mn2 = sec[0];
#pragma unroll
            for (int g = 1; g < G; ++g) {
                mn2 = __builtin_amdgcn_fmed3f(mn1, lo[g], __builtin_fminf(mn2, sec[g]));
                mn1 = __builtin_fminf(mn1, lo[g]);
            }
        }
        uint32_t par = 0;
#pragma unroll
        for (int k = 0; k + 1 < DC; k += 2)                                   // xor3
            par = __builtin_amdgcn_bitop3_b32(par, __float_as_uint(x[k][c]), __float_as_uint(x[k + 1][c]), 0x96);
        if (DC & 1) par ^= __float_as_uint(x[DC - 1][c]);
        float M1 = mn1, M2 = mn2;
        if (nms) {   // x/alpha = q + (x - q*alpha)*r, q = x*r (verified for all finite x); inf/alpha = inf
            const float q1 = mn1 * rcp, q2 = mn2 * rcp;
            const float d1 = __builtin_fmaf(__builtin_fmaf(-q1, alpha, mn1), rcp, q1);
            const float d2 = __builtin_fmaf(__builtin_fmaf(-q2, alpha, mn2), rcp, q2);
            M1 = mn1 < __builtin_huge_valf() ? d1 : mn1;
            M2 = mn2 < __builtin_huge_valf() ? d2 : mn2;
        }
        ok &= M2 < 1e30f;
        uint32_t s1 = __float_as_uint(M1) ^ (par & SIGN), s2 = __float_as_uint(M2) ^ (par & SIGN);
        asm("" : "+v"(s1), "+v"(s2));   // keep the parity out of the per-edge select
        // all compares first (separate lane masks), then the selects: no
        // compare->select hazard wait states between neighbours
        bool eq[DC];
#pragma unroll
        for (int k = 0; k < DC; ++k) eq[k] = __builtin_fabsf(x[k][c]) == mn1;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            const uint32_t m = eq[k] ? s2 : s1;
            // m ^ (v2c_k & SIGN)
            pv[k].v[c] = __uint_as_float(__builtin_amdgcn_bitop3_b32(m, __float_as_uint(x[k][c]), SIGN, 0x78));
        }
    }
    return ok;
}

// cn_fast for an fp32 pair (C = 2) with the outputs produced edge by edge: both
// codewords' minima, parity and normalised magnitudes first, then for each edge k
// the two compares and selects and sink(k, message) -- with ORDER the scheduler is
// asked to keep that per-edge order (the ping-pong kernel's scatters then overlap
// the later edges' selects, as cn_fast64's do). Same values as cn_fast<DC, 2>.
struct NoSink32 {
    __device__ __forceinline__ void operator()(int, const Pack<float, 2> &) const {}
};
#ifndef LDPC_FAST32_STORE_VALU
#define LDPC_FAST32_STORE_VALU 4
#endif
template <int DC, int DCA = DC, typename Sink = NoSink32, bool ORDER = false>
__device__ __forceinline__ bool cn_fast_pair(const Pack<float, 2> (&xin)[DCA], Pack<float, 2> (&pv)[DCA], bool nms,
                                             float alpha, float rcp, Sink sink = Sink())
{
    static_assert(DC >= 1 && DC <= DCA, "cn_fast_pair degree");
    constexpr uint32_t SIGN = 0x80000000u;
    float x[2][DC];
#pragma unroll
    for (int k = 0; k < DC; ++k)
#pragma unroll
        for (int c = 0; c < 2; ++c) x[c][k] = fsub32(xin[k].v[c], pv[k].v[c]);   // v2c (:469)
    bool ok = true;
    float mn1[2], s1f[2], s2f[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        constexpr int G = (DC + 2) / 3;
        float lo[G], sec[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int k0 = 3 * g, n = DC - k0 < 3 ? DC - k0 : 3;
            const float a0 = __builtin_fabsf(x[c][k0]);
            if (n == 3) {
                const float a1 = __builtin_fabsf(x[c][k0 + 1]), a2 = __builtin_fabsf(x[c][k0 + 2]);
                lo[g] = __builtin_fminf(__builtin_fminf(a0, a1), a2);
                sec[g] = __builtin_amdgcn_fmed3f(a0, a1, a2);
            } else if (n == 2) {
                const float a1 = __builtin_fabsf(x[c][k0 + 1]);
                lo[g] = __builtin_fminf(a0, a1);
                sec[g] = __builtin_fmaxf(a0, a1);
            } else {
                lo[g] = a0;
                sec[g] = __builtin_huge_valf();
            }
        }
        float m1, m2;
        if constexpr (G == 3) {
            m1 = __builtin_fminf(__builtin_fminf(lo[0], lo[1]), lo[2]);
            m2 = __builtin_fminf(__builtin_amdgcn_fmed3f(lo[0], lo[1], lo[2]),
                                 __builtin_fminf(__builtin_fminf(sec[0], sec[1]), sec[2]));
        } else {
            m1 = lo[0];
            m2 = sec[0];
#pragma unroll
            for (int g = 1; g < G; ++g) {
                m2 = __builtin_amdgcn_fmed3f(m1, lo[g], __builtin_fminf(m2, sec[g]));
                m1 = __builtin_fminf(m1, lo[g]);
            }
        }
        uint32_t par = 0;
#pragma unroll
        for (int k = 0; k + 1 < DC; k += 2)
            par = __builtin_amdgcn_bitop3_b32(par, __float_as_uint(x[c][k]), __float_as_uint(x[c][k + 1]), 0x96);
        if (DC & 1) par ^= __float_as_uint(x[c][DC - 1]);
        float M1 = m1, M2 = m2;
        if (nms) {   // x/alpha = q + (x - q*alpha)*r, q = x*r (verified for all finite x); inf/alpha = inf
            const float q1 = m1 * rcp, q2 = m2 * rcp;
            const float d1 = __builtin_fmaf(__builtin_fmaf(-q1, alpha, m1), rcp, q1);
            const float d2 = __builtin_fmaf(__builtin_fmaf(-q2, alpha, m2), rcp, q2);
            M1 = m1 < __builtin_huge_valf() ? d1 : m1;
            M2 = m2 < __builtin_huge_valf() ? d2 : m2;
        }
        ok &= M2 < 1e30f;
        uint32_t a1 = __float_as_uint(M1) ^ (par & SIGN), a2 = __float_as_uint(M2) ^ (par & SIGN);
        asm("" : "+v"(a1), "+v"(a2));   // keep the parity out of the per-edge select
        mn1[c] = m1;
        s1f[c] = __uint_as_float(a1);
        s2f[c] = __uint_as_float(a2);
    }
#pragma unroll
    for (int k = 0; k < DC; ++k) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint32_t m = (__builtin_fabsf(x[c][k]) == mn1[c]) ? __float_as_uint(s2f[c]) : __float_as_uint(s1f[c]);
            pv[k].v[c] = __uint_as_float(__builtin_amdgcn_bitop3_b32(m, __float_as_uint(x[c][k]), SIGN, 0x78));
        }
        sink(k, pv[k]);
        if constexpr (ORDER) {
            __builtin_amdgcn_sched_group_barrier(0x2, LDPC_FAST32_STORE_VALU, 0);   // 2 compares, 2 selects, 2 merges, address
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        }
    }
    return ok;
}

}  // namespace ldpc
