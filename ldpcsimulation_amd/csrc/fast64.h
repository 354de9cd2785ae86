// fast64.h -- the fp64 fast check node and the LDS addressing helpers shared by
// the row kernels of rows_fast.hip (k_rows_fast: one codeword per 512-thread
// block) and rows_pp.hip (k_rows_pp: two codewords per 1024-thread block, check
// and bit waves in ping-pong). Reference: src/decodeMinSum.cpp:410-450,494-515.
// The premise and the exactness argument are in rows_fast.hip's header.
#pragma once
#include "minsum_common.h"

#include <hip/hip_runtime.h>
#include <cstdint>

namespace ldpc {

// 1: premise compares on the high words as u32 (measured 2.7 % slower: the
// compiler schedules the check node worse), 0: f64 compares.
#ifndef LDPC_FAST_INTPREM
#define LDPC_FAST_INTPREM 0
#endif

constexpr double kFast64Max = 0x1p1000;    // premise bound on |yq| and |c2v|
constexpr double kFast64Tiny = 0x1p-960;   // Markstein division: minima >= this (or 0)
[[maybe_unused]] constexpr uint32_t kFast64MaxHi = 0x7e700000u;    // high word of 2^1000 (low word 0)
[[maybe_unused]] constexpr uint32_t kFast64TinyHi = 0x03f00000u;   // high word of 2^-960 (low word 0)

__device__ __forceinline__ uint32_t hi32(double d) { return (uint32_t)((unsigned long long)__double_as_longlong(d) >> 32); }
__device__ __forceinline__ uint32_t lo32(double d) { return (uint32_t)(unsigned long long)__double_as_longlong(d); }
__device__ __forceinline__ double mkd(uint32_t lo, uint32_t hi)
{
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// (m1, m2) = the two smallest of |x[K0..K0+N)| by a min/max tournament.
template <int K0, int N, int DC>
__device__ __forceinline__ void two_min(const double (&x)[DC], double &m1, double &m2)
{
    if constexpr (N == 1) {
        m1 = __builtin_fabs(x[K0]);
        m2 = __builtin_huge_val();
    } else if constexpr (N == 2) {
        m1 = __builtin_fmin(__builtin_fabs(x[K0]), __builtin_fabs(x[K0 + 1]));
        m2 = __builtin_fmax(__builtin_fabs(x[K0]), __builtin_fabs(x[K0 + 1]));
    } else if constexpr (N == 3) {
        // 4 operations instead of the split's 6 (a one-element side would carry an
        // m2 = +inf that the merge has to min away: fmin(inf, x) does not fold, NaN)
        const double a = __builtin_fabs(x[K0]), b = __builtin_fabs(x[K0 + 1]), c = __builtin_fabs(x[K0 + 2]);
        const double lo = __builtin_fmin(a, b), hi = __builtin_fmax(a, b);
        m1 = __builtin_fmin(lo, c);
        m2 = __builtin_fmin(hi, __builtin_fmax(lo, c));
    } else {
        constexpr int L = N / 2;
        double l1, l2, r1, r2;
        two_min<K0, L, DC>(x, l1, l2);
        two_min<K0 + L, N - L, DC>(x, r1, r2);
        m1 = __builtin_fmin(l1, r1);
        m2 = __builtin_fmin(__builtin_fmax(l1, r1), __builtin_fmin(l2, r2));
    }
}

template <int VAR, bool FDIV>
__device__ __forceinline__ double norm64(double m, double alpha, double rcp, double delta)
{
    if constexpr (VAR == V_NMS) {
        if constexpr (FDIV) {
            const double q = m * rcp;
            return __builtin_fma(__builtin_fma(-q, alpha, m), rcp, q);
        } else {
            return m / alpha;                                       // :498 (IEEE division)
        }
    } else if constexpr (VAR == V_OMS) {
        const double t = m - delta;                                 // :509
        return t > 0.0 ? t : 0.0;                                   // :513
    } else {
        return m;
    }
}

// fp64 fast check node over edges [0, DC) of the arrays (extent DCA >= DC; the
// entries past DC are not touched). xin: the app values gathered for the row's
// edges (padding edges read +inf); pv: in = c2v sent last iteration, out = the
// new c2v. Returns false when the premise may fail for the next iteration (or
// failed for this one's division).
// VALU instructions the scheduler places ahead of each edge's store (ORDER).
#ifndef LDPC_FAST64_CMPFIRST
#define LDPC_FAST64_CMPFIRST 0
#endif
#ifndef LDPC_FAST64_STORE_VALU
#define LDPC_FAST64_STORE_VALU 3
#endif
// ACC (the ping-pong kernel): instead of the f64 premise compare, the row folds
// hi32(M2) into the maximum *pacc (one v_max_u32; M2 >= +0 or NaN, so M2 < 2^1000 <=>
// hi32(M2) < kFast64MaxHi as u32, NaN and inf above it), and a tiny minimum forces
// *pacc to ~0; the caller tests it (per row, or once per codeword when *pacc is a
// sticky per-slot maximum: rows_pp.hip LDPC_PP_STICKY). Same set of re-decoded codewords.
struct NoSink {
    __device__ __forceinline__ void operator()(int, const Pack<double, 1> &) const {}
};
// sink(k, message) is called as each new message is formed (a store of it, say);
// with ORDER the scheduler is asked to keep that per-edge order (the selects of
// edge k, then its store), so the stores start while later edges are computed
// instead of trailing the whole row.
template <int DC, int VAR, bool FDIV, int DCA, typename Sink = NoSink, bool ORDER = false, bool ACC = false>
__device__ __forceinline__ bool cn_fast64(const Pack<double, 1> (&xin)[DCA], Pack<double, 1> (&pv)[DCA], double alpha,
                                          double rcp, double delta, Sink sink = Sink(), uint32_t *pacc = nullptr)
{
    static_assert(DC >= 1 && DC <= DCA, "cn_fast64 degree");
    constexpr uint32_t SIGN = 0x80000000u;
    double x[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) x[k] = xin[k].v[0] - pv[k].v[0];   // v2c (:469)
    double mn1, mn2;
    two_min<0, DC, DC>(x, mn1, mn2);
    uint32_t par = 0;
#pragma unroll
    for (int k = 0; k + 1 < DC; k += 2) par = __builtin_amdgcn_bitop3_b32(par, hi32(x[k]), hi32(x[k + 1]), 0x96);
    if (DC & 1) par ^= hi32(x[DC - 1]);
    const double M1 = norm64<VAR, FDIV>(mn1, alpha, rcp, delta), M2 = norm64<VAR, FDIV>(mn2, alpha, rcp, delta);
    // M2 < 2^1000 (also false for NaN; M1 <= M2 covers the row). The u32 form compares the
    // high words (M2 >= +0; 2^1000's low word is 0).
    bool ok = true;
    if constexpr (ACC) {
        const uint32_t h2 = hi32(M2);
        *pacc = *pacc > h2 ? *pacc : h2;   // v_max_u32
    } else {
#if LDPC_FAST_INTPREM
        ok = hi32(M2) < kFast64MaxHi;
#else
        ok = M2 < kFast64Max;
#endif
    }
    if constexpr (VAR == V_NMS && FDIV) {
        // minima in (0, 2^-960): the one-FMA division may round wrongly (wave-uniform skip, rare)
#if LDPC_FAST_INTPREM
        if (__builtin_amdgcn_ballot_w64(hi32(mn1) < kFast64TinyHi)) {
#else
        if (__builtin_amdgcn_ballot_w64(mn1 < kFast64Tiny)) {
#endif
            if constexpr (ACC) {
                uint32_t t = *pacc;
                asm volatile(";");   // a side effect: the rare path stays a branch (not if-converted)
                if ((mn1 > 0.0 && mn1 < kFast64Tiny) | (mn2 > 0.0 && mn2 < kFast64Tiny)) t = ~0u;
                *pacc = t;
            } else {
                ok &= !(mn1 > 0.0 && mn1 < kFast64Tiny) & !(mn2 > 0.0 && mn2 < kFast64Tiny);
            }
        }
    }
    uint32_t mk1 = SIGN, mk2 = SIGN;
    if constexpr (VAR == V_OMS) {   // a zeroed message is +0, and sgn(-0.0) = +1 (:511-513)
        mk1 = (M1 > 0.0 && mn1 != 0.0) ? SIGN : 0u;
        mk2 = (M2 > 0.0 && mn2 != 0.0) ? SIGN : 0u;
    }
    uint32_t s1 = hi32(M1) ^ (par & mk1), s2 = hi32(M2) ^ (par & mk2);
    asm("" : "+v"(s1), "+v"(s2));   // keep the parity out of the per-edge select
    const uint32_t l1 = lo32(M1), l2 = lo32(M2);
    // |v2c_k| == min1 as one v_cmp_eq_f64 with the abs source modifier, used as the select mask;
    // CMPFIRST: every edge's mask formed ahead of the per-edge selects and stores (SGPR pairs),
    // so no select waits on the compare just issued (the f64-compare -> mask-read wait states)
    [[maybe_unused]] uint64_t eqm[DC];
    if constexpr (LDPC_FAST64_CMPFIRST) {
#pragma unroll
        for (int k = 0; k < DC; ++k) eqm[k] = __builtin_amdgcn_fcmp(__builtin_fabs(x[k]), mn1, 1);
        if constexpr (ORDER) __builtin_amdgcn_sched_group_barrier(0x2, DC, 0);
    }
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const bool eq = __builtin_amdgcn_inverse_ballot_w64(
            LDPC_FAST64_CMPFIRST ? eqm[k] : __builtin_amdgcn_fcmp(__builtin_fabs(x[k]), mn1, 1));
        const uint32_t h = eq ? s2 : s1, l = eq ? l2 : l1;
        const uint32_t m = (VAR == V_OMS) ? (eq ? mk2 : mk1) : SIGN;
        pv[k].v[0] = mkd(l, __builtin_amdgcn_bitop3_b32(h, hi32(x[k]), m, 0x78));   // h ^ (v2c_k & m)
        sink(k, pv[k]);
        if constexpr (ORDER) {
            __builtin_amdgcn_sched_group_barrier(0x2, LDPC_FAST64_STORE_VALU, 0);   // VALU: compare, selects, sign merge, address
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);   // DS write: this edge's store
        }
    }
    return ok;
}

// LDS byte address of 16-bit entry k of a packed schedule row: base + 8 * entry,
// one v_mad_u32_u16 (op_sel picks the high half) instead of extract + shift-add.
template <int DC>
__device__ __forceinline__ uint32_t addr8(const uint32_t (&w)[DC / 2], int k, uint32_t base)
{
    uint32_t a;
    if (k & 1)
        asm("v_mad_u32_u16 %0, %1, 8, %2 op_sel:[1,0,0,0]" : "=v"(a) : "v"(w[k >> 1]), "v"(base));
    else
        asm("v_mad_u32_u16 %0, %1, 8, %2" : "=v"(a) : "v"(w[k >> 1]), "v"(base));
    return a;
}
// LDPC_ADDR8(DC, w, k, base, n, site): addr8 with the entry bounds-checked (entry < n)
// in LDPC_CHECK builds (check.h); in the product build exactly addr8<DC>(w, k, base)
// (n and site are not evaluated).
#ifdef LDPC_CHECK
template <int DC>
__device__ __forceinline__ uint32_t addr8c(const uint32_t (&w)[DC / 2], int k, uint32_t base, uint32_t n,
                                           unsigned site)
{
    const uint32_t e = (w[k >> 1] >> ((k & 1) * 16)) & 0xffffu;
    return base + 8u * LDPC_CHK(e, n, site);
}
#define LDPC_ADDR8(DC, w, k, base, n, site) addr8c<DC>(w, k, base, n, site)
#else
#define LDPC_ADDR8(DC, w, k, base, n, site) addr8<DC>(w, k, base)
#endif
// LDS accesses by 32-bit LDS address (no generic-pointer arithmetic: the
// address from addr8 goes straight into the ds_read / ds_write).
__device__ __forceinline__ uint32_t lds_addr_of(const void *p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
template <int B> struct LdsWord;
template <> struct LdsWord<4> { using T = unsigned int; };
template <> struct LdsWord<8> { using T = unsigned long long; };
template <> struct LdsWord<16> { using T = unsigned int __attribute__((ext_vector_type(4))); };
template <typename P>
__device__ __forceinline__ P lds_at(uint32_t addr)
{
    using U = typename LdsWord<sizeof(P)>::T;
    const U u = *(const __attribute__((address_space(3))) U *)(uintptr_t)addr;
    P p;
    __builtin_memcpy(&p, &u, sizeof(P));
    return p;
}
template <typename P>
__device__ __forceinline__ void lds_put(uint32_t addr, const P &v)
{
    using U = typename LdsWord<sizeof(P)>::T;
    U u;
    __builtin_memcpy(&u, &v, sizeof(P));
    *(__attribute__((address_space(3))) U *)(uintptr_t)addr = u;
}


}  // namespace ldpc
