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

// s += r for every codeword of a pack (one v_pk_add_f32 for two fp32 codewords).
template <typename F, int C>
__device__ __forceinline__ void padd(Pack<F, C> &s, const Pack<F, C> &r)
{
#pragma unroll
    for (int c = 0; c < C; ++c) s.v[c] += r.v[c];
}
template <>
__device__ __forceinline__ void padd<float, 2>(Pack<float, 2> &s, const Pack<float, 2> &r)
{
    using V = float __attribute__((ext_vector_type(2)));
    V a, b;
    __builtin_memcpy(&a, &s, sizeof(V));
    __builtin_memcpy(&b, &r, sizeof(V));
    a += b;
    __builtin_memcpy(&s, &a, sizeof(V));
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
template <typename F, int C, int NACT, int U, int CPT>
__device__ __forceinline__ void vn_load(const Pack<F, C> *c2v, const int (&base)[CPT], int k, Pack<F, C> (&r)[NACT][U])
{
#pragma unroll
    for (int i = 0; i < NACT; ++i)
#pragma unroll
        for (int u = 0; u < U; ++u) r[i][u] = c2v[base[i] + (k + u) * 64];
}
template <typename F, int C, int NACT, int U, int CPT>
__device__ __forceinline__ void vn_add(const Pack<F, C> (&r)[NACT][U], Pack<F, C> (&sum)[CPT])
{
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < NACT; ++i) padd(sum[i], r[i][u]);
}
template <typename F, int C, int NACT, int CPT>
__device__ __forceinline__ void vn_phase(const Pack<F, C> *c2v, const int (&base)[CPT], int &k, int kend,
                                         Pack<F, C> (&sum)[CPT])
{
    constexpr int U = NACT >= 3 ? LDPC_VN_U3 : LDPC_VN_U1;   // packs in flight per step: U * NACT
    if constexpr (LDPC_VN_PIPE) {
        // two steps in flight: step s+1's reads are issued before step s is added
        int n = (kend - k) / U;   // wave-uniform
        if (n > 0) {
            Pack<F, C> ra[NACT][U], rb[NACT][U];
            vn_load<F, C, NACT, U, CPT>(c2v, base, k, ra);
            for (;;) {
                if (n >= 2) vn_load<F, C, NACT, U, CPT>(c2v, base, k + U, rb);
                vn_add<F, C, NACT, U, CPT>(ra, sum);
                k += U;
                if (--n == 0) break;
                if (n >= 2) vn_load<F, C, NACT, U, CPT>(c2v, base, k + U, ra);
                vn_add<F, C, NACT, U, CPT>(rb, sum);
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
            for (int u = 0; u < U; ++u) r[i][u] = c2v[base[i] + (k + u) * 64];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int i = 0; i < NACT; ++i) padd(sum[i], r[i][u]);
    }
    for (; k < kend; ++k) {
        Pack<F, C> r[NACT];
#pragma unroll
        for (int i = 0; i < NACT; ++i) r[i] = c2v[base[i] + k * 64];
#pragma unroll
        for (int i = 0; i < NACT; ++i) padd(sum[i], r[i]);
    }
}
template <typename F, int C, int NACT, int CPT>
__device__ __forceinline__ void vn_phases(const Pack<F, C> *c2v, const int (&base)[CPT], const int (&gd)[CPT], int &k,
                                          Pack<F, C> (&sum)[CPT])
{
    vn_phase<F, C, NACT, CPT>(c2v, base, k, gd[NACT - 1], sum);
    if constexpr (NACT > 1) vn_phases<F, C, NACT - 1, CPT>(c2v, base, gd, k, sum);
}

}  // namespace ldpc
