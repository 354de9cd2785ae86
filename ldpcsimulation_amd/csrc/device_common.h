// device_common.h -- device helpers shared by the decoder kernels
// (kernels.hip: min-sum; gdbf.hip: GDBF / NGDBF bit flipping).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "check.h"

namespace ldpc {

// ---------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. SC'11) + Box-Muller: 4 normals per call.
// MAD64: the two 32x32->64 products of a round as v_mad_u64_u32 (same values
// either way; 20 instead of 40 quarter-rate multiplies per call). Used by gdbf.hip,
// where Philox runs every iteration, and by the ping-pong kernel's channel (12.54-12.58
// vs 12.60-12.66 ms); off in the fp64 one-codeword row kernel, where the 64-bit form
// costs 2.5 % through register allocation (16.10 vs 16.52 ms, 3 interleaved rounds).
// ---------------------------------------------------------------------
template <bool MAD64 = false>
__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1, uint32_t out[4])
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t lo0, hi0, lo1, hi1;
        if constexpr (MAD64) {
            const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
            lo0 = (uint32_t)p0; hi0 = (uint32_t)(p0 >> 32);
            lo1 = (uint32_t)p1; hi1 = (uint32_t)(p1 >> 32);
        } else {
            lo0 = 0xD2511F53u * c0; hi0 = __umulhi(0xD2511F53u, c0);
            lo1 = 0xCD9E8D57u * c2; hi1 = __umulhi(0xCD9E8D57u, c2);
        }
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// Uniforms in (0,1): (u + 1/2) * 2^-32; n0, n1 = sqrt(-2 ln r) (cos, sin)(2 pi a).
// The transform runs on the SIMD's own transcendental instructions: v_log_f32 (log2, so
// -2 ln r = -2 ln 2 * log2 r), v_sqrt_f32, and v_sin_f32 / v_cos_f32, whose argument is in
// revolutions (sin(2 pi a) is v_sin_f32(a), a in (0, 1)): five instructions where OCML's
// correctly-rounded logf / sqrtf / sincospif took ~100 with their range and denormal
// branches. r >= 2^-33 is a normal float, so the hardware log is within an ulp or two; the
// normals differ from the OCML transform's in the last bits only, which no Gaussian
// statistic resolves (test_channel_noise_statistics, the FER z-tests). LDPC_BM_OCML=1
// (variant builds) keeps the OCML transform for A/B.
#ifndef LDPC_BM_OCML
#define LDPC_BM_OCML 0
#endif
#if LDPC_BM_OCML != 0 && !defined(LDPC_AB_BUILD)
#error "LDPC_BM_OCML changes the noise the parity tests pin: variant builds only"
#endif
__device__ __forceinline__ void box_muller(uint32_t ua, uint32_t ur, float &n0, float &n1)
{
    const float a = (float)ua * 2.3283064365386963e-10f + 1.1641532182693481e-10f;
    const float r = (float)ur * 2.3283064365386963e-10f + 1.1641532182693481e-10f;
    if constexpr (!LDPC_BM_OCML) {
        const float rad = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(r));
        n0 = rad * __builtin_amdgcn_cosf(a);
        n1 = rad * __builtin_amdgcn_sinf(a);
    } else {
        const float rad = sqrtf(-2.0f * logf(r));
        float s, c;
        sincospif(2.0f * a, &s, &c);
        n0 = rad * c;
        n1 = rad * s;
    }
}
// The fp64 channel's normals: the fp32 transform above, widened to double (SURVEY
// §8 a2: Philox4x32-10 + Box-Muller in fp32). The decoders compute in fp64 on the
// widened samples y = c (1 + sigma n) exactly as on any given y; only the noise
// generator's own precision is fp32 (fp64 log / sqrt / sincospi cost 2.6 % of the fp64
// headline launch: 12.27-12.31 vs 12.60-12.66 ms). LDPC_BM64=1 (variant builds) keeps
// the fp64 transform.
#ifndef LDPC_BM64
#define LDPC_BM64 0
#endif
#if LDPC_BM64 != 0 && !defined(LDPC_AB_BUILD)
#error "LDPC_BM64 changes the noise the parity tests pin: variant builds only"
#endif
__device__ __forceinline__ void box_muller(uint32_t ua, uint32_t ur, double &n0, double &n1)
{
    if constexpr (!LDPC_BM64) {
        float f0, f1;
        box_muller(ua, ur, f0, f1);
        n0 = (double)f0;
        n1 = (double)f1;
    } else {
        const double a = ((double)ua + 0.5) * 2.3283064365386963e-10;
        const double r = ((double)ur + 0.5) * 2.3283064365386963e-10;
        const double rad = sqrt(-2.0 * log(r));
        double s, c;
        sincospi(2.0 * a, &s, &c);
        n0 = rad * c;
        n1 = rad * s;
    }
}

// Sums of NV values over the workgroup with one barrier pair; red holds 16*NV ints.
// The totals are valid in thread 0 only.
template <int NV>
__device__ __forceinline__ void block_sum_n_t0(int (&x)[NV], int *red)
{
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x[v] += __shfl_xor(x[v], o, 64);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if (l == 0)
#pragma unroll
        for (int v = 0; v < NV; ++v) red[w * NV + v] = x[v];
    __syncthreads();
    // the block totals are thread 0's (every caller reads them there): the other
    // threads skip the 16 x NV partial reads
    if (threadIdx.x == 0) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            int t = 0;
            for (int i = 0; i < nw; ++i) t += red[i * NV + v];
            x[v] = t;
        }
    }
}

// Block sums with one barrier: wave sums by shuffles, one ds_add per wave and value into
// the LDS totals tot[0..NV) (zero on entry), then thread 0 reads the totals into x and
// zeroes them. The caller orders that zeroing before its next use (a later barrier).
template <int NV>
__device__ __forceinline__ void block_sum_lds(int (&x)[NV], int *tot)
{
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x[v] += __shfl_xor(x[v], o, 64);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (x[v]) atomicAdd(&tot[v], x[v]);
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            x[v] = tot[v];
            tot[v] = 0;
        }
    }
}

}  // namespace ldpc
