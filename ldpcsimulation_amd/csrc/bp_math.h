// bp_math.h -- the fp64 transcendentals of the BP check node (src/decodeBP.cpp
// :353-377: th_k = tanh(v2c_k / 2), c2v = log((1 + p) / (1 - p))), written for
// gfx950 without branches.
//
// Why not OCML's tanh/log: they are accurate to ~0.5 ulp through double-double
// arithmetic and carry range branches; in a wave whose lanes hold messages of
// every magnitude both sides of each branch execute. The fp64 BP rows kernel
// issued ~290 VALU instructions per edge (1 096 v_add_f64 per 8-edge row) and
// ran at 0.81 of the VALU issue peak (profiles/r06_configs.jsonl). These forms
// take ~30 fp64 operations each, on one path, with the classic argument
// reductions and polynomial kernels; they agree with glibc's tanh/log to the
// ulp bounds tests/test_bp.py measures on the device (ldpc_bp_math_probe), and
// the BP decisions stay those of the oracle and of the reference's golden runs.
//
//  * tanh(x) = sign(x) E / (E + 2), E = expm1(2|x|): no cancellation at small |x|
//    (E ~ 2|x|); the denominator is kept as an unevaluated sum (2Sum) so its
//    rounding does not enter; |x| is clamped at 20, where tanh rounds to 1, so
//    that E stays finite (NaN stays NaN). expm1(y) = 2^k (1 + p) - 1 with
//    k = floor(y / ln2), r = y - k ln2 (Cody-Waite, fdlibm's ln2_hi/ln2_lo) and
//    p = expm1(r) = r + r^2 (1/2! + r/3! + ... + r^15/17!) on [0, ln2).
//    Host emulation over 4M arguments (v_rcp_f64 as 1/d): expm1 <= 1 ulp, tanh
//    <= 3 ulp (2 values of 4M at 3), log <= 1 ulp from glibc.
//  * log(z) = k ln2 + log(m), z = m 2^k, m in [sqrt(1/2), sqrt(2)): f = m - 1
//    (exact), s = f / (2 + f), log(m) = f - (hf - s (hf + R(s^2))) with
//    hf = f^2 / 2 and fdlibm's e_log.c minimax R (Lg1..Lg7, < 1 ulp); z = 0,
//    +inf and NaN by select.
//  * divisions by a reciprocal: v_rcp_f64, two Newton steps and one residual
//    correction (operands in [2, 2^60]: no scaling needed).
#pragma once
#include <hip/hip_runtime.h>

namespace ldpc {

// x / d for d in [1, 2^60] and finite x (no over/underflow in the intermediates)
__device__ __forceinline__ double bp_div_pos(double x, double d)
{
    double r = __builtin_amdgcn_rcp(d);
    r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
    r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
    const double q = x * r;
    return __builtin_fma(r, __builtin_fma(-d, q, x), q);
}

// e^y - 1 for y in [0, 40]
__device__ __forceinline__ double bp_expm1_pos(double y)
{
    const double kInvLn2 = 1.4426950408889634074;
    const double kLn2Hi = 6.93147180369123816490e-01;   // 32 trailing zero bits: k * kLn2Hi exact
    const double kLn2Lo = 1.90821492927058770002e-10;
    // k = floor(y / ln2): r in [0, ln2), so 2^k (1 + p) - 1 adds three non-negative terms
    // (no cancellation; rint's r in [-ln2/2, ln2/2] cost 2 ulp at k = 1)
    const double kd = __builtin_floor(y * kInvLn2);    // 0 .. 57
    const double hi = __builtin_fma(-kd, kLn2Hi, y);   // exact
    const double lo = kd * kLn2Lo;
    const double r = hi - lo;
    const double c = (hi - r) - lo;                    // the bits r lost
    // P(r) = 1/2! + r/3! + ... + r^15/17!  (truncation < 6e-18 relative on [0, ln2))
    double P = 2.8114572543455207632e-15;              // 1/17!
    P = __builtin_fma(P, r, 4.7794773323873852974e-14);   // 1/16!
    P = __builtin_fma(P, r, 7.6471637318198164759e-13);   // 1/15!
    P = __builtin_fma(P, r, 1.1470745597729724714e-11);   // 1/14!
    P = __builtin_fma(P, r, 1.6059043836821614599e-10);   // 1/13!
    P = __builtin_fma(P, r, 2.0876756987868098979e-09);   // 1/12!
    P = __builtin_fma(P, r, 2.5052108385441718775e-08);   // 1/11!
    P = __builtin_fma(P, r, 2.7557319223985890653e-07);   // 1/10!
    P = __builtin_fma(P, r, 2.7557319223985890653e-06);   // 1/9!
    P = __builtin_fma(P, r, 2.4801587301587301587e-05);   // 1/8!
    P = __builtin_fma(P, r, 1.9841269841269841270e-04);   // 1/7!
    P = __builtin_fma(P, r, 1.3888888888888888889e-03);   // 1/6!
    P = __builtin_fma(P, r, 8.3333333333333333333e-03);   // 1/5!
    P = __builtin_fma(P, r, 4.1666666666666666667e-02);   // 1/4!
    P = __builtin_fma(P, r, 1.6666666666666666667e-01);   // 1/3!
    P = __builtin_fma(P, r, 0.5);
    double p = __builtin_fma(r * r, P, r);             // expm1(r)
    p = __builtin_fma(c, 1.0 + p, p);                  // expm1(r + c)
    const int k = (int)kd;
    return __builtin_ldexp(p, k) + (__builtin_ldexp(1.0, k) - 1.0);
}

__device__ __forceinline__ double bp_tanh64(double x)
{
    double y = 2.0 * __builtin_fabs(x);
    y = y > 40.0 ? 40.0 : y;   // tanh(20) rounds to 1; NaN stays NaN
    const double e = bp_expm1_pos(y);
    // e / (e + 2) with the denominator's rounding error carried (2Sum: d + de = e + 2 exactly)
    const double d = e + 2.0, bb = d - e, de = (e - (d - bb)) + (2.0 - bb);
    double r = __builtin_amdgcn_rcp(d);
    r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
    r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
    const double q = e * r;
    const double res = __builtin_fma(-de, q, __builtin_fma(-d, q, e));   // e - q (d + de)
    return __builtin_copysign(__builtin_fma(r, res, q), x);
}

__device__ __forceinline__ double bp_log64(double z)
{
    const double kLn2Hi = 6.93147180369123816490e-01, kLn2Lo = 1.90821492927058770002e-10;
    const double kLg1 = 6.666666666666735130e-01, kLg2 = 3.999999999940941908e-01,
                 kLg3 = 2.857142874366239149e-01, kLg4 = 2.222219843214978396e-01,
                 kLg5 = 1.818357216161805012e-01, kLg6 = 1.531383769920937332e-01,
                 kLg7 = 1.479819860511658591e-01;
    int e = __builtin_amdgcn_frexp_exp(z);
    double m = __builtin_amdgcn_frexp_mant(z);            // [0.5, 1)
    const bool lo = m < 0.70710678118654752440;
    m = lo ? m + m : m;
    e = lo ? e - 1 : e;
    const double f = m - 1.0;                             // exact
    const double s = bp_div_pos(f, 2.0 + f);
    const double z2 = s * s, w = z2 * z2;
    const double t1 = w * __builtin_fma(w, __builtin_fma(w, kLg6, kLg4), kLg2);
    const double t2 = z2 * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, kLg7, kLg5), kLg3), kLg1);
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    const double dk = (double)e;
    const double v = dk * kLn2Hi - ((hfsq - (s * (hfsq + R) + dk * kLn2Lo)) - f);
    // z = 0 -> -inf, z = +inf -> +inf, NaN (and z < 0, never formed) -> NaN
    const double special = z == 0.0 ? -__builtin_inf() : (z > 0.0 ? z : __builtin_nan(""));
    return (z > 0.0 && z < __builtin_inf()) ? v : special;
}

}  // namespace ldpc
