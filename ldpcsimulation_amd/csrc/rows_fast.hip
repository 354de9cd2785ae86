// rows_fast.hip -- the fast-path row kernel (throughput path of the flooding
// min-sum decoder, src/decodeMinSum.cpp:247-263), fp64 first.
//
// Dataflow (same as kernels.hip's k_decode_rows): a 512-thread
// workgroup decodes C codewords at once for all T iterations with its whole
// state in LDS -- app[N+2] posteriors and the c2v messages in bit-slot-major
// order (a wave's bit-node reads are 64 consecutive words). Thread t owns
// check rows t and t+512 (RPT = 2) with their bit indices / c2v slots and
// the c2v it sent last iteration in registers, and up to CPT bit slots.
//
// What differs: the kernel holds ONLY the fast check node, compiled per
// variant (MS / NMS / OMS) and division mode, so nothing of the exact path
// or of the other variants competes for registers (the old fp64 instance
// spilled 105 VGPRs to scratch, gather addresses included: 75 ms per
// 65 536-codeword launch). Its premise (below) is checked on every row; a
// codeword group that breaks it is abandoned and appended to a re-decode
// list, which k_redo (kernels.hip: the exact one-codeword-per-block path)
// decodes right after, in the same stream. Results are therefore identical
// to the exact kernels for every input; the re-decode list is empty for any
// sane channel (fp64: it needs |c2v| >= 2^1000 or minima below 2^-960).
//
// fp64 fast check node (checkNodeUpdates :410-450, applyNormalization
// :494-499, applyOffset :503-515). Premise: every app and c2v entering the
// iteration is finite with magnitude < 2^1000 (so |v2c| < 2^1009: no inf,
// no NaN) and app is never -0 (yq is canonicalised with + 0.0; a sum that
// starts at +0 and never adds two -0s cannot be -0, and app - c2v is -0
// only when app is -0). Then
//  * sgn(v2c) (:518-523) is the sign bit of v2c's high word, the row's
//    product of signs is the xor of those words (v_bitop3 0x96), and each
//    output's sign is parity ^ sign(v2c_k) (v_bitop3 0x78) -- also for a
//    +0 magnitude, as prod*min*sgn gives;
//  * (min1, min2) = the two smallest |v2c| of the multiset, by a min/max
//    tournament (20 v_min/max_f64 for 8 edges): exactly what the
//    reference's `<=` / `<` update yields for non-NaN inputs;
//  * the argmin edge is recognised as |v2c_k| == min1 (on a tie min2 ==
//    min1, so which tied edge the reference picked does not matter);
//  * x / alpha (NMS) is IEEE division, or, for alpha = P * 2^E with an odd
//    P < 2^20 (1.25 = 5/4), Markstein's q = x*r, q += fma(-q, alpha, x)*r
//    with r = RN(1/alpha): q is within 1.5 ulp of x/alpha, the remainder
//    x - q*alpha is exact (it needs <= 22 bits), the corrected value is
//    x/alpha + d with |d| <= 1.5 ulp * 2^-53, and x/alpha, a fraction of
//    denominator P in units of the result's ulp, is at least 1/(2P) ulp
//    away from every rounding midpoint -- so the correction rounds to
//    RN(x/alpha). Valid for 2^-960 <= x < 2^1000 and x = 0;
//    other minima break the premise.
// fp32 (C = 2 codewords per block, packed as float2) uses cn_fast of
// minsum_common.h -- MS, and NMS with the device-verified reciprocal -- with
// its own premise (every |c2v| and |yq| below 1e30). Opt-in (LDPC_ROWS32=fast):
// bit-exact, but 10.05 ms per bench launch against 8.78 ms for kernels.hip's
// fp32 row kernel, which stays the fp32 default.
#include "kernels.h"
#include "device_common.h"
#include "minsum_common.h"
#include "fast64.h"

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <algorithm>

namespace ldpc {

// Progress-ordered wave priorities in the check phase: s_setprio 3 at the phase start,
// one lower after each row, 0 for the bit phase -- a wave behind outranks the ones
// ahead, so the VALU-bound phase does not end on lone waves (config 1, PEG 1008 fp64
// MS T=10: 25.6-26.0 -> 26.8-27.0 Gbit/s). 0: none.
#ifndef LDPC_FAST_PRIOBAL
#define LDPC_FAST_PRIOBAL 1
#endif
#ifndef LDPC_FAST_PREFETCH
#define LDPC_FAST_PREFETCH 1
#endif
// Timing experiments only (wrong results; `make fastvariant`): LDPC_FAST_EXP =
// 1 no c2v scatters, 2 no bit phase, 3 no barriers in the iteration loop,
// 4 check node replaced by a copy, 5 gathers all read one address.
#ifndef LDPC_FAST_EXP
#define LDPC_FAST_EXP 0
#endif
// Wrong-result timing switches build only into A/B libraries (the *variant targets define
// LDPC_AB_BUILD); a product build with one of them set is refused.
#if LDPC_FAST_EXP != 0 && !defined(LDPC_AB_BUILD)
#error "LDPC_FAST_EXP != 0 gives wrong results by design: make fastvariant only"
#endif
// 1: no staging barrier per codeword group -- the channel writes yq + 0 into app itself and
// flags the premise (raised after the channel's barrier, where thread 0 has cleared the
// flag), each thread reads its yq back, and the bit-layout padding slots are zeroed once per
// kernel (nothing else writes them); 0: the channel is staged through the c2v area and
// copied to app between two barriers, the padding slots re-zeroed every group.
#ifndef LDPC_FAST_NOB2
#define LDPC_FAST_NOB2 1
#endif
template <int RPT> struct FastShape;
#ifndef LDPC_FAST_RPT1_WAVES
#define LDPC_FAST_RPT1_WAVES 4
#endif
template <> struct FastShape<1> { static constexpr int threads = 1024, waves_per_eu = LDPC_FAST_RPT1_WAVES; };
template <> struct FastShape<2> { static constexpr int threads = 512, waves_per_eu = 4; };

template <typename F, int SRC, int C, int DC, int CPT, int RPT, int VAR, bool FDIV>
__global__ __launch_bounds__(FastShape<RPT>::threads, FastShape<RPT>::waves_per_eu) void k_rows_fast(
    DecodeArgs a, DevGraph g, RowSched rs, unsigned *redo)
{
    static_assert(sizeof(F) == 8 ? C == 1 : (C == 2 && VAR != V_OMS), "fp64 single / fp32 pair fast kernel");
    constexpr bool F64 = sizeof(F) == 8;
    const F kMax = F64 ? (F)kFast64Max : (F)1e30f;   // premise bound on |yq|
    using P = Pack<F, C>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, nt = blockDim.x;
    const int N = g.N, EA = rs.e_pad + 64;
    P *app = reinterpret_cast<P *>(smem);          // [N + 2]: bit N is the +INF sentinel of padding edges
    P *c2v = app + (N + 2);                        // [EA] bit-slot-major; last 64: per-lane dummies
    int *red = reinterpret_cast<int *>(c2v + EA);  // [31]: premise flag; [32, 128): block sums (16 waves x 6); [128, 140): acc
    const uint32_t app_base = lds_addr_of(app), c2v_base = lds_addr_of(c2v);   // LDS byte addresses

    int deg[RPT];
    uint32_t colw[RPT][DC / 2], posw[RPT][DC / 2];
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
        const int j = tid + r * nt;
        deg[r] = rs.cn_deg[j];
#pragma unroll
        for (int q = 0; q < DC / 8; ++q) {
            const uint4 xc = reinterpret_cast<const uint4 *>(rs.cn_cols + (size_t)j * DC)[q];
            const uint4 xp = reinterpret_cast<const uint4 *>(rs.cn_pos + (size_t)j * DC)[q];
            colw[r][4 * q + 0] = xc.x; colw[r][4 * q + 1] = xc.y; colw[r][4 * q + 2] = xc.z; colw[r][4 * q + 3] = xc.w;
            posw[r][4 * q + 0] = xp.x; posw[r][4 * q + 1] = xp.y; posw[r][4 * q + 2] = xp.z; posw[r][4 * q + 3] = xp.w;
        }
    }
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
    }
    if ((tid >> 6) >= (nt >> 7)) __builtin_amdgcn_s_setprio(1);   // MI355X_MICROARCH item 4
    const F alpha = (F)a.alpha, delta = (F)a.delta, rcp = F64 ? (F)(1.0 / a.alpha) : (F)a.alpha_rcp;
    const int ngrp = (a.batch + C - 1) / C;
    // the block's totals (thread 0), added to a.counts once at the end; in the
    // dynamic area (no static LDS: app starts at LDS address 0)
    // past block_sum_n_t0's area at every block size (16 waves x 3C sums; ADVICE r2: red + 96 was
    // overwritten by waves 10-12 of a 1024-thread fp32 pair block)
    static_assert(32 + 16 * 3 * C <= 128, "block sums overlap the accumulators");
    unsigned long long *acc = reinterpret_cast<unsigned long long *>(red + 128);
    if (tid == 0) {
#pragma unroll
        for (int q = 0; q < 6; ++q) acc[q] = 0;
#pragma unroll
        for (int q = 0; q < 3 * C; ++q) red[32 + q] = 0;   // block_sum_lds totals
    }
    if constexpr (LDPC_FAST_NOB2) {   // padding slots of the bit-node layout hold +0 (never written)
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int dg = (int)((rs.vn_info[tid * CPT + i] >> 16) & 0xffu);
            const int base = vgb[i] + lane, gd = vgd[i];
            P z;
#pragma unroll
            for (int c = 0; c < C; ++c) z.v[c] = F(0);
            for (int k = dg; k < gd; ++k) c2v[LDPC_CHK(base + k * 64, EA, CHK_FAST_BIT_READ)] = z;
        }
    }
    // the channel's destination: app itself (LDPC_FAST_NOB2, canonical yq) or the c2v staging area
    P *const stage = LDPC_FAST_NOB2 ? app : c2v;
    for (int grp = blockIdx.x; grp < ngrp; grp += gridDim.x) {
        // ---- channel (:214-238) ----
        if (tid == 0) red[31] = 0;
        int unc[C];
        [[maybe_unused]] bool ch_ok = true;   // LDPC_FAST_NOB2: this thread's inputs within the premise
        // LDPC_FAST_NOB2: the staged value is yq + 0 (app never holds -0), checked against the bound
        auto put = [&](int v, int c, F q) {
            if constexpr (LDPC_FAST_NOB2) {
                q = q + F(0);
                ch_ok &= dabs(q) < kMax;
            }
            stage[v].v[c] = q;
        };
        const int8_t *cvec[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            unc[c] = 0;
            cvec[c] = nullptr;
            const int b = grp * C + c;
            if (b >= a.batch) {   // missing partner of an odd batch: benign +1 samples, never a premise break
                for (int v = tid; v < N; v += nt) stage[v].v[c] = F(1);
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
                if (LDPC_FAST_NOB2 && !a.cw_table && !a.y_out && !a.quantize && !a.saturate && (N & 3) == 0) {
                    // the common case in straight-line code (the all-zero codeword, no front end,
                    // no sample output): the same values as the general loop below
                    for (int g4 = tid; g4 * 4 < N; g4 += nt) {
                        uint32_t u[4];
                        philox4x32_10<true>((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, k0, k1, u);
                        F n[4], qv[4];
                        box_muller(u[0], u[1], n[0], n[1]);
                        box_muller(u[2], u[3], n[2], n[3]);
#pragma unroll
                        for (int q4 = 0; q4 < 4; ++q4) {
                            qv[q4] = (F(1) + sigma * n[q4]) + F(0);   // (F)cv * (1 + sigma n) with cv = +1, then yq + 0
                            unc[c] += (qv[q4] > F(0) ? 1 : -1) < 0;
                            ch_ok &= dabs(qv[q4]) < kMax;
                        }
                        if constexpr (C == 1) {   // two ds_write_b128 (app at LDS address 0: 32-byte aligned groups)
                            struct alignas(16) D2 { F d[2]; };
                            lds_put<D2>(app_base + 32u * (uint32_t)g4, D2{{qv[0], qv[1]}});
                            lds_put<D2>(app_base + 32u * (uint32_t)g4 + 16u, D2{{qv[2], qv[3]}});
                        } else {
#pragma unroll
                            for (int q4 = 0; q4 < 4; ++q4) app[4 * g4 + q4].v[c] = qv[q4];
                        }
                    }
                    continue;
                }
                for (int g4 = tid; g4 * 4 < N; g4 += nt) {
                    uint32_t u[4];
                    philox4x32_10<true>((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, k0, k1, u);
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
        __syncthreads();
        P yq[CPT];
        int flag = 0;
        if constexpr (LDPC_FAST_NOB2) {
            if (__builtin_amdgcn_ballot_w64(!ch_ok)) {   // rare: an input past the premise bound
                asm volatile(";");
                if (!ch_ok) red[31] = 1;
            }
#pragma unroll
            for (int i = 0; i < CPT; ++i) {   // padding slots: +0
                yq[i] = app[LDPC_CHK(vdst(i) < N ? vdst(i) : 0, N + 2, CHK_FAST_APP_WRITE)];
                if (vdst(i) >= N)
#pragma unroll
                    for (int c = 0; c < C; ++c) yq[i].v[c] = F(0);
            }
            // the flag raised here is read after the first check phase's barrier (or below, T = 0)
            if (a.T == 0) __syncthreads();
        } else {
        bool in_ok = true;
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const P st = c2v[LDPC_CHK(vdst(i) <= N ? vdst(i) : 0, N + 2, CHK_FAST_APP_WRITE)];
            // yq + 0 maps -0 to +0, so app is never -0 (see the header)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                yq[i].v[c] = st.v[c] + F(0);
                in_ok &= dabs(yq[i].v[c]) < kMax;
            }
            app[LDPC_CHK(vdst(i), N + 2, CHK_FAST_APP_WRITE)] = yq[i];   // v2c = yq on the first pass (:364-370)
        }
        if (!in_ok) red[31] = 1;
        __syncthreads();
        // padding slots of the bit-node layout hold +0 (adding +0 changes no sum)
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int dg = (int)((rs.vn_info[tid * CPT + i] >> 16) & 0xffu);
            const int base = vgb[i] + lane, gd = vgd[i];
            P z;
#pragma unroll
            for (int c = 0; c < C; ++c) z.v[c] = F(0);
            for (int k = dg; k < gd; ++k) c2v[LDPC_CHK(base + k * 64, EA, CHK_FAST_BIT_READ)] = z;
        }
        flag = red[31];
        }
        P prev[RPT][DC];   // c2v sent on each edge last iteration: +0 before the first
#pragma unroll
        for (int r = 0; r < RPT; ++r)
#pragma unroll
            for (int k = 0; k < DC; ++k)
#pragma unroll
                for (int c = 0; c < C; ++c) prev[r][k].v[c] = F(0);

        for (int it = 0; it < a.T; ++it) {
            if (__builtin_amdgcn_readfirstlane(flag) != 0) break;
            // The packed 16-bit schedule words are opaque per iteration: otherwise
            // the compiler hoists the 32 unpacked indices out of the loop and
            // spills them (one scratch load per gather).
#pragma unroll
            for (int r = 0; r < RPT; ++r)
#pragma unroll
                for (int q = 0; q < DC / 2; ++q) asm volatile("" : "+v"(colw[r][q]), "+v"(posw[r][q]));
#pragma unroll
            for (int q = 0; q < (CPT + 1) / 2; ++q) asm volatile("" : "+v"(vdst2[q]));
            // ---- check nodes (with LDPC_FAST_PREFETCH, row r+1's gathers are issued
            // before row r is computed) ----
            if (LDPC_FAST_PRIOBAL) __builtin_amdgcn_s_setprio(3);
            P xin[LDPC_FAST_PREFETCH ? 2 : 1][DC];
#pragma unroll
            for (int k = 0; k < DC; ++k)
                xin[0][k] = lds_at<P>(LDPC_FAST_EXP == 5 ? app_base + 8 * k
                                                         : LDPC_ADDR8(DC, colw[0], k, app_base, N + 2, CHK_FAST_GATHER));
#pragma unroll
            for (int r = 0; r < RPT; ++r) {
                constexpr int NB = LDPC_FAST_PREFETCH ? 2 : 1;
                if (LDPC_FAST_PREFETCH && r + 1 < RPT) {
#pragma unroll
                    for (int k = 0; k < DC; ++k)
                        xin[(r + 1) % NB][k] = lds_at<P>(
                            LDPC_FAST_EXP == 5 ? app_base + 8 * k
                                               : LDPC_ADDR8(DC, colw[r + 1 < RPT ? r + 1 : r], k, app_base, N + 2, CHK_FAST_GATHER));
                }
                if (!LDPC_FAST_PREFETCH && r > 0) {
#pragma unroll
                    for (int k = 0; k < DC; ++k) xin[0][k] = lds_at<P>(LDPC_ADDR8(DC, colw[r], k, app_base, N + 2, CHK_FAST_GATHER));
                }
                bool ok;
                if constexpr (LDPC_FAST_EXP == 4) {
                    ok = true;
#pragma unroll
                    for (int k = 0; k < DC; ++k) prev[r][k].v[0] = xin[r % NB][k].v[0] - prev[r][k].v[0];
                } else if constexpr (F64) {
                    ok = cn_fast64<DC, VAR, FDIV>(xin[r % NB], prev[r], alpha, rcp, delta);
                } else {
                    ok = cn_fast<DC, C>(xin[r % NB], prev[r], VAR == V_NMS, (float)alpha, (float)rcp);
                }
                // a premise break (rows past M, degree 0, only write dummy slots): a skipped
                // branch, not an exec-masked flag store per row
                if (__builtin_amdgcn_ballot_w64(!ok && deg[r] > 0)) {
                    asm volatile(";");   // a side effect: stays a skipped branch
                    if (!ok && deg[r] > 0) red[31] = 1;
                }
                if (LDPC_FAST_PRIOBAL) {
                    if (r == 0) __builtin_amdgcn_s_setprio(2);
                    else __builtin_amdgcn_s_setprio(1);
                }
                if constexpr (LDPC_FAST_EXP != 1) {
#pragma unroll
                    for (int k = 0; k < DC; ++k) lds_put<P>(LDPC_ADDR8(DC, posw[r], k, c2v_base, EA, CHK_FAST_SCATTER), prev[r][k]);
                }
                if (RPT > 1) __builtin_amdgcn_sched_barrier(0);   // keep the rows' live ranges apart
            }
            if (LDPC_FAST_PRIOBAL) __builtin_amdgcn_s_setprio(0);
            if constexpr (LDPC_FAST_EXP != 3) __syncthreads();
            flag = red[31];   // in flight during the bit phase
            // ---- bit nodes: sum = yq + c2v in nlist order (:452-476) ----
            if constexpr (LDPC_FAST_EXP != 2) {
                P sum[CPT];
#pragma unroll
                for (int i = 0; i < CPT; ++i) sum[i] = yq[i];
                int k = 0;
                // the lane id recomputed here (v_mbcnt), so the lane's c2v pointer is not a
                // loop-long live value (it was spilled)
                const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
                vn_phases<F, C, CPT, CPT>(c2v + ln, vgb, vgd, k, sum, LDPC_CHK_LIM(EA - ln), CHK_FAST_BIT_READ);
#pragma unroll
                for (int i = 0; i < CPT; ++i) app[LDPC_CHK(vdst(i), N + 2, CHK_FAST_APP_WRITE)] = sum[i];
            }
            if constexpr (LDPC_FAST_EXP != 3) __syncthreads();
        }
        // Any premise failure in this group (flag set after the last barrier
        // at the latest): decode it again on the exact path.
        if (__builtin_amdgcn_readfirstlane(red[31]) != 0) {
            if (tid == 0) {
                const int nb = (grp * C + C <= a.batch) ? C : a.batch - grp * C;
                const unsigned at = atomicAdd(&redo[0], (unsigned)nb);
                for (int c = 0; c < nb; ++c) redo[1 + at + c] = (unsigned)(grp * C + c);
            }
            __syncthreads();
            continue;
        }

        // ---- decisions, error weight (:270, :382-393), syndrome, accounting ----
        int sums[3 * C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int b = grp * C + c;
            int w = 0, synd = 0;
            if (b < a.batch) {
                if (!cvec[c] && !a.d_out) {   // the common case: errors are the posteriors not > 0
#pragma unroll
                    for (int i = 0; i < CPT; ++i) {
                        const int v = vdst(i);
                        w += (v < N && !(app[v < N ? v : 0].v[c] > F(0))) ? 1 : 0;   // :471-474
                    }
                } else {
#pragma unroll
                for (int i = 0; i < CPT; ++i) {
                    const int v = vdst(i);
                    if (v < N) {
                        const int d = app[v].v[c] > F(0) ? 1 : -1;   // :471-474
                        const int cv = cvec[c] ? cvec[c][v] : 1;
                        w += (d != cv);
                        if (a.d_out) a.d_out[(size_t)b * N + v] = (int8_t)d;
                    }
                }
                }
#pragma unroll
                for (int r = 0; r < RPT; ++r) {   // padding edges read the +inf sentinel: parity 0
                    int par = 0;
#pragma unroll
                    for (int k = 0; k < DC; ++k)
                        par ^= (app[LDPC_CHK(u16_at<DC>(colw[r], k), N + 2, CHK_FAST_GATHER)].v[c] > F(0)) ? 0 : 1;
                    synd |= par;
                }
            }
            sums[3 * c] = w;
            sums[3 * c + 1] = unc[c];
            sums[3 * c + 2] = synd;
        }
        block_sum_lds<3 * C>(sums, red + 32);   // re-zeroed by thread 0; the step's last barrier orders it
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
        }
        __syncthreads();
    }
    if (tid == 0 && acc[3] > 0) {
        acc[4] = acc[3] * (unsigned long long)a.T;
#pragma unroll
        for (int q = 0; q < 6; ++q) atomicAdd(&a.counts[q], acc[q]);
    }
}

LDPC_CHECK_TU(rows_fast)

// alpha = P * 2^E with odd P < 2^20, in the range where 1/alpha is normal:
// Markstein's correction is then exact (header).
bool markstein_exact_alpha(double alpha)
{
    // |alpha| <= 2^60: a minimum >= 2^-960 then divides to >= 2^-1020, a normal
    // quotient, where the 1/(2P)-ulp midpoint argument holds
    if (!(alpha > 0x1p-900) || !(alpha <= 0x1p60)) return false;
    unsigned long long b;
    __builtin_memcpy(&b, &alpha, 8);
    const unsigned long long sig = (b & ((1ull << 52) - 1)) | (1ull << 52);   // 53-bit significand
    const int tz = __builtin_ctzll(sig);
    return (sig >> tz) < (1ull << 20);
}

template <typename F, int VAR, bool FDIV, int SRC, int DC, int CPT, int RPT>
static hipError_t launch_fast_t(const DevGraph &g, const RowSched &rs, const DecodeArgs &a, int lds, unsigned *redo,
                                hipStream_t s, int num_cus)
{
    constexpr int C = sizeof(F) == 8 ? 1 : 2;
    auto fn = k_rows_fast<F, SRC, C, DC, CPT, RPT, VAR, FDIV>;
    hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, rs.threads, lds);
    if (e != hipSuccess || per_cu < 1) per_cu = 1;
    if (const int cap = opt(LDPC_OPT_FAST_BPC)) per_cu = std::min(per_cu, cap);   // experiments
    const int ngrp = (a.batch + C - 1) / C;
    int grid = per_cu * num_cus;
    if (grid > ngrp) grid = ngrp;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(rs.threads), lds, s, a, g, rs, redo);
    return hipGetLastError();
}

template <typename F, int VAR, bool FDIV, int SRC>
static hipError_t launch_fast_shape(const DevGraph &g, const RowSched &rs, const DecodeArgs &a, int lds, unsigned *redo,
                                    hipStream_t s, int num_cus)
{
#define LDPC_FAST_CASE(DCV, CPTV, RPTV) \
    if (rs.dc == DCV && rs.cpt == CPTV && rs.rpt == RPTV) return launch_fast_t<F, VAR, FDIV, SRC, DCV, CPTV, RPTV>(g, rs, a, lds, redo, s, num_cus);
    LDPC_FAST_CASE(8, 4, 2)
    LDPC_FAST_CASE(8, 2, 1)
    LDPC_FAST_CASE(8, 4, 1)
    if constexpr (sizeof(F) == 8) {   // fp32 rows with dc > 8 hold one codeword per block: the old kernel
        LDPC_FAST_CASE(16, 4, 2)
        LDPC_FAST_CASE(16, 2, 1)
        LDPC_FAST_CASE(16, 4, 1)
    }
#undef LDPC_FAST_CASE
    return hipErrorInvalidValue;
}

bool rows_fast_supported(const RowSched &rs, bool f64)
{
    if (rs.threads <= 0) return false;
    if (rs.dc != 8 && !(f64 && rs.dc == 16)) return false;
    return (rs.rpt == 2 && rs.cpt == 4) || (rs.rpt == 1 && (rs.cpt == 2 || rs.cpt == 4));
}

bool rows_fast_f32_ok(const DecodeArgs &a) { return a.variant == V_MS || (a.variant == V_NMS && a.nms_fast); }

hipError_t launch_rows_fast(const DevGraph &g, const RowSched &rs, const DecodeArgs &a, bool f64, int lds_bytes,
                            unsigned *redo, hipStream_t s, int num_cus)
{
    const bool given = a.src == SRC_GIVEN;
#define LDPC_FAST_SRC(FT, VARV, FD)                                                                         \
    return given ? launch_fast_shape<FT, VARV, FD, SRC_GIVEN>(g, rs, a, lds_bytes, redo, s, num_cus)        \
                 : launch_fast_shape<FT, VARV, FD, SRC_PHILOX>(g, rs, a, lds_bytes, redo, s, num_cus);
    if (!f64) {   // fp32: MS, or NMS with the verified reciprocal (rows_fast_f32_ok)
        if (a.variant == V_MS) { LDPC_FAST_SRC(float, V_MS, false) }
        if (a.variant == V_NMS && a.nms_fast) { LDPC_FAST_SRC(float, V_NMS, true) }
        return hipErrorInvalidValue;
    }
    const bool fdiv = a.variant == V_NMS && markstein_exact_alpha(a.alpha);
    if (a.variant == V_MS) { LDPC_FAST_SRC(double, V_MS, false) }
    if (a.variant == V_OMS) { LDPC_FAST_SRC(double, V_OMS, false) }
    if (fdiv) { LDPC_FAST_SRC(double, V_NMS, true) }
    LDPC_FAST_SRC(double, V_NMS, false)
#undef LDPC_FAST_SRC
}

}  // namespace ldpc
