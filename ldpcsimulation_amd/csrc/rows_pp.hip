// rows_pp.hip -- the headline kernel: flooding min-sum (src/decodeMinSum.cpp
// :247-263, check node :410-450, normalisation :494-515, bit node :452-476)
// with check and bit work of two codeword slots overlapped in one workgroup.
// A slot holds one fp64 codeword (the reference's arithmetic) or an fp32 pair
// interleaved as float2 (the fp32 throughput path): the same 8-byte LDS words,
// schedule and roles either way.
//
// k_rows_fast (rows_fast.hip) decodes one codeword per 512-thread block; inside
// a block the check phase (VALU-heavy: the f64 tournament, division, selects)
// and the bit phase (LDS-latency-bound: c2v reads and dependent adds) alternate
// between barriers, so a CU's VALU and LDS pipe are each busy only about half
// the time. Here one 1024-thread block holds TWO
// codewords (slots 0 and 1, 2 x 74 KB of LDS for N=1944) and its waves are
// specialised:
//   waves 0-7  (the check role) own check rows t and t+512, as k_rows_fast's
//              threads do, with their schedule in registers;
//   waves 8-15 (the bit role) own the bit slots of k_rows_fast's thread t-512.
// Between two barriers the check role runs iteration i of one slot while the
// bit role runs the bit nodes of the other slot:
//   | check(0,0) | check(1,0)  | check(0,1)  | ... | check(1,T-1) |             |
//   |            | bit(0,0)    | bit(1,0)    | ... | bit(0,T-1)   | bit(1,T-1)  |
// so every interval carries one check phase and one bit phase, on different
// waves of the same SIMDs: 2T + 1 barrier intervals per pair instead of 4T.
// A slot's check(i+1) follows its bit(i), which follows its check(i), each an
// interval apart: the flooding schedule of each codeword is unchanged, and so
// is every value (same arithmetic as k_rows_fast: cn_fast64 of fast64.h, sums
// in nlist order), hence the decisions equal the reference's bit for bit.
//
// The c2v a row sent last iteration (the `- msg` of :469) is kept per slot in
// registers (prev: 2 slots x rows x 8 edges); re-reading it from the row's own
// c2v slots instead (8 more ds_read_b64 per row) measured slower (16.9 vs 14.7 ms).
//
// Premise failures (fast64.h for fp64, minsum_common.h cn_fast for fp32): the
// slot's flag is raised and its codeword(s) are re-decoded on the exact path
// (k_redo) after the launch; the other slot is unaffected. Rows past M (degree 0) gather app[N + 2] = +0, so
// their messages stay 0 (their scatters land in per-lane dummy slots that the
// padding edges of real rows also use; those read +inf - finite = +inf).
#include "kernels.h"
#include "device_common.h"
#include "minsum_common.h"
#include "fast64.h"

#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

namespace ldpc {

namespace {

// Timing experiments only (wrong results; `make ppvariant`): LDPC_PP_EXP =
// 1 bit role idle (barriers only), 2 check role idle, 3 check node replaced by
// a subtraction, 4 no c2v scatters, 5 gathers at lane-contiguous addresses (no
// bank conflicts), 6 scatters at lane-contiguous addresses, 7 both 5 and 6.
// LDPC_PP_BITDELAY: s_sleep units (64 cycles) the bit waves wait at an interval's start.
// fp64 premise flag: 0 = each row's hi-word maximum (fast64.h ACC) tested by a
// wave-uniform branch right after the row (no register lives across the step);
// 1 = a per-slot sticky maximum tested once after the step's last iteration (two
// VGPRs across the interval loop: the kernel setup then spills 16 B more per lane).
#ifndef LDPC_PP_STICKY
#define LDPC_PP_STICKY 0
#endif
// Timing ablations of the per-step work (results wrong by design): 1 no channel
// generation, 2 no syndrome / decisions, 4 no block reduction.
// Bit mask of the precisions (1 fp32 pairs, 2 fp64) whose step tail is folded into the
// last intervals: the bit role takes a slot's decisions and error weights from the sums of
// that slot's last bit-node pass (the values it writes to app), and the check role forms
// slot 0's syndrome in the extra interval, where it is idle; only slot 1's syndrome stays
// after the last barrier. Otherwise all of it follows the last barrier. Measured: fp32
// 7.16-7.21 -> 7.10-7.12 ms; fp64 12.28-12.29 -> 12.31 (the decisions lengthen the
// check-bound interval of bit(0,T-1)), so fp64 keeps the tail after the barrier.
#ifndef LDPC_PP_TAILFUSE
#define LDPC_PP_TAILFUSE 1
#endif
#ifndef LDPC_PP_TAILEXP
#define LDPC_PP_TAILEXP 0
#endif
#ifndef LDPC_PP_EXP
#define LDPC_PP_EXP 0
#endif
// Wrong-result timing switches build only into A/B libraries (the *variant targets define
// LDPC_AB_BUILD); a product build with one of them set is refused.
#if LDPC_PP_EXP != 0 && !defined(LDPC_AB_BUILD)
#error "LDPC_PP_EXP != 0 gives wrong results by design: make ppvariant only"
#endif
#if LDPC_PP_TAILEXP != 0 && !defined(LDPC_AB_BUILD)
#error "LDPC_PP_TAILEXP != 0 gives wrong results by design: make ppvariant only"
#endif
#ifndef LDPC_PP_BITDELAY
#define LDPC_PP_BITDELAY 0
#endif
// 0: no scheduling fence between a check wave's two rows (the compiler may interleave them)
#ifndef LDPC_PP_ROWFENCE
#define LDPC_PP_ROWFENCE 1
#endif

// Wave priority (s_setprio): 0 none, 1 check role above the bit role, 2 the reverse,
// 3 the younger half of each role (waves 4-7, 12-15) above the older half, 4 the younger
// check waves (4-7) above all others, 5 younger check > older check > bit waves.
#ifndef LDPC_PP_PRIO
#define LDPC_PP_PRIO 0
#endif
// 1: the check role issues both rows' LDS reads before computing row 0; 0: row 1's after it.
#ifndef LDPC_PP_PREFETCH
#define LDPC_PP_PREFETCH 1
#endif
// 1: the fp64 check node's scatters are pinned in per-edge order behind each message's
// selects (sched_group_barrier); 0: the machine scheduler places them (it tended to sink
// all of a row's stores behind all of its selects, a 3 % swing between builds).
#ifndef LDPC_PP_STORE_ORDER
#define LDPC_PP_STORE_ORDER 1
#endif
// 1: the scheduler is asked to issue all of an interval's gathers before the check-node
// arithmetic (sched_group_barrier); 0: left to the scheduler.
#ifndef LDPC_PP_GATHER_FIRST
#define LDPC_PP_GATHER_FIRST 0
#endif

// Diagnostic builds (-DLDPC_STAMPS, `make ppvariant`): per wave, s_memtime cycles
// spent working and waiting at the interval barriers, to a.stamps[(block*16+wave)*2].
#ifdef LDPC_STAMPS
#define PP_STAMP_DECL unsigned long long st_work = 0, st_wait = 0, st_step[5] = {}, st_t0 = __builtin_amdgcn_s_memtime()
#define PP_BARRIER()                                                        \
    do {                                                                    \
        const unsigned long long te_ = __builtin_amdgcn_s_memtime();        \
        __syncthreads();                                                    \
        const unsigned long long tb_ = __builtin_amdgcn_s_memtime();        \
        st_work += te_ - st_t0;                                             \
        st_wait += tb_ - te_;                                               \
        st_t0 = tb_;                                                        \
    } while (0)
// Per step, to a.stamps[8192 + (block*16+wave)*6 + k]: k = 0 the tail (last interval
// barrier -> the next step's top: syndrome, decisions, the block accounting), 1 the channel
// (step top -> B1), 2 the wait at B1, 3 the yq staging (B1 -> B2), 4 the wait at B2.
#define PP_STAMP_ACC(k)                                                     \
    do {                                                                    \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();         \
        st_step[k] += t_ - st_t0;                                           \
        st_t0 = t_;                                                         \
    } while (0)
#define PP_STAMP_TOP() PP_STAMP_ACC(0)
#define PP_SYNC_STAMPED(k0)                                                 \
    do {                                                                    \
        PP_STAMP_ACC(k0);                                                   \
        __syncthreads();                                                    \
        PP_STAMP_ACC(k0 + 1);                                               \
    } while (0)
#define PP_STAMP_OUT()                                                                              \
    if (a.stamps && (threadIdx.x & 63) == 0 && blockIdx.x < 256) {                                  \
        a.stamps[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 2] = st_work;                             \
        a.stamps[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 2 + 1] = st_wait;                         \
        for (int k_ = 0; k_ < 5; ++k_)                                                              \
            a.stamps[8192 + (blockIdx.x * 16 + (threadIdx.x >> 6)) * 6 + k_] = st_step[k_];         \
    }
#else
#define PP_STAMP_DECL
#define PP_BARRIER() __syncthreads()
#define PP_STAMP_TOP()
#define PP_SYNC_STAMPED(k0) __syncthreads()
#define PP_STAMP_OUT()
#endif

constexpr int kPPRole = 512;          // threads per role
constexpr int kPPWaves = 2 * kPPRole / 64;
constexpr int kPPMaxCw = 4;           // codewords per block step (2 slots x an fp32 pair)
// red[] ints: [0,2) slot flags, [32, 32 + 16 waves x 3 x 4 codewords) block sums, then acc (6 x u64)
constexpr int kPPRedSums = 32;
constexpr int kPPRedAcc = kPPRedSums + kPPWaves * 3 * kPPMaxCw;
constexpr int kPPRedInts = kPPRedAcc + 2 * 6 + 4;
static_assert(kPPRedAcc % 2 == 0 && kPPRedAcc + 2 * 6 <= kPPRedInts, "acc (6 x u64) outside red[]");

// f(integral_constant<int, I>) for I = B .. E-1: a row loop whose index is a
// compile-time constant (each row slot has its own compile-time degree)
template <int B, int E, typename Fn>
__device__ __forceinline__ void static_for(Fn &&f)
{
    if constexpr (B < E) {
        f(std::integral_constant<int, B>());
        static_for<B + 1, E>(f);
    }
}

template <typename F> struct PPCw { static constexpr int C = sizeof(F) == 8 ? 1 : 2; };   // codewords per slot

template <typename P>
struct PPSlots {
    P *app[2], *c2v[2];
    uint32_t app_base[2], c2v_base[2];   // LDS byte addresses
    int *red;
};

template <typename P>
__device__ __forceinline__ PPSlots<P> pp_slots(unsigned char *smem, int N, int EA)
{
    static_assert(sizeof(P) == 8, "one 8-byte LDS word per slot element");
    PPSlots<P> s;
    const int SL = N + 3 + EA;
    P *b = reinterpret_cast<P *>(smem);
#pragma unroll
    for (int X = 0; X < 2; ++X) {
        s.app[X] = b + X * SL;
        s.c2v[X] = s.app[X] + (N + 3);
        s.app_base[X] = lds_addr_of(s.app[X]);
        s.c2v_base[X] = lds_addr_of(s.c2v[X]);
    }
    s.red = reinterpret_cast<int *>(b + 2 * SL);
    return s;
}

// Channel of the block step's 2C codewords (:214-238) staged into app[X][v].v[c]
// (v < N; codeword grp*2C + X*C + c), by the bit role (threads t0, t0 + nt, ...),
// 4 bits (one Philox call) per thread and step; unc[X*C + c] = this thread's
// uncoded errors. A missing codeword (past the batch) is staged as +1 samples:
// never a premise break, never counted. The check role stays out of it: with the
// f64 Box-Muller inlined into its loop, the compiler hoisted the channel's loop
// invariants and spilled 14 doubles per thread around every interval loop (1.2 GB
// of scratch write-backs per bench launch).
template <typename F, int SRC>
__device__ __forceinline__ void pp_channel(const DecodeArgs &a, const PPSlots<Pack<F, PPCw<F>::C>> &s, int N, int grp,
                                           int (&unc)[2 * PPCw<F>::C], int t0, int nt)
{
    constexpr int C = PPCw<F>::C;
#pragma unroll
    for (int q = 0; q < 2 * C; ++q) unc[q] = 0;
    const int ng4 = (N + 3) / 4;
    for (int t = t0; t < 2 * C * ng4; t += nt) {
        int q = 0;   // codeword of the step (compares, not a division; selects, not a dynamic index)
#pragma unroll
        for (int k = 1; k < 2 * C; ++k) q += t >= k * ng4 ? 1 : 0;
        const int g4 = t - q * ng4, X = q >= C ? 1 : 0, c = q - X * C;
        const int b = grp * 2 * C + q;
        auto *ap = X ? s.app[1] : s.app[0];
        if (b >= a.batch) {
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4)
                if (4 * g4 + q4 < N) ap[4 * g4 + q4].v[c] = F(1);
            continue;
        }
        const uint64_t cw = a.first_cw + (uint64_t)b;
        F yv[4];
        const int8_t *cvec;
        if (SRC == SRC_GIVEN) {
            cvec = a.c ? a.c + (size_t)b * N : nullptr;
            const F *y = reinterpret_cast<const F *>(a.y) + (size_t)b * N;
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) yv[q4] = 4 * g4 + q4 < N ? y[4 * g4 + q4] : F(0);
        } else {
            cvec = a.cw_table ? a.cw_table + (size_t)(cw % (uint64_t)a.cw_rows) * N : nullptr;
            uint32_t u[4];
            philox4x32_10<true>((uint32_t)g4, (uint32_t)cw, (uint32_t)(cw >> 32), a.stream_id, (uint32_t)a.seed,
                          (uint32_t)(a.seed >> 32), u);
            F n[4];
            box_muller(u[0], u[1], n[0], n[1]);
            box_muller(u[2], u[3], n[2], n[3]);
            const F sigma = (F)a.sigma;
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int v = 4 * g4 + q4;
                const int cv = (cvec && v < N) ? cvec[v] : 1;
                yv[q4] = (F)cv * (F(1) + sigma * n[q4]);
                if (a.y_out && v < N) reinterpret_cast<F *>(a.y_out)[(size_t)b * N + v] = yv[q4];
            }
        }
        int e = 0;
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
            const int v = 4 * g4 + q4;
            if (v < N) {
                const int cv = cvec ? cvec[v] : 1;
                const F qv = front_end<F>(yv[q4], a);
                ap[v].v[c] = qv;
                e += ((qv > F(0) ? 1 : -1) * cv < 0);
            }
        }
#pragma unroll
        for (int qq = 0; qq < 2 * C; ++qq) unc[qq] += qq == q ? e : 0;
    }
}

// A wave's sum of per-lane counts 0..7, bit-sliced: three ballots and popcounts on the
// scalar unit instead of a cross-lane shuffle tree.
__device__ __forceinline__ int wave_sum3(int x)
{
    return __builtin_popcountll(__builtin_amdgcn_ballot_w64((x & 1) != 0)) +
           2 * __builtin_popcountll(__builtin_amdgcn_ballot_w64((x & 2) != 0)) +
           4 * __builtin_popcountll(__builtin_amdgcn_ballot_w64((x & 4) != 0));
}

// Block sums of the step's (bit errors, uncoded errors, syndrome) per codeword and
// the per-codeword accounting (:270-288, :382-393) by thread 0; the codewords of a
// slot whose premise failed go to the re-decode list instead. Per lane the counts are
// small -- a bit-role lane holds CPT = 4 bit slots and one Philox group of each
// codeword (N <= 2048, rows_pp_supported), so its bit and uncoded errors are <= 4; a
// check-role lane holds the 0/1 syndrome of its rows -- so each wave sums them by
// ballots (wave_sum3; the syndrome is an OR) and lane 0 adds the wave's totals into
// red[kPPRedSums ...] with LDS atomics: one barrier, and only thread 0 reads the totals
// (it clears them for the next step).
template <int C, bool HB>
__device__ __forceinline__ void pp_account(const DecodeArgs &a, int *red, int grp, int (&sums)[6 * C], unsigned *redo,
                                           unsigned long long *acc)
{
    int *tot = red + kPPRedSums;
    const bool lane0 = (threadIdx.x & 63) == 0;
    if (!(LDPC_PP_TAILEXP & 4)) {
#pragma unroll
        for (int q = 0; q < 2 * C; ++q) {
            if constexpr (HB) {
                const int w = wave_sum3(sums[3 * q]), u = wave_sum3(sums[3 * q + 1]);
                if (lane0 && w) atomicAdd(&tot[3 * q], w);
                if (lane0 && u) atomicAdd(&tot[3 * q + 1], u);
            } else {
                if (__builtin_amdgcn_ballot_w64(sums[3 * q + 2] != 0) && lane0) atomicAdd(&tot[3 * q + 2], 1);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int v = 0; v < 6 * C; ++v) {
            sums[v] = tot[v];
            tot[v] = 0;
        }
        const int fl[2] = {red[0], red[1]};
        red[0] = red[1] = 0;   // read once per step; raised again only after the next B1
#pragma unroll
        for (int q = 0; q < 2 * C; ++q) {
            const int b = grp * 2 * C + q;
            if (b >= a.batch) continue;
            if (fl[q / C]) {
                const unsigned at = atomicAdd(&redo[0], 1u);
                redo[1 + at] = (unsigned)b;
                continue;
            }
            const int w = sums[3 * q], uc = sums[3 * q + 1], sf = sums[3 * q + 2] > 0;
            acc[0] += (unsigned long long)w;
            acc[1] += (unsigned long long)(w > 0);
            acc[2] += (unsigned long long)uc;
            acc[3] += 1ull;
            acc[5] += (unsigned long long)sf;
            if (w > 0 && a.hist) atomicAdd(&a.hist[w - 1], 1ull);
            if (a.frame_res) a.frame_res[b] = make_int4(w, uc, sf, 0);
        }
    }
}

// The check node of one row: fp64 (fast64.h cn_fast64) or an fp32 pair (cn_fast,
// MS and NMS with the device-verified reciprocal; VAR picks).
// store(k, message) scatters the new message of edge k, called as each message is
// formed, in per-edge order (LDPC_PP_STORE_ORDER), so the scatters overlap the selects
// of the later edges (fp64: cn_fast64; fp32 pairs: cn_fast_pair).
// fp64: the premise is folded into the hi-word maximum *pacc (fast64.h ACC), tested by
// the caller (LDPC_PP_STICKY); the returned value is always true.
template <typename F, int DC, int VAR, bool FDIV, int C, int DCA, typename Store>
__device__ __forceinline__ bool pp_check_node(const Pack<F, C> (&xin)[DCA], Pack<F, C> (&pv)[DCA], F alpha, F rcp,
                                              F delta, Store store, uint32_t *pacc)
{
    if constexpr (sizeof(F) == 8) {
        return cn_fast64<DC, VAR, FDIV, DCA, Store, LDPC_PP_STORE_ORDER != 0, true>(xin, pv, alpha, rcp, delta, store,
                                                                                     pacc);
    } else {
        return cn_fast_pair<DC, DCA, Store, LDPC_PP_STORE_ORDER != 0>(xin, pv, VAR == V_NMS, alpha, rcp, store);
    }
}

// ---- one wave's work: R check rows of each slot, or (HB) CPT bit slots ----
// The split is per wave (an SGPR branch in the kernel): waves 0-7 hold rows t
// and t + 512 of the row schedule (R = 2), waves 8-15 the bit slots of schedule
// thread t - 512 (HB, R = 0). Row r runs a check node of compile-time degree
// DC0 (r = 0) or DC1 (r = 1): with the degree-aware slots (graph.h pp_row_slots)
// the younger check wave of each SIMD -- the SQ issues oldest-first, so it sets
// the interval -- holds only rows of degree <= 7 (DC0 = DC1 = 7) and the older
// one the degree-8 rows and the padding in its row 1 (DC1 = 8). A row of lower
// degree than its DC has padding edges: +inf gathers (no effect on min, sign or
// argmin) and scatters to the lane's dummy slot.
template <typename F, int SRC, int DC0, int DC1, int CPT, int VAR, bool FDIV, int R, bool HB>
__device__ __forceinline__ void pp_role(const DecodeArgs &a, const DevGraph &g, const RowSched &rs,
                                        const PPSlots<Pack<F, PPCw<F>::C>> &s, unsigned *redo,
                                        unsigned long long *acc)
{
    constexpr int C = PPCw<F>::C;
    using P = Pack<F, C>;
    constexpr int DCX = 8;                    // schedule stride (rs.dc)
    constexpr int RR = R > 0 ? R : 1;   // array extents
    static_assert(DC0 <= DCX && DC1 <= DCX && (R == 0) == HB, "pp_role shape");
    constexpr bool F64 = sizeof(F) == 8;
    const F kMax = F64 ? (F)kFast64Max : (F)1e30f;   // premise bound on |yq|
    const int tid = threadIdx.x, N = g.N, lane = tid & 63;
    [[maybe_unused]] const int EA = rs.e_pad + 64;   // c2v slots per codeword slot (LDPC_CHECK bounds)
    // check rows: schedule, and the c2v each sent last iteration, per slot
    // (entries past a row's DC are never touched, so they take no registers)
    [[maybe_unused]] int deg[RR];
    [[maybe_unused]] uint32_t colw[RR][DCX / 2], posw[RR][DCX / 2];
    [[maybe_unused]] P prev[2][RR][DCX];
    if constexpr (R > 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int j = tid + r * kPPRole;
            deg[r] = rs.cn_deg[j];
            const uint4 xc = reinterpret_cast<const uint4 *>(rs.cn_cols + (size_t)j * DCX)[0];
            const uint4 xp = reinterpret_cast<const uint4 *>(rs.cn_pos + (size_t)j * DCX)[0];
            colw[r][0] = xc.x; colw[r][1] = xc.y; colw[r][2] = xc.z; colw[r][3] = xc.w;
            posw[r][0] = xp.x; posw[r][1] = xp.y; posw[r][2] = xp.z; posw[r][3] = xp.w;
            if (deg[r] == 0)   // rows past M: gather the +0 entry, so their messages stay 0
#pragma unroll
                for (int q = 0; q < DCX / 2; ++q) colw[r][q] = (uint32_t)(N + 2) * 0x10001u;
        }
    }
    // bit slots of schedule thread bt
    const int bt = tid - kPPRole;
    [[maybe_unused]] int vgb[CPT], vgd[CPT];
    [[maybe_unused]] uint32_t vdst2[(CPT + 1) / 2] = {};
    if constexpr (HB) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int c = rs.vn_col[bt * CPT + i];
            vdst2[i / 2] |= (uint32_t)(c == 0xffff ? N + 1 : c) << (16 * (i & 1));
            const uint32_t info = rs.vn_info[bt * CPT + i];
            vgb[i] = __builtin_amdgcn_readfirstlane((int)(info & 0xffffu) - lane);
            vgd[i] = __builtin_amdgcn_readfirstlane((int)(info >> 24));
        }
        // padding slots of the bit-node layout hold +0 (adding +0 changes no sum); never written
        P z;
#pragma unroll
        for (int c = 0; c < C; ++c) z.v[c] = F(0);
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int dg = (int)((rs.vn_info[bt * CPT + i] >> 16) & 0xffu);
            const int base = vgb[i] + lane, gd = vgd[i];
            for (int k = dg; k < gd; ++k) {
                const int e = LDPC_CHK(base + k * 64, EA, CHK_PP_BIT_READ);
                s.c2v[0][e] = s.c2v[1][e] = z;
            }
        }
    }
    auto vdst = [&](int i) -> int { return (int)((vdst2[i / 2] >> (16 * (i & 1))) & 0xffffu); };
    const F alpha = (F)a.alpha, delta = (F)a.delta, rcp = F64 ? (F)(1.0 / a.alpha) : (F)a.alpha_rcp;
    const int nsteps = (a.batch + 2 * C - 1) / (2 * C);
    PP_STAMP_DECL;
    for (int grp = blockIdx.x; grp < nsteps; grp += gridDim.x) {
        PP_STAMP_TOP();
        [[maybe_unused]] uint32_t pacc[2] = {0u, 0u};   // fp64, LDPC_PP_STICKY: per-slot premise maximum
        constexpr bool TF = (LDPC_PP_TAILFUSE & (F64 ? 2 : 1)) != 0;
        int unc[2 * C];
        [[maybe_unused]] int wdec[2 * C];   // LDPC_PP_TAILFUSE: bit errors per codeword (bit role)
        [[maybe_unused]] int synd0[C];      // LDPC_PP_TAILFUSE: slot 0's syndrome (check role)
#pragma unroll
        for (int q = 0; q < 2 * C; ++q) unc[q] = wdec[q] = 0;
        if constexpr (HB) {
            if (!(LDPC_PP_TAILEXP & 1)) {
                pp_channel<F, SRC>(a, s, N, grp, unc, bt, kPPRole);
            } else {   // timing only: a constant channel
                for (int q = 0; q < 2 * C; ++q) unc[q] = 0;
                for (int v = bt; v < N; v += kPPRole)
                    for (int c = 0; c < C; ++c) s.app[0][v].v[c] = s.app[1][v].v[c] = F(1);
            }
        }
        PP_SYNC_STAMPED(1);   // B1: channel staged
        [[maybe_unused]] P yq[2][CPT];
        if constexpr (R > 0) {
#pragma unroll
            for (int X = 0; X < 2; ++X)
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int k = 0; k < DCX; ++k)
#pragma unroll
                        for (int c = 0; c < C; ++c) prev[X][r][k].v[c] = F(0);
        }
        if constexpr (HB) {
#pragma unroll
            for (int X = 0; X < 2; ++X) {
                bool in_ok = true;
#pragma unroll
                for (int i = 0; i < CPT; ++i) {
                    const P st = s.app[X][LDPC_CHK(vdst(i) <= N ? vdst(i) : 0, N + 3, CHK_PP_APP_WRITE)];
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        // yq + 0 maps -0 to +0, so app is never -0 (the fast check nodes' premise)
                        yq[X][i].v[c] = st.v[c] + F(0);
                        in_ok &= dabs(yq[X][i].v[c]) < kMax;
                    }
                }
#pragma unroll
                for (int i = 0; i < CPT; ++i) s.app[X][LDPC_CHK(vdst(i), N + 3, CHK_PP_APP_WRITE)] = yq[X][i];   // v2c = yq on the first pass (:364-370)
                if (!in_ok) s.red[X] = 1;
            }
            P inf, zero;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                inf.v[c] = dinf<F>();
                zero.v[c] = F(0);
            }
            if (tid == kPPRole) s.app[0][N] = s.app[1][N] = inf;
            if (tid == kPPRole + 1) s.app[0][N + 2] = s.app[1][N + 2] = zero;
        }
        PP_SYNC_STAMPED(3);   // B2: yq in app

        // Decisions and error weight of slot Y's codewords from its final posteriors
        // (bit slots; :270, :382-393), into w[Y*C + c].
        auto decide = [&](int Y, const P *post, int *w) {
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int q = Y * C + c, b = grp * 2 * C + q;
                if (b >= a.batch) continue;
                const int8_t *cvec =
                    SRC == SRC_GIVEN ? (a.c ? a.c + (size_t)b * N : nullptr)
                                     : (a.cw_table ? a.cw_table + (size_t)((a.first_cw + (uint64_t)b) % (uint64_t)a.cw_rows) * N
                                                   : nullptr);
                int e = 0;
#pragma unroll
                for (int i = 0; i < CPT; ++i) {
                    const int v = vdst(i);
                    if (v < N) {
                        const int d = post[i].v[c] > F(0) ? 1 : -1;   // :471-474
                        const int cv = cvec ? cvec[v] : 1;
                        e += (d != cv);
                        if (a.d_out) a.d_out[(size_t)b * N + v] = (int8_t)d;
                    }
                }
                w[q] = e;
            }
        };
        // Syndrome of slot X's codeword c (rows; padding edges read +inf: parity 0; rows past M skipped)
        auto syndrome = [&](int X, int c) -> int {
            int synd = 0;
            if constexpr (R > 0) {
                static_for<0, R>([&](auto rc) {
                    constexpr int r = decltype(rc)::value, DCr = r == 0 ? DC0 : DC1;
                    int par = 0;
#pragma unroll
                    for (int k = 0; k < DCr; ++k)
                        par ^= (s.app[X][LDPC_CHK(u16_at<DCX>(colw[r], k), N + 3, CHK_PP_GATHER)].v[c] > F(0)) ? 0 : 1;
                    synd |= deg[r] > 0 ? par : 0;
                });
            }
            return synd;
        };

        // One barrier interval: the rows of slot X (their reads first), the bit
        // nodes of slot 1 - X when `bits` (HB waves), then the rows' check nodes.
        auto interval = [&](auto Xc, bool rows, bool bits, bool last) {
            constexpr int X = decltype(Xc)::value, Y = 1 - X;
            [[maybe_unused]] P xin[RR][DCX];
            if constexpr (R > 0) {
                if (rows && LDPC_PP_EXP != 2) {
#pragma unroll
                    for (int r = 0; r < R; ++r)
#pragma unroll
                        for (int q = 0; q < DCX / 2; ++q) asm volatile("" : "+v"(colw[r][q]), "+v"(posw[r][q]));
                    const uint32_t ab = s.app_base[X];
                    static_for<0, (LDPC_PP_PREFETCH ? R : 1)>([&](auto rc) {
                        constexpr int r = decltype(rc)::value, DCr = r == 0 ? DC0 : DC1;
#pragma unroll
                        for (int k = 0; k < DCr; ++k)
                            xin[r][k] = lds_at<P>((LDPC_PP_EXP == 5 || LDPC_PP_EXP == 7) ? ab + 8u * (uint32_t)(lane + 64 * (k + 8 * r))
                                                                                         : LDPC_ADDR8(DCX, colw[r], k, ab, N + 3, CHK_PP_GATHER));
                    });
                    if constexpr (LDPC_PP_GATHER_FIRST && LDPC_PP_PREFETCH) {
                        // every gather of the interval issued ahead of the check-node arithmetic
                        constexpr int NG = DC0 + (R > 1 ? DC1 : 0);
                        __builtin_amdgcn_sched_group_barrier(0x2, NG, 1);     // their addresses
                        __builtin_amdgcn_sched_group_barrier(0x100, NG, 1);   // the ds_read_b64s
                    }
                }
            }
            if constexpr (HB) {
                if (LDPC_PP_BITDELAY > 0) __builtin_amdgcn_s_sleep(LDPC_PP_BITDELAY);
                if (bits && LDPC_PP_EXP != 1) {   // bit nodes: sum = yq + c2v in nlist order (:452-476)
#pragma unroll
                    for (int q = 0; q < (CPT + 1) / 2; ++q) asm volatile("" : "+v"(vdst2[q]));
                    P sum[CPT];
#pragma unroll
                    for (int i = 0; i < CPT; ++i) sum[i] = yq[Y][i];
                    int k = 0;
                    const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
                    vn_phases<F, C, CPT, CPT>(s.c2v[Y] + ln, vgb, vgd, k, sum, LDPC_CHK_LIM(EA - ln), CHK_PP_BIT_READ);
#pragma unroll
                    for (int i = 0; i < CPT; ++i) s.app[Y][LDPC_CHK(vdst(i), N + 3, CHK_PP_APP_WRITE)] = sum[i];
                    if (TF && last) decide(Y, sum, wdec);   // slot Y's final pass
                }
            }
            if constexpr (R > 0) {
                if (rows && LDPC_PP_EXP != 2) {
                    const uint32_t ab = s.app_base[X], cb = s.c2v_base[X];
                    static_for<0, R>([&](auto rc) {
                        constexpr int r = decltype(rc)::value, DCr = r == 0 ? DC0 : DC1;
                        if (!LDPC_PP_PREFETCH && r > 0) {
#pragma unroll
                            for (int k = 0; k < DCr; ++k) xin[r][k] = lds_at<P>(LDPC_ADDR8(DCX, colw[r], k, ab, N + 3, CHK_PP_GATHER));
                        }
                        bool ok = true;
                        // the scatter of edge k into the bit-slot layout (experiments: none, or lane-contiguous)
                        auto store = [&](int k, const P &m) {
                            if constexpr (LDPC_PP_EXP != 4)
                                lds_put<P>((LDPC_PP_EXP == 6 || LDPC_PP_EXP == 7)
                                               ? cb + 8u * (uint32_t)(lane + 64 * ((k + 8 * r + 16 * (tid >> 6)) % 112))
                                               : LDPC_ADDR8(DCX, posw[r], k, cb, EA, CHK_PP_SCATTER),
                                           m);
                        };
                        if constexpr (LDPC_PP_EXP == 3) {
#pragma unroll
                            for (int k = 0; k < DCr; ++k) {
#pragma unroll
                                for (int c = 0; c < C; ++c) prev[X][r][k].v[c] = xin[r][k].v[c] - prev[X][r][k].v[c];
                                store(k, prev[X][r][k]);
                            }
                        } else {
                            [[maybe_unused]] uint32_t pa = 0;
                            ok = pp_check_node<F, DCr, VAR, FDIV>(xin[r], prev[X][r], alpha, rcp, delta, store,
                                                                  LDPC_PP_STICKY ? &pacc[X] : &pa);
                            if constexpr (F64 && !LDPC_PP_STICKY) {
                                // rare: M2 >= 2^1000 (inf, NaN) or a tiny minimum in this row
                                if (__builtin_amdgcn_ballot_w64(pa >= kFast64MaxHi)) {
                                    asm volatile(";");   // a side effect: stays a skipped branch
                                    if (pa >= kFast64MaxHi && LDPC_PP_EXP == 0) s.red[X] = 1;
                                }
                            }
                        }
                        if (!ok && deg[r] > 0 && LDPC_PP_EXP == 0) s.red[X] = 1;   // experiments: never re-decode
                        if (R > 1 && LDPC_PP_ROWFENCE) __builtin_amdgcn_sched_barrier(0);   // keep the rows' live ranges apart
                    });
                }
            }
        };
        for (int it = 0; it < a.T; ++it) {
            interval(std::integral_constant<int, 0>(), true, it > 0, false);
            PP_BARRIER();   // | check(0,it) | bit(1,it-1) |
            interval(std::integral_constant<int, 1>(), true, true, it == a.T - 1);
            PP_BARRIER();   // | check(1,it) | bit(0,it) |
        }
        if (a.T > 0) {
            interval(std::integral_constant<int, 0>(), false, true, true);
            if (TF && !(LDPC_PP_TAILEXP & 2)) {   // slot 0's posteriors are final
#pragma unroll
                for (int c = 0; c < C; ++c) synd0[c] = syndrome(0, c);
            }
            PP_BARRIER();   // | syndrome(0) | bit(1,T-1) |
        }
        if constexpr (F64 && R > 0 && LDPC_PP_STICKY) {   // the premise of every iteration of the step
            if (pacc[0] >= kFast64MaxHi && LDPC_PP_EXP == 0) s.red[0] = 1;
            if (pacc[1] >= kFast64MaxHi && LDPC_PP_EXP == 0) s.red[1] = 1;
        }

        if (LDPC_PP_TAILEXP & 2) {   // timing only: no syndrome, decisions or error weights
            int sums[6 * C] = {};
            pp_account<C, HB>(a, s.red, grp, sums, redo, acc);
            continue;
        }
        // syndrome and decisions / error weight of the step's codewords (what the last
        // intervals have not formed already, LDPC_PP_TAILFUSE; T = 0: all of it here)
        const bool fused = TF && a.T > 0;
        if constexpr (HB) {
            if (!fused) {
#pragma unroll
                for (int X = 0; X < 2; ++X) {
                    P post[CPT];
#pragma unroll
                    for (int i = 0; i < CPT; ++i) post[i] = s.app[X][LDPC_CHK(vdst(i) <= N ? vdst(i) : 0, N + 3, CHK_PP_APP_WRITE)];
                    decide(X, post, wdec);
                }
            }
        }
        int sums[6 * C];
#pragma unroll
        for (int X = 0; X < 2; ++X) {
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int q = X * C + c;
                sums[3 * q] = wdec[q];
                sums[3 * q + 1] = unc[q];
                sums[3 * q + 2] = (X == 0 && fused) ? synd0[c] : syndrome(X, c);
            }
        }
        pp_account<C, HB>(a, s.red, grp, sums, redo, acc);
    }
    PP_STAMP_OUT()
}

}  // namespace

LDPC_CHECK_TU(rows_pp)

// Experiments: s_nop instructions at the kernel entry shift the code that follows by 4 bytes
// each (the code-layout sensitivity of the loops, with and without -falign-loops).
#ifndef LDPC_PP_ENTRY_NOPS
#define LDPC_PP_ENTRY_NOPS 0
#endif

// SPLIT: the schedule has degree-aware row slots (rs.dc_low == 7, graph.h
// pp_row_slots): check waves 4-7 run two 7-edge rows, waves 0-3 a 7-edge and an
// 8-edge row. Otherwise every row runs the 8-edge check node.
template <typename F, int SRC, int CPT, int VAR, bool FDIV, bool SPLIT>
__global__ __launch_bounds__(2 * kPPRole) void k_rows_pp(DecodeArgs a, DevGraph g, RowSched rs, unsigned *redo)
{
    using P = Pack<F, PPCw<F>::C>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
#pragma unroll
    for (int i = 0; i < LDPC_PP_ENTRY_NOPS; ++i) asm volatile("s_nop 0");
    const PPSlots<P> s = pp_slots<P>(smem, g.N, rs.e_pad + 64);
    unsigned long long *acc = reinterpret_cast<unsigned long long *>(s.red + kPPRedAcc);   // thread 0's block totals
    if (threadIdx.x == 0) {
        s.red[0] = s.red[1] = 0;
#pragma unroll
        for (int q = 0; q < 6; ++q) acc[q] = 0;
#pragma unroll
        for (int v = 0; v < 3 * kPPMaxCw; ++v) s.red[kPPRedSums + v] = 0;   // pp_account's totals
    }
    // the split is wave-uniform (an SGPR branch), so every wave meets every barrier
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool low = wave < kPPRole / 64;
    if (LDPC_PP_PRIO == 1 && low) __builtin_amdgcn_s_setprio(1);
    if (LDPC_PP_PRIO == 2 && !low) __builtin_amdgcn_s_setprio(1);
    if (LDPC_PP_PRIO == 3 && ((threadIdx.x >> 8) & 1)) __builtin_amdgcn_s_setprio(1);
    if (LDPC_PP_PRIO == 4 && low && wave >= kPPRole / 128) __builtin_amdgcn_s_setprio(1);
    if (LDPC_PP_PRIO == 5 && low) {
        if (wave >= kPPRole / 128) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(1);
    }
    if (!low)
        pp_role<F, SRC, 8, 8, CPT, VAR, FDIV, 0, true>(a, g, rs, s, redo, acc);
    else if (!SPLIT)
        pp_role<F, SRC, 8, 8, CPT, VAR, FDIV, 2, false>(a, g, rs, s, redo, acc);
    else if (wave >= kPPRole / 128)
        pp_role<F, SRC, 7, 7, CPT, VAR, FDIV, 2, false>(a, g, rs, s, redo, acc);
    else
        pp_role<F, SRC, 7, 8, CPT, VAR, FDIV, 2, false>(a, g, rs, s, redo, acc);
    if (threadIdx.x == 0 && acc[3] > 0) {
        acc[4] = acc[3] * (unsigned long long)a.T;
#pragma unroll
        for (int q = 0; q < 6; ++q) atomicAdd(&a.counts[q], acc[q]);
    }
}

int rows_pp_lds_bytes(const DevGraph &g, const RowSched &rs)
{
    return (int)(2 * (size_t)(g.N + 3 + rs.e_pad + 64) * 8 + kPPRedInts * sizeof(int));
}

bool rows_pp_supported(const DevGraph &g, const RowSched &rs)
{
    // N <= 4 * kPPRole: a bit-role lane then holds <= 4 bits and one Philox group per
    // codeword, the bound pp_account's ballot-sliced wave sums rely on
    return rs.threads == kPPRole && rs.rpt == 2 && rs.cpt == 4 && rs.dc == 8 && (rs.dc_low == 0 || rs.dc_low == 7) &&
           g.N <= 4 * kPPRole && g.N + 3 <= 0xffff && rows_pp_lds_bytes(g, rs) <= 160 * 1024;
}

template <typename F, int SRC, int VAR, bool FDIV>
static hipError_t launch_pp_t(const DevGraph &g, const RowSched &rs, const DecodeArgs &a, unsigned *redo,
                              hipStream_t s, int num_cus)
{
    auto fn = rs.dc_low == 7 ? k_rows_pp<F, SRC, 4, VAR, FDIV, true> : k_rows_pp<F, SRC, 4, VAR, FDIV, false>;
    const int lds = rows_pp_lds_bytes(g, rs);
    hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    constexpr int CW = 2 * PPCw<F>::C;
    const int nsteps = (a.batch + CW - 1) / CW;
    const int grid = std::min(num_cus, nsteps);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(2 * kPPRole), lds, s, a, g, rs, redo);
    return hipGetLastError();
}

hipError_t launch_rows_pp(const DevGraph &g, const RowSched &rs, const DecodeArgs &a, bool f64, unsigned *redo,
                          hipStream_t s, int num_cus)
{
    if (!rows_pp_supported(g, rs)) return hipErrorInvalidValue;
    const bool given = a.src == SRC_GIVEN;
#define LDPC_PP_SRC(FT, VARV, FD) \
    return given ? launch_pp_t<FT, SRC_GIVEN, VARV, FD>(g, rs, a, redo, s, num_cus) : launch_pp_t<FT, SRC_PHILOX, VARV, FD>(g, rs, a, redo, s, num_cus);
    if (!f64) {   // fp32 pairs: MS, or NMS with the verified reciprocal (rows_fast_f32_ok)
        if (a.variant == V_MS) { LDPC_PP_SRC(float, V_MS, false) }
        if (a.variant == V_NMS && a.nms_fast) { LDPC_PP_SRC(float, V_NMS, false) }
        return hipErrorInvalidValue;
    }
    if (a.variant == V_MS) { LDPC_PP_SRC(double, V_MS, false) }
    if (a.variant == V_OMS) { LDPC_PP_SRC(double, V_OMS, false) }
    if (markstein_exact_alpha(a.alpha)) { LDPC_PP_SRC(double, V_NMS, true) }
    LDPC_PP_SRC(double, V_NMS, false)
#undef LDPC_PP_SRC
}

}  // namespace ldpc
