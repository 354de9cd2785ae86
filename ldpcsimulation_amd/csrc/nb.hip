// nb.hip -- CDNA4 (gfx950) kernels of the non-binary GF(16) Extended Min-Sum
// decoder (BASELINE config 5; no reference counterpart:
// the reference's NB model, SystemC/NB-LDPC/inc/nodes.h, is a q^dc-LUT BP
// that does not compile). The algorithm is defined by the CPU oracle
// oracle/ems_oracle.c, which this reproduces bit for bit.
//
// Mapping: every node works on whole 16-entry message vectors held in the
// registers of ONE lane, so no cross-lane traffic is needed.
//   check node: one lane per (check, direction); the elementary check node
//     W(x) = min_a P(a) + R(a ^ x) is 256 register adds and mins, and the two
//     lanes of a check (same wave, lockstep) split the forward-backward
//     (cn_lane); messages are read and written as 4 x 16-byte chunks;
//   symbol node: one lane per symbol, entry a of an edge gathered from its
//     check-domain position h*a (GF(16) products by xtime in registers); it
//     also xors h*dec into its checks' syndrome bytes (LDS atomics), read and
//     cleared after the phase for the early stop.
// One workgroup (1024 threads for row degree <= 4, 512 for <= 8) decodes one
// codeword at a time (persistent over the batch); its edge messages (16 fp32
// per edge, in place: c2v after the check phase, v2c after the symbol phase)
// and bit LLRs live in LDS when they fit (128 KB of messages for N = 1000,
// E = 2000), else in a global slot per workgroup.
#include "nb.h"
#include "device_common.h"
#include "kernels.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

namespace ldpc {

constexpr float kInf = __builtin_huge_valf();

// Check-lane addresses recomputed per iteration (1) or hoisted by the compiler (0).
#ifndef LDPC_EMS_OPAQUE
#define LDPC_EMS_OPAQUE 1
#endif
// Timing-only ablations (wrong results; run with early stop off): 1 = no check
// nodes, 2 = no symbol nodes, 3 = no per-iteration syndrome, 4 = check and symbol
// nodes overlapped on two wave halves (one barrier interval per iteration; 5: the
// symbol nodes on the older half; 6: as 4, symbol waves at raised priority).
// 1: codewords handed out by a global ticket counter after the first grid (0: fixed stride).
#ifndef LDPC_EMS_TICKETS
#define LDPC_EMS_TICKETS 1
#endif
#ifndef LDPC_EMS_EXP
#define LDPC_EMS_EXP 0
#endif
// Wrong-result timing switches build only into A/B libraries (the *variant targets define
// LDPC_AB_BUILD); a product build with one of them set is refused.
#if LDPC_EMS_EXP != 0 && !defined(LDPC_AB_BUILD)
#error "LDPC_EMS_EXP != 0 gives wrong results by design: make nbvariant only"
#endif
// Diagnostic builds (-DLDPC_EMS_STAMPS, `make nbvariant`): per wave, s_memtime cycles
// per phase summed over the block's codewords, appended to $LDPC_EMS_STAMPS by nb_launch
// ([block][wave][8]: channel+init, check work, check wait, symbol work, symbol wait,
// syndrome, accounting, codewords). Never in the shipped kernel.
#ifdef LDPC_EMS_STAMPS
constexpr int kEmsStampBlocks = 256;
__device__ unsigned long long g_ems_stamps[kEmsStampBlocks * 16 * 8];
struct EmsStamps {
    unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long t = 0;
    __device__ void start() { t = __builtin_amdgcn_s_memtime(); }
    __device__ void lap(int k)
    {
        const unsigned long long n = __builtin_amdgcn_s_memtime();
        v[k] += n - t;
        t = n;
    }
};
#define EMS_LAP(k) st.lap(k)
#else
struct EmsStamps {
    __device__ void start() {}
};
#define EMS_LAP(k) ((void)0)
#endif
// The table reads of each thread's first symbol node (vn_pre) are issued before the
// check phase's barrier (1) or after it (0).
#ifndef LDPC_EMS_HOIST
#define LDPC_EMS_HOIST 1
#endif
// Symbol nodes of degree <= LDPC_EMS_VD keep their c2v in registers (0: re-read).
#ifndef LDPC_EMS_VD
#define LDPC_EMS_VD 2
#endif

// The graph, re-packed into LDS once per workgroup (global loads in the
// per-iteration loops would put dependent L2 round trips on every round).
// Edge slots are position-major: slot(j, k) = k*M + j for check j and mlist
// position k, so the check-node lanes of a wave (consecutive j, same k) read
// consecutive 16-byte chunks. Messages are stored in the CHECK domain,
// chunk-major: entry x of slot s at float ((x >> 2) * Ep + (s ^ (x >> 2))) * 4 + (x & 3),
// Ep = 2^k slots (nb_ep), i.e. byte (s << 4) ^ nb_lambda(x, k): XOR-linear in x, so the
// symbol node's 16 gather addresses of an edge are one XOR each (Gray order). The
// chunk index XOR-ed into the slot's low bits spreads those gathers over the banks;
// a check wave's 16-byte chunks stay one permutation of consecutive units.
struct NbSched {
    int Ep, M, sh;           // sh = log2(Ep) + 4: the chunk bits of a byte offset
    const uint8_t *cn_d;     // [M]    check degree
    const uint32_t *vn;      // [N]    first col entry << 8 | degree
    const uint16_t *vslot;   // [E]    slots of each symbol, nlist order
    const uint8_t *vh;       // [E]    their coefficients
};

typedef __attribute__((address_space(3))) float LdsF;

// GF(16) (x^4 + x + 1): v * x.
__device__ __forceinline__ int gf16_xt(int v) { return ((v << 1) & 15) ^ ((v & 8) ? 3 : 0); }

// ---- check node: one lane per (check, direction), the message vectors in registers ----
template <int Q>
__device__ __forceinline__ void load_vec(const float *msg, int Ep, int slot, float (&v)[Q])
{
    slot = LDPC_CHK(slot, Ep, CHK_EMS_SLOT);
#pragma unroll
    for (int c = 0; c < Q / 4; ++c) {
        const float4 t = *reinterpret_cast<const float4 *>(msg + ((c * Ep + (slot ^ c)) << 2));
        v[4 * c] = t.x;
        v[4 * c + 1] = t.y;
        v[4 * c + 2] = t.z;
        v[4 * c + 3] = t.w;
    }
}

// keep the nm smallest entries by (value, symbol), the rest -> +inf (oracle trunc_nm)
template <int Q>
__device__ __forceinline__ void trunc_vec(float (&v)[Q], int nm)
{
    if (nm >= Q) return;
    int r[Q];
#pragma unroll
    for (int x = 0; x < Q; ++x) {
        int c = 0;
#pragma unroll
        for (int y = 0; y < Q; ++y)
            if (y < x)
                c += v[y] <= v[x];
            else if (y > x)
                c += v[y] < v[x];
        r[x] = c;
    }
#pragma unroll
    for (int x = 0; x < Q; ++x) v[x] = r[x] < nm ? v[x] : kInf;
}

// W(x) = min_a P(a) + R(a ^ x): the oracle's ecn(), the same single adds, exact min
// (A pairwise v_pk_add_f32 formulation measured 11 % slower on MI355X.)
template <int Q>
__device__ __forceinline__ void ecn_reg(const float (&P)[Q], const float (&R)[Q], float (&W)[Q])
{
#pragma unroll
    for (int x = 0; x < Q; ++x) {
        float w = P[0] + R[x];
#pragma unroll
        for (int a = 1; a < Q; ++a) w = fminf(w, P[a] + R[a ^ x]);
        W[x] = w;
    }
}

// fill absent (+inf) entries with max finite + offset, then store
template <int Q>
__device__ __forceinline__ void store_out(float *msg, int Ep, int slot, float (&w)[Q], int nm, float offset)
{
    slot = LDPC_CHK(slot, Ep, CHK_EMS_SLOT);
    if (nm < Q) {
        float mx = -1.0f;
#pragma unroll
        for (int x = 0; x < Q; ++x) mx = fmaxf(mx, w[x] < kInf ? w[x] : -1.0f);
#pragma unroll
        for (int x = 0; x < Q; ++x) w[x] = w[x] < kInf ? w[x] : mx + offset;
    }
#pragma unroll
    for (int c = 0; c < Q / 4; ++c)
        *reinterpret_cast<float4 *>(msg + ((c * Ep + (slot ^ c)) << 2)) =
            make_float4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
}

// Forward-backward EMS of one check of degree D, split over two lanes of the
// same wave: dir = 0 walks the edges in mlist order, dir = 1 in reverse (its
// forward chain is the oracle's backward chain B; ECN is symmetric in its
// operands, each sum being one commutative add). Each lane writes the
// outputs of its half: own positions lo .. D-1, lo = ceil(D/2) / floor(D/2).
// In place and race-free: the two lanes run the same instruction stream in
// lockstep; a re-read of an input (own position kp, kp >= lo + 1 > (D-2)/2)
// comes before this lane's own store to kp and never meets a position the
// partner lane has already written (its positions > kp of its own order,
// i.e. original positions <= D-2-kp < kp of ours).
// LDPC_EMS_PRIOBAL: a wave's priority falls with the elementary check nodes it
// completes, so that the waves a SIMD arbitrates oldest-first progress together and
// the VALU-bound phase does not end on one or two lone waves (which issue at half the
// SIMD's rate). The phase starts at 3 (ems_prio(0) before the lane's check loop); in
// each check row cn_lane counts its own elementary check nodes from 1, so the priority
// after them is 2, 1, 0, 0, ... per row: the first row runs 3 -> 2 -> 1 -> 0, a later
// row starts where the previous one ended (0 for degree >= 5) and runs 2 -> 1 -> 0.
// The recorded gain was measured with exactly this pattern: 2.0 dB 10.32-10.34 ->
// 10.71-10.76 Gbit/s. 0: no priorities.
#ifndef LDPC_EMS_PRIOBAL
#define LDPC_EMS_PRIOBAL 1
#endif
__device__ __forceinline__ void ems_prio(int e)
{
    if (!LDPC_EMS_PRIOBAL) return;
    switch (e) {
    case 0: __builtin_amdgcn_s_setprio(3); break;
    case 1: __builtin_amdgcn_s_setprio(2); break;
    case 2: __builtin_amdgcn_s_setprio(1); break;
    default: __builtin_amdgcn_s_setprio(0); break;
    }
}

template <int Q, int D>
__device__ __forceinline__ void cn_lane(float *msg, int Ep, int M, int j, int dir, int nm, float offset)
{
    int ne = 0;   // elementary check nodes done (LDPC_EMS_PRIOBAL)
    auto slot = [&](int kp) { return (dir ? D - 1 - kp : kp) * M + j; };
    float F[D - 1][Q];
    float U[Q], B[Q], W[Q];
    load_vec<Q>(msg, Ep, slot(0), F[0]);
    trunc_vec<Q>(F[0], nm);
#pragma unroll
    for (int kp = 1; kp <= D - 2; ++kp) {
        load_vec<Q>(msg, Ep, slot(kp), U);
        trunc_vec<Q>(U, nm);
        ecn_reg<Q>(F[kp - 1], U, F[kp]);
        ems_prio(++ne);
        trunc_vec<Q>(F[kp], nm);
    }
    const int lo = dir ? D / 2 : (D + 1) / 2;
    load_vec<Q>(msg, Ep, slot(D - 1), B);
    trunc_vec<Q>(B, nm);
#pragma unroll
    for (int kp = D - 2; kp >= 1; --kp) {
        if (kp >= lo) {
            ecn_reg<Q>(F[kp - 1], B, W);
            ems_prio(++ne);
            trunc_vec<Q>(W, nm);
            if (kp - 1 >= lo) {   // next backward step: read input kp BEFORE this lane overwrites it
                float Bn[Q];
                load_vec<Q>(msg, Ep, slot(kp), U);
                trunc_vec<Q>(U, nm);
                ecn_reg<Q>(B, U, Bn);
                ems_prio(++ne);
                trunc_vec<Q>(Bn, nm);
                store_out<Q>(msg, Ep, slot(kp), W, nm, offset);
#pragma unroll
                for (int x = 0; x < Q; ++x) B[x] = Bn[x];
            } else {
                store_out<Q>(msg, Ep, slot(kp), W, nm, offset);
            }
        }
    }
    store_out<Q>(msg, Ep, slot(D - 1), F[D - 2], nm, offset);
}

// GF(16) products h*a for a = 0..15: h*2^i by xtime (gf16_xt), then the xor of
// the powers in a.

// ---- symbol node: one lane per symbol, the 16-entry vectors in registers ----
// This symbol's share of the parity checks of the new decisions: h * dec xor-ed
// into its checks' syndrome bytes (slot = k*M + j: check j = slot mod M, k < DC).
// GF(16) sums are xors, so the order of the atomics does not matter.
template <int DC>
__device__ __forceinline__ void syndrome_edge(int M, int s, int hv, int d, uint32_t *synd)
{
    int j = LDPC_CHK(s, M * DC, CHK_EMS_SLOT);
#pragma unroll
    for (int k = 1; k < DC; ++k) j -= j >= M ? M : 0;
    const int h1 = hv & 15, h2 = gf16_xt(h1), h4 = gf16_xt(h2), h8 = gf16_xt(h4);
    const int hd = ((d & 1) ? h1 : 0) ^ ((d & 2) ? h2 : 0) ^ ((d & 4) ? h4 : 0) ^ ((d & 8) ? h8 : 0);
    if (hd) atomicXor(&synd[j >> 2], (uint32_t)hd << (8 * (j & 3)));
}
template <int DC>
__device__ __forceinline__ void vn_syndrome(const NbSched &sc, int e0, int e1, int d, uint32_t *synd)
{
    for (int e = e0; e < e1; ++e) syndrome_edge<DC>(sc.M, sc.vslot[e], sc.vh[e], d, synd);
}

// After the symbol phase's barrier: any check unsatisfied? Every syndrome word is
// read and cleared (the next contributions come after the next check phase's barrier).
// The block-wide OR goes through one flag word per wave in the dynamic LDS (not
// __syncthreads_or, whose static LDS word would move the messages off address 0);
// a flag word is rewritten two barriers after its last read at the earliest.
__device__ __forceinline__ int syndrome_read_reset(uint32_t *synd, int nw, int *flags)
{
    int fail = 0;
    for (int w = threadIdx.x; w < nw; w += blockDim.x) {
        fail |= synd[w] != 0u;
        synd[w] = 0u;
    }
    // only the waves holding syndrome words have a flag to give (N=1000: two of 16)
    const int nwv = (int)(blockDim.x >> 6), nf = nw < (int)blockDim.x ? (nw + 63) >> 6 : nwv;
    const int any = __any(fail);
    if ((threadIdx.x & 63) == 0 && (int)(threadIdx.x >> 6) < nf) flags[threadIdx.x >> 6] = any;
    __syncthreads();
    int r = 0;
    for (int i = 0; i < nf; ++i) r |= flags[i];
    return r;
}

// Message addresses of the symbol node. Entry a of an edge is the check-domain
// position h*a, stored at (h*a) ^ f, f = the slot's XOR swizzle (0 in the plain
// layout). A check node works on its stored vectors as they are: ECN(P shifted by
// f1, R shifted by f2) is ECN(P, R) shifted by f1 ^ f2 -- the same float sums, so
// the same minima -- and the host chooses f with the XOR over every check's slots
// = 0, so each output lands at exactly its own slot's swizzle. f spreads these
// gathers over the LDS banks (nb_api.cpp nb_swizzled_coefficients).
// Byte offsets: (s << 4) ^ lambda((h*a) ^ f) with lambda XOR-linear (nb_lambda), so
// offset(a) = offset(a minus its lowest bit) ^ lambda(h * that bit): one v_xor per
// entry (the (p >> 2) * Ep + s form of the 2-mod-8 stride cost ~6 VALU per entry).
// In LDS the offsets are ds addresses: the message base (0: the kernel has no static
// LDS; any base aligned beyond the message bytes works) XOR-ed in once. In global
// memory (GS) they are byte offsets from msg.
template <int Q, bool GS>
struct MsgAddr {
    float *msg;
    int sh, xbase;
    __device__ MsgAddr(float *m, int shift)
        : msg(m), sh(shift), xbase(GS ? 0 : (int)(unsigned)(uintptr_t)(LdsF *)m) {}
    __device__ int lam(int p) const { return (p << 2) ^ ((p >> 2) << sh); }
    __device__ void edge(int s, int hv, int (&ad)[Q]) const
    {
        s = LDPC_CHK(s, 1 << (sh - 4), CHK_EMS_SLOT);   // slots [0, Ep)
        const int h1 = hv & 15, f = hv >> 4;
        const int h2 = gf16_xt(h1), h4 = gf16_xt(h2), h8 = gf16_xt(h4);
        const int L[4] = {lam(h1), lam(h2), lam(h4), lam(h8)};
        ad[0] = xbase ^ (s << 4) ^ lam(f);
#pragma unroll
        for (int a = 1; a < Q; ++a) ad[a] = ad[a & (a - 1)] ^ L[__builtin_ctz(a)];
    }
    __device__ float ld(int off) const
    {
        if constexpr (GS) return *reinterpret_cast<const float *>(reinterpret_cast<const char *>(msg) + off);
        else return *(LdsF *)(uintptr_t)(unsigned)off;
    }
    __device__ void st(int off, float x) const
    {
        if constexpr (GS) *reinterpret_cast<float *>(reinterpret_cast<char *>(msg) + off) = x;
        else *(LdsF *)(uintptr_t)(unsigned)off = x;
    }
};

// The symbol node's table reads, which depend on no message: its bit LLRs, its
// edge range and, for degree <= K, each edge's slot and coefficient. With one
// symbol per thread they are issued before the check phase's barrier
// (ems_codeword), so the symbol phase starts without two dependent LDS round trips.
template <int Q, int K>
struct VnPre {
    float lv[4];            // the symbol's bit LLRs
    int e0, e1;
    int sk[K], hk[K];
};

template <int Q, int MB, int VD, bool GS>
__device__ __forceinline__ void vn_pre(const MsgAddr<Q, GS> &ma, int v, const NbSched &sc, const float *lam,
                                       VnPre<Q, (VD > 0 ? VD : 1)> &p)
{
    static_assert(Q == 16 && MB == 4, "GF(16)");
    const float4 l4 = *reinterpret_cast<const float4 *>(lam + v * MB);
    p.lv[0] = l4.x;
    p.lv[1] = l4.y;
    p.lv[2] = l4.z;
    p.lv[3] = l4.w;
    const uint32_t vp = sc.vn[v];
    p.e0 = vp >> 8;
    p.e1 = p.e0 + (vp & 255);
    if (VD > 0 && p.e1 - p.e0 <= VD) {
#pragma unroll
        for (int k = 0; k < (VD > 0 ? VD : 1); ++k)
            if (k < p.e1 - p.e0) {
                p.sk[k] = sc.vslot[p.e0 + k];
                p.hk[k] = sc.vh[p.e0 + k];
            }
    }
}

// Entry a (symbol domain) of an edge lives at check-domain position h*a. init:
// write v2c = L on every edge. Otherwise app = L + sum of the c2v (nlist order),
// decision argmin app (first minimum), v2c = (app - c2v) - min. Both add the new
// decision's syndrome contributions (syndrome_edge).
template <int Q, int MB, int VD, int DC, bool GS>
__device__ __forceinline__ void vn_post(const MsgAddr<Q, GS> &ma, int v, const NbSched &sc, uint8_t *dec, bool init,
                                        uint32_t *synd, VnPre<Q, (VD > 0 ? VD : 1)> &p)
{
    const int e0 = p.e0, e1 = p.e1;
    float app[Q];
#pragma unroll
    for (int a = 0; a < Q; ++a) {
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < MB; ++i)
            if (((a >> i) & 1) != (p.lv[i] < 0.0f)) s += fabsf(p.lv[i]);   // oracle symbol_llr
        app[a] = s;
    }
    int ad[Q];
    if (init) {
        for (int e = e0; e < e1; ++e) {
            ma.edge(sc.vslot[e], sc.vh[e], ad);
#pragma unroll
            for (int a = 0; a < Q; ++a) ma.st(ad[a], app[a]);
        }
    } else if (VD > 0 && e1 - e0 <= VD) {
        // degree <= VD: each c2v is read once and kept in registers with its
        // addresses (the loop below re-reads and re-addresses every edge)
        constexpr int K = VD > 0 ? VD : 1;
        const int deg = e1 - e0;
        float c[K][Q];
        int ak[K][Q];
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (k < deg) {
                ma.edge(p.sk[k], p.hk[k], ak[k]);
#pragma unroll
                for (int a = 0; a < Q; ++a) c[k][a] = ma.ld(ak[k][a]);
            }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (k < deg) {
#pragma unroll
                for (int a = 0; a < Q; ++a) app[a] += c[k][a];   // nlist order
            }
        int best = 0;
        float bv = app[0];
#pragma unroll
        for (int a = 1; a < Q; ++a)
            if (app[a] < bv) {
                bv = app[a];
                best = a;
            }
        dec[v] = (uint8_t)best;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (k < deg) syndrome_edge<DC>(sc.M, p.sk[k], p.hk[k], best, synd);
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (k < deg) {
                float t[Q], mn = kInf;
#pragma unroll
                for (int a = 0; a < Q; ++a) {
                    t[a] = app[a] - c[k][a];
                    mn = fminf(mn, t[a]);
                }
#pragma unroll
                for (int a = 0; a < Q; ++a) ma.st(ak[k][a], t[a] - mn);
            }
        return;
    } else {
        for (int e = e0; e < e1; ++e) {
            ma.edge(sc.vslot[e], sc.vh[e], ad);
#pragma unroll
            for (int a = 0; a < Q; ++a) app[a] += ma.ld(ad[a]);
        }
    }
    int best = 0;
    float bv = app[0];
#pragma unroll
    for (int a = 1; a < Q; ++a)
        if (app[a] < bv) {
            bv = app[a];
            best = a;
        }
    dec[v] = (uint8_t)best;
    vn_syndrome<DC>(sc, e0, e1, best, synd);
    if (init) return;
    for (int e = e0; e < e1; ++e) {
        ma.edge(sc.vslot[e], sc.vh[e], ad);
        float t[Q], mn = kInf;
#pragma unroll
        for (int a = 0; a < Q; ++a) {
            t[a] = app[a] - ma.ld(ad[a]);
            mn = fminf(mn, t[a]);
        }
#pragma unroll
        for (int a = 0; a < Q; ++a) ma.st(ad[a], t[a] - mn);
    }
}

template <int Q, int MB, int VD, int DC, bool GS>
__device__ __forceinline__ void vn_lane(const MsgAddr<Q, GS> &ma, int v, const NbSched &sc, const float *lam,
                                        uint8_t *dec, bool init, uint32_t *synd)
{
    VnPre<Q, (VD > 0 ? VD : 1)> p;
    vn_pre<Q, MB, VD, GS>(ma, v, sc, lam, p);
    vn_post<Q, MB, VD, DC, GS>(ma, v, sc, dec, init, synd, p);
}

template <int Q, int MB, int DC, int SRC, bool GS>
__device__ __forceinline__ void ems_codeword(const NbArgs &a, const NbDevGraph &g, int b, float *msg, float *lam,
                                             uint8_t *dec, const NbSched &sc, int *red, uint32_t *synd,
                                             EmsStamps &st)
{
    st.start();
    const int tid = threadIdx.x, nt = blockDim.x;
    const int N = g.N, M = g.M, Ep = sc.Ep;
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
    // ---- initial messages v2c = L (stored at the check-domain position h*x), decisions argmin L ----
    const MsgAddr<Q, GS> ma(msg, sc.sh);
    for (int v = tid; v < N; v += nt) vn_lane<Q, MB, 0, DC, GS>(ma, v, sc, lam, dec, true, synd);
    __syncthreads();
    int fail = syndrome_read_reset(synd, (M + 3) / 4, red + 48);
    EMS_LAP(0);
    int it = 0;
    // check lanes: in each wave, lanes 0-31 take 32 consecutive checks in mlist
    // order and lanes 32-63 the same checks reversed
    const int cdir = (tid >> 5) & 1, cpr = (nt >> 6) * 32;
    const int cj0 = (tid >> 6) * 32 + (tid & 31);
    constexpr int KV = LDPC_EMS_VD > 0 ? LDPC_EMS_VD : 1;
#if LDPC_EMS_EXP >= 4 && LDPC_EMS_EXP <= 6
    // Timing experiment (results wrong by design; run without early stop): the
    // overlap a second codeword would allow, on one message array. Waves 0-7 run
    // every check node, waves 8-15 every symbol node (5: the other way round, so
    // the latency-bound symbol waves are the older ones and win the oldest-first
    // VALU arbitration; 6: as 4 with the symbol waves at s_setprio 3), concurrently in one barrier interval per iteration -- the
    // cost of an iteration if the symbol phase of one codeword overlapped the check
    // phase of another.
    while (it < a.T && (!a.early_stop || fail)) {
        const int half = nt / 2;
        const bool check_role = LDPC_EMS_EXP == 5 ? tid >= half : tid < half;
        const int rt = tid < half ? tid : tid - half;
        if (LDPC_EMS_EXP == 6 && !check_role) __builtin_amdgcn_s_setprio(3);
        if (check_role) {
            const int cpr2 = (half >> 6) * 32;
            int cj = (rt >> 6) * 32 + (rt & 31);
            asm volatile("" : "+v"(cj));
            for (int j = cj; j < M; j += cpr2) {
                switch (sc.cn_d[j]) {
                case 2: cn_lane<Q, 2>(msg, Ep, M, j, cdir, a.nm, a.offset); break;
                case 3: cn_lane<Q, 3>(msg, Ep, M, j, cdir, a.nm, a.offset); break;
                case 4: cn_lane<Q, 4>(msg, Ep, M, j, cdir, a.nm, a.offset); break;
                default: break;
                }
            }
        } else {
            for (int v = rt; v < N; v += half) vn_lane<Q, MB, LDPC_EMS_VD, DC, GS>(ma, v, sc, lam, dec, false, synd);
        }
        __syncthreads();
        fail = syndrome_read_reset(synd, (M + 3) / 4, red + 48);
        ++it;
    }
#endif
    while ((LDPC_EMS_EXP < 4 || LDPC_EMS_EXP > 6) && it < a.T && (!a.early_stop || fail)) {
        // ---- check nodes ----
        // the lane's first check, opaque per iteration: its message addresses are
        // recomputed here (a few VALU) instead of being hoisted out of the
        // iteration loop and, at 128 VGPRs, spilled and reloaded every iteration
        int cj = cj0;
        if (LDPC_EMS_OPAQUE) asm volatile("" : "+v"(cj));
        ems_prio(0);
        for (int j = cj; j < M && LDPC_EMS_EXP != 1; j += cpr) {
            switch (sc.cn_d[j]) {
            case 2: cn_lane<Q, 2>(msg, Ep, M, j, cdir, a.nm, a.offset); break;
            case 3: cn_lane<Q, 3>(msg, Ep, M, j, cdir, a.nm, a.offset); break;
            case 4: cn_lane<Q, 4>(msg, Ep, M, j, cdir, a.nm, a.offset); break;
            default:
                if (DC > 4) {
                    switch (sc.cn_d[j]) {
                    case 5: cn_lane<Q, DC >= 5 ? 5 : 2>(msg, Ep, M, j, cdir, a.nm, a.offset); break;
                    case 6: cn_lane<Q, DC >= 6 ? 6 : 2>(msg, Ep, M, j, cdir, a.nm, a.offset); break;
                    case 7: cn_lane<Q, DC >= 7 ? 7 : 2>(msg, Ep, M, j, cdir, a.nm, a.offset); break;
                    case 8: cn_lane<Q, DC >= 8 ? 8 : 2>(msg, Ep, M, j, cdir, a.nm, a.offset); break;
                    default: break;
                    }
                }
                break;
            }
        }
        if (LDPC_EMS_PRIOBAL) __builtin_amdgcn_s_setprio(0);
        EMS_LAP(1);
        // the thread's first symbol: its table reads now, behind the check nodes
        // still running
        VnPre<Q, KV> pre;
        if (LDPC_EMS_HOIST && tid < N) vn_pre<Q, MB, LDPC_EMS_VD, GS>(ma, tid, sc, lam, pre);
        __syncthreads();
        EMS_LAP(2);
        // ---- symbol nodes: lane x = variable-domain symbol, reads c2v(x) at position h*x ----
        if (LDPC_EMS_EXP != 2) {
            if (tid < N) {
                if (!LDPC_EMS_HOIST) vn_pre<Q, MB, LDPC_EMS_VD, GS>(ma, tid, sc, lam, pre);
                vn_post<Q, MB, LDPC_EMS_VD, DC, GS>(ma, tid, sc, dec, false, synd, pre);
            }
            for (int v = tid + nt; v < N; v += nt)   // codes with more symbols than threads
                vn_lane<Q, MB, LDPC_EMS_VD, DC, GS>(ma, v, sc, lam, dec, false, synd);
        }
        EMS_LAP(3);
        __syncthreads();
        EMS_LAP(4);
        if (LDPC_EMS_EXP != 3) fail = syndrome_read_reset(synd, (M + 3) / 4, red + 48);
        EMS_LAP(5);
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
    // block sums: wave shuffles, lane 0 adds into the totals red[65..67] (LDS atomics),
    // one barrier, thread 0 reads and clears them; the caller's ticket barrier ends the
    // codeword (k_ems)
    int sums[3] = {be, se, unc};
    int *tot = red + 65;
#pragma unroll
    for (int v = 0; v < 3; ++v) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sums[v] += __shfl_xor(sums[v], o, 64);
        if ((tid & 63) == 0 && sums[v]) atomicAdd(&tot[v], sums[v]);
    }
    __syncthreads();
    if (tid == 0) {
#pragma unroll
        for (int v = 0; v < 3; ++v) {
            sums[v] = tot[v];
            tot[v] = 0;
        }
        atomicAdd(&a.counts[0], (unsigned long long)sums[0]);
        atomicAdd(&a.counts[1], (unsigned long long)(sums[1] > 0));
        atomicAdd(&a.counts[2], (unsigned long long)sums[2]);
        atomicAdd(&a.counts[3], 1ull);
        atomicAdd(&a.counts[4], (unsigned long long)it);
        atomicAdd(&a.counts[5], (unsigned long long)fail);
        atomicAdd(&a.counts[6], (unsigned long long)sums[1]);
        if (a.frame_res) a.frame_res[b] = make_int4(sums[0], sums[2], fail, it);
    }
    EMS_LAP(6);
#ifdef LDPC_EMS_STAMPS
    st.v[7] += 1;
#endif
}

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }


// dynamic LDS: [msg 16*Ep f32 (ems_lds only)] [lam N*m f32] [dec N u8] [cn_d M u8]
//              [vn N u32] [vslot E u16] [vh E u8] [synd ceil(M/4) u32] [red 48 i32] [flags 16 i32]
// (no static LDS: the messages start at LDS address 0, so the symbol node's XOR-formed
// offsets are its ds addresses as they are, without an add per entry)
__host__ __device__ inline size_t aux_bytes(const NbDevGraph &g)
{
    return align16((size_t)g.N * g.m * 4) + align16((size_t)g.N) + align16((size_t)g.M) +
           align16((size_t)g.N * 4) + align16((size_t)g.E * 2) + align16((size_t)g.E) +
           align16((size_t)(g.M + 3) / 4 * 4) + (16 * 3 + 16 + 4 + 4) * 4;
}

template <int Q, int MB, int DC, int SRC, bool GSTATE, int THREADS>
__global__ __launch_bounds__(THREADS) void k_ems(NbArgs a, NbDevGraph g, float *gscratch,
                                                            size_t slot_floats)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int Ep = nb_ep(g);
    unsigned char *p = smem;
    float *msg;
    if (GSTATE) {
        msg = gscratch + slot_floats * blockIdx.x;
    } else {
        msg = reinterpret_cast<float *>(p);
        p += align16((size_t)Ep * Q * 4);
    }
    float *lam = reinterpret_cast<float *>(p);
    p += align16((size_t)g.N * MB * 4);
    uint8_t *dec = p;
    p += align16((size_t)g.N);
    uint8_t *cn_d = p;
    p += align16((size_t)g.M);
    uint32_t *vn = reinterpret_cast<uint32_t *>(p);
    p += align16((size_t)g.N * 4);
    uint16_t *vslot = reinterpret_cast<uint16_t *>(p);
    p += align16((size_t)g.E * 2);
    uint8_t *vh = p;
    p += align16((size_t)g.E);
    uint32_t *synd = reinterpret_cast<uint32_t *>(p);   // check j: byte j & 3 of word j >> 2
    p += align16((size_t)(g.M + 3) / 4 * 4);
    int *red = reinterpret_cast<int *>(p);   // [48, 64) wave flags, [64] the ticket, [65, 68) the block totals
    for (int w = threadIdx.x; w < (g.M + 3) / 4; w += blockDim.x) synd[w] = 0u;
    if (threadIdx.x < 3) red[65 + threadIdx.x] = 0;   // the block totals (ems_codeword)
    for (int j = threadIdx.x; j < g.M; j += blockDim.x) cn_d[j] = (uint8_t)(g.row_ptr[j + 1] - g.row_ptr[j]);
    for (int v = threadIdx.x; v < g.N; v += blockDim.x)
        vn[v] = ((uint32_t)g.col_ptr[v] << 8) | (uint32_t)(g.col_ptr[v + 1] - g.col_ptr[v]);
    for (int e = threadIdx.x; e < g.E; e += blockDim.x) {
        vslot[e] = (uint16_t)g.col_pslot[e];
        vh[e] = g.col_h[e];
    }
    __syncthreads();
    const NbSched sc{Ep, g.M, nb_ep_log2(Ep) + 4, cn_d, vn, vslot, vh};
    EmsStamps st;
    // Codewords: blockIdx.x first, then tickets from a.ticket (a global counter), so a
    // block whose codewords stopped early takes more -- with early stop the iterations per
    // codeword vary, and a fixed stride left the launch to the block with the most. Thread
    // 0 draws the next ticket while the current codeword decodes (its latency hidden) and
    // publishes it in red[64] after the codeword (whose barriers separate the reads).
    [[maybe_unused]] unsigned nxt = 0;
    if (LDPC_EMS_TICKETS && threadIdx.x == 0) nxt = gridDim.x + atomicAdd(a.ticket, 1u);
    for (int b = blockIdx.x; b < a.batch;) {
        ems_codeword<Q, MB, DC, SRC, GSTATE>(a, g, b, msg, lam, dec, sc, red, synd, st);
        if (LDPC_EMS_TICKETS && threadIdx.x == 0) red[64] = (int)nxt;
        __syncthreads();   // the codeword's end (its totals read, the next ticket published)
        if (LDPC_EMS_TICKETS) {
            b = red[64];
            if (threadIdx.x == 0 && b < a.batch) nxt = gridDim.x + atomicAdd(a.ticket, 1u);
        } else {
            b += gridDim.x;
        }
    }
#ifdef LDPC_EMS_STAMPS
    if ((threadIdx.x & 63) == 0 && blockIdx.x < kEmsStampBlocks && (threadIdx.x >> 6) < 16)
        for (int k = 0; k < 8; ++k) g_ems_stamps[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 + k] = st.v[k];
#endif
}

constexpr size_t kNbMaxLds = 160 * 1024;

NbChoice nb_choose(const NbDevGraph &g, int maxdc)
{
    NbChoice ch;
    ch.dc = maxdc <= 4 ? 4 : 8;
    // DC = 4: 1024 threads (4 waves per SIMD; 128 VGPRs, spills only around
    // the codeword loop: 8.12 vs 8.00 Gbit/s at 2.0 dB with 512),
    // LDPC_OPT_EMS_THREADS = 512 the other build. DC = 8: 512 (its check node needs
    // ~180 VGPRs). LDS allows one workgroup per CU either way.
    ch.threads = 512;
    if (ch.dc == 4) {
        ch.threads = 1024;
        if (opt(LDPC_OPT_EMS_THREADS) == 512) ch.threads = 512;
    }
    const size_t aux = aux_bytes(g), msgb = align16((size_t)nb_ep(g) * g.q * 4);
    // The 16-bit schedule entries are the slot indices (< maxdc * M: vslot) and the
    // symbols (< N); the chunk stride Ep (maxdc * M rounded up to a power of two, up to
    // 65 536) only enters int offsets.
    if (maxdc > kNbMaxDc || aux > kNbMaxLds || (long)g.maxdc * g.M > 65535 || g.N > 65535) {
        ch.name = "";   // unsupported: degree, LDS schedule or 16-bit indices
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

LDPC_CHECK_TU(nb)

template <int DC, int SRC, bool GS>
static hipError_t launch_t(const NbDevGraph &g, const NbArgs &a, const NbChoice &ch, void *scratch, int grid,
                           hipStream_t s)
{
    auto fn = (DC == 4 && ch.threads == 1024) ? k_ems<kNbQ, 4, DC, SRC, GS, 1024> : k_ems<kNbQ, 4, DC, SRC, GS, 512>;
    hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, ch.lds_bytes);
    if (e != hipSuccess) return e;
    if (!GS) {
        // MsgAddr XOR-s the message base into its offsets, which equals adding it only while
        // the messages sit at LDS address 0: a static __shared__ in k_ems (or in a helper it
        // inlines) would move the dynamic area and corrupt messages silently. Refuse instead.
        hipFuncAttributes fa;
        e = hipFuncGetAttributes(&fa, (const void *)fn);
        if (e != hipSuccess) return e;
        if (fa.sharedSizeBytes != 0) return hipErrorInvalidDeviceFunction;
    }
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
    if (g.q != kNbQ || g.m != 4 || !ch.name[0]) return hipErrorInvalidValue;
    int grid;
    if (ch.slot_bytes) {
        if (!scratch || slots <= 0) return hipErrorInvalidValue;
        grid = slots < a.batch ? slots : a.batch;
    } else {
        const int per_cu = (int)(kNbMaxLds / (size_t)ch.lds_bytes) >= 2 ? 2 : 1;
        grid = per_cu * num_cus;
        if (grid > a.batch) grid = a.batch;
    }
#ifdef LDPC_EMS_STAMPS
    const char *stamp_path = std::getenv("LDPC_EMS_STAMPS");
    void *sp = nullptr;
    if (stamp_path) {
        hipError_t e = hipGetSymbolAddress(&sp, HIP_SYMBOL(g_ems_stamps));
        if (e == hipSuccess) e = hipMemsetAsync(sp, 0, sizeof(g_ems_stamps), s);
        if (e != hipSuccess) return e;
    }
#endif
    if (LDPC_EMS_TICKETS) {
        if (!a.ticket) return hipErrorInvalidValue;
        const hipError_t e = hipMemsetAsync(a.ticket, 0, sizeof(unsigned), s);
        if (e != hipSuccess) return e;
    }
    const hipError_t err =
        ch.dc == 4 ? launch_dc<4>(g, a, ch, scratch, grid, s) : launch_dc<8>(g, a, ch, scratch, grid, s);
#ifdef LDPC_EMS_STAMPS
    if (stamp_path && err == hipSuccess) {
        static unsigned long long h[kEmsStampBlocks * 16 * 8];
        hipError_t e = hipMemcpyAsync(h, sp, sizeof(h), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
        if (FILE *f = std::fopen(stamp_path, "ab")) {
            std::fwrite(h, sizeof(h[0]), sizeof(h) / sizeof(h[0]), f);
            std::fclose(f);
        }
    }
#endif
    return err;
}

}  // namespace ldpc
