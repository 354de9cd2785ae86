/*
 * ems_oracle.c -- CPU ORACLE of the non-binary GF(q) Extended Min-Sum decoder
 * (test infrastructure only; see ldpc_oracle.h -- never linked by the product).
 *
 * PARITY UNPINNED against the reference: it has no EMS. Its NB-LDPC model
 * (SystemC/NB-LDPC/inc/nodes.h:82-166 symbol node, :240-293 check node) is a
 * probability-domain BP over a q^dc combination LUT and does not compile
 * (SURVEY §2, §8(f) row 4). What the reference does fix, and this follows:
 *   - the NB alist format (SystemC/NB-LDPC/src/alist.cpp:23-56: "N M q",
 *     (index, GF value) pairs per column and per row) -- parsed by
 *     ldpcsimulation_amd/codes.py and passed here as CSR arrays;
 *   - the message model: per edge a q-vector over GF(q), the H coefficient
 *     acting as a permutation of the vector (README.md "Belief Propagation
 *     For LDPC Codes"), decision = most likely symbol, stop when H z = 0.
 * The check-node rule is the EMS of Declercq & Fossorier, "Decoding
 * algorithms for nonbinary LDPC codes over GF(q)", IEEE Trans. Commun. 55(4),
 * 2007, in the forward-backward form of Voicila et al. (IEEE Trans. Commun.
 * 58(5), 2010), exactly as DESIGN.md §11 defines it. The HIP kernel
 * (ldpcsimulation_amd/csrc/nb.hip) reproduces it bit for bit; the q = 2 case
 * reduces to binary min-sum and is cross-checked against the reference-pinned
 * min-sum oracle (tests/test_ems.py).
 *
 * Messages are reliabilities: L(a) >= 0, 0 for the most likely symbol.
 * Build: oracle/Makefile (-ffp-contract=off; every sum is one IEEE fp32 add).
 */
#include "ldpc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* Primitive polynomials of GF(2^m) (bit m included). */
int orc_gf_poly(int q)
{
    switch (q) {
    case 2: return 0x3;
    case 4: return 0x7;      /* x^2+x+1 */
    case 8: return 0xB;      /* x^3+x+1 */
    case 16: return 0x13;    /* x^4+x+1 */
    case 32: return 0x25;    /* x^5+x^2+1 */
    case 64: return 0x43;    /* x^6+x+1 */
    default: return 0;
    }
}

/* a*b in GF(q): carry-less shift-and-add, reduced by the primitive polynomial. */
int orc_gf_mul(int q, int a, int b)
{
    const int poly = orc_gf_poly(q);
    int r = 0;
    while (b) {
        if (b & 1) r ^= a;
        b >>= 1;
        a <<= 1;
        if (a & q) a ^= poly;
    }
    return r;
}

static int log2i(int q)
{
    int m = 0;
    while ((1 << m) < q) ++m;
    return m;
}

/* Bit LLRs of the BPSK front-end: lam = (4*y)/N0 in fp32 (decodeBP.cpp:188's
 * 4y/N0 without the MAXLLR clip). Bit i of symbol v is sample v*m + i. */
void orc_nb_front(const float *y, int n, float n0, float *lam)
{
    for (int i = 0; i < n; ++i) lam[i] = (4.0f * y[i]) / n0;
}

/* Symbol reliabilities: L(a) = sum over bits i (ascending) that disagree with
 * the hard decision (lam_i < 0 -> 1) of |lam_i|. */
static void symbol_llr(const float *lam, int m, int q, float *L)
{
    for (int a = 0; a < q; ++a) {
        float s = 0.0f;
        for (int i = 0; i < m; ++i) {
            const float l = lam[i];
            const int hd = l < 0.0f;
            if (((a >> i) & 1) != hd) s += fabsf(l);
        }
        L[a] = s;
    }
}

/* Keep the nm smallest entries, ordered by (value, symbol); the rest -> +inf. */
static void trunc_nm(float *v, int q, int nm)
{
    if (nm >= q) return;
    float t[64];
    memcpy(t, v, sizeof(float) * (size_t)q);
    for (int x = 0; x < q; ++x) {
        int r = 0;
        for (int y = 0; y < q; ++y)
            if (t[y] < t[x] || (t[y] == t[x] && y < x)) ++r;
        if (r >= nm) v[x] = INFINITY;
    }
}

/* Elementary check node: W(x) = min over a of P(a) + Q(a ^ x). */
static void ecn(const float *P, const float *Q, float *W, int q)
{
    for (int x = 0; x < q; ++x) {
        float w = INFINITY;
        for (int a = 0; a < q; ++a) {
            const float s = P[a] + Q[a ^ x];
            w = s < w ? s : w;
        }
        W[x] = w;
    }
}

static int argmin_first(const float *v, int q)
{
    int b = 0;
    for (int a = 1; a < q; ++a)
        if (v[a] < v[b]) b = a;
    return b;
}

static int syndrome_fail(int M, int q, const int *row_ptr, const int *row_col, const int *row_h, const uint8_t *d)
{
    for (int j = 0; j < M; ++j) {
        int s = 0;
        for (int e = row_ptr[j]; e < row_ptr[j + 1]; ++e) s ^= orc_gf_mul(q, row_h[e], d[row_col[e]]);
        if (s) return 1;
    }
    return 0;
}

/* EMS decode of one frame.
 *   row_ptr[M+1], row_col[E], row_h[E]: checks in row order, edges in mlist
 *     order (edge slot e = row_ptr[j] + k), GF(q) coefficients 1..q-1;
 *   col_ptr[N+1], col_slot[E]: for each symbol its edge slots in nlist order;
 *   lam[N*m]: bit LLRs (orc_nb_front);
 *   T: maximum iterations; nm: message truncation (nm >= q: none);
 *   offset: added to the largest kept value to fill absent symbols;
 *   early_stop: stop as soon as H d = 0 (checked before every iteration).
 * Writes d[N] (symbols) and *synd_fail; returns the iterations run. */
int orc_ems_decode(int N, int M, int q, const int *row_ptr, const int *row_col, const int *row_h,
                   const int *col_ptr, const int *col_slot, const float *lam, int T, int nm, float offset,
                   int early_stop, uint8_t *d, int *synd_fail)
{
    const int m = log2i(q), E = row_ptr[M];
    int maxdc = 1;
    for (int j = 0; j < M; ++j)
        if (row_ptr[j + 1] - row_ptr[j] > maxdc) maxdc = row_ptr[j + 1] - row_ptr[j];
    float *msg = (float *)malloc(sizeof(float) * (size_t)E * q);
    float *L = (float *)malloc(sizeof(float) * (size_t)N * q);
    float *U = (float *)malloc(sizeof(float) * (size_t)maxdc * q);
    float *F = (float *)malloc(sizeof(float) * (size_t)maxdc * q);
    float *B = (float *)malloc(sizeof(float) * (size_t)maxdc * q);
    float W[64], app[64], t[64];

    for (int v = 0; v < N; ++v) {
        symbol_llr(lam + (size_t)v * m, m, q, L + (size_t)v * q);
        for (int e = col_ptr[v]; e < col_ptr[v + 1]; ++e)
            memcpy(msg + (size_t)col_slot[e] * q, L + (size_t)v * q, sizeof(float) * (size_t)q);
        d[v] = (uint8_t)argmin_first(L + (size_t)v * q, q);
    }
    int fail = syndrome_fail(M, q, row_ptr, row_col, row_h, d);
    int it = 0;
    while (it < T && (!early_stop || fail)) {
        /* ---- check nodes ---- */
        for (int j = 0; j < M; ++j) {
            const int r0 = row_ptr[j], dg = row_ptr[j + 1] - r0;
            for (int k = 0; k < dg; ++k) {
                const int h = row_h[r0 + k];
                float *u = U + (size_t)k * q;
                for (int a = 0; a < q; ++a) u[orc_gf_mul(q, h, a)] = msg[(size_t)(r0 + k) * q + a];
                trunc_nm(u, q, nm);
            }
            memcpy(F, U, sizeof(float) * (size_t)q);
            for (int k = 1; k <= dg - 2; ++k) {
                ecn(F + (size_t)(k - 1) * q, U + (size_t)k * q, F + (size_t)k * q, q);
                trunc_nm(F + (size_t)k * q, q, nm);
            }
            memcpy(B + (size_t)(dg - 1) * q, U + (size_t)(dg - 1) * q, sizeof(float) * (size_t)q);
            for (int k = dg - 2; k >= 1; --k) {
                ecn(B + (size_t)(k + 1) * q, U + (size_t)k * q, B + (size_t)k * q, q);
                trunc_nm(B + (size_t)k * q, q, nm);
            }
            for (int k = 0; k < dg; ++k) {
                const float *w;
                if (k == 0) {
                    w = B + q;
                } else if (k == dg - 1) {
                    w = F + (size_t)(k - 1) * q;
                } else {
                    ecn(F + (size_t)(k - 1) * q, B + (size_t)(k + 1) * q, W, q);
                    trunc_nm(W, q, nm);
                    w = W;
                }
                float mx = -1.0f;
                for (int x = 0; x < q; ++x)
                    if (w[x] < INFINITY && w[x] > mx) mx = w[x];
                float o[64];
                for (int x = 0; x < q; ++x) o[x] = w[x] < INFINITY ? w[x] : mx + offset;
                const int h = row_h[r0 + k];
                for (int a = 0; a < q; ++a) msg[(size_t)(r0 + k) * q + a] = o[orc_gf_mul(q, h, a)];
            }
        }
        /* ---- symbol nodes ---- */
        for (int v = 0; v < N; ++v) {
            for (int a = 0; a < q; ++a) {
                float s = L[(size_t)v * q + a];
                for (int e = col_ptr[v]; e < col_ptr[v + 1]; ++e) s += msg[(size_t)col_slot[e] * q + a];
                app[a] = s;
            }
            d[v] = (uint8_t)argmin_first(app, q);
            for (int e = col_ptr[v]; e < col_ptr[v + 1]; ++e) {
                float *mv = msg + (size_t)col_slot[e] * q;
                float mn = INFINITY;
                for (int a = 0; a < q; ++a) {
                    t[a] = app[a] - mv[a];
                    mn = t[a] < mn ? t[a] : mn;
                }
                for (int a = 0; a < q; ++a) mv[a] = t[a] - mn;
            }
        }
        fail = syndrome_fail(M, q, row_ptr, row_col, row_h, d);
        ++it;
    }
    *synd_fail = fail;
    free(msg); free(L); free(U); free(F); free(B);
    return it;
}
