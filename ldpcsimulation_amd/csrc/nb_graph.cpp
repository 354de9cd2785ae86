// nb_graph.cpp -- host-side graph code of the GF(q) EMS decoder (nb_graph.h).
#include "nb_graph.h"
#include "nb_layout.h"
#include "ldpc_hip.h"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <memory>

namespace ldpc {

namespace {
int fail(std::string &msg, int code, const char *fmt, ...) __attribute__((format(printf, 3, 4)));
int fail(std::string &msg, int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    msg = buf;
    return code;
}
}  // namespace

int gf_poly(int q)
{
    switch (q) {
    case 2: return 0x3;
    case 4: return 0x7;
    case 8: return 0xB;
    case 16: return 0x13;
    case 32: return 0x25;
    case 64: return 0x43;
    default: return 0;
    }
}

int gf_mul(int q, int a, int b)
{
    const int poly = gf_poly(q);
    int r = 0;
    while (b) {
        if (b & 1) r ^= a;
        b >>= 1;
        a <<= 1;
        if (a & q) a ^= poly;
    }
    return r;
}

// XOR swizzles of the message slots for the symbol-node gathers of nb.hip
// (vn_lane: entry a of an edge is read at check-domain position (h*a) ^ f,
// one ds_read_b32 per entry, the lanes of a wave on consecutive symbols).
// Those gathers hit random banks in the plain layout (f = 0): 3.7 LDS cycles
// per 32-lane group against 1 conflict-free (GF(16) N=1000 code). A local
// search picks f per slot under the constraint that the XOR of f over every
// check's slots is 0 (what keeps the check node's outputs in place), scoring
// the LDS bank model of the gathers: two groups of 32 lanes, bank = dword mod
// 32, cost = the most-used bank. Moves XOR the same delta into two slots of one
// check. Deterministic (fixed seed). Returned: col_h | f << 4 per column entry.
std::vector<uint8_t> nb_swizzled_coefficients(const ldpc_nb_graph &g, const std::vector<int32_t> &pslot,
                                                     const std::vector<uint8_t> &colh, const std::vector<uint8_t> &mul)
{
    std::vector<uint8_t> out(colh);
    if (g.q != kNbQ || g.E == 0) return out;
    const int Q = g.q, N = g.N, M = g.M, DV = std::max(g.maxdv, 1);
    const int lg = nb_ep_log2(nb_ep(g.maxdc, M));
    std::vector<uint8_t> f((size_t)g.maxdc * M, 0);
    std::vector<int> slot_v(f.size(), -1), slot_k(f.size(), 0);
    for (int v = 0; v < N; ++v)
        for (int e = g.col_ptr[v]; e < g.col_ptr[v + 1]; ++e) {
            slot_v[pslot[e]] = v;
            slot_k[pslot[e]] = e - g.col_ptr[v];
        }
    auto gcost = [&](int grp, int k) {   // summed over the Q entries of edge index k of a 32-symbol group
        int tot = 0;
        for (int a = 0; a < Q; ++a) {
            int cnt[32] = {0}, mx = 0;
            for (int v = grp * 32; v < std::min(N, grp * 32 + 32); ++v) {
                const int e = g.col_ptr[v] + k;
                if (e >= g.col_ptr[v + 1]) continue;
                const int sl = pslot[e], p = mul[(size_t)colh[e] * Q + a] ^ f[sl];
                mx = std::max(mx, ++cnt[((((unsigned)sl << 4) ^ (unsigned)nb_lambda(p, lg)) >> 2) & 31]);
            }
            tot += mx;
        }
        return tot;
    };
    const int ngroups = (N + 31) / 32;
    std::vector<int> C((size_t)ngroups * DV);
    for (int grp = 0; grp < ngroups; ++grp)
        for (int k = 0; k < DV; ++k) C[(size_t)grp * DV + k] = gcost(grp, k);
    uint32_t x = 0x9e3779b9u;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; };
    // a move needs two slots of one check: only checks of degree >= 2 take part
    std::vector<int> rows2;
    for (int j = 0; j < M; ++j)
        if (g.row_ptr[j + 1] - g.row_ptr[j] >= 2) rows2.push_back(j);
    if (rows2.empty()) return out;
    const long moves = std::min(200000L, 40L * g.E);
    for (long it = 0; it < moves; ++it) {
        const int j = rows2[rnd() % (uint32_t)rows2.size()], d = g.row_ptr[j + 1] - g.row_ptr[j];
        const int k1 = (int)(rnd() % (uint32_t)d);
        int k2 = (int)(rnd() % (uint32_t)(d - 1));
        if (k2 >= k1) ++k2;
        const uint8_t delta = (uint8_t)(1 + rnd() % (uint32_t)(Q - 1));
        const int s1 = k1 * M + j, s2 = k2 * M + j;
        const int a1 = (slot_v[s1] / 32) * DV + slot_k[s1], a2 = (slot_v[s2] / 32) * DV + slot_k[s2];
        const int before = C[a1] + (a2 != a1 ? C[a2] : 0);
        f[s1] ^= delta;
        f[s2] ^= delta;
        const int n1 = gcost(a1 / DV, a1 % DV), n2 = a2 != a1 ? gcost(a2 / DV, a2 % DV) : 0;
        if (n1 + n2 <= before) {
            C[a1] = n1;
            if (a2 != a1) C[a2] = n2;
        } else {
            f[s1] ^= delta;
            f[s2] ^= delta;
        }
    }
    for (int e = 0; e < g.E; ++e) out[e] = (uint8_t)(colh[e] | (f[pslot[e]] << 4));
    return out;
}

// Build the CSR views from (row, value) lists per column and (column, value) per row (0-based).
int nb_build_graph(int N, int M, int q, const NbLists &cols, const NbLists &rows, ldpc_nb_graph &g,
                   std::string &msg)
{
    if (N <= 0 || M <= 0) return fail(msg, LDPC_ERR_GRAPH, "bad dimensions N=%d M=%d", N, M);
    if (!gf_poly(q)) return fail(msg, LDPC_ERR_GRAPH, "q=%d is not a supported power of two (2..64)", q);
    g.N = N;
    g.M = M;
    g.q = q;
    g.m = 0;
    while ((1 << g.m) < q) ++g.m;
    g.row_ptr.assign(M + 1, 0);
    for (int j = 0; j < M; ++j) {
        if (rows[j].size() < 2) return fail(msg, LDPC_ERR_GRAPH, "check %d has degree %zu (< 2)", j, rows[j].size());
        g.row_ptr[j + 1] = g.row_ptr[j] + (int)rows[j].size();
        g.maxdc = std::max(g.maxdc, (int)rows[j].size());
    }
    g.E = g.row_ptr[M];
    g.row_col.resize(g.E);
    g.row_h.resize(g.E);
    std::vector<std::vector<std::pair<int, int>>> seen(N);   // (row, h) pairs from the row view
    for (int j = 0; j < M; ++j)
        for (size_t k = 0; k < rows[j].size(); ++k) {
            const int c = rows[j][k].first, h = rows[j][k].second;
            if (c < 0 || c >= N) return fail(msg, LDPC_ERR_GRAPH, "check %d: symbol index %d out of range", j, c + 1);
            if (h <= 0 || h >= q) return fail(msg, LDPC_ERR_GRAPH, "check %d: coefficient %d outside 1..q-1", j, h);
            for (const auto &pr : seen[c])
                if (pr.first == j) return fail(msg, LDPC_ERR_GRAPH, "check %d lists symbol %d twice", j, c + 1);
            g.row_col[g.row_ptr[j] + k] = c;
            g.row_h[g.row_ptr[j] + k] = (uint8_t)h;
            seen[c].push_back({j, (int)(g.row_ptr[j] + k)});
        }
    g.col_ptr.assign(N + 1, 0);
    g.col_slot.clear();
    g.col_slot.reserve(g.E);
    for (int i = 0; i < N; ++i) {
        if (cols[i].size() != seen[i].size())
            return fail(msg, LDPC_ERR_GRAPH, "symbol %d: column weight %zu but %zu rows list it", i + 1, cols[i].size(),
                       seen[i].size());
        for (const auto &ce : cols[i]) {
            const int j = ce.first;
            int slot = -1;
            for (const auto &pr : seen[i])
                if (pr.first == j) slot = pr.second;
            if (slot < 0) return fail(msg, LDPC_ERR_GRAPH, "symbol %d lists check %d, which does not list it", i + 1, j + 1);
            if (g.row_h[slot] != ce.second)
                return fail(msg, LDPC_ERR_GRAPH, "edge (%d,%d): coefficient %d in the column view, %d in the row view",
                           j + 1, i + 1, ce.second, g.row_h[slot]);
            g.col_slot.push_back(slot);
        }
        g.col_ptr[i + 1] = (int)g.col_slot.size();
        g.maxdv = std::max(g.maxdv, (int)cols[i].size());
    }
    return LDPC_OK;
}

int nb_read_alist(const char *path, ldpc_nb_graph &g, std::string &msg)
{
    std::unique_ptr<FILE, int (*)(FILE *)> f(std::fopen(path, "r"), std::fclose);
    if (!f) return fail(msg, LDPC_ERR_IO, "cannot open %s", path);
    auto rd = [&](int &v) { return std::fscanf(f.get(), "%d", &v) == 1; };
    int N = 0, M = 0, q = 0, dv = 0, dc = 0;
    if (!rd(N) || !rd(M) || !rd(q) || !rd(dv) || !rd(dc) || N <= 0 || M <= 0 || dv <= 0 || dc <= 0 ||
        N > (1 << 26) || M > (1 << 26) || dv > 1024 || dc > 1024)
        return fail(msg, LDPC_ERR_GRAPH, "%s: bad NB alist header", path);
    std::vector<int> wn(N), wm(M);
    bool ok = true;
    for (int i = 0; i < N && ok; ++i) ok = rd(wn[i]) && wn[i] >= 0 && wn[i] <= dv;
    for (int j = 0; j < M && ok; ++j) ok = rd(wm[j]) && wm[j] >= 0 && wm[j] <= dc;
    NbLists cols(N), rows(M);
    for (int i = 0; i < N && ok; ++i)
        for (int k = 0; k < dv && ok; ++k) {
            int a = 0, b = 0;
            ok = rd(a) && rd(b);
            if (k < wn[i]) cols[i].push_back({a - 1, b});
        }
    for (int j = 0; j < M && ok; ++j)
        for (int k = 0; k < dc && ok; ++k) {
            int a = 0, b = 0;
            ok = rd(a) && rd(b);
            if (k < wm[j]) rows[j].push_back({a - 1, b});
        }
    if (!ok) return fail(msg, LDPC_ERR_GRAPH, "%s: truncated or malformed NB alist", path);
    return nb_build_graph(N, M, q, cols, rows, g, msg);
}

void nb_tables(const ldpc_nb_graph &g, NbTables &t)
{
    const int q = g.q;
    t.mul.assign((size_t)q * q, 0);
    t.inv.assign(q, 0);
    for (int a = 0; a < q; ++a)
        for (int b = 0; b < q; ++b) {
            t.mul[(size_t)a * q + b] = (uint8_t)gf_mul(q, a, b);
            if (t.mul[(size_t)a * q + b] == 1) t.inv[a] = (uint8_t)b;
        }
    // position-major slot (k*M + j) and coefficient of every column entry
    t.pslot.assign(g.E, 0);
    t.colh.assign(g.E, 0);
    for (int j = 0; j < g.M; ++j)
        for (int r = g.row_ptr[j]; r < g.row_ptr[j + 1]; ++r)
            for (int e = g.col_ptr[g.row_col[r]]; e < g.col_ptr[g.row_col[r] + 1]; ++e)
                if (g.col_slot[e] == r) {
                    t.pslot[e] = (r - g.row_ptr[j]) * g.M + j;
                    t.colh[e] = g.row_h[r];
                }
    t.colh_swz = nb_swizzled_coefficients(g, t.pslot, t.colh, t.mul);
}

}  // namespace ldpc
