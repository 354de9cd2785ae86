// graph.cpp -- host-side Tanner-graph compiler and alist reader.
// See graph.h. Reference behaviour followed:
//   loadFile (C_implementations/src/alist.cpp:70-93): header "N M",
//   "maxdv maxdc", N column weights, M row weights, then exactly
//   N*maxdv and M*maxdc whitespace-separated 1-based indices (0 = pad),
//   read by fread_imatrix (src/r.cpp:277-300) irrespective of line breaks.
// Unlike the reference (which never validates and segfaults on the broken
// 802.11n files) every index and the row/column agreement is
// checked here; a malformed H is an LDPC_ERR_GRAPH, not undefined behaviour.
#include "graph.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <unordered_map>

namespace ldpc {

static std::string fmt(const char *f, long a = 0, long b = 0, long c = 0)
{
    char buf[256];
    std::snprintf(buf, sizeof buf, f, a, b, c);
    return buf;
}

std::string build_graph(int N, int M, const int *num_nlist, const int *const *nlist,
                        const int *num_mlist, const int *const *mlist, ldpc_graph &g)
{
    if (N <= 0 || M <= 0) return fmt("bad dimensions N=%ld M=%ld", N, M);
    if (!num_nlist || !nlist || !num_mlist || !mlist) return "null alist array";
    g = ldpc_graph();
    g.N = N;
    g.M = M;
    long E_rows = 0, E_cols = 0;
    for (int j = 0; j < M; ++j) {
        const int d = num_mlist[j];
        if (d < 0 || d > kMaxRowDegree)
            return fmt("check %ld has degree %ld (supported 0..%ld)", j, d, kMaxRowDegree);
        E_rows += d;
        g.maxdc = std::max(g.maxdc, d);
    }
    for (int i = 0; i < N; ++i) {
        const int d = num_nlist[i];
        if (d < 0 || d > 255) return fmt("bit %ld has degree %ld", i, d);
        E_cols += d;
        g.maxdv = std::max(g.maxdv, d);
    }
    if (E_rows != E_cols)
        return fmt("row weights sum to %ld but column weights to %ld", E_rows, E_cols);
    g.E = (int)E_rows;
    const int dcs = std::max(g.maxdc, 1);

    // Row view (mlist order) + position lookup for the column view.
    g.row_cols.assign((size_t)M * dcs, 0);
    g.row_deg.resize(M);
    std::vector<std::unordered_map<int, int>> pos(M);
    for (int j = 0; j < M; ++j) {
        g.row_deg[j] = (uint8_t)num_mlist[j];
        for (int k = 0; k < num_mlist[j]; ++k) {
            const int i = mlist[j][k] - 1;
            if (i < 0 || i >= N) return fmt("check %ld lists bit %ld (out of 1..N)", j, i + 1);
            g.row_cols[(size_t)j * dcs + k] = i;
            if (pos[j].count(i)) return fmt("check %ld lists bit %ld twice", j, i + 1);
            pos[j][i] = k;
        }
    }
    // Column view (nlist order) -> (check, position in that check's mlist).
    g.col_ptr.resize(N + 1);
    g.col_deg.resize(N);
    g.col_refs.resize(g.E);
    int e = 0;
    for (int i = 0; i < N; ++i) {
        g.col_ptr[i] = e;
        g.col_deg[i] = (uint8_t)num_nlist[i];
        for (int k = 0; k < num_nlist[i]; ++k) {
            const int j = nlist[i][k] - 1;
            if (j < 0 || j >= M) return fmt("bit %ld lists check %ld (out of 1..M)", i, j + 1);
            auto it = pos[j].find(i);
            if (it == pos[j].end())
                return fmt("bit %ld lists check %ld but that check does not list the bit", i, j + 1);
            if (it->second < 0) return fmt("bit %ld lists check %ld twice", i, j + 1);
            g.col_refs[e++] = ((uint32_t)j << kRefShift) | (uint32_t)it->second;
            it->second = -1 - it->second;   // mark used (detect duplicates)
        }
    }
    g.col_ptr[N] = e;
    return "";
}

std::string build_row_schedule(const ldpc_graph &g, int threads, int cpt, int dc, int rpt, RowSchedule &s)
{
    if (threads % 64 || (long)threads * rpt < g.M) return "rows exceed threads";
    if ((long)threads * cpt < g.N) return "bits exceed slots";
    if (g.maxdc > dc) return "row degree exceeds kernel bound";
    if (g.N > 65534) return "N exceeds 16-bit schedule";
    s = RowSchedule();
    s.threads = threads;
    s.cpt = cpt;
    s.dc = dc;
    s.rpt = rpt;
    const int rows = threads * rpt;
    // Stable sort of columns by decreasing degree -> slot order.
    std::vector<int> order(g.N);
    for (int i = 0; i < g.N; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return g.col_deg[a] > g.col_deg[b]; });
    const int nslots = threads * cpt;
    const int waves = threads / 64;
    const int ngroups = (g.N + 63) / 64;
    if (ngroups > waves * cpt) return "bits exceed slots";
    // Degree of each 64-column group (columns in decreasing-degree order) and
    // the base of its c2v block: edge kc of the group's lane l is at gbase + kc*64 + l.
    std::vector<int> gdeg(ngroups, 0), gbase(ngroups + 1, 0);
    for (int grp = 0; grp < ngroups; ++grp) {
        for (int l = 0; l < 64; ++l) {
            const int slot = grp * 64 + l;
            if (slot < g.N) gdeg[grp] = std::max(gdeg[grp], (int)g.col_deg[order[slot]]);
        }
        gbase[grp + 1] = gbase[grp] + 64 * gdeg[grp];
    }
    s.e_pad = gbase[ngroups];
    if (s.e_pad + 64 > 65535) return "padded edge count exceeds 16-bit schedule";
    if (s.e_pad < g.N) s.e_pad = g.N;   // the c2v area doubles as channel staging
    // Longest-processing-time assignment of groups to waves (a wave's bit-node
    // phase costs the sum of its groups' degrees), at most cpt groups per wave.
    std::vector<int> load(waves, 0), used(waves, 0), gw(ngroups), gi(ngroups);
    for (int grp = 0; grp < ngroups; ++grp) {   // groups are already in decreasing degree
        int best = -1;
        for (int w = 0; w < waves; ++w)
            if (used[w] < cpt && (best < 0 || load[w] < load[best])) best = w;
        gw[grp] = best;
        gi[grp] = used[best]++;
        load[best] += gdeg[grp];
    }
    s.vn_col.assign(nslots, 0xffff);
    s.vn_info.assign(nslots, 0);   // unused positions: group degree 0 (skipped)
    s.cn_cols.assign((size_t)rows * dc, 0);
    s.cn_pos.assign((size_t)rows * dc, 0);
    s.cn_deg.assign(rows, 0);
    for (int t = 0; t < rows; ++t)   // padding edges: read the +INF sentinel bit N, write the lane's dummy slot
        for (int k = 0; k < dc; ++k) {
            s.cn_cols[(size_t)t * dc + k] = (uint16_t)g.N;
            s.cn_pos[(size_t)t * dc + k] = (uint16_t)(s.e_pad + (t & 63));
        }
    for (int j = 0; j < g.M; ++j) {
        s.cn_deg[j] = g.row_deg[j];
        for (int k = 0; k < g.row_deg[j]; ++k)
            s.cn_cols[(size_t)j * dc + k] = (uint16_t)g.row_cols[(size_t)j * std::max(g.maxdc, 1) + k];
    }
    for (int grp = 0; grp < ngroups; ++grp) {
        for (int l = 0; l < 64; ++l) {
            const int slot = grp * 64 + l;
            const int t = gw[grp] * 64 + l;
            const size_t idx = (size_t)t * cpt + gi[grp];   // thread-major: a thread's slots are contiguous
            const int v = slot < g.N ? order[slot] : -1;
            const int d = v >= 0 ? g.col_deg[v] : 0;
            s.vn_col[idx] = v >= 0 ? (uint16_t)v : (uint16_t)0xffff;
            s.vn_info[idx] = (uint32_t)(gbase[grp] + l) | ((uint32_t)d << 16) | ((uint32_t)gdeg[grp] << 24);
            for (int kc = 0; kc < d; ++kc) {
                const uint32_t ref = g.col_refs[g.col_ptr[v] + kc];
                const int j = (int)(ref >> kRefShift), kr = (int)(ref & ((1u << kRefShift) - 1));
                s.cn_pos[(size_t)j * dc + kr] = (uint16_t)(gbase[grp] + kc * 64 + l);
            }
        }
    }
    // the kernel's bit-node phases rely on non-increasing group degree along a thread's slots
    for (int t = 0; t < threads; ++t)
        for (int i = 1; i < cpt; ++i)
            if ((s.vn_info[(size_t)t * cpt + i] >> 24) > (s.vn_info[(size_t)t * cpt + i - 1] >> 24))
                return "internal: bit slots not in non-increasing degree";
    return "";
}

std::string load_alist(const char *path, ldpc_graph &g)
{
    std::unique_ptr<FILE, int (*)(FILE *)> f(std::fopen(path, "r"), std::fclose);
    if (!f) return std::string("cannot open alist file: ") + (path ? path : "(null)");
    auto rd = [&](std::vector<int> &v, long n) -> bool {
        v.resize(n);
        for (long t = 0; t < n; ++t)
            if (std::fscanf(f.get(), "%d ", &v[t]) != 1) return false;
        return true;
    };
    std::vector<int> hdr, wn, wm, nl, ml;
    if (!rd(hdr, 4)) return std::string("truncated alist header: ") + path;
    const int N = hdr[0], M = hdr[1], mdv = hdr[2], mdc = hdr[3];
    if (N <= 0 || M <= 0 || mdv < 0 || mdc < 0) return std::string("bad alist header: ") + path;
    if (!rd(wn, N) || !rd(wm, M) || !rd(nl, (long)N * mdv) || !rd(ml, (long)M * mdc))
        return std::string("truncated alist body (fixed-width reader): ") + path;
    std::vector<const int *> np(N), mp(M);
    for (int i = 0; i < N; ++i) {
        if (wn[i] > mdv) return fmt("bit %ld weight %ld exceeds maxdv %ld", i, wn[i], mdv);
        np[i] = nl.data() + (size_t)i * mdv;
    }
    for (int j = 0; j < M; ++j) {
        if (wm[j] > mdc) return fmt("check %ld weight %ld exceeds maxdc %ld", j, wm[j], mdc);
        mp[j] = ml.data() + (size_t)j * mdc;
    }
    std::string err = build_graph(N, M, wn.data(), np.data(), wm.data(), mp.data(), g);
    if (!err.empty()) return err + " (" + path + ")";
    return "";
}

}  // namespace ldpc
