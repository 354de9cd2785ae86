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

std::vector<int> pp_row_slots(const ldpc_graph &g, int threads, int dc_low)
{
    const int half = threads / 2;
    if (threads % 128 || g.M > 2 * threads) return {};
    // capped slots in fill order: row 0 of every thread, then row 1 of threads half..threads-1
    std::vector<int> capped, open, out(2 * (size_t)threads, -1);
    for (int t = 0; t < threads; ++t) capped.push_back(t);
    for (int t = half; t < threads; ++t) capped.push_back(threads + t);
    for (int t = 0; t < half; ++t) open.push_back(threads + t);
    size_t nc = 0, no = 0;
    std::vector<int> rest;
    for (int j = 0; j < g.M; ++j) {
        if (g.row_deg[j] <= dc_low && nc < capped.size()) out[capped[nc++]] = j;
        else rest.push_back(j);
    }
    if (rest.size() > open.size()) return {};
    for (int j : rest) out[open[no++]] = j;
    return out;
}

std::string build_row_schedule(const ldpc_graph &g, int threads, int cpt, int dc, int rpt, RowSchedule &s,
                               const std::vector<int> *row_of_slot)
{
    if (threads % 64 || (long)threads * rpt < g.M) return "rows exceed threads";
    if (row_of_slot && row_of_slot->size() != (size_t)threads * rpt) return "row slot map has the wrong size";
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
    std::vector<int> slot_of(g.M, -1);   // row -> its slot
    for (int t = 0; t < rows; ++t) {
        const int j = row_of_slot ? (*row_of_slot)[t] : (t < g.M ? t : -1);
        if (j < -1 || j >= g.M || (j >= 0 && slot_of[j] >= 0)) return "row slot map is not a permutation";
        if (j >= 0) slot_of[j] = t;
    }
    for (int j = 0; j < g.M; ++j) {
        const int t = slot_of[j];
        if (t < 0) return "row slot map misses a row";
        s.cn_deg[t] = g.row_deg[j];
        for (int k = 0; k < g.row_deg[j]; ++k)
            s.cn_cols[(size_t)t * dc + k] = (uint16_t)g.row_cols[(size_t)j * std::max(g.maxdc, 1) + k];
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
                s.cn_pos[(size_t)slot_of[j] * dc + kr] = (uint16_t)(gbase[grp] + kc * 64 + l);
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

namespace ldpc {

// Chains from a successor vote: next[x] = the candidate with most votes (>= minv),
// each node taking at most one predecessor; the result lists every node once,
// chain by chain (cycles broken at their smallest unvisited node).
static std::vector<int> chain_order(int n, const std::vector<int> &next)
{
    std::vector<int> pred(n, -1), nx(n, -1);
    for (int x = 0; x < n; ++x)
        if (next[x] >= 0 && pred[next[x]] < 0 && next[x] != x) {
            nx[x] = next[x];
            pred[next[x]] = x;
        }
    std::vector<char> seen(n, 0);
    std::vector<int> order;
    order.reserve(n);
    auto walk = [&](int h) {
        for (int x = h; x >= 0 && !seen[x]; x = nx[x]) {
            seen[x] = 1;
            order.push_back(x);
        }
    };
    for (int x = 0; x < n; ++x)
        if (pred[x] < 0) walk(x);   // chain heads
    for (int x = 0; x < n; ++x)
        if (!seen[x]) walk(x);      // pure cycles
    return order;
}

std::string build_flood_schedule(const ldpc_graph &g, FloodSchedule &s)
{
    s = FloodSchedule();
    const int N = g.N, M = g.M, dcs = std::max(g.maxdc, 1);
    if (g.maxdc > 26) return "row degree exceeds the flood kernel's packed row state";
    s.dc = std::max(g.maxdc, 1);
    // rows of each bit
    auto rows_of = [&](int c, int e) { return (int)(g.col_refs[g.col_ptr[c] + e] >> kRefShift); };
    // ---- row chains: successor = the row holding most of (columns + 1) ----
    std::vector<int> rnext(M, -1);
    {
        std::vector<int> cnt(M, 0), touched;
        for (int j = 0; j < M; ++j) {
            touched.clear();
            const int d = g.row_deg[j];
            for (int k = 0; k < d; ++k) {
                const int c = g.row_cols[(size_t)j * dcs + k] + 1;
                if (c >= N) continue;
                for (int e = 0; e < g.col_deg[c]; ++e) {
                    const int j2 = rows_of(c, e);
                    if (cnt[j2]++ == 0) touched.push_back(j2);
                }
            }
            int best = -1;
            for (int j2 : touched) {
                if (j2 != j && cnt[j2] >= 2 && 2 * cnt[j2] >= d && (best < 0 || cnt[j2] > cnt[best])) best = j2;
            }
            for (int j2 : touched) cnt[j2] = 0;
            rnext[j] = best;
        }
    }
    const std::vector<int> rorder = chain_order(M, rnext);
    // ---- slot alignment along the chains: slot k of the next row holds the
    // column matching slot k of this row (c + 1 first, the rest in sorted order) ----
    std::vector<std::vector<int>> slots(M);   // per row: original edge index k of each slot
    std::vector<int> rpos(M);
    for (int i = 0; i < M; ++i) rpos[rorder[i]] = i;
    std::vector<char> placed(M, 0);
    for (int i = 0; i < M; ++i) {
        const int j = rorder[i];
        const int d = g.row_deg[j];
        const int *rc = &g.row_cols[(size_t)j * dcs];
        const int jp = (i > 0 && rnext[rorder[i - 1]] == j) ? rorder[i - 1] : -1;   // chain predecessor
        if (jp < 0 || !placed[jp]) {   // chain head: slots by column index
            std::vector<int> ks(d);
            for (int k = 0; k < d; ++k) ks[k] = k;
            std::sort(ks.begin(), ks.end(), [&](int a, int b) { return rc[a] < rc[b]; });
            slots[j] = ks;
        } else {
            const int *pc = &g.row_cols[(size_t)jp * dcs];
            const std::vector<int> &ps = slots[jp];
            std::vector<int> ks(d, -1);
            std::vector<char> used(d, 0);
            for (size_t t = 0; t < ps.size() && t < (size_t)d; ++t) {   // c + 1 matches
                const int want = pc[ps[t]] + 1;
                for (int k = 0; k < d; ++k)
                    if (!used[k] && rc[k] == want) { ks[t] = k; used[k] = 1; break; }
            }
            std::vector<int> restk;
            for (int k = 0; k < d; ++k)
                if (!used[k]) restk.push_back(k);
            std::sort(restk.begin(), restk.end(), [&](int a, int b) { return rc[a] < rc[b]; });
            size_t r = 0;
            for (int t = 0; t < d; ++t)
                if (ks[t] < 0) ks[t] = restk[r++];
            slots[j] = ks;
        }
        placed[j] = 1;
    }
    // ---- bit chains: c -> the column in the same slot of the next row ----
    std::vector<int> cnext(N, -1);
    {
        std::vector<std::vector<std::pair<int, int>>> votes(N);
        for (int i = 0; i + 1 < M; ++i) {
            const int j = rorder[i], j2 = rorder[i + 1];
            if (rnext[j] != j2) continue;
            const int d = std::min<int>(g.row_deg[j], g.row_deg[j2]);
            for (int t = 0; t < d; ++t) {
                const int c = g.row_cols[(size_t)j * dcs + slots[j][t]];
                const int c2 = g.row_cols[(size_t)j2 * dcs + slots[j2][t]];
                auto &v = votes[c];
                bool hit = false;
                for (auto &pr : v)
                    if (pr.first == c2) { ++pr.second; hit = true; break; }
                if (!hit) v.push_back({c2, 1});
            }
        }
        for (int c = 0; c < N; ++c) {
            int best = -1, bv = 0;
            for (auto &pr : votes[c])
                if (pr.second > bv) { bv = pr.second; best = pr.first; }
            cnext[c] = best;
        }
    }
    // storage order: column chains in order of first use by (row order, slot)
    std::vector<int> corder0 = chain_order(N, cnext);
    std::vector<int> chain_id(N, -1), chain_start;
    {
        // split corder0 into chains (a chain continues while cnext links consecutive entries)
        for (int t = 0; t < N; ++t) {
            if (t == 0 || cnext[corder0[t - 1]] != corder0[t]) chain_start.push_back(t);
            chain_id[corder0[t]] = (int)chain_start.size() - 1;
        }
    }
    chain_start.push_back(N);
    std::vector<int> corder;
    corder.reserve(N);
    {
        std::vector<char> done(chain_start.size(), 0);
        auto emit = [&](int ch) {
            if (done[ch]) return;
            done[ch] = 1;
            for (int t = chain_start[ch]; t < chain_start[ch + 1]; ++t) corder.push_back(corder0[t]);
        };
        for (int i = 0; i < M; ++i) {
            const int j = rorder[i];
            for (int t = 0; t < (int)slots[j].size(); ++t)
                emit(chain_id[g.row_cols[(size_t)j * dcs + slots[j][t]]]);
        }
        for (int ch = 0; ch + 1 < (int)chain_start.size(); ++ch) emit(ch);
    }
    // ---- layouts ----
    s.ngroups = (N + 63) / 64;
    const int NP = s.ngroups * 64;
    s.pos_of_bit.assign(N, -1);
    s.bit_at.assign(NP, -1);
    s.pdeg.assign(NP, 0);
    for (int p = 0; p < N; ++p) {
        s.pos_of_bit[corder[p]] = p;
        s.bit_at[p] = corder[p];
        s.pdeg[p] = g.col_deg[corder[p]];
    }
    s.gbase.assign(s.ngroups, 0);
    long base = 0;
    for (int gi = 0; gi < s.ngroups; ++gi) {
        int gd = 0;
        for (int l = 0; l < 64; ++l) gd = std::max(gd, (int)s.pdeg[gi * 64 + l]);
        s.gbase[gi] = (int32_t)base;
        base += 64L * gd;
    }
    if (base + 64 > INT32_MAX) return "graph too large for the flood schedule";
    s.e_pad = (int)base;
    // c2v element of each edge (row j, original position k)
    std::vector<int32_t> qpos((size_t)M * dcs, -1);
    for (int c = 0; c < N; ++c) {
        const int p = s.pos_of_bit[c];
        for (int e = 0; e < g.col_deg[c]; ++e) {
            const uint32_t ref = g.col_refs[g.col_ptr[c] + e];
            const int j = (int)(ref >> kRefShift), k = (int)(ref & ((1u << kRefShift) - 1));
            qpos[(size_t)j * dcs + k] = s.gbase[p / 64] + 64 * e + (p % 64);
        }
    }
    s.chain_head.assign(M, 1);
    for (int i = 1; i < M; ++i) s.chain_head[i] = rnext[rorder[i - 1]] == rorder[i] ? 0 : 1;
    s.M_pad = (M + 63) / 64 * 64;
    s.row_of.assign(s.M_pad, -1);
    s.rdeg.assign(s.M_pad, 0);
    s.sp.assign((size_t)s.dc * s.M_pad, NP);   // padding slots: the +inf sentinel position NP
    s.sq.assign((size_t)s.dc * s.M_pad, 0);
    long coal = 0, tot = 0;
    for (int i = 0; i < s.M_pad; ++i) {
        for (int t = 0; t < s.dc; ++t) s.sq[(size_t)t * s.M_pad + i] = s.e_pad + (i & 63);
        if (i >= M) continue;
        const int j = rorder[i];
        s.row_of[i] = j;
        s.rdeg[i] = g.row_deg[j];
        for (int t = 0; t < g.row_deg[j]; ++t) {
            const int k = slots[j][t];
            s.sp[(size_t)t * s.M_pad + i] = s.pos_of_bit[g.row_cols[(size_t)j * dcs + k]];
            s.sq[(size_t)t * s.M_pad + i] = qpos[(size_t)j * dcs + k];
            if (i & 63) {
                ++tot;
                coal += s.sp[(size_t)t * s.M_pad + i] == s.sp[(size_t)t * s.M_pad + i - 1] + 1;
            }
        }
    }
    s.coalesced = tot ? (double)coal / (double)tot : 0.0;
    return "";
}

std::string build_layers(const ldpc_graph &g, const FloodSchedule &s, LayerSchedule &ls)
{
    ls = LayerSchedule();
    const int M = g.M, N = g.N;
    if ((int)s.row_of.size() < M) return "flood schedule missing";
    const int dcs = std::max(g.maxdc, 1);
    // Chain-level first-fit colouring. The flood schedule's row chains (a
    // quasi-cyclic block row: DVB-S2's 360-row groups) are split where a row
    // shares a bit with an earlier row of the same piece; each piece joins the
    // lowest layer none of its bits is in yet. Whole chains per layer keep the
    // gathers of consecutive lanes on consecutive positions (DVB-S2: 3.2
    // instead of 11.5 cache lines per 64-lane gather with row-level colouring,
    // at the same 17 layers). Pieces shorter than 32 rows (codes without
    // long chains, e.g. PEG) are coloured row by row.
    std::vector<int32_t> piece_start;
    {
        std::vector<int32_t> mark(N, -1);
        int cur = -1;
        for (int i = 0; i < M; ++i) {
            const int j = s.row_of[i];
            if (j < 0) return "padding inside the row order";
            const int32_t *rc = &g.row_cols[(size_t)j * dcs];
            bool clash = false;
            for (int k = 0; k < g.row_deg[j]; ++k) clash |= cur >= 0 && mark[rc[k]] == cur;
            if (cur < 0 || clash || (i < (int)s.chain_head.size() && s.chain_head[i])) {
                piece_start.push_back(i);
                cur = (int)piece_start.size() - 1;
            }
            for (int k = 0; k < g.row_deg[j]; ++k) mark[rc[k]] = cur;
        }
        piece_start.push_back(M);
        // pieces shorter than a wave gain no coalescing: colour their rows one by one
        std::vector<int32_t> ps;
        for (size_t c = 0; c + 1 < piece_start.size(); ++c) {
            if (piece_start[c + 1] - piece_start[c] >= 32) ps.push_back(piece_start[c]);
            else
                for (int i = piece_start[c]; i < piece_start[c + 1]; ++i) ps.push_back(i);
        }
        ps.push_back(M);
        piece_start.swap(ps);
    }
    std::vector<std::vector<int32_t>> bit_layers(N);
    std::vector<int32_t> layer_of(M, -1), forbid;
    int nlayers = 0;
    for (size_t c = 0; c + 1 < piece_start.size(); ++c) {
        forbid.clear();
        for (int i = piece_start[c]; i < piece_start[c + 1]; ++i) {
            const int j = s.row_of[i];
            const int32_t *rc = &g.row_cols[(size_t)j * dcs];
            for (int k = 0; k < g.row_deg[j]; ++k)
                for (int32_t L : bit_layers[rc[k]]) forbid.push_back(L);
        }
        std::sort(forbid.begin(), forbid.end());
        int L = 0;
        for (int32_t f : forbid) {
            if (f == L) ++L;
            else if (f > L) break;
        }
        nlayers = std::max(nlayers, L + 1);
        for (int i = piece_start[c]; i < piece_start[c + 1]; ++i) {
            layer_of[i] = L;
            const int j = s.row_of[i];
            for (int k = 0; k < g.row_deg[j]; ++k) bit_layers[g.row_cols[(size_t)j * dcs + k]].push_back(L);
        }
    }
    // layered order: layer by layer, chain order inside a layer
    std::vector<int32_t> cnt(nlayers + 1, 0), pos_i(M);
    for (int i = 0; i < M; ++i) ++cnt[layer_of[i] + 1];
    for (int L = 0; L < nlayers; ++L) cnt[L + 1] += cnt[L];
    ls.lptr = cnt;
    for (int i = 0; i < M; ++i) pos_i[cnt[layer_of[i]]++] = i;
    ls.dc = s.dc;
    ls.M_pad = (M + 63) / 64 * 64;
    const int NP = s.ngroups * 64;
    ls.row_order.assign(M, -1);
    ls.rdeg.assign(ls.M_pad, 0);
    // positions ranked by degree, high first (stable: chains of equal-degree bits stay consecutive)
    std::vector<int32_t> by_deg(NP), rank(NP + 1);
    for (int p = 0; p < NP; ++p) by_deg[p] = p;
    std::stable_sort(by_deg.begin(), by_deg.end(), [&](int32_t x, int32_t y) { return s.pdeg[x] > s.pdeg[y]; });
    for (int q = 0; q < NP; ++q) rank[by_deg[q]] = q;
    rank[NP] = NP;   // the +inf sentinel keeps its place
    ls.pos_of_bit.resize(N);
    for (int v = 0; v < N; ++v) ls.pos_of_bit[v] = rank[s.pos_of_bit[v]];
    ls.sp.assign((size_t)ls.dc * ls.M_pad, NP);
    for (int n = 0; n < M; ++n) {
        const int i = pos_i[n];
        ls.row_order[n] = s.row_of[i];
        ls.rdeg[n] = s.rdeg[i];
        for (int k = 0; k < s.dc; ++k) ls.sp[(size_t)k * ls.M_pad + n] = rank[s.sp[(size_t)k * s.M_pad + i]];
    }
    return "";
}

}  // namespace ldpc
