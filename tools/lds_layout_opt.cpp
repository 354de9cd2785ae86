// lds_layout_opt -- how far can the free choices of the ping-pong kernel's static
// schedule (graph.h build_row_schedule + pp_row_slots) cut its LDS bank conflicts?
// Host-only study tool (no device, not part of the library).
//
// Free choices that change no value (flooding rows are independent, the check node
// is symmetric in its edges, the bit node keeps its nlist order):
//   (a) which row a row slot holds, within the degree-aware classes of pp_row_slots;
//   (b) the order of a row's edges in its slot (gather k and scatter k move together);
//   (c) the (group, lane) of a column in the bit-slot-major c2v layout, among columns
//       of equal degree.
// Bank model (MI355X_MICROARCH LDS table): ds_read_b64 = 2 groups of 32 lanes, an
// 8-B word w on banks 2w, 2w+1 of 64 -> word bank w mod 32; ds_write_b64 = 4 groups
// of 16 lanes, word bank w mod 16; a group costs the most distinct words on one bank.
// Reported: array cycles per codeword-iteration, conflict-free vs the given
// schedule vs after a simulated-annealing search over (a)-(c).
//
// usage: lds_layout_opt ALIST [iterations] [seed]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

struct Code {
    int N = 0, M = 0;
    std::vector<std::vector<int>> rows, cols;   // 0-based, alist order
};

static Code load(const char *path)
{
    Code c;
    FILE *f = std::fopen(path, "r");
    if (!f) { std::perror(path); std::exit(1); }
    int maxdv, maxdc;
    if (std::fscanf(f, "%d %d %d %d", &c.N, &c.M, &maxdv, &maxdc) != 4) std::exit(1);
    std::vector<int> dv(c.N), dcv(c.M);
    for (auto &x : dv) if (std::fscanf(f, "%d", &x) != 1) std::exit(1);
    for (auto &x : dcv) if (std::fscanf(f, "%d", &x) != 1) std::exit(1);
    c.cols.resize(c.N);
    c.rows.resize(c.M);
    for (int i = 0; i < c.N; ++i)
        for (int k = 0; k < maxdv; ++k) {
            int v;
            if (std::fscanf(f, "%d", &v) != 1) std::exit(1);
            if (v > 0) c.cols[i].push_back(v - 1);
        }
    for (int j = 0; j < c.M; ++j)
        for (int k = 0; k < maxdc; ++k) {
            int v;
            if (std::fscanf(f, "%d", &v) != 1) std::exit(1);
            if (v > 0) c.rows[j].push_back(v - 1);
        }
    std::fclose(f);
    return c;
}

constexpr int T = 512, RPT = 2, CPT = 4, DC = 8, DCL = 7, SLOTS = T * RPT, BW = T / 64;

struct Layout {
    const Code *c;
    std::vector<int> slot_row;                 // [SLOTS] row or -1
    std::vector<std::vector<int>> ord;         // [M] column at edge position k
    std::vector<int> grp_of, lane_of;          // [N] column placement
    std::vector<int> gbase, gdeg;              // per group
    std::vector<std::vector<int>> at;          // [ngroups][64] column or -1
    std::vector<int> kc_of_edge;               // helper: (row, col) -> index in col's nlist, via map
    int e_pad = 0, ngroups = 0;
    std::vector<int> gw, gi;                   // group -> bit wave, slot index

    int kc(int j, int col) const
    {
        const auto &L = c->cols[col];
        for (int q = 0; q < (int)L.size(); ++q)
            if (L[q] == j) return q;
        std::abort();
    }
    static int slot_dc(int s) { const int r = s / T, t = s % T; return (t >= T / 2 || r == 0) ? DCL : DC; }
    // word of the gather of edge k of slot s
    int gword(int s, int k) const
    {
        const int j = slot_row[s];
        if (j < 0) return c->N + 2;
        if (k >= (int)c->rows[j].size()) return c->N;
        return ord[j][k];
    }
    int sword(int s, int k) const
    {
        const int j = slot_row[s];
        if (j < 0 || k >= (int)c->rows[j].size()) return e_pad + (s % T) % 64;
        const int col = ord[j][k];
        return gbase[grp_of[col]] + kc(j, col) * 64 + lane_of[col];
    }
    // cost of one lane group
    static int group_cost(const int *w, int n, int banks)
    {
        int cnt[64] = {0};
        int uniq[64];
        int nu = 0;
        for (int i = 0; i < n; ++i) {
            bool seen = false;
            for (int q = 0; q < nu; ++q) if (uniq[q] == w[i]) { seen = true; break; }
            if (!seen) { uniq[nu++] = w[i]; cnt[w[i] % banks]++; }
        }
        int m = 0;
        for (int b = 0; b < banks; ++b) m = std::max(m, cnt[b]);
        return m;
    }
    // gather half h (0,1) of instruction (wave w, row r, edge k)
    int gather_cost(int w, int r, int k, int h) const
    {
        int ws[32];
        for (int l = 0; l < 32; ++l) ws[l] = gword(r * T + 64 * w + 32 * h + l, k);
        return group_cost(ws, 32, 32);
    }
    int scatter_cost(int w, int r, int k, int q) const
    {
        int ws[16];
        for (int l = 0; l < 16; ++l) ws[l] = sword(r * T + 64 * w + 16 * q + l, k);
        return group_cost(ws, 16, 16);
    }
    int appw_cost(int bw, int i, int q) const
    {
        int ws[16];
        for (int l = 0; l < 16; ++l) {
            // the column at (bit wave bw, slot i, lane 16q + l)
            int col = -1;
            for (int g = 0; g < ngroups; ++g)
                if (gw[g] == bw && gi[g] == i) { col = at[g][16 * q + l]; break; }
            ws[l] = col >= 0 ? col : c->N + 1;
        }
        return group_cost(ws, 16, 16);
    }
    long total(long *parts = nullptr) const
    {
        long g = 0, s = 0, a = 0;
        for (int w = 0; w < BW; ++w)
            for (int r = 0; r < RPT; ++r) {
                const int dcr = slot_dc(r * T + 64 * w);
                for (int k = 0; k < dcr; ++k) {
                    for (int h = 0; h < 2; ++h) g += gather_cost(w, r, k, h);
                    for (int q = 0; q < 4; ++q) s += scatter_cost(w, r, k, q);
                }
            }
        for (int bw = 0; bw < BW; ++bw)
            for (int i = 0; i < CPT; ++i)
                for (int q = 0; q < 4; ++q) a += appw_cost(bw, i, q);
        if (parts) { parts[0] = g; parts[1] = s; parts[2] = a; }
        return g + s + a;
    }
};

static Layout initial(const Code &c)
{
    Layout L;
    L.c = &c;
    // pp_row_slots
    L.slot_row.assign(SLOTS, -1);
    std::vector<int> capped, open;
    for (int t = 0; t < T; ++t) capped.push_back(t);
    for (int t = T / 2; t < T; ++t) capped.push_back(T + t);
    for (int t = 0; t < T / 2; ++t) open.push_back(T + t);
    size_t nc = 0, no = 0;
    std::vector<int> rest;
    for (int j = 0; j < c.M; ++j) {
        if ((int)c.rows[j].size() <= DCL && nc < capped.size()) L.slot_row[capped[nc++]] = j;
        else rest.push_back(j);
    }
    for (int j : rest) L.slot_row[open[no++]] = j;
    L.ord = c.rows;
    // build_row_schedule: columns by decreasing degree (stable), 64-column groups, LPT waves
    std::vector<int> order(c.N);
    for (int i = 0; i < c.N; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return c.cols[a].size() > c.cols[b].size(); });
    L.ngroups = (c.N + 63) / 64;
    L.gdeg.assign(L.ngroups, 0);
    L.gbase.assign(L.ngroups + 1, 0);
    L.at.assign(L.ngroups, std::vector<int>(64, -1));
    L.grp_of.assign(c.N, -1);
    L.lane_of.assign(c.N, -1);
    for (int g = 0; g < L.ngroups; ++g) {
        for (int l = 0; l < 64; ++l) {
            const int sl = g * 64 + l;
            if (sl < c.N) {
                const int v = order[sl];
                L.at[g][l] = v;
                L.grp_of[v] = g;
                L.lane_of[v] = l;
                L.gdeg[g] = std::max(L.gdeg[g], (int)c.cols[v].size());
            }
        }
        L.gbase[g + 1] = L.gbase[g] + 64 * L.gdeg[g];
    }
    L.e_pad = std::max(L.gbase[L.ngroups], c.N);
    std::vector<int> load(BW, 0), used(BW, 0);
    L.gw.assign(L.ngroups, 0);
    L.gi.assign(L.ngroups, 0);
    for (int g = 0; g < L.ngroups; ++g) {
        int best = -1;
        for (int w = 0; w < BW; ++w)
            if (used[w] < CPT && (best < 0 || load[w] < load[best])) best = w;
        L.gw[g] = best;
        L.gi[g] = used[best]++;
        load[best] += L.gdeg[g];
    }
    return L;
}

int main(int argc, char **argv)
{
    if (argc < 2) { std::fprintf(stderr, "usage: %s ALIST [iterations] [seed]\n", argv[0]); return 2; }
    const Code c = load(argv[1]);
    const long iters = argc > 2 ? std::atol(argv[2]) : 200000;
    std::mt19937_64 rng(argc > 3 ? std::atol(argv[3]) : 1);
    Layout L = initial(c);
    long parts[3];
    // conflict-free reference: every group 1 cycle
    long ideal_g = 0, ideal_s = 0, ideal_a = 0;
    for (int w = 0; w < BW; ++w)
        for (int r = 0; r < RPT; ++r) { const int d = Layout::slot_dc(r * T + 64 * w); ideal_g += 2 * d; ideal_s += 4 * d; }
    ideal_a = BW * CPT * 4;
    long cur = L.total(parts);
    std::printf("conflict-free group cycles: gather %ld scatter %ld app_write %ld\n", ideal_g, ideal_s, ideal_a);
    std::printf("given schedule:             gather %ld scatter %ld app_write %ld  (extra %ld)\n", parts[0], parts[1],
                parts[2], cur - ideal_g - ideal_s - ideal_a);
    std::uniform_real_distribution<double> U(0, 1);
    double temp = 2.0;
    long best = cur;
    for (long it = 0; it < iters; ++it) {
        temp = 1e-9;
        const int mv = rng() % 3;
        if (mv == 0) {   // swap two row slots (classes respected)
            const int a = rng() % SLOTS, b = rng() % SLOTS;
            const int ja = L.slot_row[a], jb = L.slot_row[b];
            auto fits = [&](int s, int j) { return j < 0 || (int)c.rows[j].size() <= Layout::slot_dc(s); };
            if (a == b || !fits(a, jb) || !fits(b, ja)) continue;
            std::swap(L.slot_row[a], L.slot_row[b]);
            const long nv = L.total();
            if (nv <= cur || U(rng) < std::exp((cur - nv) / temp)) cur = nv;
            else std::swap(L.slot_row[a], L.slot_row[b]);
        } else if (mv == 1) {   // swap two edges of one row
            const int j = rng() % c.M, d = (int)c.rows[j].size();
            const int k1 = rng() % d, k2 = rng() % d;
            if (k1 == k2) continue;
            std::swap(L.ord[j][k1], L.ord[j][k2]);
            const long nv = L.total();
            if (nv <= cur || U(rng) < std::exp((cur - nv) / temp)) cur = nv;
            else std::swap(L.ord[j][k1], L.ord[j][k2]);
        } else {   // swap two columns of equal degree (group, lane)
            const int a = rng() % c.N, b = rng() % c.N;
            if (a == b || c.cols[a].size() != c.cols[b].size()) continue;
            auto sw = [&]() {
                std::swap(L.at[L.grp_of[a]][L.lane_of[a]], L.at[L.grp_of[b]][L.lane_of[b]]);
                std::swap(L.grp_of[a], L.grp_of[b]);
                std::swap(L.lane_of[a], L.lane_of[b]);
            };
            sw();
            const long nv = L.total();
            if (nv <= cur || U(rng) < std::exp((cur - nv) / temp)) cur = nv;
            else sw();
        }
        best = std::min(best, cur);
        if (it % (iters / 10 + 1) == 0) { std::fprintf(stderr, "it %ld cur %ld\n", it, cur); }
    }
    L.total(parts);
    std::printf("after search:               gather %ld scatter %ld app_write %ld  (extra %ld)\n", parts[0], parts[1],
                parts[2], cur - ideal_g - ideal_s - ideal_a);
    return 0;
}
