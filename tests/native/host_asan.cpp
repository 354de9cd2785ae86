// Host-code sanitizer pass: the Tanner-graph compiler of
// libldpc_hip.so (ldpcsimulation_amd/csrc/graph.cpp: load_alist, build_graph,
// build_row_schedule, build_flood_schedule, build_layers) and the CPU oracle
// (oracle/*.c) built with -fsanitize=address,undefined and run over every code
// given on the command line, plus malformed inputs. Built and run by
// `make asan` (tests/test_host_asan.py); any sanitizer report aborts with a
// non-zero status.
#include "graph.h"
extern "C" {
#include "ldpc_oracle.h"
}

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

static int fails = 0;
#define CHECK(c, ...)                      \
    do {                                   \
        if (!(c)) {                        \
            std::printf("FAIL: " __VA_ARGS__); \
            std::printf("\n");             \
            ++fails;                       \
        }                                  \
    } while (0)

static void one_code(const char *path)
{
    ldpc_graph g;
    const std::string err = ldpc::load_alist(path, g);
    orc_alist H{};
    const int orc = orc_alist_load(path, &H);
    if (!err.empty()) {   // the reference's broken files must be rejected, not crash
        std::printf("%s: rejected (%s)\n", path, err.c_str());
        if (orc == 0) orc_alist_free(&H);
        return;
    }
    CHECK(orc == 0, "%s: oracle loader failed", path);
    CHECK(H.N == g.N && H.M == g.M, "%s: loaders disagree on N/M", path);
    // the same graph through build_graph from alist_struct-style arrays
    std::vector<const int *> nl(H.N), ml(H.M);
    for (int i = 0; i < H.N; ++i) nl[i] = H.nlist + (size_t)i * H.maxdv;
    for (int j = 0; j < H.M; ++j) ml[j] = H.mlist + (size_t)j * H.maxdc;
    ldpc_graph g2;
    const std::string e2 = ldpc::build_graph(H.N, H.M, H.deg_n, nl.data(), H.deg_m, ml.data(), g2);
    CHECK(e2.empty() && g2.E == g.E && g2.col_refs == g.col_refs, "%s: build_graph differs (%s)", path, e2.c_str());
    // every schedule shape the library may build
    int rows = 0;
    for (int threads : {64, 256, 512, 1024})
        for (int rpt : {1, 2, 3})
            for (int cpt : {1, 2, 4})
                for (int dc : {8, 16, 32}) {
                    ldpc::RowSchedule rs;
                    if (ldpc::build_row_schedule(g, threads, cpt, dc, rpt, rs).empty()) {
                        ++rows;
                        CHECK((int)rs.cn_cols.size() == threads * rpt * dc, "%s: row schedule size", path);
                    }
                }
    // the ping-pong kernel's degree-aware row slots: a permutation of the rows in which
    // every capped slot (row 0 of every thread, row 1 of the upper half) holds degree <= 7
    for (int threads : {128, 512}) {
        const std::vector<int> slots = ldpc::pp_row_slots(g, threads, 7);
        if (slots.empty()) continue;
        std::vector<int> seen(g.M, 0);
        for (size_t t = 0; t < slots.size(); ++t) {
            const int j = slots[t];
            if (j < 0) continue;
            CHECK(j < g.M && !seen[j]++, "%s: pp_row_slots not a permutation", path);
            const bool capped = t < (size_t)threads || (int)(t % threads) >= threads / 2;
            CHECK(!capped || g.row_deg[j] <= 7, "%s: degree-%d row in a capped slot", path, (int)g.row_deg[j]);
        }
        for (int j = 0; j < g.M; ++j) CHECK(seen[j] == 1, "%s: row %d missing from pp_row_slots", path, j);
        ldpc::RowSchedule rs;
        const std::string er = ldpc::build_row_schedule(g, threads, 4, 8, 2, rs, &slots);
        CHECK(er.empty() || er == "bits exceed slots", "%s: pp row schedule (%s)", path, er.c_str());
        ++rows;
    }
    ldpc::FloodSchedule fs;
    const std::string ef = ldpc::build_flood_schedule(g, fs);
    if (ef.empty()) {
        ldpc::LayerSchedule ls;
        const std::string el = ldpc::build_layers(g, fs, ls);
        CHECK(el.empty() && (int)ls.row_order.size() == g.M, "%s: layers (%s)", path, el.c_str());
    }
    // the oracle decodes a few frames (fp64 and fp32, flooding and layered) and runs the frame loop
    const int N = H.N;
    std::vector<double> y(N);
    std::vector<float> yf(N);
    std::vector<int8_t> d(N);
    orc_rng rng;
    orc_srandom(&rng, 7);
    for (int i = 0; i < N; ++i) {
        y[i] = 1.0 + 0.8 * orc_rann(&rng);
        yf[i] = (float)y[i];
    }
    orc_cfg cfg{};
    cfg.variant = ORC_NMS;
    cfg.alpha = 1.25;
    const int T = N > 20000 ? 2 : 5;
    orc_decode_f64(&H, y.data(), T, &cfg, d.data());
    orc_decode_f32(&H, yf.data(), T, &cfg, d.data());
    orc_decode_layered_f64(&H, y.data(), T, &cfg, nullptr, d.data());
    orc_stats st{};
    const int64_t fr = orc_minsum_run(&H, 0.5, 1.0, T, &cfg, 3, nullptr, 0, 3, nullptr, 0, &st);
    CHECK(fr == 3 && st.words == 3, "%s: frame loop", path);
    std::printf("%s: N=%d M=%d E=%d, %d row schedules, flood %s (coalesced slot accesses %.3f, %d groups)\n", path,
                g.N, g.M, g.E, rows, ef.empty() ? "ok" : ef.c_str(), fs.coalesced, fs.ngroups);
    orc_alist_free(&H);
}

int main(int argc, char **argv)
{
    for (int a = 1; a < argc; ++a) one_code(argv[a]);
    // malformed graphs: rejected with a message, never a crash
    {
        const int nn[2] = {1, 1}, nm[1] = {3};
        const int c0[1] = {1}, c1[1] = {1};
        const int *nl[2] = {c0, c1};
        const int r0[3] = {1, 2, 3};   // bit 3 does not exist
        const int *ml[1] = {r0};
        ldpc_graph g;
        CHECK(!ldpc::build_graph(2, 1, nn, nl, nm, ml, g).empty(), "out-of-range bit accepted");
    }
    {
        ldpc_graph g;
        CHECK(!ldpc::load_alist("/nonexistent/x.alist", g).empty(), "missing file accepted");
    }
    std::printf("%s (%d failures)\n", fails ? "FAILED" : "ok", fails);
    return fails ? 1 : 0;
}
