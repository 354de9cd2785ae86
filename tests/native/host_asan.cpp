// Host-code sanitizer pass: the Tanner-graph compiler of
// libldpc_hip.so (ldpcsimulation_amd/csrc/graph.cpp: load_alist, build_graph,
// build_row_schedule, build_flood_schedule, build_layers), the GF(q) graph code
// of the EMS decoder (nb_graph.cpp: the NB alist reader, the CSR build, the GF
// tables and the message-slot swizzle search), the CLIs' argument-file parsing
// (cli_common.h: codeword files, alist headers) and the CPU oracle (oracle/*.c),
// built with -fsanitize=address,undefined and run over every code given on the
// command line, plus malformed inputs. Built and run by `make asan`
// (tests/test_host_asan.py); any sanitizer report aborts with a non-zero status.
//   usage: host_asan [binary.alist ...] [--nb nb.alist ...] [--cw codeword-file ...] [--tmp DIR]
#include "graph.h"
#include "nb_graph.h"
#include "nb_layout.h"
#include "cli_common.h"
#include "ldpc_hip.h"
extern "C" {
#include "ldpc_oracle.h"
}

#include <sstream>

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

// An NB alist (SystemC/NB-LDPC/src/alist.cpp:23-56 format) through the loader and,
// when it loads, the tables the EMS context uploads; GF(16) codes get the slot swizzle,
// whose per-check XOR must be 0 (what keeps the check node's outputs in place).
static void one_nb(const char *path)
{
    ldpc_nb_graph g;
    std::string msg;
    const int rc = ldpc::nb_read_alist(path, g, msg);
    if (rc != LDPC_OK) {
        std::printf("%s: NB rejected (%d: %s)\n", path, rc, msg.c_str());
        CHECK(!msg.empty(), "%s: rejection without a message", path);
        return;
    }
    CHECK(g.row_ptr.size() == (size_t)g.M + 1 && g.col_ptr.size() == (size_t)g.N + 1 && (int)g.col_slot.size() == g.E,
          "%s: NB CSR sizes", path);
    ldpc::NbTables t;
    ldpc::nb_tables(g, t);
    CHECK((int)t.pslot.size() == g.E && (int)t.colh_swz.size() == g.E, "%s: NB tables", path);
    for (int a = 1; a < g.q; ++a) CHECK(t.mul[(size_t)a * g.q + t.inv[a]] == 1, "%s: GF inverse of %d", path, a);
    if (g.q == ldpc::kNbQ) {
        std::vector<int> x(g.M, 0);
        for (int e = 0; e < g.E; ++e) {
            CHECK((t.colh_swz[e] & 15) == t.colh[e], "%s: swizzle changed a coefficient", path);
            x[t.pslot[e] % g.M] ^= t.colh_swz[e] >> 4;
        }
        for (int j = 0; j < g.M; ++j) CHECK(x[j] == 0, "%s: check %d swizzles do not XOR to 0", path, j);
    }
    std::printf("%s: NB N=%d M=%d q=%d E=%d maxdv=%d maxdc=%d\n", path, g.N, g.M, g.q, g.E, g.maxdv, g.maxdc);
}

static std::string write_tmp(const std::string &dir, const std::string &name, const std::string &text)
{
    const std::string p = dir + "/" + name;
    FILE *f = std::fopen(p.c_str(), "wb");
    if (!f) { std::printf("FAIL: cannot write %s\n", p.c_str()); ++fails; return p; }
    std::fwrite(text.data(), 1, text.size(), f);
    std::fclose(f);
    return p;
}

// Malformed NB alists: each must be rejected with a message (never a crash).
static void nb_malformed(const std::string &dir)
{
    const char *bad[][2] = {
        {"empty", ""},
        {"header_only", "4 2 16\n2 4\n"},
        {"truncated", "4 2 16\n1 2\n1 1 1 1\n2 2\n1 3 0 0\n"},
        {"neg_header", "-4 2 16\n1 2\n"},
        {"huge_header", "100000000 2 16\n1 2\n"},
        {"q_not_pow2", "2 1 12\n1 2\n1 1\n2\n1 3 0 0\n1 3\n1 3 2 3\n"},
        {"degree1_check", "2 2 16\n1 1\n1 1\n1 1\n1 3\n2 4\n1 3\n2 4\n"},
        {"degree0_check", "2 2 16\n1 2\n1 1\n2 0\n1 3\n1 4\n1 3 2 4\n0 0 0 0\n"},
        {"index_out_of_range", "2 1 16\n1 2\n1 1\n2\n1 3\n1 4\n1 3 7 4\n"},
        {"coef_zero", "2 1 16\n1 2\n1 1\n2\n1 0\n1 4\n1 0 2 4\n"},
        {"coef_q", "2 1 16\n1 2\n1 1\n2\n1 16\n1 4\n1 16 2 4\n"},
        {"views_disagree", "2 1 16\n1 2\n1 1\n2\n1 3\n1 4\n1 5 2 4\n"},
        {"weight_above_max", "2 1 16\n1 2\n3 1\n2\n1 3\n1 4\n1 3 2 4\n"},
        {"weight_negative", "2 1 16\n1 2\n-1 1\n2\n1 3\n1 4\n1 3 2 4\n"},
        {"text", "this is not an alist\n"},
    };
    for (const auto &b : bad) {
        const std::string p = write_tmp(dir, std::string("nb_") + b[0] + ".alist", b[1]);
        ldpc_nb_graph g;
        std::string msg;
        const int rc = ldpc::nb_read_alist(p.c_str(), g, msg);
        CHECK(rc == LDPC_ERR_GRAPH && !msg.empty(), "NB %s accepted (rc %d)", b[0], rc);
    }
    // a valid two-symbol GF(16) code, then the same through the list interface
    const std::string ok = write_tmp(dir, "nb_ok.alist", "2 1 16\n1 2\n1 1\n2\n1 3\n1 4\n1 3 2 4\n");
    ldpc_nb_graph g;
    std::string msg;
    CHECK(ldpc::nb_read_alist(ok.c_str(), g, msg) == LDPC_OK, "NB valid code rejected (%s)", msg.c_str());
    ldpc::NbTables t;
    if (g.E) ldpc::nb_tables(g, t);
    ldpc_nb_graph g2;
    CHECK(ldpc::nb_build_graph(2, 1, 16, {{{0, 3}}, {{0, 4}}}, {{{0, 3}, {1, 4}}}, g2, msg) == LDPC_OK, "NB lists");
    CHECK(ldpc::nb_build_graph(0, 1, 16, {}, {{}}, g2, msg) == LDPC_ERR_GRAPH, "NB N = 0 accepted");
    CHECK(ldpc::nb_read_alist((dir + "/does_not_exist.alist").c_str(), g2, msg) == LDPC_ERR_IO, "NB missing file");
    for (int q : {2, 4, 8, 16, 32, 64})   // every field: a * inv(a) = 1 through the tables
        for (int a = 1; a < q; ++a) {
            int inv = 0;
            for (int b = 1; b < q; ++b) if (ldpc::gf_mul(q, a, b) == 1) inv = b;
            CHECK(inv != 0, "GF(%d): %d has no inverse", q, a);
        }
    CHECK(ldpc::nb_ep(4, 8200) == 65536 && ldpc::nb_ep_log2(65536) == 16, "chunk stride");
}

// The CLIs' codeword files (cli_common.h, decodeMinSum.cpp:136-143,193-212): the
// reference's eof/rewind rule and the per-symbol conversion over odd inputs.
static void one_codeword_file(const char *path, int N)
{
    const std::vector<std::string> lines = reference_codeword_lines(path);
    CHECK(!lines.empty(), "%s: no codeword line", path);
    std::vector<int8_t> c(N, 1);
    std::ostringstream log;
    for (const auto &l : lines) apply_codeword_line(l, N, c, log);
    for (int i = 0; i < N; ++i) CHECK(c[i] == 1 || c[i] == -1, "%s: symbol %d not bipolar", path, i);
    std::printf("%s: %zu codeword line(s), %zu bytes of invalid-symbol reports\n", path, lines.size(), log.str().size());
}

static void cli_inputs(const std::string &dir)
{
    const std::pair<const char *, std::string> files[] = {
        {"cw_empty", ""},
        {"cw_one_unterminated", "0101"},
        {"cw_two_unterminated", "0101\n1100"},
        {"cw_terminated", "0101\n1100\n"},
        {"cw_junk", std::string("01\x00\xff\r\n\n\n2x", 11)},
        {"cw_long", std::string(100000, '1') + "\n"},
        {"cw_crlf", "0101\r\n1100\r\n"},
    };
    for (const auto &f : files) {
        const std::string p = write_tmp(dir, f.first, f.second);
        for (int N : {0, 1, 4, 7, 4096}) one_codeword_file(p.c_str(), N);
    }
    one_codeword_file((dir + "/does_not_exist.enc").c_str(), 8);   // unreadable: one empty line, all invalid
    const std::pair<const char *, std::string> hdrs[] = {
        {"hdr_empty", ""}, {"hdr_short", "8 4\n"}, {"hdr_text", "N M\n"}, {"hdr_ok", "8 4\n3 6\n"},
        {"hdr_neg", "8 4\n-3 -6\n"}};
    for (const auto &h : hdrs) {
        const std::string p = write_tmp(dir, h.first, h.second);
        int dv = -7, dc = -7;
        alist_header(p.c_str(), dv, dc);
        CHECK(dv != -7 && dc != -7, "%s: alist_header left its outputs unset", h.first);
    }
    int dv = -7, dc = -7;
    alist_header((dir + "/does_not_exist.alist").c_str(), dv, dc);
    CHECK(dv == 0 && dc == 0, "alist_header of a missing file");
}

int main(int argc, char **argv)
{
    std::string tmp = "/tmp";
    std::vector<const char *> bin, nb, cw;
    std::vector<const char *> *cur = &bin;
    for (int a = 1; a < argc; ++a) {
        const std::string s = argv[a];
        if (s == "--nb") cur = &nb;
        else if (s == "--cw") cur = &cw;
        else if (s == "--tmp" && a + 1 < argc) tmp = argv[++a];
        else cur->push_back(argv[a]);
    }
    for (const char *p : bin) one_code(p);
    for (const char *p : nb) one_nb(p);
    for (const char *p : cw) one_codeword_file(p, 1008);
    nb_malformed(tmp);
    cli_inputs(tmp);
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
