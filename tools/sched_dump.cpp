// sched_dump -- write the row kernel's static schedule (graph.h RowSchedule) of an
// alist to a binary file, for host-side LDS bank models (scripts/lds_bank_model.py).
// Host only: loads the alist through the C ABI, no device call.
#include <cstdio>
#include <cstdlib>
#include "ldpc_hip.h"
#include "graph.h"

int main(int argc, char **argv)
{
    if (argc < 4) { std::fprintf(stderr, "usage: %s alist threads out.bin [cpt dc rpt [pp_dc_low]]\n", argv[0]); return 2; }
    ldpc_graph *g = nullptr;
    if (ldpc_graph_load_alist(argv[1], &g) != LDPC_OK) { std::fprintf(stderr, "%s\n", ldpc_last_error()); return 1; }
    const int threads = std::atoi(argv[2]);
    const int cpt = argc > 4 ? std::atoi(argv[4]) : 4, dc = argc > 5 ? std::atoi(argv[5]) : 8, rpt = argc > 6 ? std::atoi(argv[6]) : 2;
    ldpc::RowSchedule s;
    // pp_dc_low > 0: the ping-pong kernel's degree-aware row slots (graph.h pp_row_slots)
    const int dc_low = argc > 7 ? std::atoi(argv[7]) : 0;
    const std::vector<int> slots = dc_low > 0 ? ldpc::pp_row_slots(*g, threads, dc_low) : std::vector<int>();
    if (dc_low > 0 && slots.empty()) { std::fprintf(stderr, "rows do not fit the degree split\n"); return 1; }
    const std::string err = ldpc::build_row_schedule(*g, threads, cpt, dc, rpt, s, dc_low > 0 ? &slots : nullptr);
    if (!err.empty()) { std::fprintf(stderr, "%s\n", err.c_str()); return 1; }
    FILE *f = std::fopen(argv[3], "wb");
    const int hdr[8] = {g->N, g->M, s.threads, s.cpt, s.dc, s.e_pad, s.rpt, 0};
    std::fwrite(hdr, 4, 8, f);
    std::fwrite(s.cn_cols.data(), 2, s.cn_cols.size(), f);
    std::fwrite(s.cn_pos.data(), 2, s.cn_pos.size(), f);
    std::fwrite(s.cn_deg.data(), 1, s.cn_deg.size(), f);
    std::fwrite(s.vn_col.data(), 2, s.vn_col.size(), f);
    std::fwrite(s.vn_info.data(), 4, s.vn_info.size(), f);
    std::fclose(f);
    ldpc_graph_destroy(g);
    return 0;
}
