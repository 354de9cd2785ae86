// graph.h -- host-side Tanner-graph compiler (internal to libldpc_hip.so).
//
// Replaces the reference's alist_struct + find() edge search
// (C_implementations/inc/alist.h:21-36, src/decodeMinSum.cpp:527-536) with
// flat arrays the kernels index directly:
//   row_cols[j*maxdc + k]  0-based bit index of the k-th edge of check j, in
//                          mlist order (pads = 0, bounded by row_deg[j]);
//   col_ptr[i]..col_ptr[i+1]  edges of bit i in nlist order (the order the
//                          reference sums c2v in symNodeUpdates, :456-463);
//   col_refs[e] = (j << 6) | k  the check j and the position k of bit i in
//                          mlist[j] -- what find(mlist[j], ., i) returns.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

struct ldpc_graph {
    int N = 0, M = 0, E = 0, maxdv = 0, maxdc = 0;
    std::vector<int32_t> row_cols;   // [M * maxdc]
    std::vector<uint8_t> row_deg;    // [M]
    std::vector<int32_t> col_ptr;    // [N + 1]
    std::vector<uint32_t> col_refs;  // [E]
    std::vector<uint8_t> col_deg;    // [N]
};

namespace ldpc {
constexpr int kMaxRowDegree = 58;   // sign bits that fit the packed row state
constexpr int kRefShift = 6;

// Static work schedule of the row-parallel kernel (kernels.hip, k_decode_rows):
// RPT check rows per thread (thread t owns rows t, t + threads, ...) and up to
// CPT bit-node slots per thread. Columns are sorted by degree (stable) and cut into 64-column groups
// of near-uniform degree; edge kc (nlist order) of the group's column l lives
// at c2v element gbase + kc*64 + l, so a wave's bit-node reads are 64
// consecutive words (conflict-free LDS). Groups are assigned to waves by
// longest-processing-time so the bit-node phase is balanced across waves.
struct RowSchedule {
    int threads = 0, cpt = 0, dc = 0, e_pad = 0, rpt = 1;
    int dc_low = 0;                  // > 0: rows placed by pp_row_slots (slots it caps hold degree <= dc_low)
    std::vector<uint16_t> cn_cols;   // [threads * rpt * dc]  bit index of edge k of row j
    std::vector<uint16_t> cn_pos;    // [threads * rpt * dc]  c2v element of edge k of row j
    std::vector<uint8_t> cn_deg;     // [threads * rpt]       (row j -> thread j % threads)
    std::vector<uint16_t> vn_col;    // [threads * cpt] column of slot s (0xffff = none)
    std::vector<uint32_t> vn_info;   // [threads * cpt] (gbase+lane) | deg << 16 | group degree << 24
};

// Build from alist_struct-style arrays (1-based). Returns "" on success or
// an error message.
std::string build_graph(int N, int M, const int *num_nlist, const int *const *nlist,
                        const int *num_mlist, const int *const *mlist, ldpc_graph &g);
// Static schedule of the global-memory flooding kernel (kernels.hip,
// k_decode_flood) for codes whose state does not fit on chip (DVB-S2 N=64800).
// Quasi-cyclic structure is discovered, not assumed: every row is chained to
// the row that holds most of its columns + 1, edge slots are aligned along the
// chains, and columns are chained the same way (column c -> the column the
// aligned slot of the next row holds). Rows are processed in chain order and
// bits are stored in column-chain order, so the 64 lanes of a wave, working on
// 64 consecutive rows of a chain, gather and scatter 64 consecutive words
// (DVB-S2: 90 row chains and the bit chains of length 360; 802.11n: Z=81).
// Nothing depends on the discovery succeeding: a code without the structure
// gets an arbitrary but valid order.
struct FloodSchedule {
    int M_pad = 0;                    // rows rounded up to 64
    int dc = 0;                       // max row degree
    int ngroups = 0, e_pad = 0;       // 64-bit groups of the c2v layout, its size
    std::vector<int32_t> row_of;      // [M_pad] check row at order position i (-1: padding)
    std::vector<uint8_t> chain_head;  // [M] 1 where order position i starts a row chain
    std::vector<uint8_t> rdeg;        // [M_pad]
    std::vector<int32_t> sp;          // [dc * M_pad] slot-major: bit position (storage order) of slot k (pads: ngroups*64, the +inf sentinel)
    std::vector<int32_t> sq;          // [dc * M_pad] slot-major: c2v element of slot k (pads: e_pad + i%64)
    std::vector<int32_t> pos_of_bit;  // [N] storage position of bit v
    std::vector<int32_t> bit_at;      // [ngroups * 64] bit at storage position p (-1: padding)
    std::vector<uint8_t> pdeg;        // [ngroups * 64] degree of the bit at position p
    std::vector<int32_t> gbase;       // [ngroups]: edge e (nlist order) of position p at gbase[p/64] + 64e + p%64
    double coalesced = 0;             // diagnostic: share of slot accesses whose lane neighbour is +1
};
std::string build_flood_schedule(const ldpc_graph &g, FloodSchedule &s);

// Layered schedule (kernels.hip, k_decode_layered_*): rows grouped into
// layers of rows that share no bit, by first-fit colouring of whole row
// chains of the flood schedule (each chain -- split where it would share a
// bit with itself -- joins the lowest layer none of its bits is in yet), so a
// quasi-cyclic block row stays together and rows keep their chain neighbours
// (coalesced gathers). The serial row order is layer by layer, each layer in
// chain order; updating a layer's rows in
// parallel equals updating them serially in that order (bit-disjoint rows
// commute), which is the oracle's row-serial definition.
struct LayerSchedule {
    int M_pad = 0, dc = 0;
    std::vector<int32_t> row_order;   // [M] check row at layered position n
    std::vector<int32_t> lptr;        // [nlayers + 1] layered positions of each layer
    std::vector<int32_t> sp;          // [dc * M_pad] slot-major layered position of edge k of the row at
                                      // layered position n (pads: the +inf sentinel, ngroups * 64)
    std::vector<uint8_t> rdeg;        // [M_pad]
    std::vector<int32_t> pos_of_bit;  // [N] layered position of bit v: the FloodSchedule positions ranked
                                      // by bit degree (stable), so the most-gathered bits come first --
                                      // the global kernel keeps positions [0, P) in LDS
};
std::string build_layers(const ldpc_graph &g, const FloodSchedule &s, LayerSchedule &ls);

// Reference loadFile() semantics (src/alist.cpp:70-93, fixed-width lines).
std::string load_alist(const char *path, ldpc_graph &g);
// Row schedule for `threads` threads (multiple of 64, >= M), `cpt` bit slots
// per thread (threads*cpt >= N) and row-degree bound dc. Returns "" or why the
// graph does not fit (the caller then uses the generic kernel).
// row_of_slot (optional, [threads * rpt], -1 = padding): the check row each row
// slot holds; by default slot j holds row j. Any assignment gives the same
// values (flooding rows are independent); it only moves work between waves.
std::string build_row_schedule(const ldpc_graph &g, int threads, int cpt, int dc, int rpt, RowSchedule &s,
                               const std::vector<int> *row_of_slot = nullptr);
// Degree-aware row slots of the ping-pong kernel (rows_pp.hip; 512 check threads,
// 2 rows each, dc 8): every row-0 slot and the row-1 slots of threads 256..511
// -- the younger check wave of each SIMD runs only those -- hold rows of degree
// <= dc_low (a 7-edge check node: 7 gathers, 7 scatters, a 7-input tournament);
// the degree-8 rows, the remaining rows and the padding go to the row-1 slots
// of threads 0..255. Rows keep their order within each class (quasi-cyclic
// neighbours stay lane neighbours: coalesced gathers and scatters). Empty when
// the rows do not fit that split.
std::vector<int> pp_row_slots(const ldpc_graph &g, int threads, int dc_low);
}  // namespace ldpc
