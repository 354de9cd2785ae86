// nb_graph.h -- host-side graph code of the GF(q) EMS decoder (nb_graph.cpp):
// the NB alist reader (semantics of SystemC/NB-LDPC/src/alist.cpp:23-56, plus
// validation), the CSR views, GF(q) tables and the message-slot swizzles the
// device context uploads (nb_api.cpp). No HIP: the host sanitizer build
// (Makefile `asan`, tests/native/host_asan.cpp) compiles it with g++.
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

struct ldpc_nb_graph {
    int N = 0, M = 0, q = 0, m = 0, E = 0, maxdv = 0, maxdc = 0;
    std::vector<int32_t> row_ptr, row_col, col_ptr, col_slot;
    std::vector<uint8_t> row_h;
};

namespace ldpc {

using NbLists = std::vector<std::vector<std::pair<int, int>>>;   // per column / row: (0-based index, GF value)

int gf_poly(int q);                 // primitive polynomial of GF(q), q = 2..64 (0: unsupported)
int gf_mul(int q, int a, int b);

// The CSR views from the column and row lists; validates that both describe the same
// edges and coefficients. Returns LDPC_OK or a negative ldpc_status, msg = why.
int nb_build_graph(int N, int M, int q, const NbLists &cols, const NbLists &rows, ldpc_nb_graph &g, std::string &msg);
// NB alist file (N M q / maxdv maxdc / weights / (index, value) pairs, zero padded).
int nb_read_alist(const char *path, ldpc_nb_graph &g, std::string &msg);

// What the device context uploads beside the CSR views.
struct NbTables {
    std::vector<uint8_t> mul, inv;     // GF(q) multiplication [q*q] and inverse [q]
    std::vector<int32_t> pslot;        // [E] column entry -> position-major slot k*M + j
    std::vector<uint8_t> colh;         // [E] its coefficient
    std::vector<uint8_t> colh_swz;     // [E] coefficient | slot XOR swizzle << 4 (GF(16) only; else = colh)
};
void nb_tables(const ldpc_nb_graph &g, NbTables &t);
std::vector<uint8_t> nb_swizzled_coefficients(const ldpc_nb_graph &g, const std::vector<int32_t> &pslot,
                                              const std::vector<uint8_t> &colh, const std::vector<uint8_t> &mul);

}  // namespace ldpc
