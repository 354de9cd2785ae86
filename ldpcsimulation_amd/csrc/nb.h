// nb.h -- internal interface of the non-binary GF(q) EMS kernels (nb.hip)
// and their C ABI (nb_api.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>

#include "nb_layout.h"

namespace ldpc {

struct NbDevGraph {
    int N, M, q, m, E, maxdc;
    const int32_t *row_ptr;       // [M + 1]  edge slot of (check j, mlist position k) = row_ptr[j] + k
    const int32_t *row_col;       // [E]      symbol of each slot
    const uint8_t *row_h;         // [E]      GF(q) coefficient of each slot
    const int32_t *col_ptr;       // [N + 1]
    const int32_t *col_slot;      // [E]      row-major slots of each symbol, nlist order
    const int32_t *col_pslot;     // [E]      the same edges as position-major slots k*M + j
    const uint8_t *col_h;         // [E]      their coefficients (low nibble) | slot XOR swizzle << 4 (nb.hip vn_lane)
    const uint8_t *gf_mul;        // [q * q]  multiplication table
    const uint8_t *gf_inv;        // [q]
};

struct NbArgs {
    int batch, T, nm, early_stop, src;
    float offset, n0, sigma;
    const float *y;               // SRC_GIVEN: [batch][N * m] channel samples
    const uint8_t *c;             // SRC_GIVEN: [batch][N] transmitted symbols or null (all-zero)
    uint64_t seed, first_cw;
    uint32_t stream_id;
    uint8_t *d_out;               // [batch][N] decided symbols or null
    float *y_out;                 // SRC_PHILOX: generated samples [batch][N * m] or null
    int4 *frame_res;              // [batch] {bit_err, uncoded, syndrome_fail, iterations} or null
    unsigned long long *counts;   // [7] bit, frame, uncoded, frames, iters, syndrome_fail, symbol errors
    unsigned *ticket;             // codewords past the first grid's are handed out by this counter
                                  // (nb_launch zeroes it): early stop makes codewords unequal
};

struct NbChoice {
    const char *name = "";        // "ems_lds" | "ems_global"
    int lds_bytes = 0, threads = 0, dc = 0;
    size_t slot_bytes = 0;        // ems_global: message bytes per resident codeword
};

// the chunk stride of a device graph's message layout (nb_layout.h)
__host__ __device__ inline int nb_ep(const NbDevGraph &g) { return nb_ep(g.maxdc, g.M); }

NbChoice nb_choose(const NbDevGraph &g, int maxdc);
hipError_t nb_launch(const NbDevGraph &g, const NbArgs &a, const NbChoice &ch, void *scratch, int slots,
                     int num_cus, hipStream_t s);

// ldpc_last_error() of api.cpp.
int set_last_error(int code, const std::string &msg);

}  // namespace ldpc
