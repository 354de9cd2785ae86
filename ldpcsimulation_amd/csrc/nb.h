// nb.h -- internal interface of the non-binary GF(q) EMS kernels (nb.hip)
// and their C ABI (nb_api.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>

namespace ldpc {

constexpr int kNbQ = 16;          // field size the kernels are built for (GF(16), BASELINE config 5)
constexpr int kNbMaxDc = 8;       // row degree bound (DC template 4 / 8)

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
};

struct NbChoice {
    const char *name = "";        // "ems_lds" | "ems_global"
    int lds_bytes = 0, threads = 0, dc = 0;
    size_t slot_bytes = 0;        // ems_global: message bytes per resident codeword
};

// Position-major message slot count (maxdc * M) rounded up to a power of two
// (at least 4): the chunk stride of the message layout of nb.hip, where the byte
// offset of entry p of slot s is (s << 4) ^ nb_lambda(p) -- XOR-linear in p.
__host__ __device__ inline int nb_ep(const NbDevGraph &g)
{
    int e = 4;
    while (e < g.maxdc * g.M) e <<= 1;
    return e;
}
__host__ __device__ inline int nb_ep_log2(int ep)
{
    int k = 0;
    while ((1 << k) < ep) ++k;
    return k;
}
// Byte offset of entry p (0..15) relative to its slot's s << 4, chunk stride 2^k slots:
// chunk p >> 2 at (p >> 2) << (k + 4), the slot XOR-ed with the chunk index (bits 4-5),
// the entry within its 16-byte chunk at (p & 3) << 2.
__host__ __device__ inline int nb_lambda(int p, int k) { return (p << 2) ^ ((p >> 2) << (k + 4)); }

NbChoice nb_choose(const NbDevGraph &g, int maxdc);
hipError_t nb_launch(const NbDevGraph &g, const NbArgs &a, const NbChoice &ch, void *scratch, int slots,
                     int num_cus, hipStream_t s);

// ldpc_last_error() of api.cpp.
int set_last_error(int code, const std::string &msg);

}  // namespace ldpc
