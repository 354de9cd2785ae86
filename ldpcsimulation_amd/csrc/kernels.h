// kernels.h -- internal launch interface between api.cpp and kernels.hip.
#pragma once
#include "options.h"
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ldpc {

struct DevGraph {
    int N, M, dcs;                  // dcs = row stride of row_cols (max(maxdc,1))
    const int32_t *row_cols;        // [M * dcs]
    const uint8_t *row_deg;         // [M]
    const int32_t *col_ptr;         // [N + 1]
    const uint32_t *col_refs;       // [E]  (check << 6) | position
};

enum { SRC_GIVEN = 0, SRC_PHILOX = 1 };
enum { VARIANT_BP = 3 };   // ldpc_variant LDPC_BP

struct DecodeArgs {
    int batch, T, variant, quantize, saturate;
    double ymax, nq, alpha, delta;
    double n0, max_llr;             // BP front-end: yq = 4*y/n0 clipped to +-max_llr
    // fp32 NMS: q = x*r, q += fma(-q, alpha, x)*r equals x/alpha for every
    // finite float x (verified on the device by verify_div_by_reciprocal)
    int nms_fast;
    float alpha_rcp;
    int src;
    const void *y;                  // SRC_GIVEN: [batch][N] float|double (device)
    const int8_t *c;                // SRC_GIVEN: [batch][N] bipolar, or null (+1)
    const int8_t *cw_table;         // SRC_PHILOX: [cw_rows][N] bipolar, or null
    int cw_rows;
    uint64_t seed, first_cw;
    uint32_t stream_id;
    double sigma;
    int8_t *d_out;                  // [batch][N] or null
    void *y_out;                    // SRC_PHILOX: channel samples [batch][N] F (pre front-end) or null
    int4 *frame_res;                // [batch] {bit_err, uncoded, syndrome_fail, 0} or null
    unsigned long long *counts;     // [6] accumulated
    unsigned long long *hist;       // [N] accumulated (weight w -> hist[w-1])
    unsigned long long *stamps;     // diagnostic builds (-DLDPC_STAMPS): [grid][4] cycle sums, else null
};

// Device copy of graph.h's RowSchedule (row-parallel kernel).
struct RowSched {
    int threads, cpt, dc, e_pad, rpt;
    int dc_low;                     // > 0: degree-aware row slots (graph.h pp_row_slots)
    const uint16_t *cn_cols;       // [threads * rpt * dc]  (row j = thread j % threads, r = j / threads)
    const uint16_t *cn_pos;         // [threads * rpt * dc]
    const uint8_t *cn_deg;          // [threads * rpt]
    const uint16_t *vn_col;         // [threads * cpt]
    const uint32_t *vn_info;        // [threads * cpt]
};

// Device copy of graph.h's FloodSchedule (global-memory flooding kernel).
struct FloodSched {
    int M_pad, dc, ngroups, e_pad;
    int dv;                         // max column degree
    const int32_t *sp, *sq;         // [dc * M_pad] slot-major bit position / c2v element
    const uint8_t *rdeg;            // [M_pad]
    const int32_t *pos_of_bit;      // [N]
    const int32_t *bit_at;          // [ngroups * 64]
    const uint8_t *pdeg;            // [ngroups * 64]
    const int32_t *gbase;           // [ngroups]
    const uint32_t *eref;           // [e_pad + 64] per c2v element: (row << 5) | position in the row
};

// Device copy of graph.h's LayerSchedule.
struct LayerSched {
    int nlayers = 0, max_layer = 0, M_pad = 0;
    const int32_t *lptr = nullptr;  // [nlayers + 1] layered row positions of each layer
    const int32_t *sp = nullptr;    // [dc * M_pad] slot-major layered positions (graph.h LayerSchedule)
    const uint8_t *rdeg = nullptr;  // [M_pad]
    const int32_t *pos_of_bit = nullptr;   // [N] layered position of each bit
};

struct KernelChoice {
    const char *name;               // "rows", "lds", "flood" or "global"
    int lds_bytes;                  // dynamic LDS per block
    size_t scratch_per_block;       // global kernel
    int threads;
    int cw_per_block;               // rows kernel: codewords decoded together per block
};

// Pick the kernel for a graph / precision. rs (may be null) is the row
// schedule when the graph admits one; force selects "lds"/"global" for tests.
// fs (may be null): the flood schedule, used for codes whose state exceeds LDS.
KernelChoice choose_kernel(const DevGraph &g, bool f64, const RowSched *rs, const char *force = nullptr,
                           const FloodSched *fs = nullptr);
// Launch the decode. gscratch must hold choice.scratch_per_block * grid bytes
// for the global kernel (grid returned through *grid_out, may be null).
hipError_t launch_decode(const DevGraph &g, const DecodeArgs &a, bool f64, const KernelChoice &kc,
                         void *gscratch, int gscratch_blocks, hipStream_t s, const RowSched *rs = nullptr,
                         int num_cus = 256, const FloodSched *fs = nullptr);
int blocks_per_cu(const DevGraph &g, bool f64, const KernelChoice &kc);
// Flooding of codes beyond LDS as one launch per phase over an Infinity-Cache-
// resident set of codewords (kernels.hip k_flood_*); gscratch as for "flood".
// aux (may be null): a second stream with fork/join events; the resident set is
// then split in two halves, one per stream, so one half's launch boundaries
// overlap the other half's kernels.
struct AuxStream {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
};
hipError_t launch_flood_phase(const DevGraph &g, const FloodSched &fs, const DecodeArgs &a, bool f64,
                              const KernelChoice &kc, void *gscratch, size_t gscratch_bytes, hipStream_t s,
                              const AuxStream *aux = nullptr);

// Layered schedule (k_decode_layered_*): state in LDS when it fits
// ("layered_lds"), else in a global slot per block ("layered_global").
// Requires the flood schedule (row order, storage order) and row degree <= kPackedMaxDc.
KernelChoice choose_layered(const DevGraph &g, bool f64, const FloodSched &fs, const LayerSched &ls,
                            const char *force = nullptr);
hipError_t launch_layered(const DevGraph &g, const DecodeArgs &a, bool f64, const KernelChoice &kc,
                          const FloodSched &fs, const LayerSched &ls, void *gscratch, int gscratch_blocks,
                          hipStream_t s);
int layered_blocks_per_cu(bool f64, const KernelChoice &kc);
size_t layered_resident_bytes(const FloodSched &fs, const LayerSched &ls, bool f64);
// Packed check state of the flood and layered kernels: a 5-bit argmin and one
// sign bit per edge in a 32-bit meta word.
constexpr int kPackedMaxDc = 26;

// Exhaustive device check that dividing by alpha through its correctly rounded
// reciprocal plus one FMA correction step reproduces IEEE x/alpha for all
// 2^31 - 2^23 finite non-negative floats x (the only operands the check-node
// normalisation divides: |v2c| minima). *mismatches receives the count.
hipError_t verify_div_by_reciprocal(float alpha, float rcp, unsigned long long *mismatches_dev, hipStream_t s);

// Fast-path row kernel (rows_fast.hip): fp64 (one codeword per block) and fp32
// (a pair, dc <= 8), same LDS layout and schedule as the "rows" kernel
// (lds_bytes of its KernelChoice), check node compiled per variant; codeword
// groups whose premise fails are appended to redo (redo[0] = count, must be 0
// at launch; redo[1..] batch indices, capacity batch), and launch_redo
// (kernels.hip) decodes them on the exact path. fp32 takes it only for MS and
// for NMS with the verified reciprocal (rows_fast_f32_ok, after nms_setup).
bool rows_fast_supported(const RowSched &rs, bool f64);
bool rows_fast_f32_ok(const DecodeArgs &a);
hipError_t launch_rows_fast(const DevGraph &g, const RowSched &rs, const DecodeArgs &a, bool f64, int lds_bytes,
                            unsigned *redo, hipStream_t s, int num_cus);
// alpha for which the fast fp64 NMS division x*r + one fma correction is exact
bool markstein_exact_alpha(double alpha);
size_t redo_lds_bytes(const DevGraph &g, bool f64);
hipError_t launch_redo(const DevGraph &g, const DecodeArgs &a, bool f64, const unsigned *redo, hipStream_t s,
                       int num_cus);

// Ping-pong row kernel (rows_pp.hip): two slots per 1024-thread block -- an
// fp64 codeword or an fp32 pair (float2) each -- check waves and bit waves
// overlapped (schedule: 512 threads, 2 rows and 4 bit slots each, dc 8, the
// degree-aware row slots when rs.dc_low == 7); redo as above (fp32: MS and NMS
// with the verified reciprocal, rows_fast_f32_ok).
bool rows_pp_supported(const DevGraph &g, const RowSched &rs);
int rows_pp_lds_bytes(const DevGraph &g, const RowSched &rs);
hipError_t launch_rows_pp(const DevGraph &g, const RowSched &rs, const DecodeArgs &a, bool f64, unsigned *redo,
                          hipStream_t s, int num_cus);

// Row-kernel template bounds (host picks the smallest that fits).
constexpr int kRowsMaxThreads = 1024;
constexpr int kRowsCpt[] = {2, 4, 8};
// rows per thread -> block threads cap
constexpr int kRowsMaxThreadsForRpt[] = {0, 1024, 512, 384};
constexpr int kRowsDc[] = {8, 16, 32};

}  // namespace ldpc
