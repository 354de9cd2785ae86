// gdbf.h -- internal launch interface of the GDBF / NGDBF kernels (gdbf.hip).
#pragma once
#include "kernels.h"

namespace ldpc {

// The -D switches of src/decodeGDBF.cpp (values = LDPC_GDBF_* of ldpc_hip.h).
enum {
    GDBF_NOISE = 1, GDBF_ADAPT = 2, GDBF_WEIGHT = 4, GDBF_SMOOTH = 8, GDBF_SATURATE = 16, GDBF_QUANTIZE = 32,
    GDBF_SEQUENTIAL = 64, GDBF_MODESWITCH = 128, GDBF_QPROB = 256
};

struct GdbfArgs {
    int batch, T, flags, windowsize, src, tswitch;
    double theta0, lambda, w, noise_sigma, ymax, qmax, sigma;
    double qsigma;                  // GDBF_QPROB: the normalCDF sigma (noiseSigma)
    const void *y;                  // SRC_GIVEN: raw channel samples [batch][N] (F)
    const void *pert;               // SRC_GIVEN with GDBF_NOISE: perturbations [batch][T][N] (F);
                                    // with GDBF_QPROB: the ranu() draws [batch][T][N] (F)
    const int8_t *c;                // SRC_GIVEN: bipolar codewords [batch][N] or null (+1)
    const int8_t *cw_table;         // SRC_PHILOX: codeword table [cw_rows][N] or null
    int cw_rows;
    uint64_t seed, first_cw;
    uint32_t stream_id;
    int8_t *d_out;                  // [batch][N] or null
    int4 *frame_res;                // [batch] {bit_err, uncoded, syndrome_fail, iterations} or null
    unsigned long long *counts;     // [6] accumulated (iters = sum of iterations run)
    unsigned long long *hist;       // [N] error-weight histogram
    unsigned *ticket;               // gdbf_rows: codewords past the first grid's are handed out by
                                    // this counter (gdbf_launch zeroes it): early stop makes them unequal
};

struct GdbfChoice {
    const char *name = "";          // "gdbf_rows" | "gdbf_lds" | "gdbf_global"
    int lds_bytes = 0, threads = 0;
    size_t slot_bytes = 0;          // global kernel: state bytes per resident codeword
    int dvm = 0;                    // gdbf_rows: bit-degree bound of the register schedule (4 or 12)
};

// flags: the decoder's GDBF_* switches; maxdv / maxdc: the code's largest
// column / row degree. LDPC_GDBF_KERNEL=generic in the environment forces the
// one-workgroup-per-codeword kernels (tests compare the two).
GdbfChoice gdbf_choose(const DevGraph &g, bool f64, int flags, int maxdv, int maxdc);
// scratch: slots * choice.slot_bytes bytes for the global kernel (persistent grid of `slots`);
// num_cus sizes the persistent grid of gdbf_rows.
hipError_t gdbf_launch(const DevGraph &g, const GdbfArgs &a, bool f64, const GdbfChoice &ch, void *scratch,
                       int slots, int num_cus, hipStream_t s);

}  // namespace ldpc
