// bp.h -- internal launch interface of the belief-propagation kernels (bp.hip).
#pragma once
#include "kernels.h"

namespace ldpc {

constexpr int kBpMaxDc = 32;   // row degree bound of the BP check node (per-thread tanh array)

// "bp_rows" (graph in registers, persistent; N <= 4096, row degree <= 8),
// "bp_lds" (state in LDS) or "bp_global" (a global slot per resident block).
// E: the code's edge count; num_cus sizes bp_rows' persistent grid.
KernelChoice bp_choose(const DevGraph &g, bool f64, int E);
// ldpc_bp_math_probe: tanh and log of bp_math.h over n device values (verification)
hipError_t bp_math_probe(const double *x, double *t, double *l, int n, hipStream_t s);
// checked builds (LDPC_CHECK): one out-of-range index on purpose (ldpc_check_selftest)
hipError_t check_selftest_launch(hipStream_t s);
hipError_t bp_launch(const DevGraph &g, const DecodeArgs &a, bool f64, const KernelChoice &kc, void *gscratch,
                     int gblocks, int E, int num_cus, hipStream_t s);

}  // namespace ldpc
