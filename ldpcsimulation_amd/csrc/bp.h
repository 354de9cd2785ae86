// bp.h -- internal launch interface of the belief-propagation kernels (bp.hip).
#pragma once
#include "kernels.h"

namespace ldpc {

constexpr int kBpMaxDc = 32;   // row degree bound of the BP check node (per-thread tanh array)

// "bp_lds" (state in LDS) or "bp_global" (a global slot per resident block).
KernelChoice bp_choose(const DevGraph &g, bool f64);
hipError_t bp_launch(const DevGraph &g, const DecodeArgs &a, bool f64, const KernelChoice &kc, void *gscratch,
                     int gblocks, hipStream_t s);

}  // namespace ldpc
