// options.h -- the kernel-selection options of a context (include/ldpc_hip.h
// ldpc_option, ldpc_ctx_set_option): tests and A/B measurements override the
// library's kernel choice through the C ABI, never through the environment.
//
// The launch helpers deep in the kernel files (kernels.hip, nb.hip, bp.hip,
// gdbf.hip, rows_fast.hip) read them through opt(): each ABI entry point that
// chooses or launches a kernel installs its context's options for the duration
// of the call (OptScope). Outside such a call every option reads 0, the
// library's own choice.
#pragma once
#include "ldpc_hip.h"

namespace ldpc {

struct Options {
    int v[LDPC_OPT_COUNT] = {};
};

// Valid range of each option's value (ldpc_ctx_set_option refuses others).
bool option_value_ok(int option, int value);

// The EMS options belong to the GF(q) context (ldpc_nb_ctx_set_option) and only there;
// the binary context refuses them, and the nb context refuses every other option.
inline bool option_is_ems(int option) { return option == LDPC_OPT_EMS_THREADS || option == LDPC_OPT_EMS_SWIZZLE; }

// The options installed on this thread (all zero when none is).
const Options &cur_opts();
inline int opt(int option) { return cur_opts().v[option]; }

class OptScope {
public:
    explicit OptScope(const Options &o);
    ~OptScope();
    OptScope(const OptScope &) = delete;
    OptScope &operator=(const OptScope &) = delete;

private:
    const Options *prev_;
};

}  // namespace ldpc
