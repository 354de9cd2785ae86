// check.h -- device bounds checks of the schedule-derived indices (a
// bounds-checked debug build of the kernels; `make checked`, -DLDPC_CHECK).
//
// Index safety in the kernels rests on the host: graph.cpp / nb_graph.cpp validate
// the alist and build every schedule (the reference validates nothing,
// alist.cpp:22-95). The checked build re-proves it on the device: every LDS or
// global index that a kernel computes from a schedule goes through LDPC_CHK(i, n,
// site), which in the product build is `i` itself (no instruction, the product
// .so is unchanged) and in the checked build tests 0 <= i < n. A violation is
// recorded -- the first one's site, index, bound, block and thread, and a count --
// in the translation unit's g_ldpc_check record, and the index is replaced by 0 so
// that it never becomes an out-of-bounds access (no trap, no fault); the ABI call
// that ran the launch then fails with LDPC_ERR_DEVICE naming the site
// (api.cpp check_device_indices).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ldpc {

// sites (check_site_name in api.cpp prints them)
enum CheckSite : unsigned {
    CHK_PP_GATHER = 1,     // rows_pp: app entry of a check row's edge      (< N + 3)
    CHK_PP_SCATTER,        // rows_pp: c2v slot of a check row's edge       (< e_pad + 64)
    CHK_PP_BIT_READ,       // rows_pp: c2v slot a bit slot reads            (< e_pad + 64)
    CHK_PP_APP_WRITE,      // rows_pp: app entry a bit slot writes          (< N + 3)
    CHK_FAST_GATHER,       // rows_fast: as above                           (< N + 2)
    CHK_FAST_SCATTER,      //                                               (< e_pad + 64)
    CHK_FAST_BIT_READ,     //                                               (< e_pad + 64)
    CHK_FAST_APP_WRITE,    //                                               (< N + 2)
    CHK_FLOOD_APP,         // flood / layered: bit position of a row's edge (< ngroups * 64)
    CHK_FLOOD_C2V,         // flood: c2v / eref slot                        (< slots)
    CHK_FLOOD_ROW,         // flood: row of a packed-state reference       (< M_pad)
    CHK_GDBF_BIT,          // gdbf_rows: bit a check row gathers            (< np)
    CHK_GDBF_CHECK,        // gdbf_rows: check term slot a bit reads/writes (< sidx(M) + 1)
    CHK_EMS_SLOT,          // EMS: message slot of a check / symbol edge    (< Ep)
    CHK_BP_COL,            // bp_rows: bit a check row gathers              (< N + 1)
    CHK_BP_MSG,            // bp_rows: message slot                         (< E + 1)
    CHK_SITES
};

struct CheckRec {
    unsigned count, site, idx, bound, block, thread, pad0, pad1;
};

#if defined(LDPC_CHECK) && defined(__HIP__)
// one record per translation unit (no relocatable device code): each kernel file
// defines its host reader with LDPC_CHECK_TU(name)
static __device__ CheckRec g_ldpc_check;

static __device__ __noinline__ void chk_record(uint32_t i, uint32_t n, unsigned site)
{
    if (atomicAdd(&g_ldpc_check.count, 1u) == 0u) {
        g_ldpc_check.site = site;
        g_ldpc_check.idx = i;
        g_ldpc_check.bound = n;
        g_ldpc_check.block = blockIdx.x;
        g_ldpc_check.thread = threadIdx.x;
    }
}
__device__ __forceinline__ uint32_t chk_idx(uint32_t i, uint32_t n, unsigned site)
{
    if (__builtin_expect(i >= n, 0)) {
        chk_record(i, n, site);
        return 0u;
    }
    return i;
}
#define LDPC_CHK(i, n, site) ((__typeof__(i))::ldpc::chk_idx((uint32_t)(i), (uint32_t)(n), (site)))
#define LDPC_CHK_LIM(n) (n)   // a bound passed down to a helper (vn_phases): evaluated in checked builds only
// host: read and clear this translation unit's record
#define LDPC_CHECK_TU(name)                                                                             \
    hipError_t check_take_##name(CheckRec *out)                                                        \
    {                                                                                                  \
        hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ldpc_check), sizeof(CheckRec), 0,         \
                                           hipMemcpyDeviceToHost);                                     \
        if (e != hipSuccess) return e;                                                                 \
        const CheckRec z{};                                                                            \
        return hipMemcpyToSymbol(HIP_SYMBOL(g_ldpc_check), &z, sizeof(CheckRec), 0, hipMemcpyHostToDevice); \
    }
#else
#define LDPC_CHK(i, n, site) (i)
#define LDPC_CHK_LIM(n) 0x7fffffff
#define LDPC_CHECK_TU(name)
#endif

#ifdef LDPC_CHECK
// After a launch (checked builds): synchronise `s`, read and clear every translation
// unit's record; the number of violations (0: none), the first one described in msg.
// api.cpp; a negative value is a HIP error.
long check_collect(hipStream_t s, char *msg, size_t msg_len);
hipError_t check_take_rows_pp(CheckRec *out);
hipError_t check_take_rows_fast(CheckRec *out);
hipError_t check_take_kernels(CheckRec *out);
hipError_t check_take_gdbf(CheckRec *out);
hipError_t check_take_nb(CheckRec *out);
hipError_t check_take_bp(CheckRec *out);
#endif

}  // namespace ldpc
