// api.cpp -- C ABI of libldpc_hip.so (include/ldpc_hip.h).
//
// Owns device state (graph upload, counters, staging buffers, events) and
// maps the reference's per-frame loop onto batched kernel launches. No C++
// exception crosses the ABI; every HIP failure becomes LDPC_ERR_DEVICE with
// a message in ldpc_last_error().
#include "ldpc_hip.h"
#include "gdbf.h"
#include "bp.h"
#include "nb.h"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <new>
#include <string>
#include <vector>

#include "graph.h"
#include "kernels.h"
#include "check.h"

static thread_local std::string g_last_error;

static int set_err(int code, const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                           \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) {                                                                 \
            (void)hipGetLastError();                                                            \
            return set_err(LDPC_ERR_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                           __FILE__, __LINE__);                                                 \
        }                                                                                       \
    } while (0)

#ifdef LDPC_CHECK
namespace ldpc {
static const char *check_site_name(unsigned s)
{
    static const char *const names[CHK_SITES] = {
        "?", "rows_pp gather (app entry)", "rows_pp scatter (c2v slot)", "rows_pp bit read (c2v slot)",
        "rows_pp app write", "rows_fast gather (app entry)", "rows_fast scatter (c2v slot)",
        "rows_fast bit read (c2v slot)", "rows_fast app write", "flood/layered bit position",
        "flood c2v / eref slot", "flood packed-state row", "gdbf_rows bit", "gdbf_rows check term slot",
        "EMS message slot", "bp_rows bit", "bp_rows message slot"};
    return s < CHK_SITES ? names[s] : "?";
}
long check_collect(hipStream_t s, char *msg, size_t msg_len)
{
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return -(long)e;
    hipError_t (*const take[])(CheckRec *) = {check_take_rows_pp, check_take_rows_fast, check_take_kernels,
                                              check_take_gdbf, check_take_nb, check_take_bp};
    long total = 0;
    for (auto fn : take) {
        CheckRec r{};
        if ((e = fn(&r)) != hipSuccess) return -(long)e;
        if (r.count && !total)
            std::snprintf(msg, msg_len, "LDPC_CHECK: %s index %u >= bound %u (block %u, thread %u)",
                          check_site_name(r.site), r.idx, r.bound, r.block, r.thread);
        total += r.count;
    }
    return total;
}
}  // namespace ldpc
// checked builds: every launch is synchronised and its indices' record read
#define LDPC_CHECK_AFTER_LAUNCH(stream)                                                              \
    do {                                                                                             \
        char m_[192];                                                                                \
        const long n_ = ldpc::check_collect((stream), m_, sizeof m_);                                \
        if (n_ < 0) return set_err(LDPC_ERR_DEVICE, "check_collect: %s", hipGetErrorString((hipError_t)-n_)); \
        if (n_ > 0) return set_err(LDPC_ERR_DEVICE, "%s; %ld violations", m_, n_);                   \
    } while (0)
#else
#define LDPC_CHECK_AFTER_LAUNCH(stream) ((void)0)
#endif

struct DevBuf {
    void *p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t bytes)
    {
        if (bytes <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipSuccess) n = bytes;
        return e;
    }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

struct ldpc_ctx {
    int device = 0;
    const ldpc_graph *g = nullptr;
    int max_batch = 0;
    int num_cus = 0;
    hipStream_t own = nullptr, stream = nullptr;
    ldpc::DevGraph dg{};
    DevBuf graph, counts, hist, y_stage, c_stage, d_stage, fw_stage, cw_table, gscratch, p_stage;
    int cw_rows = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t handoff = nullptr;  // orders the launches of a context across ldpc_ctx_set_stream
    ldpc::AuxStream aux;          // second stream of the flooding phase launches (kernels.h)
    bool timed = false;
    ldpc::Options opts;           // kernel-selection options (ldpc_ctx_set_option), tests and A/B only
    bool has_rs = false;
    ldpc::RowSched rs{};
    DevBuf sched;
    bool has_rs_pp = false;                               // the ping-pong kernel's degree-aware row slots
    ldpc::RowSched rs_pp{};
    DevBuf sched_pp;
    bool has_fs = false;
    ldpc::FloodSched fs{};
    DevBuf fsched;                                        // flood kernel schedule (codes beyond LDS)
    bool has_ls = false;
    ldpc::LayerSched ls{};                                // layered schedule (row order = fs order)
    DevBuf lsched;
    DevBuf divcheck;                                      // mismatch counter of verify_div_by_reciprocal
    DevBuf redo;                                          // re-decode list of the fast row kernel
    bool last_fast = false;                               // last min-sum launch used the fast row kernel
    std::vector<std::pair<float, bool>> div_ok;           // alpha -> reciprocal division exact
};

namespace ldpc {
int set_last_error(int code, const std::string &msg)
{
    g_last_error = msg;
    return code;
}

static const Options kNoOptions{};
static thread_local const Options *t_opts = nullptr;
const Options &cur_opts() { return t_opts ? *t_opts : kNoOptions; }
OptScope::OptScope(const Options &o) : prev_(t_opts) { t_opts = &o; }
OptScope::~OptScope() { t_opts = prev_; }

bool option_value_ok(int option, int v)
{
    switch (option) {
    case LDPC_OPT_ROWS64:
    case LDPC_OPT_ROWS32: return v >= 0 && v <= 2;
    case LDPC_OPT_PP_SLOTS:
    case LDPC_OPT_FLOOD_MODE:
    case LDPC_OPT_FLOOD_MSG:
    case LDPC_OPT_BP_KERNEL:
    case LDPC_OPT_GDBF_KERNEL:
    case LDPC_OPT_EMS_SWIZZLE: return v == 0 || v == 1;
    case LDPC_OPT_KERNEL: return v >= 0 && v <= 3;
    case LDPC_OPT_FLOOD_SPS_CHECK:
    case LDPC_OPT_FLOOD_SPS_BIT: return v >= 0 && v <= 4;
    case LDPC_OPT_FLOOD_RESIDENT: return v >= 0 && v <= 4096;
    case LDPC_OPT_FLOOD_STREAMS: return v >= 0 && v <= 2;
    case LDPC_OPT_FLOOD_BPC:
    case LDPC_OPT_LAYERED_BPC:
    case LDPC_OPT_ROWS_BPC:
    case LDPC_OPT_FAST_BPC: return v >= 0 && v <= 64;
    case LDPC_OPT_LAYERED_LDS_POS: return v >= 0 && v <= 65536;
    case LDPC_OPT_LAYERED_ROWS64: return v >= 0 && v <= 2;
    case LDPC_OPT_LAYERED_THREADS:
    case LDPC_OPT_EMS_THREADS: return v == 0 || v == 512 || v == 1024;
    default: return false;
    }
}
}  // namespace ldpc

// Device copy of a host row schedule (graph.cpp build_row_schedule).
static hipError_t upload_row_sched(const ldpc::RowSchedule &hs, DevBuf &buf, ldpc::RowSched &rs)
{
    auto al = [](size_t n) { return (n + 255) & ~(size_t)255; };
    const size_t b_cc = al(2 * hs.cn_cols.size()), b_cp = al(2 * hs.cn_pos.size()), b_cd = al(hs.cn_deg.size()),
                 b_vc = al(2 * hs.vn_col.size()), b_vi = al(4 * hs.vn_info.size());
    hipError_t e = buf.ensure(b_cc + b_cp + b_cd + b_vc + b_vi);
    if (e != hipSuccess) return e;
    unsigned char *sb = (unsigned char *)buf.p;
    const std::pair<const void *, size_t> parts[] = {{hs.cn_cols.data(), 2 * hs.cn_cols.size()},
                                                     {hs.cn_pos.data(), 2 * hs.cn_pos.size()},
                                                     {hs.cn_deg.data(), hs.cn_deg.size()},
                                                     {hs.vn_col.data(), 2 * hs.vn_col.size()},
                                                     {hs.vn_info.data(), 4 * hs.vn_info.size()}};
    const size_t offs[] = {0, b_cc, b_cc + b_cp, b_cc + b_cp + b_cd, b_cc + b_cp + b_cd + b_vc};
    for (int i = 0; i < 5; ++i)
        if (parts[i].second && (e = hipMemcpy(sb + offs[i], parts[i].first, parts[i].second, hipMemcpyHostToDevice)) != hipSuccess)
            return e;
    rs.threads = hs.threads;
    rs.cpt = hs.cpt;
    rs.dc = hs.dc;
    rs.e_pad = hs.e_pad;
    rs.rpt = hs.rpt;
    rs.dc_low = hs.dc_low;
    rs.cn_cols = (const uint16_t *)sb;
    rs.cn_pos = (const uint16_t *)(sb + offs[1]);
    rs.cn_deg = (const uint8_t *)(sb + offs[2]);
    rs.vn_col = (const uint16_t *)(sb + offs[3]);
    rs.vn_info = (const uint32_t *)(sb + offs[4]);
    return hipSuccess;
}

extern "C" {

int ldpc_abi_version(void) { return LDPC_ABI_VERSION; }
int ldpc_f64_nms_fast_division(double alpha) { return ldpc::markstein_exact_alpha(alpha) ? 1 : 0; }
const char *ldpc_last_error(void) { return g_last_error.c_str(); }

// ----------------------------------------------------------------- graph
int ldpc_graph_create(int N, int M, const int *num_nlist, const int *const *nlist, const int *num_mlist,
                      const int *const *mlist, ldpc_graph **out)
{
    if (!out) return set_err(LDPC_ERR_INVALID, "out is null");
    *out = nullptr;
    ldpc_graph *g = new (std::nothrow) ldpc_graph();
    if (!g) return set_err(LDPC_ERR_NOMEM, "graph allocation failed");
    std::string err;
    try {
        err = ldpc::build_graph(N, M, num_nlist, nlist, num_mlist, mlist, *g);
    } catch (const std::bad_alloc &) {
        delete g;
        return set_err(LDPC_ERR_NOMEM, "graph build out of memory");
    }
    if (!err.empty()) {
        delete g;
        return set_err(LDPC_ERR_GRAPH, "%s", err.c_str());
    }
    *out = g;
    return LDPC_OK;
}

int ldpc_graph_load_alist(const char *path, ldpc_graph **out)
{
    if (!out || !path) return set_err(LDPC_ERR_INVALID, "null argument");
    *out = nullptr;
    ldpc_graph *g = new (std::nothrow) ldpc_graph();
    if (!g) return set_err(LDPC_ERR_NOMEM, "graph allocation failed");
    std::string err;
    try {
        err = ldpc::load_alist(path, *g);
    } catch (const std::bad_alloc &) {
        delete g;
        return set_err(LDPC_ERR_NOMEM, "alist load out of memory");
    }
    if (!err.empty()) {
        delete g;
        const bool io = err.rfind("cannot open", 0) == 0;
        return set_err(io ? LDPC_ERR_IO : LDPC_ERR_GRAPH, "%s", err.c_str());
    }
    *out = g;
    return LDPC_OK;
}

int ldpc_graph_info(const ldpc_graph *g, int *N, int *M, int *E, int *maxdv, int *maxdc)
{
    if (!g) return set_err(LDPC_ERR_INVALID, "graph is null");
    if (N) *N = g->N;
    if (M) *M = g->M;
    if (E) *E = g->E;
    if (maxdv) *maxdv = g->maxdv;
    if (maxdc) *maxdc = g->maxdc;
    return LDPC_OK;
}

void ldpc_graph_destroy(ldpc_graph *g) { delete g; }

int ldpc_graph_layers(const ldpc_graph *g, int32_t *row_order, int32_t *layer_ptr, int *nlayers)
{
    if (!g || !nlayers) return set_err(LDPC_ERR_INVALID, "null argument");
    ldpc::FloodSchedule fh;
    ldpc::LayerSchedule lh;
    std::string err;
    try {
        err = ldpc::build_flood_schedule(*g, fh);
        if (err.empty()) err = ldpc::build_layers(*g, fh, lh);
    } catch (const std::bad_alloc &) {
        return set_err(LDPC_ERR_NOMEM, "layer schedule out of memory");
    }
    if (!err.empty()) return set_err(LDPC_ERR_GRAPH, "%s", err.c_str());
    *nlayers = (int)lh.lptr.size() - 1;
    if (row_order)
        for (int i = 0; i < g->M; ++i) row_order[i] = lh.row_order[i];
    if (layer_ptr)
        for (size_t L = 0; L < lh.lptr.size(); ++L) layer_ptr[L] = lh.lptr[L];
    return LDPC_OK;
}

// ----------------------------------------------------------------- context
int ldpc_bp_math_probe(int device, const double *x, int n, double *tanh_out, double *log_out)
{
    if (!x || n < 0) return set_err(LDPC_ERR_INVALID, "x is null or n < 0");
    if (n == 0) return LDPC_OK;
    HIP_TRY(hipSetDevice(device));
    const size_t bytes = sizeof(double) * (size_t)n;
    double *dx = nullptr, *dt = nullptr, *dl = nullptr;
    hipError_t e = hipMalloc(&dx, 3 * bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return set_err(LDPC_ERR_NOMEM, "hipMalloc(%zu): %s", 3 * bytes, hipGetErrorString(e));
    }
    dt = dx + n;
    dl = dt + n;
    e = hipMemcpy(dx, x, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = ldpc::bp_math_probe(dx, tanh_out ? dt : nullptr, log_out ? dl : nullptr, n, nullptr);
    if (e == hipSuccess && tanh_out) e = hipMemcpy(tanh_out, dt, bytes, hipMemcpyDeviceToHost);
    if (e == hipSuccess && log_out) e = hipMemcpy(log_out, dl, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(dx);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return set_err(LDPC_ERR_DEVICE, "bp math probe: %s", hipGetErrorString(e));
    }
    return LDPC_OK;
}

int ldpc_check_selftest(int device)
{
#ifdef LDPC_CHECK
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(ldpc::check_selftest_launch(nullptr));
    LDPC_CHECK_AFTER_LAUNCH(nullptr);
    return set_err(LDPC_ERR_DEVICE, "LDPC_CHECK self-test: the violation was not recorded");
#else
    (void)device;
    return set_err(LDPC_ERR_UNSUPPORTED, "this library has no device index checks (build `make checked`)");
#endif
}

int ldpc_device_count(int *n)
{
    if (!n) return set_err(LDPC_ERR_INVALID, "n is null");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        *n = 0;
        return set_err(LDPC_ERR_DEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *n = c;
    return LDPC_OK;
}

static void ctx_free(ldpc_ctx *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (DevBuf *b : {&c->graph, &c->counts, &c->hist, &c->y_stage, &c->c_stage, &c->d_stage, &c->fw_stage,
                      &c->cw_table, &c->gscratch, &c->sched, &c->sched_pp, &c->divcheck, &c->fsched, &c->lsched, &c->p_stage,
                      &c->redo})
        b->release();
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->handoff) (void)hipEventDestroy(c->handoff);
    if (c->aux.fork) (void)hipEventDestroy(c->aux.fork);
    if (c->aux.join) (void)hipEventDestroy(c->aux.join);
    if (c->aux.s) (void)hipStreamDestroy(c->aux.s);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

int ldpc_ctx_create(int device, const ldpc_graph *g, int max_batch, ldpc_ctx **out)
{
    if (!out || !g) return set_err(LDPC_ERR_INVALID, "null argument");
    *out = nullptr;
    if (max_batch <= 0) return set_err(LDPC_ERR_INVALID, "max_batch must be > 0");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return set_err(LDPC_ERR_INVALID, "device %d of %d", device, ndev);
    ldpc_ctx *c = new (std::nothrow) ldpc_ctx();
    if (!c) return set_err(LDPC_ERR_NOMEM, "ctx allocation failed");
    c->device = device;
    c->g = g;
    c->max_batch = max_batch;
    auto fail = [&](int rc) {
        ctx_free(c);
        return rc;
    };
    hipError_t e;
#define CTX_TRY(expr)                                                                                   \
    do {                                                                                                \
        e = (expr);                                                                                     \
        if (e != hipSuccess) {                                                                          \
            (void)hipGetLastError();                                                                    \
            return fail(set_err(LDPC_ERR_DEVICE, "%s failed: %s", #expr, hipGetErrorString(e)));       \
        }                                                                                               \
    } while (0)
    CTX_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    CTX_TRY(hipGetDeviceProperties(&prop, device));
    c->num_cus = prop.multiProcessorCount;
    CTX_TRY(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
    c->stream = c->own;
    CTX_TRY(hipEventCreate(&c->ev0));
    CTX_TRY(hipEventCreate(&c->ev1));
    CTX_TRY(hipStreamCreateWithFlags(&c->aux.s, hipStreamNonBlocking));
    CTX_TRY(hipEventCreateWithFlags(&c->aux.fork, hipEventDisableTiming));
    CTX_TRY(hipEventCreateWithFlags(&c->aux.join, hipEventDisableTiming));

    // Graph upload: one allocation, 256-B aligned sections.
    const int dcs = g->maxdc > 0 ? g->maxdc : 1;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t s_rc = al(sizeof(int32_t) * (size_t)g->M * dcs), s_rd = al((size_t)g->M),
                 s_cp = al(sizeof(int32_t) * (size_t)(g->N + 1)), s_cr = al(sizeof(uint32_t) * (size_t)(g->E + 1));
    CTX_TRY(c->graph.ensure(s_rc + s_rd + s_cp + s_cr));
    unsigned char *gb = (unsigned char *)c->graph.p;
    CTX_TRY(hipMemcpy(gb, g->row_cols.data(), sizeof(int32_t) * g->row_cols.size(), hipMemcpyHostToDevice));
    CTX_TRY(hipMemcpy(gb + s_rc, g->row_deg.data(), g->row_deg.size(), hipMemcpyHostToDevice));
    CTX_TRY(hipMemcpy(gb + s_rc + s_rd, g->col_ptr.data(), sizeof(int32_t) * g->col_ptr.size(),
                      hipMemcpyHostToDevice));
    if (g->E > 0)
        CTX_TRY(hipMemcpy(gb + s_rc + s_rd + s_cp, g->col_refs.data(), sizeof(uint32_t) * g->col_refs.size(),
                          hipMemcpyHostToDevice));
    c->dg.N = g->N;
    c->dg.M = g->M;
    c->dg.dcs = dcs;
    c->dg.row_cols = (const int32_t *)gb;
    c->dg.row_deg = (const uint8_t *)(gb + s_rc);
    c->dg.col_ptr = (const int32_t *)(gb + s_rc + s_rd);
    c->dg.col_refs = (const uint32_t *)(gb + s_rc + s_rd + s_cp);

    // Row-parallel schedule (the throughput kernel) when the graph fits it.
    {
        // Rows per thread: 1 up to 512 rows (512-thread blocks), 2 up to 1024 rows
        // (512 threads, two blocks per CU: their barriers overlap; measured 1.13x
        // over one 1024-thread block with 1 row per thread on the N=1944 code).
        const int rpt = g->M <= 512 ? 1 : 2;
        int threads = ((((g->M + rpt - 1) / rpt) + 63) / 64) * 64;
        if (threads < 64) threads = 64;
        int dc = 0, cpt = 0;
        for (int d : ldpc::kRowsDc)
            if (!dc && g->maxdc <= d) dc = d;
        static const int cpt_for_rpt[][3] = {{0, 0, 0}, {2, 4, 0}, {4, 0, 0}};
        for (int q : cpt_for_rpt[rpt])
            if (q && !cpt && (long)(threads / 64) * q >= (g->N + 63) / 64) cpt = q;
        ldpc::RowSchedule hs;
        if (threads <= ldpc::kRowsMaxThreadsForRpt[rpt] && dc && cpt &&
            ldpc::build_row_schedule(*g, threads, cpt, dc, rpt, hs).empty()) {
            CTX_TRY(upload_row_sched(hs, c->sched, c->rs));
            c->has_rs = true;
            // the ping-pong kernel's copy: degree-7 rows on the younger check waves (graph.h pp_row_slots)
            const std::vector<int> slots = ldpc::pp_row_slots(*g, threads, 7);
            ldpc::RowSchedule hp;
            if (rpt == 2 && dc == 8 && cpt == 4 && !slots.empty() &&
                ldpc::build_row_schedule(*g, threads, cpt, dc, rpt, hp, &slots).empty()) {
                hp.dc_low = 7;
                CTX_TRY(upload_row_sched(hp, c->sched_pp, c->rs_pp));
                c->has_rs_pp = true;
            }
        }
    }
    // Flood schedule (global-memory kernel for codes whose state exceeds LDS;
    // also selectable with LDPC_KERNEL=flood for tests).
    {
        ldpc::FloodSchedule fh;
        if (ldpc::build_flood_schedule(*g, fh).empty()) {
            const size_t n_sp = fh.sp.size(), n_rd = fh.rdeg.size(), n_pb = fh.pos_of_bit.size(),
                         n_ba = fh.bit_at.size(), n_pd = fh.pdeg.size(), n_gb = fh.gbase.size();
            const size_t o_sq = al(4 * n_sp), o_rd = o_sq + al(4 * n_sp), o_pb = o_rd + al(n_rd),
                         o_ba = o_pb + al(4 * n_pb), o_pd = o_ba + al(4 * n_ba), o_gb = o_pd + al(n_pd),
                         o_er = o_gb + al(4 * n_gb), n_er = (size_t)fh.e_pad + 64, tot = o_er + al(4 * n_er);
            // element -> (row, position) of the c2v layout: the packed-message bit phase
            // (kernels.hip k_flood_bit_packed) rebuilds a message from its row's state
            std::vector<uint32_t> eref(n_er, 0);
            for (int i = 0; i < fh.M_pad; ++i)
                for (int k = 0; k < fh.rdeg[i]; ++k)
                    eref[fh.sq[(size_t)k * fh.M_pad + i]] = ((uint32_t)i << 5) | (uint32_t)k;
            CTX_TRY(c->fsched.ensure(tot));
            unsigned char *fb = (unsigned char *)c->fsched.p;
            CTX_TRY(hipMemcpy(fb, fh.sp.data(), 4 * n_sp, hipMemcpyHostToDevice));
            CTX_TRY(hipMemcpy(fb + o_sq, fh.sq.data(), 4 * n_sp, hipMemcpyHostToDevice));
            CTX_TRY(hipMemcpy(fb + o_rd, fh.rdeg.data(), n_rd, hipMemcpyHostToDevice));
            CTX_TRY(hipMemcpy(fb + o_pb, fh.pos_of_bit.data(), 4 * n_pb, hipMemcpyHostToDevice));
            CTX_TRY(hipMemcpy(fb + o_ba, fh.bit_at.data(), 4 * n_ba, hipMemcpyHostToDevice));
            CTX_TRY(hipMemcpy(fb + o_pd, fh.pdeg.data(), n_pd, hipMemcpyHostToDevice));
            CTX_TRY(hipMemcpy(fb + o_gb, fh.gbase.data(), 4 * n_gb, hipMemcpyHostToDevice));
            CTX_TRY(hipMemcpy(fb + o_er, eref.data(), 4 * n_er, hipMemcpyHostToDevice));
            c->fs.M_pad = fh.M_pad;
            c->fs.dc = fh.dc;
            c->fs.ngroups = fh.ngroups;
            c->fs.e_pad = fh.e_pad;
            c->fs.dv = g->maxdv;
            c->fs.sp = (const int32_t *)fb;
            c->fs.sq = (const int32_t *)(fb + o_sq);
            c->fs.rdeg = (const uint8_t *)(fb + o_rd);
            c->fs.pos_of_bit = (const int32_t *)(fb + o_pb);
            c->fs.bit_at = (const int32_t *)(fb + o_ba);
            c->fs.pdeg = (const uint8_t *)(fb + o_pd);
            c->fs.gbase = (const int32_t *)(fb + o_gb);
            c->fs.eref = (const uint32_t *)(fb + o_er);
            c->has_fs = true;
            ldpc::LayerSchedule lh;
            if (fh.dc <= ldpc::kPackedMaxDc && ldpc::build_layers(*g, fh, lh).empty()) {
                const size_t n_lp = lh.lptr.size(), n_sp = lh.sp.size(), n_rd = lh.rdeg.size(),
                             n_pb = lh.pos_of_bit.size();
                const size_t o_sp = al(4 * n_lp), o_rd = o_sp + al(4 * n_sp), o_pb = o_rd + al(n_rd),
                             tot = o_pb + al(4 * n_pb);
                CTX_TRY(c->lsched.ensure(tot));
                unsigned char *lb = (unsigned char *)c->lsched.p;
                CTX_TRY(hipMemcpy(lb, lh.lptr.data(), 4 * n_lp, hipMemcpyHostToDevice));
                CTX_TRY(hipMemcpy(lb + o_sp, lh.sp.data(), 4 * n_sp, hipMemcpyHostToDevice));
                CTX_TRY(hipMemcpy(lb + o_rd, lh.rdeg.data(), n_rd, hipMemcpyHostToDevice));
                CTX_TRY(hipMemcpy(lb + o_pb, lh.pos_of_bit.data(), 4 * n_pb, hipMemcpyHostToDevice));
                c->ls.pos_of_bit = (const int32_t *)(lb + o_pb);
                c->ls.nlayers = (int)n_lp - 1;
                c->ls.M_pad = lh.M_pad;
                c->ls.lptr = (const int32_t *)lb;
                c->ls.sp = (const int32_t *)(lb + o_sp);
                c->ls.rdeg = (const uint8_t *)(lb + o_rd);
                for (int L = 0; L < c->ls.nlayers; ++L)
                    c->ls.max_layer = std::max(c->ls.max_layer, lh.lptr[L + 1] - lh.lptr[L]);
                c->has_ls = true;
            }
        }
    }
    CTX_TRY(c->counts.ensure(8 * sizeof(unsigned long long)));
    CTX_TRY(hipMemset(c->counts.p, 0, c->counts.n));
    CTX_TRY(c->hist.ensure(sizeof(unsigned long long) * (size_t)g->N));
    CTX_TRY(hipMemset(c->hist.p, 0, c->hist.n));
#undef CTX_TRY
    *out = c;
    return LDPC_OK;
}

int ldpc_ctx_set_stream(ldpc_ctx *c, void *s)
{
    if (!c) return set_err(LDPC_ERR_INVALID, "ctx is null");
    const hipStream_t ns = s ? (hipStream_t)s : c->own;
    if (ns != c->stream) {
        // The launches of one context share its counters (the GDBF/EMS codeword ticket
        // included), staging and re-decode buffers: the new stream starts after everything
        // already queued on the old one, so launches never overlap across a stream change.
        HIP_TRY(hipSetDevice(c->device));
        if (!c->handoff) HIP_TRY(hipEventCreateWithFlags(&c->handoff, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(c->handoff, c->stream));
        HIP_TRY(hipStreamWaitEvent(ns, c->handoff, 0));
    }
    c->stream = ns;
    return LDPC_OK;
}

int ldpc_ctx_synchronize(ldpc_ctx *c)
{
    if (!c) return set_err(LDPC_ERR_INVALID, "ctx is null");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return LDPC_OK;
}

void ldpc_ctx_destroy(ldpc_ctx *c) { ctx_free(c); }

int ldpc_ctx_set_option(ldpc_ctx *c, int option, int value)
{
    if (!c) return set_err(LDPC_ERR_INVALID, "ctx is null");
    if (!ldpc::option_value_ok(option, value))
        return set_err(LDPC_ERR_INVALID, "option %d: unknown, or value %d out of range", option, value);
    if (ldpc::option_is_ems(option))
        return set_err(LDPC_ERR_INVALID, "option %d is an EMS option (ldpc_nb_ctx_set_option)", option);
    c->opts.v[option] = value;
    return LDPC_OK;
}

int ldpc_ctx_get_option(const ldpc_ctx *c, int option, int *value)
{
    if (!c || !value) return set_err(LDPC_ERR_INVALID, "null argument");
    if (option <= 0 || option >= LDPC_OPT_COUNT) return set_err(LDPC_ERR_INVALID, "unknown option %d", option);
    *value = c->opts.v[option];
    return LDPC_OK;
}

// ----------------------------------------------------------------- helpers
static bool is_device_ptr(const void *p)
{
    if (!p) return false;
    hipPointerAttribute_t at;
    hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
}

static int check_cfg(const ldpc_ctx *c, const ldpc_decoder_cfg *cfg)
{
    if (!cfg) return set_err(LDPC_ERR_INVALID, "cfg is null");
    if (cfg->variant < LDPC_MS || cfg->variant > LDPC_BP) return set_err(LDPC_ERR_INVALID, "bad variant %d", cfg->variant);
    if (cfg->variant == LDPC_BP) {
        if (cfg->schedule != LDPC_FLOODING) return set_err(LDPC_ERR_UNSUPPORTED, "BP is flooding only");
        if (c->g->maxdc > ldpc::kBpMaxDc)
            return set_err(LDPC_ERR_UNSUPPORTED, "BP supports row degree <= %d", ldpc::kBpMaxDc);
        if (cfg->max_llr < 0) return set_err(LDPC_ERR_INVALID, "max_llr must be >= 0");
    }
    if (cfg->precision != LDPC_F32 && cfg->precision != LDPC_F64)
        return set_err(LDPC_ERR_INVALID, "bad precision %d", cfg->precision);
    if (cfg->T < 0) return set_err(LDPC_ERR_INVALID, "T must be >= 0");
    if ((cfg->quantize || cfg->saturate) && !(cfg->ymax > 0))
        return set_err(LDPC_ERR_INVALID, "quantize/saturate need ymax > 0");
    if (cfg->quantize && (cfg->qbits < 1 || cfg->qbits > 30)) return set_err(LDPC_ERR_INVALID, "qbits out of range");
    if (cfg->schedule != LDPC_FLOODING && cfg->schedule != LDPC_LAYERED)
        return set_err(LDPC_ERR_INVALID, "bad schedule %d", cfg->schedule);
    if (cfg->schedule == LDPC_LAYERED && !c->has_ls)
        return set_err(LDPC_ERR_UNSUPPORTED, "layered schedule unavailable for this graph (row degree > %d)",
                       ldpc::kPackedMaxDc);
    return LDPC_OK;
}

static void fill_common(ldpc::DecodeArgs &a, ldpc_ctx *c, const ldpc_decoder_cfg *cfg, int batch)
{
    std::memset(&a, 0, sizeof a);
    a.batch = batch;
    a.T = cfg->T;
    a.variant = cfg->variant;
    a.quantize = cfg->quantize;
    a.saturate = cfg->saturate;
    a.ymax = cfg->ymax;
    a.nq = std::pow(2.0, (double)cfg->qbits);   // Nq = pow(2.0, Q) (:121)
    a.alpha = cfg->alpha;
    a.delta = cfg->delta;
    a.n0 = cfg->n0;
    a.max_llr = cfg->max_llr > 0 ? cfg->max_llr : 20.0;   // MAXLLR = 20 (decodeBP.cpp:58)
    a.counts = (unsigned long long *)c->counts.p;
    a.hist = (unsigned long long *)c->hist.p;
}

static_assert(sizeof(ldpc_frame_result) == sizeof(int4), "frame result layout");

// fp32 NMS: use the reciprocal division only after the device has checked it
// against IEEE x/alpha for every finite non-negative float (cached per alpha).
static int nms_setup(ldpc_ctx *c, const ldpc_decoder_cfg *cfg, ldpc::DecodeArgs &a)
{
    a.nms_fast = 0;
    a.alpha_rcp = 0.f;
    if (cfg->variant != LDPC_NMS || cfg->precision != LDPC_F32) return LDPC_OK;
    const float alpha = (float)cfg->alpha;
    if (!(alpha > 0.f) || !std::isfinite(alpha)) return LDPC_OK;
    const float rcp = 1.0f / alpha;
    bool ok = false, known = false;
    for (const auto &e : c->div_ok)
        if (e.first == alpha) { ok = e.second; known = true; }
    if (!known) {
        HIP_TRY(c->divcheck.ensure(sizeof(unsigned long long)));
        HIP_TRY(ldpc::verify_div_by_reciprocal(alpha, rcp, (unsigned long long *)c->divcheck.p, c->stream));
        unsigned long long bad = 1;
        HIP_TRY(hipMemcpyAsync(&bad, c->divcheck.p, sizeof bad, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        ok = bad == 0;
        c->div_ok.emplace_back(alpha, ok);
    }
    if (ok) {
        a.nms_fast = 1;
        a.alpha_rcp = rcp;
    }
    return LDPC_OK;
}

// LDPC_OPT_KERNEL: the generic kernel a test forces (kernels.hip choose_kernel).
static const char *forced_kernel(const ldpc_ctx *c)
{
    static const char *const names[] = {nullptr, "lds", "flood", "global"};
    return names[c->opts.v[LDPC_OPT_KERNEL]];
}

static ldpc::KernelChoice select_kernel(const ldpc_ctx *c, bool f64, int schedule, int variant)
{
    const ldpc::OptScope os(c->opts);
    if (variant == LDPC_BP) return ldpc::bp_choose(c->dg, f64, c->g->E);
    if (schedule == LDPC_LAYERED) return ldpc::choose_layered(c->dg, f64, c->fs, c->ls, forced_kernel(c));
    return ldpc::choose_kernel(c->dg, f64, c->has_rs ? &c->rs : nullptr, forced_kernel(c), c->has_fs ? &c->fs : nullptr);
}

static bool is_layered(const ldpc::KernelChoice &kc) { return kc.name[0] == 'l' && kc.name[1] == 'a'; }

// The ping-pong kernel's schedule: the degree-aware row slots (graph.h
// pp_row_slots) when the code admits them, else the row kernel's.
static const ldpc::RowSched &pp_sched(const ldpc_ctx *c)
{
    if (c->opts.v[LDPC_OPT_PP_SLOTS] == 1) return c->rs;   // tests / A/B: the row kernel's slots
    return c->has_rs_pp ? c->rs_pp : c->rs;
}

// Row graphs on the fast path: a kernel holding only the fast check node plus the
// exact re-decode (k_redo) of the codewords whose premise failed.
//   fp64: the ping-pong kernel (rows_pp.hip: two codewords per 1024-thread block,
//         check and bit waves overlapped) when the schedule fits it, else the
//         one-codeword-per-block k_rows_fast (LDPC_OPT_ROWS64 = 1 forces the latter);
//   fp32: pairs as float2 -- MS and NMS with the verified reciprocal (a after
//         nms_setup) -- on the ping-pong kernel (7.4 vs 8.8 ms per bench launch for
//         the row kernel), on the pair instance of k_rows_fast with
//         LDPC_OPT_ROWS32 = 1, on the row kernel (kernels.hip k_decode_rows, fast and
//         exact loops in one) with LDPC_OPT_ROWS32 = 2 and for everything else (OMS,
//         codes the ping-pong schedule does not fit).
// LDPC_OPT_ROWS64 = 2 keeps the row kernel for fp64 too.
enum class FastKind { none, pp, fast };
static FastKind fast_kind(const ldpc_ctx *c, const ldpc::KernelChoice &kc, bool f64, const ldpc::DecodeArgs &a)
{
    const int r64 = c->opts.v[LDPC_OPT_ROWS64], r32 = c->opts.v[LDPC_OPT_ROWS32];
    if (f64 && r64 == 2) return FastKind::none;
    if (kc.name[0] != 'r' || !c->has_rs || ldpc::redo_lds_bytes(c->dg, f64) > 160 * 1024) return FastKind::none;
    const bool pp_ok = ldpc::rows_pp_supported(c->dg, pp_sched(c));
    if (f64) {
        if (pp_ok && r64 == 0) return FastKind::pp;
        return ldpc::rows_fast_supported(c->rs, true) ? FastKind::fast : FastKind::none;
    }
    if (!ldpc::rows_fast_f32_ok(a)) return FastKind::none;
    if (r32 == 1) return ldpc::rows_fast_supported(c->rs, false) ? FastKind::fast : FastKind::none;
    if (r32 == 2) return FastKind::none;
    return pp_ok ? FastKind::pp : FastKind::none;
}
static bool use_rows_fast(const ldpc_ctx *c, const ldpc::KernelChoice &kc, bool f64, const ldpc::DecodeArgs &a)
{
    return fast_kind(c, kc, f64, a) != FastKind::none;
}
static bool use_rows_pp(const ldpc_ctx *c, const ldpc::KernelChoice &kc, bool f64, const ldpc::DecodeArgs &a)
{
    return fast_kind(c, kc, f64, a) == FastKind::pp;
}

// Flooding of codes beyond LDS: one launch per phase over an Infinity-Cache-
// resident set (default; 1.5x the persistent kernel on DVB-S2) or the
// persistent workgroup-per-codeword kernel (LDPC_OPT_FLOOD_MODE = 1).
static bool use_flood_phase(const ldpc_ctx *c) { return c->opts.v[LDPC_OPT_FLOOD_MODE] != 1; }

// Resident-state budget of the global layered kernel (bytes its resident codewords touch):
// within MI355X's 256 MiB Infinity Cache with room for the schedule and the rest of the
// working set (measured knee: 208.5 MiB fine, 216 MiB 1.2x slower; api.cpp run_kernel).
static constexpr size_t kLayeredResidentBudget = (size_t)208 << 20;

static int run_kernel(ldpc_ctx *c, const ldpc::DecodeArgs &a, bool f64, int schedule)
{
    const ldpc::OptScope os(c->opts);
    const ldpc::KernelChoice kc = select_kernel(c, f64, schedule, a.variant);
    const bool layered = is_layered(kc);
    if (a.variant == ldpc::VARIANT_BP) {
        int gblocks = 0;
        if (kc.scratch_per_block) {
            gblocks = std::min(a.batch, 4 * c->num_cus);
            HIP_TRY(c->gscratch.ensure(kc.scratch_per_block * (size_t)gblocks + 65536));   // + the phase kernels' counters
        }
        HIP_TRY(hipEventRecord(c->ev0, c->stream));
        HIP_TRY(ldpc::bp_launch(c->dg, a, f64, kc, c->gscratch.p, gblocks, c->g->E, c->num_cus, c->stream));
        HIP_TRY(hipEventRecord(c->ev1, c->stream));
        c->timed = true;
        LDPC_CHECK_AFTER_LAUNCH(c->stream);
        return LDPC_OK;
    }
    int gblocks = layered ? c->num_cus : 0;
    if (kc.scratch_per_block) {
        int per_cu = layered ? ldpc::layered_blocks_per_cu(f64, kc) : ldpc::blocks_per_cu(c->dg, f64, kc);
        // Global layered kernel: at most one codeword per CU, and no more resident
        // codewords than the Infinity Cache holds (kLayeredResidentBudget: DVB-S2 fp64,
        // 1.01 MB touched per codeword, runs 6.4 ms per codeword round at 184-216
        // resident codewords and 7.6 / 8.7 / 9.3 ms at 224 / 240 / 256 -- the state
        // spills to HBM; 2 per CU measured 1.5x slower); LDPC_OPT_LAYERED_BPC
        // overrides both (experiments).
        if (layered) {
            const int want = c->opts.v[LDPC_OPT_LAYERED_BPC] > 0 ? c->opts.v[LDPC_OPT_LAYERED_BPC] : 1;
            per_cu = std::min(per_cu, want);
        } else if (const int cap = c->opts.v[LDPC_OPT_FLOOD_BPC]) {   // global flooding kernel (experiments)
            per_cu = std::min(per_cu, cap);
        }
        if (per_cu <= 0) per_cu = 1;
        gblocks = per_cu * c->num_cus;
        if (layered && c->opts.v[LDPC_OPT_LAYERED_BPC] <= 0) {
            const size_t fp = ldpc::layered_resident_bytes(c->fs, c->ls, f64);
            gblocks = (int)std::min<size_t>((size_t)gblocks, std::max<size_t>(1, kLayeredResidentBudget / fp));
        }
        if (gblocks > a.batch) gblocks = a.batch;
        if (layered) {   // the same number of codeword rounds on fewer resident codewords
            const int rounds = (a.batch + gblocks - 1) / gblocks;
            gblocks = (a.batch + rounds - 1) / rounds;
        }
        HIP_TRY(c->gscratch.ensure(kc.scratch_per_block * (size_t)gblocks + 65536));   // + the phase kernels' counters
    }
#ifdef LDPC_STAMPS
    // diagnostic builds: per-block phase cycle sums appended to $LDPC_STAMPS
    static DevBuf stamp_buf;
    ldpc::DecodeArgs as = a;
    const char *stamp_path = std::getenv("LDPC_STAMPS");
    if (stamp_path) {
        HIP_TRY(stamp_buf.ensure(8192 * 4 * sizeof(unsigned long long)));
        HIP_TRY(hipMemsetAsync(stamp_buf.p, 0, stamp_buf.n, c->stream));
        as.stamps = (unsigned long long *)stamp_buf.p;
    }
#define a as
#endif
    // fp64 row graphs: the fast-path kernel plus the exact re-decode of any
    // codeword whose premise failed (LDPC_ROWS=old keeps the old row kernel).
    const bool fast = use_rows_fast(c, kc, f64, a);
    if (fast) HIP_TRY(c->redo.ensure(sizeof(unsigned) * ((size_t)c->max_batch + 1)));
    HIP_TRY(hipEventRecord(c->ev0, c->stream));
    c->last_fast = fast;
    if (fast) {
        HIP_TRY(hipMemsetAsync(c->redo.p, 0, sizeof(unsigned), c->stream));
        if (use_rows_pp(c, kc, f64, a))
            HIP_TRY(ldpc::launch_rows_pp(c->dg, pp_sched(c), a, f64, (unsigned *)c->redo.p, c->stream, c->num_cus));
        else
            HIP_TRY(ldpc::launch_rows_fast(c->dg, c->rs, a, f64, kc.lds_bytes, (unsigned *)c->redo.p, c->stream,
                                           c->num_cus));
        HIP_TRY(ldpc::launch_redo(c->dg, a, f64, (const unsigned *)c->redo.p, c->stream, c->num_cus));
    } else if (layered) {
        HIP_TRY(ldpc::launch_layered(c->dg, a, f64, kc, c->fs, c->ls, c->gscratch.p, gblocks, c->stream));
    } else if (kc.name[0] == 'f' && use_flood_phase(c))
        HIP_TRY(ldpc::launch_flood_phase(c->dg, c->fs, a, f64, kc, c->gscratch.p, c->gscratch.n, c->stream, &c->aux));
    else
        HIP_TRY(ldpc::launch_decode(c->dg, a, f64, kc, c->gscratch.p, gblocks, c->stream,
                                    c->has_rs ? &c->rs : nullptr, c->num_cus, c->has_fs ? &c->fs : nullptr));
    HIP_TRY(hipEventRecord(c->ev1, c->stream));
    c->timed = true;
#ifdef LDPC_STAMPS
#undef a
    if (stamp_path) {
        std::vector<unsigned long long> h(8192 * 4);
        HIP_TRY(hipMemcpyAsync(h.data(), stamp_buf.p, stamp_buf.n, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (FILE *f = std::fopen(stamp_path, "ab")) {
            std::fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
            std::fclose(f);
        }
    }
#endif
    LDPC_CHECK_AFTER_LAUNCH(c->stream);
    return LDPC_OK;
}


static int read_counts(ldpc_ctx *c, ldpc_counts *out, int reset)
{
    unsigned long long h[8];
    HIP_TRY(hipMemcpyAsync(h, c->counts.p, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (out) {
        out->bit_err = (int64_t)h[0];
        out->frame_err = (int64_t)h[1];
        out->uncoded_bit_err = (int64_t)h[2];
        out->frames = (int64_t)h[3];
        out->iters = (int64_t)h[4];
        out->syndrome_fail = (int64_t)h[5];
    }
    if (reset) HIP_TRY(hipMemsetAsync(c->counts.p, 0, c->counts.n, c->stream));
    return LDPC_OK;
}

static void accumulate(ldpc_counts *acc, const ldpc_counts &d)
{
    acc->bit_err += d.bit_err;
    acc->frame_err += d.frame_err;
    acc->uncoded_bit_err += d.uncoded_bit_err;
    acc->frames += d.frames;
    acc->iters += d.iters;
    acc->syndrome_fail += d.syndrome_fail;
}

// ----------------------------------------------------------------- decode
int ldpc_decode_batch(ldpc_ctx *c, const void *y, int batch, const ldpc_decoder_cfg *cfg, const int8_t *cw,
                      int8_t *d_out, ldpc_frame_result *frame_weights, ldpc_counts *counts)
{
    if (!c || !y) return set_err(LDPC_ERR_INVALID, "null argument");
    int rc = check_cfg(c, cfg);
    if (rc) return rc;
    if (batch <= 0 || batch > c->max_batch)
        return set_err(LDPC_ERR_INVALID, "batch %d outside 1..max_batch=%d", batch, c->max_batch);
    HIP_TRY(hipSetDevice(c->device));
    if (cfg->variant == LDPC_BP && !(cfg->n0 > 0)) return set_err(LDPC_ERR_INVALID, "BP needs cfg->n0 > 0");
    const bool f64 = cfg->precision == LDPC_F64;
    const int N = c->g->N;
    const size_t ybytes = (size_t)batch * N * (f64 ? 8 : 4);
    const size_t nbytes = (size_t)batch * N;

    ldpc::DecodeArgs a;
    fill_common(a, c, cfg, batch);
    a.src = ldpc::SRC_GIVEN;
    {
        const int nrc = nms_setup(c, cfg, a);
        if (nrc) return nrc;
    }
    // Inputs: stage host buffers.
    if (is_device_ptr(y)) {
        a.y = y;
    } else {
        HIP_TRY(c->y_stage.ensure(ybytes));
        HIP_TRY(hipMemcpyAsync(c->y_stage.p, y, ybytes, hipMemcpyHostToDevice, c->stream));
        a.y = c->y_stage.p;
    }
    if (cw) {
        if (is_device_ptr(cw)) {
            a.c = cw;
        } else {
            HIP_TRY(c->c_stage.ensure(nbytes));
            HIP_TRY(hipMemcpyAsync(c->c_stage.p, cw, nbytes, hipMemcpyHostToDevice, c->stream));
            a.c = (const int8_t *)c->c_stage.p;
        }
    }
    const bool d_host = d_out && !is_device_ptr(d_out);
    const bool w_host = frame_weights && !is_device_ptr(frame_weights);
    if (d_host) {
        HIP_TRY(c->d_stage.ensure(nbytes));
        a.d_out = (int8_t *)c->d_stage.p;
    } else {
        a.d_out = d_out;
    }
    if (w_host) {
        HIP_TRY(c->fw_stage.ensure(sizeof(ldpc_frame_result) * (size_t)batch));
        a.frame_res = (int4 *)c->fw_stage.p;
    } else {
        a.frame_res = (int4 *)frame_weights;
    }
    ldpc_counts before;
    rc = read_counts(c, &before, 0);
    if (rc) return rc;
    rc = run_kernel(c, a, f64, cfg->schedule);
    if (rc) return rc;
    if (d_host) HIP_TRY(hipMemcpyAsync(d_out, c->d_stage.p, nbytes, hipMemcpyDeviceToHost, c->stream));
    if (w_host)
        HIP_TRY(hipMemcpyAsync(frame_weights, c->fw_stage.p, sizeof(ldpc_frame_result) * (size_t)batch,
                               hipMemcpyDeviceToHost, c->stream));
    ldpc_counts after;
    rc = read_counts(c, &after, 0);
    if (rc) return rc;
    if (counts) {
        ldpc_counts d;
        d.bit_err = after.bit_err - before.bit_err;
        d.frame_err = after.frame_err - before.frame_err;
        d.uncoded_bit_err = after.uncoded_bit_err - before.uncoded_bit_err;
        d.frames = after.frames - before.frames;
        d.iters = after.iters - before.iters;
        d.syndrome_fail = after.syndrome_fail - before.syndrome_fail;
        accumulate(counts, d);
    }
    return LDPC_OK;
}

// ----------------------------------------------------------------- Monte-Carlo
int ldpc_sim_set_codewords(ldpc_ctx *c, const uint8_t *bits, int rows)
{
    if (!c) return set_err(LDPC_ERR_INVALID, "ctx is null");
    if (rows < 0 || (rows > 0 && !bits)) return set_err(LDPC_ERR_INVALID, "bad codeword table");
    HIP_TRY(hipSetDevice(c->device));
    c->cw_rows = 0;
    if (rows == 0) return LDPC_OK;
    const size_t n = (size_t)rows * c->g->N;
    std::vector<int8_t> bip(n);
    for (size_t i = 0; i < n; ++i) {
        if (bits[i] > 1) return set_err(LDPC_ERR_INVALID, "codeword bit %zu is %d (want 0/1)", i, bits[i]);
        bip[i] = bits[i] ? -1 : +1;   // '1' -> c = -1, '0' -> c = +1 (:204-207)
    }
    HIP_TRY(c->cw_table.ensure(n));
    HIP_TRY(hipMemcpy(c->cw_table.p, bip.data(), n, hipMemcpyHostToDevice));
    c->cw_rows = rows;
    return LDPC_OK;
}

static int sim_launch_impl(ldpc_ctx *c, double ebn0_db, double R, const ldpc_decoder_cfg *cfg, uint64_t seed,
                           uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames_dev,
                           void *y_out_dev, int8_t *d_out_dev)
{
    if (!c) return set_err(LDPC_ERR_INVALID, "ctx is null");
    int rc = check_cfg(c, cfg);
    if (rc) return rc;
    if (batch <= 0 || batch > c->max_batch)
        return set_err(LDPC_ERR_INVALID, "batch %d outside 1..max_batch=%d", batch, c->max_batch);
    if (!(R > 0)) return set_err(LDPC_ERR_INVALID, "rate must be > 0");
    HIP_TRY(hipSetDevice(c->device));
    ldpc::DecodeArgs a;
    fill_common(a, c, cfg, batch);
    a.src = ldpc::SRC_PHILOX;
    {
        const int nrc = nms_setup(c, cfg, a);
        if (nrc) return nrc;
    }
    const double N0 = std::pow(10.0, -ebn0_db / 10.0) / R;   // :146
    a.sigma = std::sqrt(N0 / 2.0);                            // :147
    if (cfg->variant == LDPC_BP) a.n0 = N0;                   // 4*y/N0 (decodeBP.cpp:104,188)
    a.seed = seed;
    a.stream_id = stream_id;
    a.first_cw = first_cw;
    a.cw_table = c->cw_rows ? (const int8_t *)c->cw_table.p : nullptr;
    a.cw_rows = c->cw_rows;
    a.frame_res = (int4 *)frames_dev;
    a.y_out = y_out_dev;
    a.d_out = d_out_dev;
    return run_kernel(c, a, cfg->precision == LDPC_F64, cfg->schedule);
}

int ldpc_sim_launch(ldpc_ctx *c, double ebn0_db, double R, const ldpc_decoder_cfg *cfg, uint64_t seed,
                    uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames_dev)
{
    if (frames_dev && !is_device_ptr(frames_dev))
        return set_err(LDPC_ERR_INVALID, "frames_dev must be a device pointer");
    return sim_launch_impl(c, ebn0_db, R, cfg, seed, stream_id, first_cw, batch, frames_dev, nullptr, nullptr);
}

int ldpc_ctx_read_counts(ldpc_ctx *c, ldpc_counts *out, int reset)
{
    if (!c) return set_err(LDPC_ERR_INVALID, "ctx is null");
    HIP_TRY(hipSetDevice(c->device));
    return read_counts(c, out, reset);
}

int ldpc_ctx_read_histogram(ldpc_ctx *c, int64_t *out, int reset)
{
    if (!c || !out) return set_err(LDPC_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(out, c->hist.p, c->hist.n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (reset) HIP_TRY(hipMemsetAsync(c->hist.p, 0, c->hist.n, c->stream));
    return LDPC_OK;
}

// Synchronous sim with optional host-or-device outputs (staged when host).
static int sim_sync_impl(ldpc_ctx *c, double ebn0_db, double R, const ldpc_decoder_cfg *cfg, uint64_t seed,
                         uint32_t stream_id, uint64_t first_cw, int batch, void *y_out, int8_t *d_out,
                         ldpc_frame_result *frames, ldpc_counts *accum)
{
    if (!c) return set_err(LDPC_ERR_INVALID, "ctx is null");
    int rc = check_cfg(c, cfg);
    if (rc) return rc;
    if (batch <= 0 || batch > c->max_batch)
        return set_err(LDPC_ERR_INVALID, "batch %d outside 1..max_batch=%d", batch, c->max_batch);
    HIP_TRY(hipSetDevice(c->device));
    const size_t nb = (size_t)batch * c->g->N;
    const size_t ybytes = nb * (cfg->precision == LDPC_F64 ? 8 : 4);
    ldpc_counts before;
    rc = read_counts(c, &before, 0);
    if (rc) return rc;
    const bool w_host = frames && !is_device_ptr(frames);
    const bool y_host = y_out && !is_device_ptr(y_out);
    const bool d_host = d_out && !is_device_ptr(d_out);
    ldpc_frame_result *fw_dev = frames;
    void *y_dev = y_out;
    int8_t *d_dev = d_out;
    if (w_host) {
        HIP_TRY(c->fw_stage.ensure(sizeof(ldpc_frame_result) * (size_t)batch));
        fw_dev = (ldpc_frame_result *)c->fw_stage.p;
    }
    if (y_host) {
        HIP_TRY(c->y_stage.ensure(ybytes));
        y_dev = c->y_stage.p;
    }
    if (d_host) {
        HIP_TRY(c->d_stage.ensure(nb));
        d_dev = (int8_t *)c->d_stage.p;
    }
    rc = sim_launch_impl(c, ebn0_db, R, cfg, seed, stream_id, first_cw, batch, fw_dev, y_dev, d_dev);
    if (rc) return rc;
    if (w_host)
        HIP_TRY(hipMemcpyAsync(frames, fw_dev, sizeof(ldpc_frame_result) * (size_t)batch, hipMemcpyDeviceToHost,
                               c->stream));
    if (y_host) HIP_TRY(hipMemcpyAsync(y_out, y_dev, ybytes, hipMemcpyDeviceToHost, c->stream));
    if (d_host) HIP_TRY(hipMemcpyAsync(d_out, d_dev, nb, hipMemcpyDeviceToHost, c->stream));
    ldpc_counts after;
    rc = read_counts(c, &after, 0);
    if (rc) return rc;
    if (accum) {
        ldpc_counts d;
        d.bit_err = after.bit_err - before.bit_err;
        d.frame_err = after.frame_err - before.frame_err;
        d.uncoded_bit_err = after.uncoded_bit_err - before.uncoded_bit_err;
        d.frames = after.frames - before.frames;
        d.iters = after.iters - before.iters;
        d.syndrome_fail = after.syndrome_fail - before.syndrome_fail;
        accumulate(accum, d);
    }
    return LDPC_OK;
}

int ldpc_sim_batch(ldpc_ctx *c, double ebn0_db, double R, const ldpc_decoder_cfg *cfg, uint64_t seed,
                   uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames, ldpc_counts *accum)
{
    return sim_sync_impl(c, ebn0_db, R, cfg, seed, stream_id, first_cw, batch, nullptr, nullptr, frames, accum);
}

int ldpc_sim_trace(ldpc_ctx *c, double ebn0_db, double R, const ldpc_decoder_cfg *cfg, uint64_t seed,
                   uint32_t stream_id, uint64_t first_cw, int batch, void *y_out, int8_t *d_out,
                   ldpc_frame_result *frames, ldpc_counts *accum)
{
    return sim_sync_impl(c, ebn0_db, R, cfg, seed, stream_id, first_cw, batch, y_out, d_out, frames, accum);
}

int ldpc_ctx_last_kernel_ms(ldpc_ctx *c, float *ms)
{
    if (!c || !ms) return set_err(LDPC_ERR_INVALID, "null argument");
    if (!c->timed) return set_err(LDPC_ERR_INVALID, "no kernel launched yet");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipEventSynchronize(c->ev1));
    HIP_TRY(hipEventElapsedTime(ms, c->ev0, c->ev1));
    return LDPC_OK;
}

int ldpc_ctx_row_sched_info(ldpc_ctx *c, const ldpc_decoder_cfg *cfg, int32_t *info)
{
    if (!c || !cfg || !info) return set_err(LDPC_ERR_INVALID, "null argument");
    const bool f64 = cfg->precision == LDPC_F64;
    int rc = check_cfg(c, cfg);
    if (rc) return rc;
    const ldpc::KernelChoice kc = select_kernel(c, f64, cfg->schedule, cfg->variant);
    if (cfg->variant == LDPC_BP || !c->has_rs || std::strcmp(kc.name, "rows") != 0)
        return set_err(LDPC_ERR_UNSUPPORTED, "the row kernel does not decode this cfg (kernel %s)", kc.name);
    info[0] = c->rs.threads;
    info[1] = c->rs.rpt;
    info[2] = c->rs.cpt;
    info[3] = c->rs.dc;
    info[4] = c->rs.e_pad;
    info[5] = kc.cw_per_block;
    info[6] = kc.lds_bytes;
    info[7] = ldpc::blocks_per_cu(c->dg, f64, kc);
    ldpc::DecodeArgs a;
    fill_common(a, c, cfg, 1);
    rc = nms_setup(c, cfg, a);   // fp32 NMS: whether the verified reciprocal (and so the fast kernels) applies
    if (rc) return rc;
    info[8] = 0;
    info[9] = c->rs.threads * c->rs.rpt * c->rs.dc;   // check edge slots issued per codeword-iteration
    if (use_rows_pp(c, kc, f64, a)) {   // one 1024-thread block per CU
        const ldpc::RowSched &rs = pp_sched(c);
        info[6] = ldpc::rows_pp_lds_bytes(c->dg, rs);
        info[7] = 1;
        info[8] = rs.dc_low;
        // degree-aware slots (rows_pp.hip k_rows_pp SPLIT): every row-0 slot and the row-1 slots of
        // threads >= threads/2 run a dc_low-edge check node, the other row-1 slots a dc-edge one
        if (rs.dc_low) info[9] = (rs.threads + rs.threads / 2) * rs.dc_low + (rs.threads / 2) * rs.dc;
    }
    return LDPC_OK;
}

int ldpc_ctx_redo_count(ldpc_ctx *c, int64_t *n)
{
    if (!c || !n) return set_err(LDPC_ERR_INVALID, "null argument");
    *n = 0;
    if (!c->last_fast || !c->redo.p) return LDPC_OK;
    HIP_TRY(hipSetDevice(c->device));
    unsigned h = 0;
    HIP_TRY(hipMemcpyAsync(&h, c->redo.p, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    *n = (int64_t)h;
    return LDPC_OK;
}

int ldpc_ctx_kernel_info(ldpc_ctx *c, const ldpc_decoder_cfg *cfg, char *name, int name_len, int *lds_bytes,
                         int *bpc)
{
    if (!c || !cfg) return set_err(LDPC_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    const bool f64 = cfg->precision == LDPC_F64;
    int rc = check_cfg(c, cfg);
    if (rc) return rc;
    const ldpc::KernelChoice kc = select_kernel(c, f64, cfg->schedule, cfg->variant);
    ldpc::DecodeArgs a;
    fill_common(a, c, cfg, 1);
    rc = nms_setup(c, cfg, a);   // fp32 NMS: whether the verified reciprocal (and so the fast kernel) applies
    if (rc) return rc;
    if (name && name_len > 0)
        std::snprintf(name, (size_t)name_len, "%s",
                      cfg->variant != LDPC_BP && use_rows_fast(c, kc, f64, a) ? (use_rows_pp(c, kc, f64, a) ? "rows_pp" : "rows_fast")
                                                                                : kc.name);
    if (lds_bytes) *lds_bytes = kc.lds_bytes;
    if (bpc) *bpc = cfg->variant == LDPC_BP ? 0 : is_layered(kc) ? (kc.lds_bytes ? 0 : ldpc::layered_blocks_per_cu(f64, kc))
                                   : ldpc::blocks_per_cu(c->dg, f64, kc);
    if (cfg->variant != LDPC_BP && use_rows_pp(c, kc, f64, a)) {
        if (lds_bytes) *lds_bytes = ldpc::rows_pp_lds_bytes(c->dg, pp_sched(c));
        if (bpc) *bpc = 1;
    }
    return LDPC_OK;
}


// ----------------------------------------------------------------- GDBF / NGDBF
static int gdbf_check_cfg(const ldpc_gdbf_cfg *cfg)
{
    if (!cfg) return set_err(LDPC_ERR_INVALID, "cfg is null");
    if (cfg->precision != LDPC_F32 && cfg->precision != LDPC_F64)
        return set_err(LDPC_ERR_INVALID, "bad precision %d", cfg->precision);
    if (cfg->T < 0 || cfg->T > 4094) return set_err(LDPC_ERR_INVALID, "T must be in 0..4094");
    if (cfg->flags & ~511) return set_err(LDPC_ERR_INVALID, "unknown GDBF flags 0x%x", cfg->flags);
    if ((cfg->flags & LDPC_GDBF_ADAPT) && (cfg->flags & (LDPC_GDBF_SEQUENTIAL | LDPC_GDBF_MODESWITCH)))
        return set_err(LDPC_ERR_UNSUPPORTED, "threshold adaptation with single-bit flips is not supported");
    if ((cfg->flags & LDPC_GDBF_QPROB) && (cfg->flags & LDPC_GDBF_NOISE))
        return set_err(LDPC_ERR_UNSUPPORTED, "QPROB with NOISE is not supported");
    if ((cfg->flags & LDPC_GDBF_MODESWITCH) && cfg->tswitch < 0) return set_err(LDPC_ERR_INVALID, "tswitch < 0");
    if ((cfg->flags & (LDPC_GDBF_SATURATE | LDPC_GDBF_QUANTIZE)) && !(cfg->ymax > 0))
        return set_err(LDPC_ERR_INVALID, "saturate/quantize need ymax > 0");
    if ((cfg->flags & LDPC_GDBF_QUANTIZE) && (cfg->nq < 1 || cfg->nq > 30))
        return set_err(LDPC_ERR_INVALID, "nq out of range");
    if ((cfg->flags & LDPC_GDBF_SMOOTH) && (cfg->windowsize < 0 || cfg->windowsize > 32767))
        return set_err(LDPC_ERR_INVALID, "windowsize out of range");
    return LDPC_OK;
}

static void gdbf_fill(ldpc::GdbfArgs &a, ldpc_ctx *c, const ldpc_gdbf_cfg *cfg, int batch)
{
    std::memset(&a, 0, sizeof a);
    a.batch = batch;
    a.T = cfg->T;
    a.flags = cfg->flags;
    a.windowsize = cfg->windowsize;
    a.theta0 = cfg->theta;
    a.lambda = cfg->lambda;
    a.w = (cfg->flags & LDPC_GDBF_WEIGHT) ? cfg->alpha : 1.0;   // :541-551
    a.ymax = cfg->ymax;
    a.qmax = std::pow(2, (cfg->nq - 1));                       // :490
    a.tswitch = cfg->tswitch;
    a.qsigma = cfg->qsigma;
    a.counts = (unsigned long long *)c->counts.p;
    a.hist = (unsigned long long *)c->hist.p;
    a.ticket = reinterpret_cast<unsigned *>((unsigned long long *)c->counts.p + 7);   // the 8th word of counts
}

static int gdbf_run(ldpc_ctx *c, const ldpc::GdbfArgs &a, bool f64)
{
    const ldpc::OptScope os(c->opts);
    const ldpc::GdbfChoice ch = ldpc::gdbf_choose(c->dg, f64, a.flags, c->g->maxdv, c->g->maxdc);
    int slots = 0;
    if (ch.slot_bytes) {
        slots = std::min(a.batch, 2 * c->num_cus);
        HIP_TRY(c->gscratch.ensure(ch.slot_bytes * (size_t)slots));
    }
    HIP_TRY(hipEventRecord(c->ev0, c->stream));
    HIP_TRY(ldpc::gdbf_launch(c->dg, a, f64, ch, c->gscratch.p, slots, c->num_cus, c->stream));
    HIP_TRY(hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    LDPC_CHECK_AFTER_LAUNCH(c->stream);
    return LDPC_OK;
}

static int counts_delta(ldpc_ctx *c, const ldpc_counts &before, ldpc_counts *acc)
{
    ldpc_counts after;
    int rc = read_counts(c, &after, 0);
    if (rc) return rc;
    if (acc) {
        ldpc_counts d;
        d.bit_err = after.bit_err - before.bit_err;
        d.frame_err = after.frame_err - before.frame_err;
        d.uncoded_bit_err = after.uncoded_bit_err - before.uncoded_bit_err;
        d.frames = after.frames - before.frames;
        d.iters = after.iters - before.iters;
        d.syndrome_fail = after.syndrome_fail - before.syndrome_fail;
        accumulate(acc, d);
    }
    return LDPC_OK;
}

int ldpc_gdbf_decode_batch(ldpc_ctx *c, const void *y, const void *pert, int batch, const ldpc_gdbf_cfg *cfg,
                           const int8_t *cw, int8_t *d_out, ldpc_frame_result *frames, ldpc_counts *counts)
{
    if (!c || !y) return set_err(LDPC_ERR_INVALID, "null argument");
    int rc = gdbf_check_cfg(cfg);
    if (rc) return rc;
    if (batch <= 0 || batch > c->max_batch)
        return set_err(LDPC_ERR_INVALID, "batch %d outside 1..max_batch=%d", batch, c->max_batch);
    if ((cfg->flags & (LDPC_GDBF_NOISE | LDPC_GDBF_QPROB)) && !pert)
        return set_err(LDPC_ERR_INVALID, "NOISE / QPROB need pert");
    if ((cfg->flags & LDPC_GDBF_QPROB) && !(cfg->qsigma > 0)) return set_err(LDPC_ERR_INVALID, "QPROB needs qsigma > 0");
    HIP_TRY(hipSetDevice(c->device));
    const bool f64 = cfg->precision == LDPC_F64;
    const int N = c->g->N;
    const size_t fsz = f64 ? 8 : 4, nb = (size_t)batch * N;
    ldpc::GdbfArgs a;
    gdbf_fill(a, c, cfg, batch);
    a.src = ldpc::SRC_GIVEN;
    if (is_device_ptr(y)) {
        a.y = y;
    } else {
        HIP_TRY(c->y_stage.ensure(nb * fsz));
        HIP_TRY(hipMemcpyAsync(c->y_stage.p, y, nb * fsz, hipMemcpyHostToDevice, c->stream));
        a.y = c->y_stage.p;
    }
    if (cfg->flags & (LDPC_GDBF_NOISE | LDPC_GDBF_QPROB)) {
        const size_t pb = nb * (size_t)cfg->T * fsz;
        if (is_device_ptr(pert)) {
            a.pert = pert;
        } else {
            HIP_TRY(c->p_stage.ensure(pb));
            HIP_TRY(hipMemcpyAsync(c->p_stage.p, pert, pb, hipMemcpyHostToDevice, c->stream));
            a.pert = c->p_stage.p;
        }
    }
    if (cw) {
        if (is_device_ptr(cw)) {
            a.c = cw;
        } else {
            HIP_TRY(c->c_stage.ensure(nb));
            HIP_TRY(hipMemcpyAsync(c->c_stage.p, cw, nb, hipMemcpyHostToDevice, c->stream));
            a.c = (const int8_t *)c->c_stage.p;
        }
    }
    const bool d_host = d_out && !is_device_ptr(d_out);
    const bool w_host = frames && !is_device_ptr(frames);
    if (d_host) {
        HIP_TRY(c->d_stage.ensure(nb));
        a.d_out = (int8_t *)c->d_stage.p;
    } else {
        a.d_out = d_out;
    }
    if (w_host) {
        HIP_TRY(c->fw_stage.ensure(sizeof(ldpc_frame_result) * (size_t)batch));
        a.frame_res = (int4 *)c->fw_stage.p;
    } else {
        a.frame_res = (int4 *)frames;
    }
    ldpc_counts before;
    rc = read_counts(c, &before, 0);
    if (rc) return rc;
    rc = gdbf_run(c, a, f64);
    if (rc) return rc;
    if (d_host) HIP_TRY(hipMemcpyAsync(d_out, c->d_stage.p, nb, hipMemcpyDeviceToHost, c->stream));
    if (w_host)
        HIP_TRY(hipMemcpyAsync(frames, c->fw_stage.p, sizeof(ldpc_frame_result) * (size_t)batch,
                               hipMemcpyDeviceToHost, c->stream));
    return counts_delta(c, before, counts);
}

static int gdbf_sim_impl(ldpc_ctx *c, double ebn0_db, double R, const ldpc_gdbf_cfg *cfg, uint64_t seed,
                         uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames_dev)
{
    if (!c) return set_err(LDPC_ERR_INVALID, "ctx is null");
    int rc = gdbf_check_cfg(cfg);
    if (rc) return rc;
    if (batch <= 0 || batch > c->max_batch)
        return set_err(LDPC_ERR_INVALID, "batch %d outside 1..max_batch=%d", batch, c->max_batch);
    if (!(R > 0)) return set_err(LDPC_ERR_INVALID, "rate must be > 0");
    if (stream_id >= (1u << 20)) return set_err(LDPC_ERR_INVALID, "stream_id must be < 2^20");
    HIP_TRY(hipSetDevice(c->device));
    ldpc::GdbfArgs a;
    gdbf_fill(a, c, cfg, batch);
    a.src = ldpc::SRC_PHILOX;
    const double N0 = std::pow(10.0, -ebn0_db / 10.0) / R;   // :175-176
    a.sigma = std::sqrt(N0 / 2.0);
    a.noise_sigma = a.sigma * cfg->noise_scale;               // :296
    a.qsigma = a.noise_sigma;                                  // symNodeUpdates' sigma (:353, :563)
    a.seed = seed;
    a.stream_id = stream_id;
    a.first_cw = first_cw;
    a.cw_table = c->cw_rows ? (const int8_t *)c->cw_table.p : nullptr;
    a.cw_rows = c->cw_rows;
    a.frame_res = (int4 *)frames_dev;
    return gdbf_run(c, a, cfg->precision == LDPC_F64);
}

int ldpc_gdbf_sim_launch(ldpc_ctx *c, double ebn0_db, double R, const ldpc_gdbf_cfg *cfg, uint64_t seed,
                         uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames_dev)
{
    if (frames_dev && !is_device_ptr(frames_dev))
        return set_err(LDPC_ERR_INVALID, "frames_dev must be a device pointer");
    return gdbf_sim_impl(c, ebn0_db, R, cfg, seed, stream_id, first_cw, batch, frames_dev);
}

int ldpc_gdbf_sim_batch(ldpc_ctx *c, double ebn0_db, double R, const ldpc_gdbf_cfg *cfg, uint64_t seed,
                        uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames,
                        ldpc_counts *accum)
{
    if (!c) return set_err(LDPC_ERR_INVALID, "ctx is null");
    HIP_TRY(hipSetDevice(c->device));
    ldpc_counts before;
    int rc = read_counts(c, &before, 0);
    if (rc) return rc;
    const bool w_host = frames && !is_device_ptr(frames);
    ldpc_frame_result *fw_dev = frames;
    if (w_host) {
        HIP_TRY(c->fw_stage.ensure(sizeof(ldpc_frame_result) * (size_t)std::max(batch, 1)));
        fw_dev = (ldpc_frame_result *)c->fw_stage.p;
    }
    rc = gdbf_sim_impl(c, ebn0_db, R, cfg, seed, stream_id, first_cw, batch, fw_dev);
    if (rc) return rc;
    if (w_host)
        HIP_TRY(hipMemcpyAsync(frames, fw_dev, sizeof(ldpc_frame_result) * (size_t)batch, hipMemcpyDeviceToHost,
                               c->stream));
    return counts_delta(c, before, accum);
}

int ldpc_gdbf_kernel_info(ldpc_ctx *c, const ldpc_gdbf_cfg *cfg, char *name, int name_len, int *lds_bytes)
{
    int rc = gdbf_check_cfg(cfg);
    if (rc) return rc;
    if (!c) return set_err(LDPC_ERR_INVALID, "ctx is null");
    const ldpc::OptScope os(c->opts);
    const ldpc::GdbfChoice ch = ldpc::gdbf_choose(c->dg, cfg->precision == LDPC_F64, cfg->flags, c->g->maxdv, c->g->maxdc);
    if (name && name_len > 0) std::snprintf(name, (size_t)name_len, "%s", ch.name);
    if (lds_bytes) *lds_bytes = ch.lds_bytes;
    return LDPC_OK;
}

}  // extern "C"
