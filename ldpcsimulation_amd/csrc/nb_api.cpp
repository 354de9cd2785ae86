// nb_api.cpp -- C ABI of the non-binary GF(q) EMS decoder (include/ldpc_hip.h,
// "non-binary" section): NB alist loading with the semantics of the
// reference's SystemC/NB-LDPC/src/alist.cpp:23-56 (plus validation), device
// contexts, decode of given channel samples and the fused Monte-Carlo.
#include "ldpc_hip.h"
#include "nb.h"
#include "nb_graph.h"
#include "check.h"
#include "kernels.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

namespace {

int err(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int err(int code, const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return ldpc::set_last_error(code, buf);
}

#define NB_HIP_TRY(expr)                                                                                   \
    do {                                                                                                   \
        hipError_t e_ = (expr);                                                                            \
        if (e_ != hipSuccess) {                                                                            \
            (void)hipGetLastError();                                                                       \
            return err(LDPC_ERR_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                       __LINE__);                                                                          \
        }                                                                                                  \
    } while (0)

struct Buf {
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

bool is_device_ptr(const void *p)
{
    if (!p) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
}

}  // namespace

struct ldpc_nb_ctx {
    int device = 0, max_batch = 0, num_cus = 0;
    const ldpc_nb_graph *g = nullptr;
    hipStream_t own = nullptr, stream = nullptr;
    ldpc::NbDevGraph dg{};
    Buf graph, counts, y_stage, c_stage, d_stage, fr_stage, scratch;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t handoff = nullptr;         // orders the launches of a context across ldpc_nb_ctx_set_stream
    bool timed = false;
    const uint8_t *col_h_swz = nullptr;   // device: col_h with the slot swizzles (nb_swizzled_coefficients)
    ldpc::Options opts;                   // kernel-selection options (ldpc_nb_ctx_set_option)
};

// LDPC_OPT_EMS_SWIZZLE = 1 keeps the plain message layout (A/B).
static bool nb_swizzle_enabled() { return ldpc::opt(LDPC_OPT_EMS_SWIZZLE) != 1; }

extern "C" {

int ldpc_nb_graph_create(int N, int M, int q, const int *num_nlist, const int *const *nlist, const int *const *nvals,
                         const int *num_mlist, const int *const *mlist, const int *const *mvals, ldpc_nb_graph **out)
{
    if (!out || !num_nlist || !nlist || !nvals || !num_mlist || !mlist || !mvals)
        return err(LDPC_ERR_INVALID, "null argument");
    *out = nullptr;
    if (N <= 0 || M <= 0) return err(LDPC_ERR_GRAPH, "bad dimensions N=%d M=%d", N, M);
    try {
        ldpc::NbLists cols(N), rows(M);
        for (int i = 0; i < N; ++i)
            for (int k = 0; k < num_nlist[i]; ++k) cols[i].push_back({nlist[i][k] - 1, nvals[i][k]});
        for (int j = 0; j < M; ++j)
            for (int k = 0; k < num_mlist[j]; ++k) rows[j].push_back({mlist[j][k] - 1, mvals[j][k]});
        std::unique_ptr<ldpc_nb_graph> g(new ldpc_nb_graph());
        std::string msg;
        const int rc = ldpc::nb_build_graph(N, M, q, cols, rows, *g, msg);
        if (rc) return err(rc, "%s", msg.c_str());
        *out = g.release();
    } catch (const std::bad_alloc &) {
        return err(LDPC_ERR_NOMEM, "graph build out of memory");
    }
    return LDPC_OK;
}

int ldpc_nb_graph_load_alist(const char *path, ldpc_nb_graph **out)
{
    if (!path || !out) return err(LDPC_ERR_INVALID, "null argument");
    *out = nullptr;
    try {
        std::unique_ptr<ldpc_nb_graph> g(new ldpc_nb_graph());
        std::string msg;
        const int rc = ldpc::nb_read_alist(path, *g, msg);
        if (rc) return err(rc, "%s", msg.c_str());
        *out = g.release();
    } catch (const std::bad_alloc &) {
        return err(LDPC_ERR_NOMEM, "alist load out of memory");
    }
    return LDPC_OK;
}

int ldpc_nb_graph_info(const ldpc_nb_graph *g, int *N, int *M, int *q, int *E, int *maxdv, int *maxdc)
{
    if (!g) return err(LDPC_ERR_INVALID, "graph is null");
    if (N) *N = g->N;
    if (M) *M = g->M;
    if (q) *q = g->q;
    if (E) *E = g->E;
    if (maxdv) *maxdv = g->maxdv;
    if (maxdc) *maxdc = g->maxdc;
    return LDPC_OK;
}

void ldpc_nb_graph_destroy(ldpc_nb_graph *g) { delete g; }

int ldpc_nb_ctx_create(int device, const ldpc_nb_graph *g, int max_batch, ldpc_nb_ctx **out)
{
    if (!g || !out) return err(LDPC_ERR_INVALID, "null argument");
    *out = nullptr;
    if (max_batch <= 0) return err(LDPC_ERR_INVALID, "max_batch must be > 0");
    if (g->q != ldpc::kNbQ) return err(LDPC_ERR_UNSUPPORTED, "the EMS kernels are built for GF(16), got q=%d", g->q);
    if (g->maxdc > ldpc::kNbMaxDc) return err(LDPC_ERR_UNSUPPORTED, "row degree %d > %d", g->maxdc, ldpc::kNbMaxDc);
    if (g->maxdv > 255) return err(LDPC_ERR_UNSUPPORTED, "column degree %d > 255", g->maxdv);
    int ndev = 0;
    NB_HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return err(LDPC_ERR_INVALID, "device %d outside 0..%d", device, ndev - 1);
    NB_HIP_TRY(hipSetDevice(device));
    auto *c = new (std::nothrow) ldpc_nb_ctx();
    if (!c) return err(LDPC_ERR_NOMEM, "context allocation failed");
    c->device = device;
    c->max_batch = max_batch;
    c->g = g;
    hipDeviceProp_t prop;
    NB_HIP_TRY(hipGetDeviceProperties(&prop, device));
    c->num_cus = prop.multiProcessorCount;
    NB_HIP_TRY(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
    c->stream = c->own;
    NB_HIP_TRY(hipEventCreate(&c->ev0));
    NB_HIP_TRY(hipEventCreate(&c->ev1));
    // graph upload: row_ptr | row_col | col_ptr | col_slot | row_h | gf_mul | gf_inv | pslot | colh | colh_swz
    const int q = g->q;
    ldpc::NbTables tb;
    ldpc::nb_tables(*g, tb);
    const std::vector<uint8_t> &mul = tb.mul, &inv = tb.inv, &colh = tb.colh, &colhs = tb.colh_swz;
    const std::vector<int32_t> &pslot = tb.pslot;
    const size_t n_rp = (g->M + 1) * 4, n_rc = (size_t)g->E * 4, n_cp = (g->N + 1) * 4, n_cs = (size_t)g->E * 4;
    const size_t total = n_rp + n_rc + n_cp + 2 * n_cs + 3 * (size_t)g->E + mul.size() + inv.size() + 256;
    std::vector<uint8_t> blob(total, 0);
    size_t off = 0;
    auto put = [&](const void *src, size_t n) {
        const size_t o = off;
        std::memcpy(blob.data() + off, src, n);
        off = (off + n + 15) & ~(size_t)15;
        return o;
    };
    blob.resize(total + 256);
    const size_t o_rp = put(g->row_ptr.data(), n_rp), o_rc = put(g->row_col.data(), n_rc),
                 o_cp = put(g->col_ptr.data(), n_cp), o_cs = put(g->col_slot.data(), n_cs),
                 o_h = put(g->row_h.data(), g->E), o_mul = put(mul.data(), mul.size()),
                 o_inv = put(inv.data(), inv.size()), o_ps = put(pslot.data(), n_cs),
                 o_ch = put(colh.data(), g->E), o_chs = put(colhs.data(), g->E);
    NB_HIP_TRY(c->graph.ensure(off));
    NB_HIP_TRY(hipMemcpy(c->graph.p, blob.data(), off, hipMemcpyHostToDevice));
    auto *base = (uint8_t *)c->graph.p;
    c->dg.N = g->N;
    c->dg.M = g->M;
    c->dg.q = q;
    c->dg.m = g->m;
    c->dg.E = g->E;
    c->dg.row_ptr = (const int32_t *)(base + o_rp);
    c->dg.row_col = (const int32_t *)(base + o_rc);
    c->dg.col_ptr = (const int32_t *)(base + o_cp);
    c->dg.col_slot = (const int32_t *)(base + o_cs);
    c->dg.row_h = base + o_h;
    c->dg.gf_mul = base + o_mul;
    c->dg.gf_inv = base + o_inv;
    c->dg.col_pslot = (const int32_t *)(base + o_ps);
    c->dg.col_h = base + o_ch;
    c->col_h_swz = base + o_chs;
    c->dg.maxdc = g->maxdc;
    if (!ldpc::nb_choose(c->dg, g->maxdc).name[0]) {
        ldpc_nb_ctx_destroy(c);
        return err(LDPC_ERR_UNSUPPORTED, "code too large for the EMS kernels (N=%d, E=%d)", g->N, g->E);
    }
    NB_HIP_TRY(c->counts.ensure(8 * sizeof(unsigned long long)));
    NB_HIP_TRY(hipMemset(c->counts.p, 0, 8 * sizeof(unsigned long long)));
    *out = c;
    return LDPC_OK;
}

int ldpc_nb_ctx_set_stream(ldpc_nb_ctx *c, void *hip_stream)
{
    if (!c) return err(LDPC_ERR_INVALID, "ctx is null");
    const hipStream_t ns = hip_stream ? (hipStream_t)hip_stream : c->own;
    if (ns != c->stream) {
        // one context's launches share its counters and codeword ticket: the new stream
        // starts after everything already queued on the old one (no overlap across streams)
        NB_HIP_TRY(hipSetDevice(c->device));
        if (!c->handoff) NB_HIP_TRY(hipEventCreateWithFlags(&c->handoff, hipEventDisableTiming));
        NB_HIP_TRY(hipEventRecord(c->handoff, c->stream));
        NB_HIP_TRY(hipStreamWaitEvent(ns, c->handoff, 0));
    }
    c->stream = ns;
    return LDPC_OK;
}

void ldpc_nb_ctx_destroy(ldpc_nb_ctx *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->own);
    for (Buf *b : {&c->graph, &c->counts, &c->y_stage, &c->c_stage, &c->d_stage, &c->fr_stage, &c->scratch})
        b->release();
    if (c->handoff) (void)hipEventDestroy(c->handoff);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

static int check_ems(const ldpc_nb_ctx *c, const ldpc_ems_cfg *cfg, int batch)
{
    if (!c || !cfg) return err(LDPC_ERR_INVALID, "null argument");
    if (batch <= 0 || batch > c->max_batch)
        return err(LDPC_ERR_INVALID, "batch %d outside 1..max_batch=%d", batch, c->max_batch);
    if (cfg->T < 0) return err(LDPC_ERR_INVALID, "T must be >= 0");
    if (cfg->nm < 1) return err(LDPC_ERR_INVALID, "nm must be >= 1");
    if (!(cfg->offset >= 0)) return err(LDPC_ERR_INVALID, "offset must be >= 0");
    return LDPC_OK;
}

static int read_counts_raw(ldpc_nb_ctx *c, unsigned long long *v)
{
    NB_HIP_TRY(hipMemcpyAsync(v, c->counts.p, 7 * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    NB_HIP_TRY(hipStreamSynchronize(c->stream));
    return LDPC_OK;
}

static void add_counts(ldpc_nb_counts *acc, const unsigned long long *after, const unsigned long long *before)
{
    acc->bit_err += (int64_t)(after[0] - before[0]);
    acc->frame_err += (int64_t)(after[1] - before[1]);
    acc->uncoded_bit_err += (int64_t)(after[2] - before[2]);
    acc->frames += (int64_t)(after[3] - before[3]);
    acc->iters += (int64_t)(after[4] - before[4]);
    acc->syndrome_fail += (int64_t)(after[5] - before[5]);
    acc->symbol_err += (int64_t)(after[6] - before[6]);
}

static int run(ldpc_nb_ctx *c, const ldpc::NbArgs &a)
{
    const ldpc::OptScope os(c->opts);
    const ldpc::NbChoice ch = ldpc::nb_choose(c->dg, c->g->maxdc);
    int slots = 0;
    if (ch.slot_bytes) {
        slots = std::min(a.batch, c->num_cus);
        NB_HIP_TRY(c->scratch.ensure(ch.slot_bytes * (size_t)slots));
    }
    NB_HIP_TRY(hipEventRecord(c->ev0, c->stream));
    ldpc::NbDevGraph dg = c->dg;
    // untruncated messages (nm >= q): the XOR-swizzled layout; truncation ranks
    // entries by symbol on ties, so it keeps the plain one (nb.hip vn_lane)
    if (a.nm >= dg.q && nb_swizzle_enabled()) dg.col_h = c->col_h_swz;
    NB_HIP_TRY(ldpc::nb_launch(dg, a, ch, c->scratch.p, slots, c->num_cus, c->stream));
    NB_HIP_TRY(hipEventRecord(c->ev1, c->stream));
    c->timed = true;
#ifdef LDPC_CHECK
    {   // checked builds: the launch's index record (check.h)
        char m[192];
        const long n = ldpc::check_collect(c->stream, m, sizeof m);
        if (n < 0) return err(LDPC_ERR_DEVICE, "check_collect: %s", hipGetErrorString((hipError_t)-n));
        if (n > 0) return err(LDPC_ERR_DEVICE, "%s; %ld violations", m, n);
    }
#endif
    return LDPC_OK;
}

static void fill_cfg(ldpc::NbArgs &a, ldpc_nb_ctx *c, const ldpc_ems_cfg *cfg, int batch)
{
    std::memset(&a, 0, sizeof a);
    a.batch = batch;
    a.T = cfg->T;
    a.nm = cfg->nm;
    a.early_stop = cfg->early_stop ? 1 : 0;
    a.offset = (float)cfg->offset;
    a.counts = (unsigned long long *)c->counts.p;
    a.ticket = reinterpret_cast<unsigned *>((unsigned long long *)c->counts.p + 7);   // the 8th word of counts
}

int ldpc_ems_decode_batch(ldpc_nb_ctx *c, const float *y, int batch, double n0, const ldpc_ems_cfg *cfg,
                          const uint8_t *cw, uint8_t *d_out, ldpc_frame_result *frames, ldpc_nb_counts *counts)
{
    int rc = check_ems(c, cfg, batch);
    if (rc) return rc;
    if (!y) return err(LDPC_ERR_INVALID, "y is null");
    if (!(n0 > 0)) return err(LDPC_ERR_INVALID, "n0 must be > 0");
    NB_HIP_TRY(hipSetDevice(c->device));
    const int N = c->g->N, m = c->g->m;
    ldpc::NbArgs a;
    fill_cfg(a, c, cfg, batch);
    a.src = ldpc::SRC_GIVEN;
    a.n0 = (float)n0;
    const size_t yb = (size_t)batch * N * m * sizeof(float), nb = (size_t)batch * N;
    if (is_device_ptr(y)) {
        a.y = y;
    } else {
        NB_HIP_TRY(c->y_stage.ensure(yb));
        NB_HIP_TRY(hipMemcpyAsync(c->y_stage.p, y, yb, hipMemcpyHostToDevice, c->stream));
        a.y = (const float *)c->y_stage.p;
    }
    if (cw) {
        for (size_t i = 0; !is_device_ptr(cw) && i < nb; ++i)
            if (cw[i] >= (unsigned)c->g->q) return err(LDPC_ERR_INVALID, "codeword symbol %zu is %d (q=%d)", i, cw[i], c->g->q);
        if (is_device_ptr(cw)) {
            a.c = cw;
        } else {
            NB_HIP_TRY(c->c_stage.ensure(nb));
            NB_HIP_TRY(hipMemcpyAsync(c->c_stage.p, cw, nb, hipMemcpyHostToDevice, c->stream));
            a.c = (const uint8_t *)c->c_stage.p;
        }
    }
    const bool d_host = d_out && !is_device_ptr(d_out), f_host = frames && !is_device_ptr(frames);
    if (d_host) {
        NB_HIP_TRY(c->d_stage.ensure(nb));
        a.d_out = (uint8_t *)c->d_stage.p;
    } else {
        a.d_out = d_out;
    }
    if (f_host) {
        NB_HIP_TRY(c->fr_stage.ensure(sizeof(ldpc_frame_result) * (size_t)batch));
        a.frame_res = (int4 *)c->fr_stage.p;
    } else {
        a.frame_res = (int4 *)frames;
    }
    unsigned long long before[7], after[7];
    rc = read_counts_raw(c, before);
    if (rc) return rc;
    rc = run(c, a);
    if (rc) return rc;
    if (d_host) NB_HIP_TRY(hipMemcpyAsync(d_out, c->d_stage.p, nb, hipMemcpyDeviceToHost, c->stream));
    if (f_host)
        NB_HIP_TRY(hipMemcpyAsync(frames, c->fr_stage.p, sizeof(ldpc_frame_result) * (size_t)batch,
                                  hipMemcpyDeviceToHost, c->stream));
    rc = read_counts_raw(c, after);
    if (rc) return rc;
    if (counts) add_counts(counts, after, before);
    return LDPC_OK;
}

static int sim_impl(ldpc_nb_ctx *c, double ebn0_db, double R, const ldpc_ems_cfg *cfg, uint64_t seed,
                    uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames_dev, float *y_dev,
                    uint8_t *d_dev)
{
    int rc = check_ems(c, cfg, batch);
    if (rc) return rc;
    if (!(R > 0)) return err(LDPC_ERR_INVALID, "rate must be > 0");
    NB_HIP_TRY(hipSetDevice(c->device));
    ldpc::NbArgs a;
    fill_cfg(a, c, cfg, batch);
    a.src = ldpc::SRC_PHILOX;
    const double N0 = std::pow(10.0, -ebn0_db / 10.0) / R;   // decodeMinSum.cpp:146-147
    a.n0 = (float)N0;
    a.sigma = (float)std::sqrt(N0 / 2.0);
    a.seed = seed;
    a.stream_id = stream_id;
    a.first_cw = first_cw;
    a.frame_res = (int4 *)frames_dev;
    a.y_out = y_dev;
    a.d_out = d_dev;
    return run(c, a);
}

int ldpc_ems_sim_launch(ldpc_nb_ctx *c, double ebn0_db, double R, const ldpc_ems_cfg *cfg, uint64_t seed,
                        uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames_dev)
{
    if (frames_dev && !is_device_ptr(frames_dev)) return err(LDPC_ERR_INVALID, "frames_dev must be device memory");
    return sim_impl(c, ebn0_db, R, cfg, seed, stream_id, first_cw, batch, frames_dev, nullptr, nullptr);
}

int ldpc_ems_sim_trace(ldpc_nb_ctx *c, double ebn0_db, double R, const ldpc_ems_cfg *cfg, uint64_t seed,
                       uint32_t stream_id, uint64_t first_cw, int batch, float *y_out, uint8_t *d_out,
                       ldpc_frame_result *frames, ldpc_nb_counts *accum)
{
    int rc = check_ems(c, cfg, batch);
    if (rc) return rc;
    const int N = c->g->N, m = c->g->m;
    const size_t yb = (size_t)batch * N * m * sizeof(float), nb = (size_t)batch * N;
    const bool y_host = y_out && !is_device_ptr(y_out), d_host = d_out && !is_device_ptr(d_out),
               f_host = frames && !is_device_ptr(frames);
    float *yd = y_out;
    uint8_t *dd = d_out;
    ldpc_frame_result *fd = frames;
    if (y_host) {
        NB_HIP_TRY(c->y_stage.ensure(yb));
        yd = (float *)c->y_stage.p;
    }
    if (d_host) {
        NB_HIP_TRY(c->d_stage.ensure(nb));
        dd = (uint8_t *)c->d_stage.p;
    }
    if (f_host) {
        NB_HIP_TRY(c->fr_stage.ensure(sizeof(ldpc_frame_result) * (size_t)batch));
        fd = (ldpc_frame_result *)c->fr_stage.p;
    }
    unsigned long long before[7], after[7];
    rc = read_counts_raw(c, before);
    if (rc) return rc;
    rc = sim_impl(c, ebn0_db, R, cfg, seed, stream_id, first_cw, batch, fd, yd, dd);
    if (rc) return rc;
    if (y_host) NB_HIP_TRY(hipMemcpyAsync(y_out, yd, yb, hipMemcpyDeviceToHost, c->stream));
    if (d_host) NB_HIP_TRY(hipMemcpyAsync(d_out, dd, nb, hipMemcpyDeviceToHost, c->stream));
    if (f_host)
        NB_HIP_TRY(hipMemcpyAsync(frames, fd, sizeof(ldpc_frame_result) * (size_t)batch, hipMemcpyDeviceToHost,
                                  c->stream));
    rc = read_counts_raw(c, after);
    if (rc) return rc;
    if (accum) add_counts(accum, after, before);
    return LDPC_OK;
}

int ldpc_ems_sim_batch(ldpc_nb_ctx *c, double ebn0_db, double R, const ldpc_ems_cfg *cfg, uint64_t seed,
                       uint32_t stream_id, uint64_t first_cw, int batch, ldpc_frame_result *frames,
                       ldpc_nb_counts *accum)
{
    return ldpc_ems_sim_trace(c, ebn0_db, R, cfg, seed, stream_id, first_cw, batch, nullptr, nullptr, frames, accum);
}

int ldpc_nb_ctx_read_counts(ldpc_nb_ctx *c, ldpc_nb_counts *out, int reset)
{
    if (!c || !out) return err(LDPC_ERR_INVALID, "null argument");
    NB_HIP_TRY(hipSetDevice(c->device));
    unsigned long long v[7], z[7] = {0, 0, 0, 0, 0, 0, 0};
    int rc = read_counts_raw(c, v);
    if (rc) return rc;
    std::memset(out, 0, sizeof *out);
    add_counts(out, v, z);
    if (reset) {
        NB_HIP_TRY(hipMemsetAsync(c->counts.p, 0, 7 * sizeof(unsigned long long), c->stream));
        NB_HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return LDPC_OK;
}

int ldpc_nb_ctx_last_kernel_ms(ldpc_nb_ctx *c, float *ms)
{
    if (!c || !ms) return err(LDPC_ERR_INVALID, "null argument");
    if (!c->timed) return err(LDPC_ERR_INVALID, "no kernel launched yet");
    NB_HIP_TRY(hipEventSynchronize(c->ev1));
    NB_HIP_TRY(hipEventElapsedTime(ms, c->ev0, c->ev1));
    return LDPC_OK;
}

int ldpc_ems_kernel_info(ldpc_nb_ctx *c, char *name, int name_len, int *lds_bytes)
{
    if (!c) return err(LDPC_ERR_INVALID, "ctx is null");
    const ldpc::OptScope os(c->opts);
    const ldpc::NbChoice ch = ldpc::nb_choose(c->dg, c->g->maxdc);
    if (name && name_len > 0) std::snprintf(name, (size_t)name_len, "%s", ch.name);
    if (lds_bytes) *lds_bytes = ch.lds_bytes;
    return LDPC_OK;
}

int ldpc_nb_ctx_set_option(ldpc_nb_ctx *c, int option, int value)
{
    if (!c) return err(LDPC_ERR_INVALID, "ctx is null");
    if (!ldpc::option_is_ems(option))
        return err(LDPC_ERR_INVALID, "option %d is not an EMS option", option);
    if (!ldpc::option_value_ok(option, value)) return err(LDPC_ERR_INVALID, "option %d: value %d out of range", option, value);
    c->opts.v[option] = value;
    return LDPC_OK;
}

}  // extern "C"
