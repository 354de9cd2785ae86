"""Belief propagation, tanh rule (reference src/decodeBP.cpp).

Oracle tier (CPU): oracle/bp_oracle.c restates decodeBP.cpp and reproduces the
reference's own runs frame by frame (tests/test_oracle.py, golden runs of
oracle/_ref/decodeBP compiled from the unmodified sources).
GPU tier: tanh and log are the device's (OCML) functions, which agree with
glibc's to about one ulp but not bit for bit, so the GPU is held to
  - fp64: the oracle's decisions and the reference's whole golden runs (totals
    and the sequence of per-frame error weights) -- a one-ulp difference in a
    message does not move a decision at these sizes;
  - fp32: at most 0.1% of decisions differing from the fp32 oracle on the same
    y (tolerance written in the test), identical results on frames the oracle
    decodes, and a frame-error rate consistent with the reference's
    (two-proportion z-test, |z| < 3).
"""
import math

import numpy as np
import pytest

from conftest import code_path, golden_runs
from helpers import cw_lines, final_numbers
from oracle import oracle as O

CODES = ["PEGReg504x1008.alist", "80211n_1944_r12.alist", "4000.2000.4.244.alist"]
F32_BIT_TOL = 1e-3      # fraction of fp32 decisions allowed to differ from the fp32 oracle


def _n0(ebn0, R=0.5):
    return 10 ** (-ebn0 / 10) / R


def _glibc_frames(N, nframes, ebn0, R, seed):
    g = O.GlibcRandom(seed)
    sigma = math.sqrt(_n0(ebn0, R) / 2)
    return np.stack([g.channel(np.ones(N, dtype=np.int32), sigma) for _ in range(nframes)])


def test_oracle_bp_front_end_clips_at_maxllr():
    A = O.Alist(code_path("PEGReg504x1008.alist"))
    yq = A.bp_front(np.array([0.1, -3.0, 7.0, -0.0]), N0=0.5)
    assert yq[0] == 4 * 0.1 / 0.5 and yq[1] == -20.0 and yq[2] == 20.0 and yq[3] == 0.0


def test_oracle_bp_f32_clip_keeps_messages_finite():
    """fp32: tanhf(10) == 1 would make c2v infinite and v2c NaN; the c2v clip
    keeps a clean high-SNR frame decoding to the all-zero codeword."""
    A = O.Alist(code_path("80211n_1944_r12.alist"))
    y = _glibc_frames(A.N, 2, 6.0, 0.5, seed=5)
    yq = np.clip(4 * y / _n0(6.0), -20, 20).astype(np.float32)
    d, c2v = A.bp_decode(yq, 30, want_c2v=True)
    assert (d == 1).all()
    assert np.isfinite(c2v).all() and np.abs(c2v).max() <= 20.0


def _native():
    from ldpcsimulation_amd import native
    return native


@pytest.mark.gpu
@pytest.mark.parametrize("code", CODES)
def test_bp_f64_decisions_match_oracle(gpu_ctx_factory, code):
    native = _native()
    ctx = gpu_ctx_factory(code)
    A = O.Alist(code_path(code))
    ebn0 = 2.0
    y = _glibc_frames(A.N, 12, ebn0, 0.5, seed=321)
    yq = np.array([A.bp_front(row, _n0(ebn0)) for row in y])
    for T in (0, 1, 4, 20):
        cfg = native.DecoderConfig(variant=native.BP, T=T, precision=native.F64, n0=_n0(ebn0))
        d, fr, cnt = ctx.decode(y, cfg)
        want = A.bp_decode(yq, T)
        assert int((d != want).sum()) == 0, f"T={T}"
        w = (want != 1).sum(axis=1)
        assert np.array_equal(fr["bit_err"], w) and cnt.bit_err == int(w.sum()) and cnt.iters == T * len(y)
        assert np.array_equal(fr["uncoded_bit_err"], (yq < 0).sum(axis=1))


@pytest.mark.gpu
@pytest.mark.parametrize("code", CODES)
def test_bp_f32_decisions_within_tolerance(gpu_ctx_factory, code):
    native = _native()
    ctx = gpu_ctx_factory(code)
    A = O.Alist(code_path(code))
    ebn0 = 2.0
    y = _glibc_frames(A.N, 12, ebn0, 0.5, seed=99).astype(np.float32)
    n0 = _n0(ebn0)
    yq = np.clip((np.float32(4) * y) / np.float32(n0), -20, 20).astype(np.float32)
    for T in (0, 1, 4, 20):
        cfg = native.DecoderConfig(variant=native.BP, T=T, precision=native.F32, n0=n0)
        d, fr, _ = ctx.decode(y, cfg)
        want = A.bp_decode(yq, T)
        assert (d != want).mean() <= F32_BIT_TOL, f"T={T}: {(d != want).sum()} decisions differ"
        ok = (want == 1).all(axis=1)
        assert (fr["bit_err"][ok] == 0).all(), f"T={T}: a frame the oracle decodes failed on the GPU"


@pytest.mark.gpu
@pytest.mark.parametrize("run", golden_runs("bp"), ids=lambda r: r["name"])
def test_gpu_reproduces_reference_bp_run(gpu_ctx_factory, run):
    """decodeBP's own Monte-Carlo run (reference noise drawn on the host), decoded in fp64 on the GPU:
    same totals and the same per-frame error weights as the reference binary printed."""
    native = _native()
    R, snr, T = float(run["args"][0]), float(run["args"][1]), int(run["args"][2])
    ctx = gpu_ctx_factory(run["code"], 1024)
    N = ctx.graph.N
    lines = cw_lines(run)
    g = O.GlibcRandom(run["seed"])
    sigma = math.sqrt(_n0(snr, R) / 2)
    cfg = native.DecoderConfig(variant=native.BP, T=T, precision=native.F64, n0=_n0(snr, R))
    min_we = 20 if N <= 10000 else (10 if N <= 50000 else 5)   # decodeBP.cpp:145-147
    errors = words = word_errors = unc = f = 0
    ferr = []
    done = False
    while not done:
        B = 128
        cw = np.ones((B, N), dtype=np.int8)
        ys = np.empty((B, N))
        for k in range(B):
            if lines:
                cw[k] = [-1 if ch == "1" else 1 for ch in lines[(f + k) % len(lines)][:N]]
            ys[k] = g.channel(cw[k].astype(np.int32), sigma)
        _, fr, _ = ctx.decode(ys, cfg, c=cw if lines else None, want_decisions=False)
        f += B
        for r in fr:
            if not (errors < 200 or word_errors < min_we):
                done = True
                break
            unc += int(r["uncoded_bit_err"])
            if r["bit_err"] > 0:
                errors += int(r["bit_err"])
                word_errors += 1
                ferr.append(int(r["bit_err"]))
            words += 1
    assert (errors, words, unc) == final_numbers(run["final"])
    assert ferr == run["ferr_weights"]


@pytest.mark.gpu
def test_bp_sim_on_device_noise_matches_oracle(gpu_ctx_factory):
    native = _native()
    ctx = gpu_ctx_factory("80211n_1944_r12.alist")
    A = O.Alist(code_path("80211n_1944_r12.alist"))
    cfg = native.DecoderConfig(variant=native.BP, T=20, precision=native.F64)
    y, d, fr, cnt = ctx.sim_trace(1.5, 0.5, cfg, seed=41, stream_id=2, first_cw=500, batch=16)
    yq = np.array([A.bp_front(row, _n0(1.5)) for row in y])
    want = A.bp_decode(yq, 20)
    assert int((d != want).sum()) == 0
    assert cnt.frames == 16 and cnt.bit_err == int((want != 1).sum())


@pytest.mark.gpu
def test_bp_fer_matches_reference_statistically(gpu_ctx_factory):
    """fp32 BP with on-device Philox noise against the reference's decodeBP run on
    802.11n N=1944 at 1.5 dB, T=30 (golden bp_1944_1.5_T30_s4): |z| < 3."""
    native = _native()
    from ldpcsimulation_amd.sim import two_proportion_z
    run = [r for r in golden_runs("bp") if r["name"] == "bp_1944_1.5_T30_s4"][0]
    ctx = gpu_ctx_factory(run["code"], 8192)
    cfg = native.DecoderConfig(variant=native.BP, T=30, precision=native.F32)
    fr, cnt = ctx.sim_batch(1.5, 0.5, cfg, seed=2029, stream_id=7, first_cw=0, batch=8192)
    _, words, _ = final_numbers(run["final"])
    z = two_proportion_z(cnt.frame_err, cnt.frames, len(run["ferr_weights"]), words)
    assert abs(z) < 3, (cnt.frame_err, cnt.frames, z)
    assert cnt.frames == 8192 and cnt.iters == 30 * 8192


@pytest.mark.gpu
def test_bp_sim_independent_of_batch_split(gpu_ctx_factory):
    native = _native()
    ctx = gpu_ctx_factory("PEGReg504x1008.alist")
    cfg = native.DecoderConfig(variant=native.BP, T=10)
    full, _ = ctx.sim_batch(2.0, 0.5, cfg, seed=3, stream_id=0, first_cw=0, batch=300)
    a, _ = ctx.sim_batch(2.0, 0.5, cfg, seed=3, stream_id=0, first_cw=0, batch=120)
    b, _ = ctx.sim_batch(2.0, 0.5, cfg, seed=3, stream_id=0, first_cw=120, batch=180)
    assert np.array_equal(full, np.concatenate([a, b]))


@pytest.mark.gpu
@pytest.mark.parametrize("code", CODES)
@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_bp_rows_kernel_equals_generic_kernel(gpu_ctx_factory, monkeypatch, code, prec):
    """The register-schedule BP kernel (bp_rows) and the one-workgroup-per-codeword
    kernel give identical channel samples, decisions and per-frame results on the
    on-device Philox path (same arithmetic in the same order)."""
    native = _native()
    ctx = gpu_ctx_factory(code, 1024)
    cfg = native.DecoderConfig(variant=native.BP, T=12, precision=native.F32 if prec == "f32" else native.F64)
    if code.startswith("4000") and prec == "f64":   # app + messages: 160 KB, beyond one workgroup's LDS
        assert ctx.kernel_info(cfg)["kernel"] != "bp_rows"
        return
    assert ctx.kernel_info(cfg)["kernel"] == "bp_rows"
    got = [ctx.sim_trace(e, 0.5, cfg, seed=17, stream_id=3, first_cw=64, batch=1024) for e in (1.0, 2.0)]
    ctx.set_option("bp_kernel", "generic")
    assert ctx.kernel_info(cfg)["kernel"] != "bp_rows"
    for e, (y, d, fr, cnt) in zip((1.0, 2.0), got):
        y2, d2, fr2, cnt2 = ctx.sim_trace(e, 0.5, cfg, seed=17, stream_id=3, first_cw=64, batch=1024)
        assert np.array_equal(y, y2) and np.array_equal(fr, fr2), e
        assert int((d != d2).sum()) == 0, e
        assert cnt.as_dict() == cnt2.as_dict()
    assert got[0][3].frame_err > 0   # failing frames are compared too


BP_TANH_ULP_TOL = 3     # device tanh (bp_math.h) vs glibc, max ulps over the check node's domain
BP_LOG_ULP_TOL = 1      # device log vs glibc


def _ulps(got, want):
    got, want = np.asarray(got), np.asarray(want)
    both_inf = np.isinf(got) & np.isinf(want) & (np.sign(got) == np.sign(want))
    same = (got == want) | both_inf | (np.isnan(got) & np.isnan(want))
    sp = np.spacing(np.abs(np.where(np.isfinite(want), want, 0.0)))
    u = np.where(same, 0.0, np.abs(got - want) / np.where(sp > 0, sp, np.inf))
    return np.where(np.isfinite(u) | same, u, np.inf)


@pytest.mark.gpu
def test_bp_f64_math_within_ulps_of_glibc():
    """The fp64 BP check node's tanh and log (bp_math.h, branch-free, on the device through
    ldpc_bp_math_probe) against glibc's (math.tanh / math.log: decodeBP.cpp:353-377 calls
    them), over the arguments the check node forms -- v2c/2 in [-10, 10] (|v2c| <= MAXLLR
    = 20), tiny and huge magnitudes, (1+p)/(1-p) for p in (-1, 1) -- and the specials.
    Tolerances: BP_TANH_ULP_TOL and BP_LOG_ULP_TOL ulps."""
    import ctypes as C
    native = _native()
    L = native.lib()
    rng = np.random.default_rng(2026)
    xt = np.concatenate([rng.uniform(-10, 10, 300000), rng.uniform(-1e-3, 1e-3, 30000),
                         np.sign(rng.uniform(-1, 1, 30000)) * 10.0 ** rng.uniform(-310, 2.5, 30000),
                         [0.0, -0.0, 5e-324, -5e-324, 19.0, 20.0, 25.0, -25.0, 1e300, np.inf, -np.inf, np.nan]])
    p = np.concatenate([rng.uniform(-1, 1, 300000), 1 - 10.0 ** rng.uniform(-16, 0, 30000),
                        -1 + 10.0 ** rng.uniform(-16, 0, 30000), rng.uniform(-1e-6, 1e-6, 30000)])
    with np.errstate(divide="ignore"):
        xl = np.concatenate([(1 + p) / (1 - p), 10.0 ** rng.uniform(-320, 308, 30000),
                             [0.0, 5e-324, 1.0, np.nextafter(1.0, 2), np.nextafter(1.0, 0), np.inf, np.nan]])
    for x, fn, tol, name in ((xt, math.tanh, BP_TANH_ULP_TOL, "tanh"), (xl, math.log, BP_LOG_ULP_TOL, "log")):
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = np.empty_like(x)
        args = (out.ctypes.data, None) if name == "tanh" else (None, out.ctypes.data)
        assert L.ldpc_bp_math_probe(0, x.ctypes.data, len(x), *args) == 0, native.lib().ldpc_last_error()
        want = np.array([fn(v) if not (name == "log" and v == 0) else -math.inf for v in x.tolist()])
        u = _ulps(out, want)
        hist = {k: int((u == k).sum()) for k in range(0, tol + 1)}
        print(f"{name}: max {u.max()} ulp over {len(x)} values; histogram {hist}")
        assert u.max() <= tol, (name, x[np.argmax(u)], out[np.argmax(u)], want[np.argmax(u)])
