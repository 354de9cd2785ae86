"""GPU parity: the HIP decoder (through the C ABI) against the oracle and the reference.

Tiers:
  (a) identical channel samples y -> decisions bit-exact with the oracle, in
      fp64 (the reference's precision) and fp32 (oracle run in float);
  (b) whole reference runs (tests/golden/reference_runs.json, produced by the
      compiled reference) reproduced through the GPU: same totals, same
      sequence of per-frame error weights;
  (c) statistical: on-device Philox noise and FER against the reference.
"""
import math

import os

import numpy as np
import pytest

from conftest import code_path, golden_runs
from helpers import cw_lines, final_numbers, run_config
from oracle import oracle as O

pytestmark = pytest.mark.gpu

CODES = ["PEGReg504x1008.alist", "80211n_1944_r12.alist", "4000.2000.4.244.alist"]
VARIANTS = {
    "ms": dict(variant=0),
    "nms": dict(variant=1, alpha=1.25),
    "oms": dict(variant=2, delta=0.15),
    "qnms": dict(variant=1, alpha=1.25, quantize=True, ymax=1.5, qbits=4),
    "qoms": dict(variant=2, delta=0.15, quantize=True, ymax=1.5, qbits=4),
    "sat_ms": dict(variant=0, saturate=True, ymax=1.2),
}


def _native():
    from ldpcsimulation_amd import native
    return native


def _glibc_frames(N, nframes, ebn0, R, seed, c=None):
    g = O.GlibcRandom(seed)
    sigma = math.sqrt(10 ** (-ebn0 / 10) / R / 2)
    c = np.ones(N, dtype=np.int32) if c is None else c
    return np.stack([g.channel(c, sigma) for _ in range(nframes)])


def _oracle_front(y, v, f32):
    if v.get("quantize"):
        q = O.quantize_f32 if f32 else O.quantize
        flat = np.array([q(float(x), v["ymax"], v["qbits"]) for x in y.ravel()],
                        dtype=np.float32 if f32 else np.float64)
        return flat.reshape(y.shape)
    if v.get("saturate"):
        ym = np.float32(v["ymax"]) if f32 else v["ymax"]
        return np.clip(y, -ym, ym)
    return y


@pytest.mark.parametrize("code", CODES)
@pytest.mark.parametrize("vname", list(VARIANTS))
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_decisions_bit_exact_vs_oracle(gpu_ctx_factory, code, vname, prec):
    native = _native()
    ctx = gpu_ctx_factory(code)
    N = ctx.graph.N
    v = VARIANTS[vname]
    f32 = prec == "f32"
    y = _glibc_frames(N, 12, 1.8, 0.5, seed=1234 + len(vname))
    if f32:
        y = y.astype(np.float32)
    A = O.Alist(code_path(code))
    from ldpcsimulation_amd import codes
    H = codes.read_alist(code_path(code))
    yq = _oracle_front(y, v, f32)
    for T in (0, 1, 3, 10):
        cfg = native.DecoderConfig(T=T, precision=native.F32 if f32 else native.F64, **v)
        d, fr, cnt = ctx.decode(y, cfg)
        want = A.decode(yq, T, O.Cfg(**{k: v[k] for k in v}))
        mism = int((d != want).sum())
        assert mism == 0, f"T={T}: {mism} decision mismatches"
        w = (want != 1).sum(axis=1)
        assert np.array_equal(fr["bit_err"], w)
        assert cnt.frames == len(y) and cnt.bit_err == int(w.sum())
        assert cnt.frame_err == int((w > 0).sum()) and cnt.iters == T * len(y)
        sf = [int(any(H.syndrome(row != 1))) for row in want]
        assert list(fr["syndrome_fail"]) == sf and cnt.syndrome_fail == sum(sf)


@pytest.mark.parametrize("run", golden_runs(), ids=lambda r: r["name"])
def test_gpu_reproduces_reference_run(gpu_ctx_factory, run):
    """The reference's own Monte-Carlo run, with the reference's noise, decoded on the GPU in fp64."""
    native = _native()
    R, snr, T, c = run_config(run)
    bit_ref, words_ref, unc_ref = final_numbers(run["final"])
    ctx = gpu_ctx_factory(run["code"], 1024)
    N = ctx.graph.N
    lines = cw_lines(run)
    g = O.GlibcRandom(run["seed"])
    sigma = math.sqrt(10 ** (-snr / 10) / R / 2)
    cfg = native.DecoderConfig(T=T, precision=native.F64, **c)
    errors = words = word_errors = unc = 0
    ferr = []
    f = 0
    done = False
    while not done:
        B = 256
        cw = np.ones((B, N), dtype=np.int8)
        ys = np.empty((B, N))
        for k in range(B):
            if lines:
                cw[k] = [-1 if ch == "1" else 1 for ch in lines[(f + k) % len(lines)][:N]]
            ys[k] = g.channel(cw[k].astype(np.int32), sigma)
        _, fr, _ = ctx.decode(ys, cfg, c=cw if lines else None, want_decisions=False)
        f += B
        for r in fr:
            if not (errors < 200 or word_errors < 40):
                done = True
                break
            unc += int(r["uncoded_bit_err"])
            if r["bit_err"] > 0:
                errors += int(r["bit_err"])
                word_errors += 1
                ferr.append(int(r["bit_err"]))
            words += 1
    assert (errors, words, unc) == (bit_ref, words_ref, unc_ref)
    assert ferr == run["ferr_weights"]


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_fused_sim_matches_oracle_on_device_noise(gpu_ctx_factory, prec):
    """AWGN -> decode -> count in one kernel: decisions equal the oracle's on the y it generated."""
    native = _native()
    ctx = gpu_ctx_factory("80211n_1944_r12.alist")
    f32 = prec == "f32"
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=20,
                               precision=native.F32 if f32 else native.F64)
    y, d, fr, cnt = ctx.sim_trace(1.25, 0.5, cfg, seed=77, stream_id=3, first_cw=1000, batch=24)
    A = O.Alist(code_path("80211n_1944_r12.alist"))
    want = A.decode(y, 20, O.Cfg(variant=1, alpha=1.25))
    assert int((d != want).sum()) == 0
    w = (want != 1).sum(axis=1)
    assert np.array_equal(fr["bit_err"], w)
    assert np.array_equal(fr["uncoded_bit_err"], (y <= 0).sum(axis=1))
    assert cnt.bit_err == int(w.sum()) and cnt.frames == 24


def test_sim_independent_of_batch_split(gpu_ctx_factory):
    native = _native()
    ctx = gpu_ctx_factory("80211n_1944_r12.alist")
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=10)
    full, c_full = ctx.sim_batch(1.0, 0.5, cfg, seed=5, stream_id=0, first_cw=0, batch=512)
    a, c_a = ctx.sim_batch(1.0, 0.5, cfg, seed=5, stream_id=0, first_cw=0, batch=200)
    b, c_b = ctx.sim_batch(1.0, 0.5, cfg, seed=5, stream_id=0, first_cw=200, batch=312)
    assert np.array_equal(full, np.concatenate([a, b]))
    assert c_full.bit_err == c_a.bit_err + c_b.bit_err
    other, _ = ctx.sim_batch(1.0, 0.5, cfg, seed=6, stream_id=0, first_cw=0, batch=512)
    assert not np.array_equal(full["uncoded_bit_err"], other["uncoded_bit_err"])


@pytest.mark.parametrize("code", CODES)
def test_all_kernels_bit_identical(monkeypatch, code):
    """The row-parallel, per-codeword-LDS, flood (global, coalesced) and generic global kernels give
    identical results."""
    native = _native()
    g = native.Graph.from_alist(code_path(code))
    ctxs = {}
    for k in ("default", "lds", "flood", "global"):
        ctxs[k] = native.Context(g, 0, 300)
        if k != "default":
            ctxs[k].set_option("kernel", k)
    cfgs = [native.DecoderConfig(variant=native.OMS, delta=0.1, T=15, quantize=True, ymax=1.5, qbits=5),
            native.DecoderConfig(variant=native.NMS, alpha=1.25, T=15),
            native.DecoderConfig(variant=native.MS, T=15)]
    for cfg, prec in ((c, p) for c in cfgs for p in (native.F32, native.F64)):
        cfg.precision = prec
        names = {k: c.kernel_info(cfg)["kernel"] for k, c in ctxs.items()}
        assert names["lds"] == "lds" and names["global"] == "global" and names["flood"] == "flood"
        if code != "4000.2000.4.244.alist":
            # fp64: the ping-pong kernel (rows_pp.hip, M in 513..1024) or the one-codeword
            # fast-path kernel (rows_fast.hip); fp32: the row kernel
            pp_code = code == "80211n_1944_r12.alist"
            f64_default = "rows_pp" if pp_code else "rows_fast"
            # fp32: pairs on the ping-pong kernel for MS / verified-reciprocal NMS, else the row kernel
            f32_default = "rows_pp" if pp_code and cfg.variant != native.OMS else "rows"
            assert names["default"] == (f64_default if prec == native.F64 else f32_default)
        outs = {k: c.sim_trace(2.0, 0.5, cfg, 9, 0, 0, 300) for k, c in ctxs.items()}
        cd = ctxs["default"]
        cd.set_option("rows64", "fast")   # fp64: the one-codeword fast kernel where pp is the default
        outs["rows_fast"] = cd.sim_trace(2.0, 0.5, cfg, 9, 0, 0, 300)
        cd.set_option("rows64", "rows")   # the previous row kernel (exact + fast loops in one)
        outs["rows_old"] = cd.sim_trace(2.0, 0.5, cfg, 9, 0, 0, 300)
        cd.set_option("rows64", "pp")
        cd.set_option("rows32", "fast")   # fp32: the pair instance of rows_fast (opt-in)
        outs["rows_fast32"] = cd.sim_trace(2.0, 0.5, cfg, 9, 0, 0, 300)
        cd.set_option("rows32", "rows")   # fp32: the row kernel
        outs["rows32"] = cd.sim_trace(2.0, 0.5, cfg, 9, 0, 0, 300)
        cd.set_option("rows32", "pp")
        ref = outs["global"]
        for k, o in outs.items():
            for a, b in zip(o[:3], ref[:3]):
                assert np.array_equal(a, b), k


def test_channel_noise_statistics(gpu_ctx_factory):
    """Philox + Box-Muller noise: mean/variance/tails of (y-1)/sigma over 24M samples."""
    native = _native()
    ctx = gpu_ctx_factory("80211n_1944_r12.alist", 4096)
    cfg = native.DecoderConfig(T=0, precision=native.F64)
    sigma = math.sqrt(10 ** (-1.5 / 10) / 0.5 / 2)
    n = []
    for k in range(3):
        y, _, _, _ = ctx.sim_trace(1.5, 0.5, cfg, seed=11, stream_id=k, first_cw=0, batch=4096)
        n.append(((y - 1.0) / sigma).ravel())
    n = np.concatenate(n)
    m = n.size
    assert abs(n.mean()) < 5 / math.sqrt(m)
    assert abs(n.var() - 1) < 5 * math.sqrt(2 / m)
    for t in (1.0, 2.0, 3.0):
        p = math.erfc(t / math.sqrt(2))
        got = float((np.abs(n) > t).mean())
        assert abs(got - p) < 6 * math.sqrt(p * (1 - p) / m), (t, got, p)
    # independence of consecutive samples
    assert abs(np.corrcoef(n[:-1], n[1:])[0, 1]) < 5 / math.sqrt(m)


def test_syndrome_and_codeword_mode(gpu_ctx_factory):
    """Codeword-file mode decodes the transmitted codeword; decoded frames have zero syndrome."""
    native = _native()
    ctx = gpu_ctx_factory("PEGReg504x1008.alist", 2048)
    lines = [l.strip() for l in open(code_path("PEGReg504x1008_data20.enc")) if l.strip()]
    bits = np.array([[int(ch) for ch in l] for l in lines], dtype=np.uint8)
    ctx.set_codewords(bits)
    try:
        cfg = native.DecoderConfig(T=20)
        y, d, fr, cnt = ctx.sim_trace(2.5, 0.5, cfg, seed=3, stream_id=0, first_cw=0, batch=400)
        rows = np.arange(400) % len(lines)
        c = 1 - 2 * bits[rows].astype(np.int8)
        assert np.array_equal(fr["bit_err"], (d != c).sum(axis=1))
        ok = fr["bit_err"] == 0
        assert ok.sum() > 300
        assert (fr["syndrome_fail"][ok] == 0).all()
        # channel symmetry: the same noise on the all-zero word gives the same weights
        ctx.set_codewords(None)
        fr0, _ = ctx.sim_batch(2.5, 0.5, cfg, 3, 0, 0, 400)
        assert np.array_equal(fr0["bit_err"], fr["bit_err"])
    finally:
        ctx.set_codewords(None)


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_fer_matches_reference_statistically(gpu_ctx_factory, prec):
    """802.11n N=1944 NMS a=1.25 T=50, on-device Philox channel: GPU FER vs the
    reference's own decodeNMS over 10 seeds per point (tests/golden/reference_fer.json,
    scripts/ref_fer.py: 400 frame errors per point, decodeMinSum.cpp:189 stop rule),
    two-proportion z-test |z| < 3 at all four SURVEY §8(d) points. The GPU side
    decodes 16k-256k frames (>= 250 frame errors per point), so a FER shift of
    ~20 % would show as |z| > 3. fp64 is the reference's arithmetic; fp32 is the
    throughput path (its decision gap to fp64 is tests/test_precision_gap.py)."""
    import json
    native = _native()
    from ldpcsimulation_amd.sim import two_proportion_z
    with open(os.path.join(os.path.dirname(__file__), "golden", "reference_fer.json")) as f:
        ref = {p["ebn0_db"]: (p["frame_err"], p["frames"]) for p in json.load(f)["points"]}
    ctx = gpu_ctx_factory("80211n_1944_r12.alist", 16384)
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=50,
                               precision=native.F64 if prec == "f64" else native.F32)
    rounds = {1.0: 1, 1.25: 1, 1.5: 4, 1.75: 16}
    for ebn0, (k_ref, n_ref) in sorted(ref.items()):
        assert k_ref >= 400
        ferr = frames = 0
        for r in range(rounds[ebn0]):
            _, cnt = ctx.sim_batch(ebn0, 0.5, cfg, seed=2026, stream_id=int(ebn0 * 100), first_cw=r * 16384,
                                   batch=16384, want_frames=False)
            ferr += cnt.frame_err
            frames += cnt.frames
        assert frames == rounds[ebn0] * 16384
        z = two_proportion_z(ferr, frames, k_ref, n_ref)
        assert abs(z) < 3, (ebn0, ferr, frames, k_ref, n_ref, z)
        assert ferr >= 200, (ebn0, ferr, frames)


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("vname", ["ms", "nms"])
def test_degree_one_check_infinities_exact(tmp_path, prec, vname):
    """A degree-1 check sends +-inf (min2 of one edge, :419-447); the sums then hit
    inf - inf = NaN. The fast fp32 check-node path must hand over to the exact path
    so decisions still equal the oracle's (reference semantics for inf/NaN)."""
    from ldpcsimulation_amd import codes
    native = _native()
    H = codes.read_alist(code_path("PEGReg504x1008.alist"))
    rows = H.rows + [[5], [17, 900]]                     # add a degree-1 and a degree-2 check
    H2 = codes.ParityCheck.from_rows(H.N, rows)
    path = str(tmp_path / "peg_deg1.alist")
    codes.write_alist(H2, path)
    ctx = native.Context(native.Graph.from_alist(path), 0, 64)
    f32 = prec == "f32"
    v = VARIANTS[vname]
    y = _glibc_frames(H.N, 8, 2.0, 0.5, seed=99)
    if f32:
        y = y.astype(np.float32)
    A = O.Alist(path)
    for T in (1, 2, 5, 12):
        cfg = native.DecoderConfig(T=T, precision=native.F32 if f32 else native.F64, **v)
        d, fr, cnt = ctx.decode(y, cfg)
        want = A.decode(y, T, O.Cfg(**v))
        assert int((d != want).sum()) == 0, T


@pytest.mark.parametrize("vname", ["ms", "nms", "oms"])
def test_signed_zeros_and_ties_exact(vname):
    """Channel values drawn from {+-0, +-0.5, +-1, +-2}: exact zero messages
    (sgn(-0) = +1, :518-523), tied minima (:428-437) and -0 channel samples. The
    fast fp32 check node reads v2c signs from bit patterns, which holds only
    because yq is canonicalised to +0; decisions must equal the oracle's."""
    native = _native()
    path = code_path("PEGReg504x1008.alist")
    ctx = native.Context(native.Graph.from_alist(path), 0, 64)
    A = O.Alist(path)
    rng = np.random.default_rng(7)
    vals = np.array([-0.0, 0.0, -0.5, 0.5, -1.0, 1.0, -2.0, 2.0], dtype=np.float32)
    y = vals[rng.integers(0, len(vals), size=(16, A.N))]
    y[:4] = np.where(rng.random((4, A.N)) < 0.5, np.float32(-0.0), np.float32(0.0))   # all-zero frames
    v = VARIANTS[vname]
    for T in (1, 2, 3, 8):
        cfg = native.DecoderConfig(T=T, precision=native.F32, **v)
        d, fr, cnt = ctx.decode(y, cfg)
        want = A.decode(y, T, O.Cfg(**v))
        assert int((d != want).sum()) == 0, T


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_dvbs2_flood_decisions_vs_oracle(gpu_ctx_factory, prec):
    """DVB-S2 N=64800 (state beyond LDS: the flood kernel) -- decisions equal the oracle's."""
    native = _native()
    ctx = gpu_ctx_factory("dvbs2_1_2.alist", 64)
    f32 = prec == "f32"
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=6, precision=native.F32 if f32 else native.F64)
    assert ctx.kernel_info(cfg)["kernel"] == "flood"
    y, d, fr, cnt = ctx.sim_trace(0.8, 0.5, cfg, seed=5, stream_id=1, first_cw=3, batch=3)
    A = O.Alist(code_path("dvbs2_1_2.alist"))
    want = A.decode(y, 6, O.Cfg(variant=1, alpha=1.25))
    assert int((d != want).sum()) == 0
    assert np.array_equal(fr["bit_err"], (want != 1).sum(axis=1))


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_flood_heavy_column_vs_oracle(tmp_path, monkeypatch, prec):
    """Phase flooding on a code with a column of degree 40: the packed-message bit
    phase is built for column degrees <= 32, so such a code takes the
    c2v-array bit phase (any degree); decisions equal the oracle's."""
    from ldpcsimulation_amd import codes
    native = _native()
    rng = np.random.default_rng(40)
    N, M = 600, 300
    rows = [sorted(set(rng.choice(np.arange(1, N), size=6, replace=False).tolist())) for _ in range(M)]
    for j in range(40):                       # bit 0 in 40 checks
        rows[j] = sorted(set(rows[j]) | {0})
    path = str(tmp_path / "heavy_col.alist")
    codes.write_alist(codes.ParityCheck.from_rows(N, rows), path)
    ctx = native.Context(native.Graph.from_alist(path), 0, 64)
    ctx.set_option("kernel", "flood")
    f32 = prec == "f32"
    y = _glibc_frames(N, 16, 3.0, 0.5, seed=41)
    if f32:
        y = y.astype(np.float32)
    A = O.Alist(path)
    assert sum(0 in r for r in rows) == 40
    for v in (VARIANTS["ms"], VARIANTS["nms"]):
        for T in (1, 7):
            cfg = native.DecoderConfig(T=T, precision=native.F32 if f32 else native.F64, **v)
            assert ctx.kernel_info(cfg)["kernel"] == "flood"
            d, fr, cnt = ctx.decode(y, cfg)
            want = A.decode(y, T, O.Cfg(**v))
            assert int((d != want).sum()) == 0, (v, T)
