"""The fast-path row kernel (ldpcsimulation_amd/csrc/rows_fast.hip): fp64 decode of
every row-kernel graph, fast check node compiled per variant, exact re-decode of
codewords that break its premise.

CPU tests pin the fp64 division rule it uses (Markstein's one-FMA correction of
x * RN(1/alpha), checked against IEEE x / alpha by the oracle's C helper) and the
host-side argument checks. GPU tests compare its decisions with the fp64 oracle
(the restatement of decodeMinSum.cpp:247-263, 410-515) on the headline
configuration, and force the premise to fail (huge, tiny, infinite and NaN
channel values) so the re-decode path runs and must give the oracle's answer too.
"""
import math

import numpy as np
import pytest

from conftest import code_path
from oracle import oracle as O


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("alpha", [1.25, 1.5, 0.75, 1.125, 2.0, 5.0, 0.625, 1.3125])
def test_markstein_division_matches_ieee(alpha):
    """alpha = P*2^E, odd P < 2^20: the fast fp64 NMS division equals x/alpha on a
    sample of 2M random x over 2^-960..2^1000 plus binade edges and x near k*alpha."""
    assert O.markstein_mismatch(alpha, 2_000_000, seed=11) == 0


@pytest.mark.parametrize("alpha,fast", [
    (1.25, 1), (0.75, 1), (5.0, 1), (1.5, 1), (2.0 ** 60, 1), (3.0 * 2.0 ** 55, 1),
    (1.1, 0), (2.0 ** -950, 0), (2.0 ** 61, 0), (3.0 * 2.0 ** 60, 0), (1.0 + 2.0 ** -30, 0),
    (0.0, 0), (-1.25, 0), (float("inf"), 0), (float("nan"), 0)])
def test_markstein_alpha_gate(alpha, fast):
    """The kernel takes the fast division only for alpha it can prove (rows_fast.hip
    markstein_exact_alpha, through ldpc_f64_nms_fast_division): alpha = P*2^E with odd
    P < 2^20 and 2^-900 < alpha <= 2^60 (above 2^60 a minimum near 2^-960 divides to a
    subnormal quotient); 1.1 and 1 + 2^-30 have P >= 2^20."""
    from ldpcsimulation_amd import native
    assert native.lib().ldpc_f64_nms_fast_division(alpha) == fast


@pytest.mark.parametrize("alpha", [2.0 ** 60, 3.0 * 2.0 ** 55])
def test_markstein_division_matches_ieee_large_alpha(alpha):
    """At the gate's upper end the fast division still equals IEEE x / alpha."""
    assert O.markstein_mismatch(alpha, 500_000, seed=13) == 0


class _FakeGraph:
    N = 8


def test_decode_rejects_wrong_tensor_dtypes():
    """Context.decode checks torch tensors' dtype before any device call."""
    torch = pytest.importorskip("torch")
    from ldpcsimulation_amd import native
    ctx = native.Context.__new__(native.Context)
    ctx.graph = _FakeGraph()
    ctx._h = None
    cfg64 = native.DecoderConfig(precision=native.F64)
    cfg32 = native.DecoderConfig(precision=native.F32)
    with pytest.raises(TypeError):
        ctx.decode(torch.zeros(2, 8, dtype=torch.float32), cfg64)
    with pytest.raises(TypeError):
        ctx.decode(torch.zeros(2, 8, dtype=torch.float64), cfg32)
    with pytest.raises(TypeError):
        ctx.decode(torch.zeros(2, 8, dtype=torch.float64), cfg64, c=torch.ones(2, 8, dtype=torch.int32))
    with pytest.raises(ValueError):
        ctx.decode(torch.zeros(3, 5, dtype=torch.float64), cfg64)
    with pytest.raises(ValueError):
        ctx.decode(torch.zeros(2, 8, dtype=torch.float64), cfg64, c=torch.ones(1, 8, dtype=torch.int8))


# ------------------------------------------------------------------ GPU
def _glibc_frames(N, nframes, ebn0, R, seed):
    g = O.GlibcRandom(seed)
    sigma = math.sqrt(10 ** (-ebn0 / 10) / R / 2)
    c = np.ones(N, dtype=np.int32)
    return np.stack([g.channel(c, sigma) for _ in range(nframes)])


@pytest.mark.gpu
@pytest.mark.parametrize("code", ["80211n_1944_r12.alist", "PEGReg504x1008.alist"])
def test_fast_kernel_is_the_f64_row_kernel(gpu_ctx_factory, code):
    """fp64 row graphs take a fast-path kernel: the ping-pong kernel (rows_pp.hip) for
    the 802.11n code (M = 972: 512 threads x 2 rows), k_rows_fast otherwise or with
    option rows64 = fast (the kernel the tests of this file exercise)."""
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory(code)
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=5, precision=native.F64)
    assert ctx.kernel_info(cfg)["kernel"] == ("rows_pp" if code == "80211n_1944_r12.alist" else "rows_fast")
    ctx.set_option("rows64", "fast")
    assert ctx.kernel_info(cfg)["kernel"] == "rows_fast"
    cfg.precision = native.F32                       # fp32: pairs on the ping-pong kernel where it fits
    assert ctx.kernel_info(cfg)["kernel"] == ("rows_pp" if code == "80211n_1944_r12.alist" else "rows")
    ctx.set_option("rows32", "rows")
    assert ctx.kernel_info(cfg)["kernel"] == "rows"


@pytest.mark.gpu
def test_f32_pair_fast_kernel_opt_in(gpu_ctx_factory):
    """Option rows32 = fast selects the fp32 pair instance of rows_fast for MS and
    verified-reciprocal NMS; OMS keeps the row kernel."""
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory("80211n_1944_r12.alist")
    ctx.set_option("rows32", "fast")
    for v, want in ((native.MS, "rows_fast"), (native.NMS, "rows_fast"), (native.OMS, "rows")):
        cfg = native.DecoderConfig(variant=v, alpha=1.25, delta=0.1, T=5, precision=native.F32)
        assert ctx.kernel_info(cfg)["kernel"] == want


@pytest.mark.gpu
@pytest.mark.parametrize("code", ["80211n_1944_r12.alist", "PEGReg504x1008.alist"])
@pytest.mark.parametrize("vname,v", [("ms", dict(variant=0)), ("nms", dict(variant=1, alpha=1.25)),
                                     ("nms_ieee", dict(variant=1, alpha=1.1)),
                                     ("oms", dict(variant=2, delta=0.15))])
def test_premise_breaks_are_redecoded_exactly(gpu_ctx_factory, code, vname, v):
    """Frames built to break the fast premise (|y| >= 2^1000, minima below 2^-960, inf,
    NaN, values growing past 2^1000 mid-decode) are re-decoded on the exact path:
    decisions, error weights and counters equal the fp64 oracle's for every frame,
    and the re-decode list holds exactly the frames that broke it. (k_rows_fast; the
    ping-pong kernel's twin is tests/test_rows_pp.py.)"""
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory(code)
    ctx.set_option("rows64", "fast")
    N = ctx.graph.N
    y = _glibc_frames(N, 16, 1.5, 0.5, seed=4242)
    y[1] *= 1e305                     # input premise: |yq| >= 2^1000
    y[2] *= 1e-305                    # minima far below 2^-960 (NMS fast division premise)
    y[3, 5] = np.inf                  # non-finite input
    y[4, 7] = np.nan
    y[5] *= 2.0 ** 995                # grows past 2^1000 after a few iterations
    y[6, ::3] = -0.0                  # signed zeros: canonicalised, never a premise break
    y[7] = np.where(np.arange(N) % 2 == 0, 0.5, -1.0)   # ties in every row
    A = O.Alist(code_path(code))
    for T in (1, 7, 30):
        cfg = native.DecoderConfig(T=T, precision=native.F64, **v)
        d, fr, cnt = ctx.decode(y, cfg)
        redo = ctx.redo_count()
        want = A.decode(y, T, O.Cfg(**v), workers=8)
        mism = (d != want).sum(axis=1)
        assert int(mism.sum()) == 0, f"T={T}: mismatching frames {np.nonzero(mism)[0].tolist()}"
        w = (want != 1).sum(axis=1)
        assert np.array_equal(fr["bit_err"], w)
        assert cnt.frames == len(y) and cnt.bit_err == int(w.sum()) and cnt.iters == T * len(y)
        # frames 1, 3, 4 always break it; 2 under the fast NMS division (tiny minima); 5 once it grows
        assert redo >= 3, redo
        assert redo <= 5, redo


@pytest.mark.gpu
@pytest.mark.parametrize("code", ["80211n_1944_r12.alist", "PEGReg504x1008.alist"])
@pytest.mark.parametrize("vname,v", [("ms", dict(variant=0)), ("nms", dict(variant=1, alpha=1.25))])
def test_f32_premise_breaks_are_redecoded_exactly(gpu_ctx_factory, code, vname, v):
    """fp32: frames that break the fast premise (|yq| >= 1e30, inf, NaN, values growing
    past 1e30 mid-decode) -- the pair instance of rows_fast (option rows32 = fast) re-decodes
    them on the exact path, the row kernel hands them over to its exact loop; both give
    the fp32 oracle's decisions and counters."""
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory(code)
    ctx.set_option("rows32", "fast")
    N = ctx.graph.N
    y = _glibc_frames(N, 16, 1.5, 0.5, seed=4243).astype(np.float32)
    y[1] *= np.float32(1e31)          # input premise: |yq| >= 1e30
    y[3, 5] = np.inf                  # non-finite input
    y[4, 7] = np.nan
    y[5] *= np.float32(2.0 ** 92)     # grows past 1e30 after a few iterations
    y[6, ::3] = -0.0                  # signed zeros: canonicalised, never a premise break
    y[7] = np.where(np.arange(N) % 2 == 0, 0.5, -1.0)   # ties in every row
    y[9] = y[8]                       # the pair partner of an unbroken frame is decoded alike
    A = O.Alist(code_path(code))
    for T in (1, 7, 30):
        cfg = native.DecoderConfig(T=T, precision=native.F32, **v)
        assert ctx.kernel_info(cfg)["kernel"] == "rows_fast"
        d, fr, cnt = ctx.decode(y, cfg)
        redo = ctx.redo_count()
        want = A.decode(y, T, O.Cfg(**v), workers=8)
        mism = (d != want).sum(axis=1)
        assert int(mism.sum()) == 0, f"T={T}: mismatching frames {np.nonzero(mism)[0].tolist()}"
        w = (want != 1).sum(axis=1)
        assert np.array_equal(fr["bit_err"], w)
        assert cnt.frames == len(y) and cnt.bit_err == int(w.sum()) and cnt.iters == T * len(y)
        # pairs (0,1), (2,3), (4,5) break (frame 5 shares frame 4's pair); a pair is re-decoded whole
        assert redo == 6, redo
        ctx.set_option("rows32", "rows")
        assert ctx.kernel_info(cfg)["kernel"] == "rows"
        d_old, fr_old, cnt_old = ctx.decode(y, cfg)
        ctx.set_option("rows32", "fast")
        assert np.array_equal(d_old, d) and np.array_equal(fr_old, fr) and cnt_old.bit_err == cnt.bit_err


@pytest.mark.gpu
@pytest.mark.parametrize("ebn0", [1.5, 1.75])
@pytest.mark.parametrize("vname,v", [("nms", dict(variant=1, alpha=1.25)), ("ms", dict(variant=0))])
@pytest.mark.parametrize("kernel", ["pp", "fast"])
def test_f64_headline_config_bit_exact(gpu_ctx_factory, kernel, ebn0, vname, v):
    """The bench configuration in fp64 (802.11n N=1944, T=50, on-device Philox channel):
    2048 codewords per point, decisions identical to the fp64 oracle on the same y,
    and no codeword needed the exact path -- for the bench's kernel (the ping-pong
    kernel, rows_pp.hip) and for k_rows_fast."""
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory("80211n_1944_r12.alist")
    ctx.set_option("rows64", kernel)
    cfg = native.DecoderConfig(T=50, precision=native.F64, **v)
    assert ctx.kernel_info(cfg)["kernel"] == "rows_" + kernel
    y, d, fr, cnt = ctx.sim_trace(ebn0, 0.5, cfg, seed=20261016, stream_id=1, first_cw=0, batch=2048)
    assert ctx.redo_count() == 0
    want = O.Alist(code_path("80211n_1944_r12.alist")).decode(y, 50, O.Cfg(**v), workers=16)
    assert int((d != want).sum()) == 0
    w = (want != 1).sum(axis=1)
    assert np.array_equal(fr["bit_err"], w)
    assert cnt.frame_err == int((w > 0).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("ebn0", [1.5, 1.75])
@pytest.mark.parametrize("vname,v", [("nms", dict(variant=1, alpha=1.25)), ("ms", dict(variant=0))])
def test_f32_bench_kernel_bit_exact_at_T50(gpu_ctx_factory, ebn0, vname, v):
    """The fp32 bench kernel (k_decode_rows<float, PHILOX, 2, 8, 4, 2>: fast check node,
    reciprocal NMS, fast->exact hand-over) at the bench's T=50 on 2048 codewords per
    point: decisions identical to the fp32 oracle on the same y, to
    the opt-in pair instance of rows_fast (option rows32 = fast) and to the fp32 default,
    the ping-pong kernel's float2 slots (rows_pp.hip)."""
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory("80211n_1944_r12.alist")
    cfg = native.DecoderConfig(T=50, precision=native.F32, **v)
    ctx.set_option("rows32", "rows")
    assert ctx.kernel_info(cfg)["kernel"] == "rows"
    y, d, fr, cnt = ctx.sim_trace(ebn0, 0.5, cfg, seed=20261017, stream_id=2, first_cw=0, batch=2048)
    for k32, name in (("fast", "rows_fast"), ("pp", "rows_pp")):   # the opt-in pair kernel, the fp32 default
        ctx.set_option("rows32", k32)
        assert ctx.kernel_info(cfg)["kernel"] == name
        y_f, d_f, fr_f, _ = ctx.sim_trace(ebn0, 0.5, cfg, seed=20261017, stream_id=2, first_cw=0, batch=2048)
        assert ctx.redo_count() == 0
        assert np.array_equal(y_f, y) and np.array_equal(d_f, d) and np.array_equal(fr_f, fr), k32
    want = O.Alist(code_path("80211n_1944_r12.alist")).decode(y, 50, O.Cfg(**v), workers=16)
    assert int((d != want).sum()) == 0
    assert np.array_equal(fr["bit_err"], (want != 1).sum(axis=1))
