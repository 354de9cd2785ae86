"""Layered (row-serial) min-sum: SURVEY §8(f) row 2, BASELINE config 3.

The reference only floods (src/decodeMinSum.cpp:247-263), so the layered
schedule has no reference output to pin it: its oracle is the row-serial
restatement oracle/ldpc_oracle.c:orc_decode_layered_* (same check-node rule
as the reference's :410-450/:494-515; "parity unpinned" against the
reference, pinned against that oracle). Bit-exact tier: identical y ->
identical decisions for every variant, fp32 and fp64.

CPU tests: the layer partition (bit-disjoint row sets by first-fit colouring of
row chains: 17 layers on DVB-S2 N=64800, the 12 block rows of Z=81 on 802.11n N=1944) and
the commutation property the GPU kernel relies on (any order of the rows
inside a layer gives the same result). GPU tests: the HIP kernels against the oracle.
"""
import math

import numpy as np
import pytest

from conftest import code_path
from oracle import oracle as O

CODES = ["PEGReg504x1008.alist", "80211n_1944_r12.alist", "4000.2000.4.244.alist"]
VARIANTS = {
    "ms": dict(variant=0),
    "nms": dict(variant=1, alpha=1.25),
    "oms": dict(variant=2, delta=0.15),
    "qoms": dict(variant=2, delta=0.15, quantize=True, ymax=1.5, qbits=4),
}


def _native():
    from ldpcsimulation_amd import native
    return native


def _layers(code):
    native = _native()
    g = native.Graph.from_alist(code_path(code))
    order, ptr = g.layers()
    return g, order, ptr


def _frames(N, n, ebn0, seed, dtype=np.float64):
    g = O.GlibcRandom(seed)
    sigma = math.sqrt(10 ** (-ebn0 / 10) / 0.5 / 2)
    c = np.ones(N, dtype=np.int32)
    return np.stack([g.channel(c, sigma) for _ in range(n)]).astype(dtype)


@pytest.mark.parametrize("code,want", [("dvbs2_1_2.alist", None), ("80211n_1944_r12.alist", (12, 81)),
                                       ("PEGReg504x1008.alist", None)])
def test_layer_partition_is_bit_disjoint(code, want):
    """Layers: bit-disjoint row sets (chain-level first-fit colouring, graph.cpp build_layers); the
    802.11n N=1944 code comes out as its 12 block rows of Z=81."""
    from ldpcsimulation_amd import codes
    g, order, ptr = _layers(code)
    H = codes.read_alist(code_path(code))
    assert sorted(order.tolist()) == list(range(g.M))
    assert ptr[0] == 0 and ptr[-1] == g.M and np.all(np.diff(ptr) > 0)
    layer_bits = []
    for L in range(len(ptr) - 1):
        cols = [c for j in order[ptr[L]:ptr[L + 1]] for c in H.rows[j]]
        assert len(cols) == len(set(cols)), f"layer {L} rows share a bit"
        layer_bits.append(set(cols))
    # first fit over whole row chains: every layer L > 0 clashes with each earlier layer
    for L in range(1, len(ptr) - 1):
        assert all(layer_bits[L] & layer_bits[K] for K in range(L))
    if want:
        assert (len(ptr) - 1, int(np.diff(ptr).max())) == want
        assert np.all(np.diff(ptr) == want[1])
    else:
        assert len(ptr) - 1 <= 2 * max(len(c) for c in H.cols) + 2


@pytest.mark.parametrize("vname", ["ms", "nms", "oms"])
def test_oracle_layers_commute(vname):
    """Rows inside a layer may be updated in any order (what the kernel's parallel layer does)."""
    _, order, ptr = _layers("80211n_1944_r12.alist")
    A = O.Alist(code_path("80211n_1944_r12.alist"))
    y = _frames(A.N, 3, 1.5, seed=21)
    rng = np.random.default_rng(3)
    shuffled = order.copy()
    for L in range(len(ptr) - 1):
        rng.shuffle(shuffled[ptr[L]:ptr[L + 1]])
    cfg = O.Cfg(**VARIANTS[vname])
    for dt in (np.float64, np.float32):
        a = A.decode_layered(y.astype(dt), 8, cfg, order)
        b = A.decode_layered(y.astype(dt), 8, cfg, shuffled)
        assert np.array_equal(a, b)


def test_oracle_layered_converges_faster_than_flooding():
    """Sanity of the restatement: at equal T the layered schedule leaves fewer errors."""
    _, order, _ = _layers("80211n_1944_r12.alist")
    A = O.Alist(code_path("80211n_1944_r12.alist"))
    y = _frames(A.N, 40, 1.75, seed=8)
    cfg = O.Cfg(variant=1, alpha=1.25)
    lay = int((A.decode_layered(y, 4, cfg, order) != 1).sum())
    flo = int((A.decode(y, 4, cfg) != 1).sum())
    assert lay < flo


@pytest.mark.gpu
@pytest.mark.parametrize("code", CODES)
@pytest.mark.parametrize("vname", list(VARIANTS))
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_layered_decisions_bit_exact_vs_oracle(gpu_ctx_factory, code, vname, prec):
    native = _native()
    ctx = gpu_ctx_factory(code)
    g, order, _ = _layers(code)
    v = VARIANTS[vname]
    f32 = prec == "f32"
    y = _frames(g.N, 8, 1.8, seed=4321 + len(vname), dtype=np.float32 if f32 else np.float64)
    A = O.Alist(code_path(code))
    yq = y
    if v.get("quantize"):
        q = O.quantize_f32 if f32 else O.quantize
        yq = np.array([q(float(x), v["ymax"], v["qbits"]) for x in y.ravel()], dtype=y.dtype).reshape(y.shape)
    for T in (0, 1, 3, 10):
        cfg = native.DecoderConfig(T=T, precision=native.F32 if f32 else native.F64,
                                   schedule=native.LAYERED, **v)
        assert ctx.kernel_info(cfg)["kernel"] == "layered_lds"
        d, fr, cnt = ctx.decode(y, cfg)
        want = A.decode_layered(yq, T, O.Cfg(**v), order)
        assert int((d != want).sum()) == 0, f"T={T}"
        assert np.array_equal(fr["bit_err"], (want != 1).sum(axis=1))
        assert cnt.iters == T * len(y)


@pytest.mark.gpu
@pytest.mark.parametrize("code", ["80211n_1944_r12.alist", "PEGReg504x1008.alist"])
def test_layered_lds_and_global_identical(monkeypatch, code):
    native = _native()
    g = native.Graph.from_alist(code_path(code))
    cg = native.Context(g, 0, 200)
    cg.set_option("kernel", "global")
    cl = native.Context(g, 0, 200)
    for prec in (native.F32, native.F64):
        cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=12, precision=prec, schedule=native.LAYERED)
        assert cg.kernel_info(cfg)["kernel"] == "layered_global"
        assert cl.kernel_info(cfg)["kernel"] == "layered_lds"
        a = cg.sim_trace(1.5, 0.5, cfg, 9, 0, 0, 200)
        b = cl.sim_trace(1.5, 0.5, cfg, 9, 0, 0, 200)
        for x, z in zip(a[:3], b[:3]):
            assert np.array_equal(x, z)


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_dvbs2_layered_decisions_vs_oracle(gpu_ctx_factory, prec):
    """DVB-S2 N=64800 layered (state beyond LDS: the global layered kernel) against the oracle."""
    native = _native()
    ctx = gpu_ctx_factory("dvbs2_1_2.alist", 64)
    _, order, _ = _layers("dvbs2_1_2.alist")
    f32 = prec == "f32"
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=5, precision=native.F32 if f32 else native.F64,
                               schedule=native.LAYERED)
    assert ctx.kernel_info(cfg)["kernel"] == "layered_global"
    y, d, fr, cnt = ctx.sim_trace(0.8, 0.5, cfg, seed=5, stream_id=1, first_cw=3, batch=3)
    A = O.Alist(code_path("dvbs2_1_2.alist"))
    want = A.decode_layered(y, 5, O.Cfg(variant=1, alpha=1.25), order)
    assert int((d != want).sum()) == 0
    assert np.array_equal(fr["bit_err"], (want != 1).sum(axis=1))


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_dvbs2_layered_frames_independent_of_grid(prec):
    """The global layered kernel sizes its grid to the batch (resident codewords inside the
    Infinity Cache, the same number of codeword rounds on fewer blocks, api.cpp run_kernel):
    every codeword's result is the same in one 461-frame launch (3 rounds on 154 blocks) as
    in launches of 1, 230 (one round) and 230 frames."""
    native = _native()
    g = native.Graph.from_alist(code_path("dvbs2_1_2.alist"))
    ctx = native.Context(g, 0, 461)
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=3, schedule=native.LAYERED,
                               precision=native.F64 if prec == "f64" else native.F32)
    assert ctx.kernel_info(cfg)["kernel"] == "layered_global"
    whole, cw = ctx.sim_batch(0.9, 0.5, cfg, 11, 2, 5, 461)
    parts = [ctx.sim_batch(0.9, 0.5, cfg, 11, 2, 5 + f, n)[0] for f, n in ((0, 1), (1, 230), (231, 230))]
    assert np.array_equal(whole, np.concatenate(parts))
    assert cw.frames == 461 and int(whole["bit_err"].sum()) > 0


@pytest.mark.gpu
def test_dvbs2_layered_beats_flooding_fer():
    """Config 3 sanity at 1.0 dB, T=50 (NMS a=1.25): the layered FER is well below the flooding
    FER on the same frames (measured 194 vs 1212 of 2048)."""
    native = _native()
    g = native.Graph.from_alist(code_path("dvbs2_1_2.alist"))
    ctx = native.Context(g, 0, 256)
    res = {}
    for sched in (native.FLOODING, native.LAYERED):
        cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=50, schedule=sched)
        _, cnt = ctx.sim_batch(1.0, 0.5, cfg, seed=1, stream_id=0, first_cw=0, batch=256)
        res[sched] = cnt.frame_err
    assert 2 * res[native.LAYERED] < res[native.FLOODING], res
