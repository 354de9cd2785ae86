"""The ping-pong fp64 row kernel (ldpcsimulation_amd/csrc/rows_pp.hip): two codewords
per 1024-thread block, check waves and bit waves overlapped, one barrier interval
per codeword-iteration.

Its arithmetic is k_rows_fast's (fast64.h), so every output must equal the
one-codeword-per-block kernel's and the fp64 oracle's (decodeMinSum.cpp:247-263,
410-515): decisions, per-frame results and counters, for every variant, odd
batches (the last pair's second slot empty), T = 0 and 1, and frames that break
the fast premise -- those are re-decoded exactly, one codeword at a time, and the
other codeword of their pair is unaffected.
"""
import math

import numpy as np
import pytest

from conftest import code_path
from oracle import oracle as O

CODE = "80211n_1944_r12.alist"


def _kernel(ctx, name):
    ctx.set_option("rows64", name)


@pytest.mark.gpu
def test_pp_kernel_selected_for_the_bench_code(gpu_ctx_factory):
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory(CODE)
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=50, precision=native.F64)
    _kernel(ctx, "pp")
    assert ctx.kernel_info(cfg)["kernel"] == "rows_pp"
    _kernel(ctx, "fast")
    assert ctx.kernel_info(cfg)["kernel"] == "rows_fast"
    ctx.reset_options()
    info = ctx.kernel_info(cfg)
    assert info["kernel"] == "rows_pp"      # the default
    # two slots of app[N+3] + c2v[e_pad+64] in one block per CU
    assert info["blocks_per_cu"] == 1 and 2 * 8 * (ctx.graph.N + 3) < info["lds_bytes"] <= 160 * 1024
    si = ctx.row_sched_info(cfg)
    assert si["lds_bytes"] == info["lds_bytes"] and si["blocks_per_cu"] == 1
    # PEG 504x1008 has M <= 512: one row per thread, the one-codeword kernel
    assert gpu_ctx_factory("PEGReg504x1008.alist").kernel_info(cfg)["kernel"] == "rows_fast"


@pytest.mark.gpu
@pytest.mark.parametrize("batch,T,v", [
    (2048, 50, dict(variant=1, alpha=1.25)),     # the bench configuration
    (1001, 50, dict(variant=0)),                 # odd batch: the last pair has one codeword
    (257, 7, dict(variant=2, delta=0.15)),
    (64, 1, dict(variant=1, alpha=1.1)),         # IEEE division (alpha not P*2^E)
    (3, 0, dict(variant=1, alpha=1.25)),         # no iteration: decisions of the channel
    (1, 13, dict(variant=0)),                    # one codeword, empty partner slot
])
def test_pp_equals_rows_fast_and_oracle(gpu_ctx_factory, batch, T, v):
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory(CODE)
    cfg = native.DecoderConfig(T=T, precision=native.F64, **v)
    _kernel(ctx, "fast")
    y0, d0, f0, c0 = ctx.sim_trace(1.5, 0.5, cfg, seed=77, stream_id=5, first_cw=123, batch=batch)
    _kernel(ctx, "pp")
    y1, d1, f1, c1 = ctx.sim_trace(1.5, 0.5, cfg, seed=77, stream_id=5, first_cw=123, batch=batch)
    assert ctx.redo_count() == 0
    assert np.array_equal(y0, y1)
    assert np.array_equal(d0, d1)
    assert np.array_equal(f0, f1)
    assert c0.as_dict() == c1.as_dict()
    n = min(batch, 256)
    want = O.Alist(code_path(CODE)).decode(y1[:n], T, O.Cfg(**v), workers=16)
    assert int((d1[:n] != want).sum()) == 0
    assert np.array_equal(f1["bit_err"][:n], (want != 1).sum(axis=1))


def _glibc_frames(N, nframes, ebn0, R, seed):
    g = O.GlibcRandom(seed)
    sigma = math.sqrt(10 ** (-ebn0 / 10) / R / 2)
    c = np.ones(N, dtype=np.int32)
    return np.stack([g.channel(c, sigma) for _ in range(nframes)])


@pytest.mark.gpu
@pytest.mark.parametrize("vname,v", [("nms", dict(variant=1, alpha=1.25)), ("ms", dict(variant=0)),
                                     ("oms", dict(variant=2, delta=0.15))])
def test_pp_premise_breaks_are_redecoded_exactly(gpu_ctx_factory, vname, v):
    """Frames 1-5 break the fast premise (|y| >= 2^1000, tiny minima, inf, NaN, growth
    past 2^1000); their pair partners (0, and the unbroken frames 6-9 sharing no pair
    with them) decode normally. Everything equals the fp64 oracle; the re-decode list
    holds the broken codewords only (not whole pairs)."""
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory(CODE)
    _kernel(ctx, "pp")
    N = ctx.graph.N
    y = _glibc_frames(N, 12, 1.5, 0.5, seed=4244)
    y[1] *= 1e305
    y[2] *= 1e-305
    y[3, 5] = np.inf
    y[4, 7] = np.nan
    y[5] *= 2.0 ** 995
    y[6, ::3] = -0.0
    y[7] = np.where(np.arange(N) % 2 == 0, 0.5, -1.0)
    A = O.Alist(code_path(CODE))
    for T in (1, 7, 30):
        cfg = native.DecoderConfig(T=T, precision=native.F64, **v)
        assert ctx.kernel_info(cfg)["kernel"] == "rows_pp"
        d, fr, cnt = ctx.decode(y, cfg)
        redo = ctx.redo_count()
        want = A.decode(y, T, O.Cfg(**v), workers=8)
        mism = (d != want).sum(axis=1)
        assert int(mism.sum()) == 0, f"T={T}: mismatching frames {np.nonzero(mism)[0].tolist()}"
        w = (want != 1).sum(axis=1)
        assert np.array_equal(fr["bit_err"], w)
        assert cnt.frames == len(y) and cnt.bit_err == int(w.sum()) and cnt.iters == T * len(y)
        assert 3 <= redo <= 5, redo      # frames 1, 3, 4 always; 2 (fast division) and 5 (growth) may


def _random_code(tmp_path, name, N, M, row_deg, seed):
    """A random code with the given row degrees (a list, one per row, sum >= N) in which
    every bit is in at least one check: the first N edge slots take a permutation of the
    bits, the rest random bits (redrawn on a duplicate within the row)."""
    from ldpcsimulation_amd import codes
    rng = np.random.default_rng(seed)
    assert sum(row_deg) >= N
    pool = list(rng.permutation(N)) + list(rng.integers(0, N, size=sum(row_deg) - N))
    rows, at = [], 0
    for j in range(M):
        r = []
        for _ in range(row_deg[j]):
            v = int(pool[at])
            at += 1
            while v in r:
                v = int(rng.integers(N))
            r.append(v)
        rows.append(sorted(r))
    path = str(tmp_path / name)
    codes.write_alist(codes.ParityCheck.from_rows(N, rows), path)
    return path


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["bench", "all_deg8", "low_deg"])
def test_pp_row_slot_layouts_equal_each_other_and_oracle(tmp_path, shape):
    """The degree-aware row slots (graph.h pp_row_slots: the younger check wave of each
    SIMD runs two 7-edge check nodes) and the plain slots give the same values: rows of
    a flooding iteration are independent (decodeMinSum.cpp:410-450), so moving them
    between waves, and running a degree-<=7 row through a 7-edge check node, changes
    nothing. Codes (M in 897..1024: 512 check threads, two rows each): the bench code
    (810 degree-7 and 162 degree-8 rows, split), 950 degree-8 rows (no split: only 256
    slots take degree 8), 950 rows of degree 4-6 (split; 7-edge check nodes with
    padding edges)."""
    from ldpcsimulation_amd import native
    if shape == "bench":
        path = code_path(CODE)
    elif shape == "all_deg8":
        path = _random_code(tmp_path, "d8.alist", 1900, 950, [8] * 950, seed=8)
    else:
        rng = np.random.default_rng(6)
        path = _random_code(tmp_path, "d46.alist", 1900, 950, rng.integers(4, 7, size=950).tolist(), seed=6)
    ctx = native.Context(native.Graph.from_alist(path), 0, 1024)
    cfg = native.DecoderConfig(variant=1, alpha=1.25, T=30, precision=native.F64)
    outs = {}
    for slots in ("plain", "split"):
        ctx.set_option("pp_slots", slots)
        assert ctx.kernel_info(cfg)["kernel"] == "rows_pp"
        outs[slots] = ctx.sim_trace(2.5, 0.5, cfg, seed=31, stream_id=2, first_cw=0, batch=515)
        assert ctx.redo_count() == 0
    ctx.set_option("pp_slots", "split")
    _kernel(ctx, "fast")
    outs["fast"] = ctx.sim_trace(2.5, 0.5, cfg, seed=31, stream_id=2, first_cw=0, batch=515)
    for k in ("split", "fast"):
        for a, b in zip(outs[k][:3], outs["plain"][:3]):
            assert np.array_equal(a, b), k
        assert outs[k][3].as_dict() == outs["plain"][3].as_dict(), k
    y, d = outs["split"][0], outs["split"][1]
    want = O.Alist(path).decode(y[:64], 30, O.Cfg(variant=1, alpha=1.25), workers=16)
    assert int((d[:64] != want).sum()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("batch,T,v", [
    (2048, 50, dict(variant=1, alpha=1.25)),     # the bench configuration
    (1003, 50, dict(variant=0)),                 # batch 1003 = 250 steps of 4 + 3: the last step's partner missing
    (2, 7, dict(variant=1, alpha=1.25)),         # one pair, the other slot empty
    (5, 0, dict(variant=0)),                     # no iteration
])
def test_pp_fp32_pairs_equal_row_kernel_and_oracle(gpu_ctx_factory, batch, T, v):
    """fp32 pairs on the ping-pong kernel (the fp32 default: two float2 slots, four codewords
    per block step) give the fp32 row kernel's channel, decisions, per-frame results and
    counters, and the fp32 oracle's decisions (decodeMinSum.cpp:410-476 in float)."""
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory(CODE)
    cfg = native.DecoderConfig(T=T, precision=native.F32, **v)
    ctx.set_option("rows32", "rows")
    assert ctx.kernel_info(cfg)["kernel"] == "rows"
    y0, d0, f0, c0 = ctx.sim_trace(1.5, 0.5, cfg, seed=78, stream_id=6, first_cw=321, batch=batch)
    ctx.set_option("rows32", "pp")                    # the fp32 default
    assert ctx.kernel_info(cfg)["kernel"] == "rows_pp"
    y1, d1, f1, c1 = ctx.sim_trace(1.5, 0.5, cfg, seed=78, stream_id=6, first_cw=321, batch=batch)
    assert ctx.redo_count() == 0
    assert np.array_equal(y0, y1) and np.array_equal(d0, d1) and np.array_equal(f0, f1)
    assert c0.as_dict() == c1.as_dict()
    n = min(batch, 128)
    want = O.Alist(code_path(CODE)).decode(y1[:n], T, O.Cfg(**v), workers=16)
    assert int((d1[:n] != want).sum()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("vname,v", [("nms", dict(variant=1, alpha=1.25)), ("ms", dict(variant=0))])
def test_pp_fp32_premise_breaks_are_redecoded_exactly(gpu_ctx_factory, vname, v):
    """fp32 pairs: frames whose inputs or messages leave the fast premise (|y| >= 1e30,
    inf, NaN, growth past 1e30) hand their pair to the exact re-decode; every decision
    equals the fp32 oracle's and the other pair of the step is unaffected."""
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory(CODE)
    ctx.set_option("rows32", "pp")
    N = ctx.graph.N
    y = _glibc_frames(N, 12, 1.5, 0.5, seed=4245).astype(np.float32)
    y[1] *= np.float32(1e31)
    y[3, 5] = np.inf
    y[4, 7] = np.nan
    y[6, ::3] = -0.0
    y[9] *= np.float32(1e28)
    A = O.Alist(code_path(CODE))
    for T in (1, 7, 30):
        cfg = native.DecoderConfig(T=T, precision=native.F32, **v)
        assert ctx.kernel_info(cfg)["kernel"] == "rows_pp"
        d, fr, cnt = ctx.decode(y, cfg)
        want = A.decode(y, T, O.Cfg(**v), workers=8)
        mism = (d != want).sum(axis=1)
        assert int(mism.sum()) == 0, f"T={T}: mismatching frames {np.nonzero(mism)[0].tolist()}"
        assert np.array_equal(fr["bit_err"], (want != 1).sum(axis=1))
        assert cnt.frames == len(y) and cnt.iters == T * len(y)
        assert ctx.redo_count() >= 4        # the pairs of frames 1, 3, 4 (and 9 once it grows)


@pytest.mark.gpu
def test_environment_cannot_reroute_the_product(monkeypatch):
    """with every former kernel-choice variable set to a non-default
    value, a fresh context still decodes the bench configuration on rows_pp (fp64) with
    the degree-aware slots, and gives the same results as the same context after
    ldpc_ctx_set_option has switched it to rows_fast and back."""
    from test_abi import FORMER_KNOBS, KNOB_VALUES
    from ldpcsimulation_amd import native
    for k in FORMER_KNOBS:
        monkeypatch.setenv(k, KNOB_VALUES.get(k, "1"))
    ctx = native.Context(native.Graph.from_alist(code_path(CODE)), 0, 1024)
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=50, precision=native.F64)
    assert ctx.kernel_info(cfg)["kernel"] == "rows_pp"
    assert all(ctx.get_option(k) == 0 for k in native.OPTIONS if not k.startswith("ems"))
    cfg32 = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=50, precision=native.F32)
    assert ctx.kernel_info(cfg32)["kernel"] == "rows_pp"
    a = ctx.sim_trace(1.5, 0.5, cfg, seed=5, stream_id=0, first_cw=0, batch=512)
    ctx.set_option("rows64", "fast")
    assert ctx.kernel_info(cfg)["kernel"] == "rows_fast"
    b = ctx.sim_trace(1.5, 0.5, cfg, seed=5, stream_id=0, first_cw=0, batch=512)
    ctx.set_option("rows64", "pp")
    assert ctx.kernel_info(cfg)["kernel"] == "rows_pp"
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y)
    assert a[3].as_dict() == b[3].as_dict()


@pytest.mark.gpu
def test_binary_context_refuses_ems_options_and_orders_stream_changes():
    """the EMS options (20, 21) belong to the nb context, so the binary context
    refuses them; reset_options skips them by name. A stream change orders the context's
    next launch after the previous stream's work (ldpc_ctx_set_stream's event), so two
    async launches of one context on two streams give the same counts as one stream."""
    import torch
    from ldpcsimulation_amd import native
    ctx = native.Context(native.Graph.from_alist(code_path(CODE)), 0, 4096)
    for name in native.EMS_OPTIONS:
        with pytest.raises(native.LdpcError):
            ctx.set_option(name, 0)
    ctx.reset_options()
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=50, precision=native.F64)
    ref = ctx.sim_batch(1.5, 0.5, cfg, seed=11, stream_id=0, first_cw=0, batch=4096)[1]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    ctx.read_counts(reset=True)
    ctx.set_stream(s1.cuda_stream)
    ctx.sim_launch(1.5, 0.5, cfg, seed=11, stream_id=0, first_cw=0, batch=2048)
    ctx.set_stream(s2.cuda_stream)
    ctx.sim_launch(1.5, 0.5, cfg, seed=11, stream_id=0, first_cw=2048, batch=2048)
    ctx.synchronize()
    ctx.set_stream(None)
    got = ctx.read_counts(reset=True)
    assert got.as_dict() == ref.as_dict()
    # the GDBF rows kernel hands out codewords from the context's ticket word (cleared per
    # launch): more codewords than one grid, two launches on two streams
    gcfg = native.GdbfConfig(T=60)
    gref = ctx.gdbf_sim_batch(3.5, 0.5, gcfg, seed=3, stream_id=0, first_cw=0, batch=4096)[1]
    ctx.read_counts(reset=True)
    ctx.set_stream(s1.cuda_stream)
    ctx.gdbf_sim_launch(3.5, 0.5, gcfg, seed=3, stream_id=0, first_cw=0, batch=2048)
    ctx.set_stream(s2.cuda_stream)
    ctx.gdbf_sim_launch(3.5, 0.5, gcfg, seed=3, stream_id=0, first_cw=2048, batch=2048)
    ctx.synchronize()
    ctx.set_stream(None)
    assert ctx.read_counts(reset=True).as_dict() == gref.as_dict()


@pytest.mark.gpu
@pytest.mark.parametrize("prec,batch", [("f64", 4096), ("f64", 1001), ("f32", 4096), ("f32", 1003)])
def test_pp_channel_fast_step_equals_general_loop(gpu_ctx_factory, prec, batch):
    """The channel's straight-line common step (rows_pp.hip pp_channel: all codewords of the
    step in the batch, no codeword table, no front end, no sample output) gives the general
    loop's values: sim_batch takes the fast step, sim_trace (which writes the samples) the
    general loop, on the same seed -- per-frame results, counters and the re-decode list
    identical; a ragged batch runs its last step on the general loop in both."""
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory(CODE)
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=20,
                               precision=native.F64 if prec == "f64" else native.F32)
    assert ctx.kernel_info(cfg)["kernel"] == "rows_pp"
    f_fast, c_fast = ctx.sim_batch(1.25, 0.5, cfg, seed=5150, stream_id=2, first_cw=999, batch=batch)
    r_fast = ctx.redo_count()
    y, d, f_gen, c_gen = ctx.sim_trace(1.25, 0.5, cfg, seed=5150, stream_id=2, first_cw=999, batch=batch)
    assert np.array_equal(f_fast, f_gen)
    assert c_fast.as_dict() == c_gen.as_dict() and r_fast == ctx.redo_count() == 0
    assert c_gen.frame_err > 0 and c_gen.uncoded_bit_err > 0
