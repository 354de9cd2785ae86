#!/usr/bin/env python3
"""Ping-pong kernel (rows_pp.hip) against k_rows_fast and the fp64 oracle on the
bench code: same Philox channel, decisions/per-frame results/counters equal."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401  (one HIP runtime: torch first)
from ldpcsimulation_amd import codes, native  # noqa: E402
from oracle import oracle as O  # noqa: E402

path = codes.ensure_80211n_1944()
g = native.Graph.from_alist(path)
ctx = native.Context(g, 0, 4096)
bad = 0
for batch, T, vk in ((2048, 50, dict(variant=native.NMS, alpha=1.25)), (257, 7, dict(variant=native.MS)),
                     (33, 1, dict(variant=native.OMS, delta=0.15)), (5, 0, dict(variant=native.NMS, alpha=1.1))):
    cfg = native.DecoderConfig(T=T, precision=native.F64, **vk)
    os.environ["LDPC_ROWS"] = "fast"
    y0, d0, f0, c0 = ctx.sim_trace(1.5, 0.5, cfg, seed=99, stream_id=3, first_cw=0, batch=batch)
    os.environ["LDPC_ROWS"] = "pp"
    assert ctx.kernel_info(cfg)["kernel"] == "rows_pp", ctx.kernel_info(cfg)
    y1, d1, f1, c1 = ctx.sim_trace(1.5, 0.5, cfg, seed=99, stream_id=3, first_cw=0, batch=batch)
    ok = np.array_equal(y0, y1) and np.array_equal(d0, d1) and np.array_equal(f0, f1) and c0.as_dict() == c1.as_dict()
    print(f"batch={batch} T={T} {vk}: pp == fast: {ok}; counts {c1.as_dict()} redo {ctx.redo_count()}", flush=True)
    if batch <= 257:
        want = O.Alist(path).decode(y1, T, O.Cfg(**{k: v for k, v in vk.items()}), workers=16)
        m = int((d1 != want).sum())
        print(f"   vs oracle: {m} differing decisions", flush=True)
        bad += m
    bad += 0 if ok else 1
print("PP_CHECK", "OK" if bad == 0 else f"FAIL {bad}")
sys.exit(1 if bad else 0)
