#!/usr/bin/env python3
"""Ping-pong kernel (rows_pp.hip) against the other row kernels and the oracle on the
bench code: same Philox channel, decisions/per-frame results/counters equal.
fp64: pp vs k_rows_fast (option rows64 = fast); fp32 pairs: pp vs the row kernel
(rows32 = rows) and the pair instance of k_rows_fast (rows32 = fast).
usage: pp_check.py [--lib ab/libldpc_hip_NAME.so]   (a variant build under A/B)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401  (one HIP runtime: torch first)
from ldpcsimulation_amd import codes, native  # noqa: E402
from oracle import oracle as O  # noqa: E402

if len(sys.argv) > 2 and sys.argv[1] == "--lib":
    native.use_library(os.path.abspath(sys.argv[2]))

path = codes.ensure_80211n_1944()
g = native.Graph.from_alist(path)
ctx = native.Context(g, 0, 4096)
bad = 0
CASES = ((2048, 50, dict(variant=native.NMS, alpha=1.25)), (257, 7, dict(variant=native.MS)),
         (33, 1, dict(variant=native.OMS, delta=0.15)), (5, 0, dict(variant=native.NMS, alpha=1.1)),
         (4095, 50, dict(variant=native.NMS, alpha=1.25)), (6, 3, dict(variant=native.MS)))
for prec in (native.F64, native.F32):
    for batch, T, vk in CASES:
        cfg = native.DecoderConfig(T=T, precision=prec, **vk)
        arms = {"f64": [("fast", dict(rows64="fast")), ("pp", {})],
                "f32": [("rows", dict(rows32="rows")), ("fast32", dict(rows32="fast")), ("pp", {})]}
        res = {}
        for name, opts in arms["f64" if prec == native.F64 else "f32"]:
            ctx.reset_options()
            ctx.set_options(opts)
            kern = ctx.kernel_info(cfg)["kernel"]
            res[name] = (kern, ctx.sim_trace(1.5, 0.5, cfg, seed=99, stream_id=3, first_cw=0, batch=batch),
                         ctx.redo_count())
        ref_name = next(iter(res))
        y0, d0, f0, c0 = res[ref_name][1]
        for name, (kern, (y1, d1, f1, c1), redo) in res.items():
            ok = np.array_equal(y0, y1) and np.array_equal(d0, d1) and np.array_equal(f0, f1) and \
                c0.as_dict() == c1.as_dict()
            print(f"{'f64' if prec == native.F64 else 'f32'} batch={batch} T={T} {vk}: {name} ({kern}) == "
                  f"{ref_name}: {ok}; redo {redo}", flush=True)
            bad += 0 if ok else 1
        if batch <= 257:
            want = O.Alist(path).decode(y0, T, O.Cfg(**vk), workers=16)
            m = int((d0 != want).sum())
            print(f"   vs oracle: {m} differing decisions", flush=True)
            bad += m
print("PP_CHECK", "OK" if bad == 0 else f"FAIL {bad}")
sys.exit(1 if bad else 0)
