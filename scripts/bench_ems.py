#!/usr/bin/env python3
"""Throughput of the GF(16) EMS decoder (BASELINE config 5): fused on-device
AWGN -> EMS -> error count over a batch, one MI355X. Prints one JSON line.

    python scripts/bench_ems.py [--batch B --T T --nm NM --ebn0 E --steps K]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=16384)
    p.add_argument("--T", type=int, default=20)
    p.add_argument("--nm", type=int, default=16)
    p.add_argument("--offset", type=float, default=0.0)
    p.add_argument("--ebn0", type=float, nargs="+", default=[1.5, 2.0])
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--no-early-stop", action="store_true")
    p.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                   help="an EMS option of the context (ems_threads, ems_swizzle), A/B only")
    p.add_argument("--lib", default=None, help="another build of the decoder library (A/B only)")
    a = p.parse_args()
    from ldpcsimulation_amd import codes, native
    if a.lib:
        native.use_library(os.path.abspath(a.lib))
    g = native.NbGraph.from_alist(codes.ensure_gf16_code())
    ctx = native.NbContext(g, 0, a.batch)
    for o in a.option:
        k, _, v = o.partition("=")
        ctx.set_option(k, int(v) if v.isdigit() else v)
    cfg = native.EmsConfig(T=a.T, nm=a.nm, offset=a.offset, early_stop=not a.no_early_stop)
    for ebn0 in a.ebn0:
        ctx.sim_batch(ebn0, 0.5, cfg, seed=1, stream_id=0, first_cw=0, batch=min(a.batch, 1024))   # warm-up
        ctx.read_counts(reset=True)
        kms = []
        t0 = time.perf_counter()
        for k in range(a.steps):
            ctx.sim_launch(ebn0, 0.5, cfg, seed=1, stream_id=0, first_cw=k * a.batch, batch=a.batch)
            kms.append(ctx.last_kernel_ms())
        wall = time.perf_counter() - t0
        c = ctx.read_counts(reset=True)
        bits = c.frames * g.N * g.m
        print(json.dumps({"code": "gf16_N1000_dv2_dc4 (N=1000 GF(16) symbols, 4000 bits, R=1/2)",
                          "ebn0_db": ebn0, "T_max": a.T, "nm": a.nm, "offset": a.offset,
                          "early_stop": cfg.early_stop, "batch": a.batch, "steps": a.steps,
                          "kernel": ctx.kernel_info(), "kernel_ms": sum(kms) / len(kms),
                          "coded_mbit_s_kernel": bits / (sum(kms) / 1e3) / 1e6,
                          "coded_mbit_s_wall": bits / wall / 1e6,
                          "fer": c.frame_err / c.frames, "ber": c.bit_err / bits,
                          "avg_iters": c.iters / c.frames, "frames": c.frames}), flush=True)


if __name__ == "__main__":
    main()
