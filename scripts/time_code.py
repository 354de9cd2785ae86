#!/usr/bin/env python3
"""Time the fused on-device simulation for one code: decoded Mbit/s and the kernel chosen.

usage: time_code.py ALIST [--batch B] [--T T] [--snr DB] [--variant ms|nms|oms] [--prec f32|f64] [--reps R]
                    [--schedule flooding|layered]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ldpcsimulation_amd import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("alist")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--T", type=int, default=50)
    ap.add_argument("--snr", type=float, default=1.0)
    ap.add_argument("--rate", type=float, default=0.5)
    ap.add_argument("--variant", default="nms")
    ap.add_argument("--prec", default="f32")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--schedule", choices=["flooding", "layered"], default="flooding")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="a kernel-choice option of the context (native.OPTIONS), A/B only")
    ap.add_argument("--lib", default=None, help="another build of the decoder library (A/B only)")
    ap.add_argument("--decoder", choices=["minsum", "gdbf"], default="minsum",
                    help="gdbf: SMNGDBF (theta -0.6, eta 0.75, lambda 0.99, w 0.8, window 16, Ymax 2.5)")
    a = ap.parse_args()
    if a.lib:
        native.use_library(os.path.abspath(a.lib))
    g = native.Graph.from_alist(a.alist)
    ctx = native.Context(g, 0, a.batch)
    for o in a.option:
        k, _, v = o.partition("=")
        ctx.set_option(k, int(v) if v.isdigit() else v)
    v = {"ms": dict(variant=native.MS), "nms": dict(variant=native.NMS, alpha=1.25),
         "oms": dict(variant=native.OMS, delta=0.15), "bp": dict(variant=native.BP)}[a.variant]
    cfg = native.DecoderConfig(T=a.T, precision=native.F32 if a.prec == "f32" else native.F64,
                               schedule=native.LAYERED if a.schedule == "layered" else native.FLOODING, **v)
    if a.decoder == "gdbf":
        cfg = native.GdbfConfig(T=a.T, precision=cfg.precision)
        info = ctx.gdbf_kernel_info(cfg)
        run = ctx.gdbf_sim_batch
    else:
        info = ctx.kernel_info(cfg)
        run = ctx.sim_batch
    run(a.snr, a.rate, cfg, seed=1, stream_id=0, first_cw=0, batch=a.batch)   # warm-up
    best = 1e30
    for r in range(a.reps):
        t0 = time.perf_counter()
        _, cnt = run(a.snr, a.rate, cfg, seed=1, stream_id=0, first_cw=(r + 1) * a.batch, batch=a.batch)
        dt = time.perf_counter() - t0
        best = min(best, dt)
    mbit = g.N * a.batch / best / 1e6
    print(f"{os.path.basename(a.alist)} N={g.N} batch={a.batch} T={a.T} {a.variant}/{a.prec}: "
          f"{a.decoder}/{a.schedule} {best*1e3:.1f} ms/batch  {mbit:.1f} Mbit/s  kernel={info}  last FER={cnt.frame_err}/{cnt.frames}  avg it={cnt.iters / cnt.frames:.2f}")


if __name__ == "__main__":
    main()
