#!/usr/bin/env python3
"""Phase-per-launch flooding (LDPC_FLOOD_MODE=phase) against the persistent
flood kernel on DVB-S2: identical decisions on the same on-device channel, and
the decode rate of both. Usage: LDPC_FLOOD_MODE=phase python flood_phase_check.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np  # noqa: E402

from conftest import code_path  # noqa: E402
from ldpcsimulation_amd import native  # noqa: E402


def main():
    g = native.Graph.from_alist(code_path("dvbs2_1_2.alist"))
    B = int(os.environ.get("BATCH", "2048"))
    ctx = native.Context(g, 0, B)
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=int(os.environ.get("T", "50")),
                               precision=native.F64 if os.environ.get("PREC", "f32") == "f64" else native.F32)
    print("mode", os.environ.get("LDPC_FLOOD_MODE", "persistent"), ctx.kernel_info(cfg), flush=True)
    y, d, fr, cnt = ctx.sim_trace(1.0, 0.5, cfg, seed=3, stream_id=0, first_cw=0, batch=64)
    np.save(os.path.join(os.environ.get("OUT", "gpurun_out"), f"flood_d_{os.environ.get('LDPC_FLOOD_MODE', 'p')}.npy"), d)
    print("trace frame_err", cnt.frame_err, "bit_err", cnt.bit_err, flush=True)
    ctx.sim_batch(1.0, 0.5, cfg, seed=1, stream_id=0, first_cw=0, batch=B, want_frames=False)
    for r in range(2):
        t0 = time.perf_counter()
        _, cnt = ctx.sim_batch(1.0, 0.5, cfg, seed=1, stream_id=0, first_cw=(r + 1) * B, batch=B, want_frames=False)
        dt = time.perf_counter() - t0
        print(f"batch {B}: {dt * 1e3:.1f} ms  {g.N * B / dt / 1e6:.1f} Mbit/s  FER {cnt.frame_err}/{cnt.frames}",
              flush=True)


if __name__ == "__main__":
    main()
