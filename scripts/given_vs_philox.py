#!/usr/bin/env python3
"""Kernel time of the row kernel fed device-resident channel samples (SRC_GIVEN)
vs the fused on-device Philox channel (SRC_PHILOX), N=1944 NMS 1.25 T=50, 65536
codewords, fp64 and fp32. Tells whether generating the channel inside the decode
kernel costs more than a separate pass would."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from ldpcsimulation_amd import codes, native  # noqa: E402


def main():
    g = native.Graph.from_alist(codes.ensure_80211n_1944())
    B = 65536
    ctx = native.Context(g, 0, B)
    for prec, dt in (("f64", torch.float64), ("f32", torch.float32)):
        cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=50,
                                   precision=native.F64 if prec == "f64" else native.F32)
        sigma = (10 ** (-1.5 / 10) / 0.5 / 2) ** 0.5
        y = (1 + sigma * torch.randn((B, g.N), dtype=torch.float64, device="cuda")).to(dt)
        frames = torch.empty((B, 4), dtype=torch.int32, device="cuda")
        res = {}
        for name in ("given", "philox", "given", "philox"):
            ms = []
            for r in range(3):
                if name == "given":
                    ctx.decode(y, cfg, want_decisions=False, want_frames=False)
                else:
                    ctx.sim_launch(1.5, 0.5, cfg, 5, 0, r * B, B, frames)
                    ctx.synchronize()
                ms.append(ctx.last_kernel_ms())
            res.setdefault(name, []).extend(ms)
        print(prec, {k: round(min(v), 3) for k, v in res.items()}, "ms (min of 6)", flush=True)


if __name__ == "__main__":
    main()
