#!/usr/bin/env python3
"""Summarise the layered kernel's per-wave phase stamps (a -DLDPC_STAMPS build, LayStamps
in kernels.hip): the last launch's record of $LDPC_STAMPS, averaged over the launch's blocks.

usage: lay_stamps.py STAMPS_BIN
"""
import sys

import numpy as np

NAMES = ["schedule loads", "gathers + state", "check rule", "scatter drain", "layer barrier",
         "channel, init, decisions", "scatter issue"]


def main():
    raw = np.fromfile(sys.argv[1], dtype=np.uint64)
    rec = raw[-8192 * 4:].reshape(256, 16, 8).astype(np.float64)
    rec = rec[rec[:, :, 7].sum(axis=1) > 0]          # the launch's blocks (the grid may be < 256)
    nb = len(rec)
    print(f"blocks: {nb}")
    tot = rec[:, :, :7].sum(axis=2)                 # cycles per wave over the launch
    passes = rec[:, :, 7]
    print(f"cycles per wave (mean over blocks and waves): {tot.mean():.0f}; passes per wave {passes.mean():.1f}")
    for k, n in enumerate(NAMES):
        frac = rec[:, :, k].sum() / tot.sum()
        per = rec[:, :, k].sum() / max(passes.sum(), 1.0)
        print(f"  {n:24s} {frac * 100:5.1f} %   {per:8.0f} cycles per pass")
    for w0 in (0, 4, 8, 12):
        sl = rec[:, w0:w0 + 4, :]
        p = sl[:, :, 7].sum()
        print(f"  waves {w0:2d}-{w0 + 3:2d}: passes {p / (4 * nb):.1f}/wave, per pass " +
              " ".join(f"{sl[:, :, k].sum() / max(p, 1):7.0f}" for k in (0, 1, 2, 6, 3)) +
              f"  barrier/wave {sl[:, :, 4].sum() / (4 * nb):.0f}")


if __name__ == "__main__":
    main()
