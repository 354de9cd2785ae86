#!/usr/bin/env python3
"""Summarise LDPC_EMS_STAMPS dumps of the EMS kernel (nb.hip, -DLDPC_EMS_STAMPS):
per wave, s_memtime cycles per codeword and per iteration in each phase.
usage: ems_stamps.py DUMP [AVG_ITERS]"""
import sys
import numpy as np

names = ["channel+init", "check work", "check wait", "symbol work", "symbol wait", "syndrome", "accounting"]
a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 256, 16, 8).astype(np.float64)
iters = float(sys.argv[2]) if len(sys.argv) > 2 else None
for i, l in enumerate(a):
    used = l[l[:, 0, 7] > 0]
    cw = used[:, :, 7:8]
    per = (used[:, :, :7] / cw).mean(axis=(0, 1))
    tot = per.sum()
    print(f"launch {i}: blocks={len(used)} codewords/block={cw.mean():.1f} cycles/codeword {tot:.0f}")
    for n, v in zip(names, per):
        extra = f"  {v / iters:8.0f} per iteration" if iters and n not in ("channel+init", "accounting") else ""
        print(f"  {n:13s} {v:9.0f} ({100 * v / tot:5.1f} %){extra}")
