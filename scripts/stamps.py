#!/usr/bin/env python3
"""Summarise LDPC_STAMPS dumps: per launch, mean per-block cycles in each phase."""
import sys
import numpy as np
a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8192, 4)
for i, l in enumerate(a):
    used = l[l.sum(axis=1) > 0].astype(np.float64)
    tot = used.sum(axis=1)
    m = used.mean(axis=0)
    print(f"launch {i}: blocks={len(used)} mean cycles chan={m[0]:.3e} cn={m[1]:.3e} vn={m[2]:.3e} acct={m[3]:.3e} "
          f"| shares chan={m[0]/tot.mean():.3f} cn={m[1]/tot.mean():.3f} vn={m[2]/tot.mean():.3f} acct={m[3]/tot.mean():.3f}")
