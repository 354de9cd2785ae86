#!/usr/bin/env python3
"""Summarise LDPC_STAMPS dumps of the ping-pong kernel (rows_pp.hip, -DLDPC_STAMPS):
per role, s_memtime cycles per barrier interval spent working and waiting.
usage: pp_stamps.py DUMP INTERVALS_PER_BLOCK [STEPS_PER_BLOCK]"""
import sys
import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8192 * 4)
iv = float(sys.argv[2])
for i, l in enumerate(a):
    s = l[: 256 * 16 * 2].reshape(256, 16, 2).astype(np.float64)
    used = s[s[:, :, 0].sum(axis=1) > 0]
    for name, w in (("check 0-3", slice(0, 4)), ("check 4-7", slice(4, 8)), ("bit 8-11", slice(8, 12)),
                    ("bit 12-15", slice(12, 16))):
        work = used[:, w, 0] / iv
        wait = used[:, w, 1] / iv
        print(f"launch {i} {name:9s}: blocks={len(used)} work {work.mean():7.1f} (min {work.min():7.1f} max "
              f"{work.max():7.1f})  wait {wait.mean():7.1f}  cycles/interval")
    # per step (kernels that record them): syndrome + decisions (last interval barrier ->
    # the block accounting), the accounting (-> next step top), channel (top -> B1), B1 wait,
    # yq staging (B1 -> B2), B2 wait
    st = l[8192: 8192 + 256 * 16 * 6].reshape(256, 16, 6).astype(np.float64)
    if st.sum() > 0 and len(sys.argv) > 3:
        steps = float(sys.argv[3])
        st = st[s[:, :, 0].sum(axis=1) > 0]
        for name, w in (("check 0-3", slice(0, 4)), ("check 4-7", slice(4, 8)), ("bit 8-11", slice(8, 12)),
                        ("bit 12-15", slice(12, 16))):
            m = [st[:, w, k].mean() / steps for k in range(6)]
            print(f"launch {i} {name:9s}: syndrome+decisions {m[5]:7.1f}  accounting {m[0]:7.1f}  channel {m[1]:7.1f}  "
                  f"B1 wait {m[2]:7.1f}  staging {m[3]:7.1f}  B2 wait {m[4]:7.1f}  cycles/step")
