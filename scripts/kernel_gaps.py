#!/usr/bin/env python3
"""Launch-boundary gaps from a rocprofv3 --kernel-trace CSV: for consecutive
dispatches on one queue (sorted by start), gap = next start - previous end.
Prints, per kernel-name transition, the count and gap percentiles, and the
total busy vs idle time between the first and last dispatch matching PATTERN.
usage: kernel_gaps.py TRACE.csv [PATTERN] [--json OUT]"""
import csv
import json
import sys

import numpy as np


def short(n):
    n = n.split("(")[0]
    return n.replace("void ", "").replace("ldpc::", "")


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "flood"
    rows = [r for r in csv.DictReader(open(path))]
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]) for r in rows]
    rows.sort()
    sel = [i for i, r in enumerate(rows) if pat in r[2]]
    if not sel:
        sys.exit(f"no dispatch matches {pat}")
    lo, hi = sel[0], sel[-1]
    seg = rows[lo:hi + 1]
    busy = sum(e - s for s, e, _, _ in seg)
    span = seg[-1][1] - seg[0][0]
    trans = {}
    gaps = []
    for a, b in zip(seg, seg[1:]):
        g = b[0] - a[1]
        gaps.append(g)
        trans.setdefault(f"{a[2].split('<')[0]} -> {b[2].split('<')[0]}", []).append(g)
    gaps = np.array(gaps) / 1e3
    out = {"dispatches": len(seg), "span_us": span / 1e3, "busy_us": busy / 1e3, "idle_us": (span - busy) / 1e3,
           "busy_frac": busy / span,
           "gap_us_percentiles": {p: float(np.percentile(gaps, p)) for p in (5, 25, 50, 75, 95, 99)},
           "gap_us_mean": float(gaps.mean()),
           "histogram_us": dict(zip([f"{a:.0f}-{b:.0f}" for a, b in zip([0, 1, 2, 4, 8, 16, 32, 64], [1, 2, 4, 8, 16, 32, 64, 1e9])],
                                    np.histogram(gaps, bins=[-1e9, 1, 2, 4, 8, 16, 32, 64, 1e9])[0].tolist())),
           "by_transition": {k: {"n": len(v), "median_us": float(np.median(v) / 1e3), "mean_us": float(np.mean(v) / 1e3)}
                             for k, v in sorted(trans.items(), key=lambda kv: -len(kv[1]))},
           "kernel_us": {}}
    per = {}
    for s, e, n, _ in seg:
        per.setdefault(n.split("<")[0], []).append((e - s) / 1e3)
    out["kernel_us"] = {k: {"n": len(v), "mean_us": float(np.mean(v))} for k, v in per.items()}
    print(json.dumps(out, indent=1))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
