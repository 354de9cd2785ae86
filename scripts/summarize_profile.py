#!/usr/bin/env python3
"""Summarise a scripts/profile_round.sh output directory into profiles/.

Writes <name>_kernel_stats.csv (the rocprofv3 --stats table), <name>_pmc.json
(per-dispatch counter averages of the kernel whose name contains the
pattern argument; default "decode") and, for bench.py's
`roofline.traffic`, profiles/traffic_latest.json with the HBM bytes per launch:
FETCH_SIZE and WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE counts
wide coalesced reads at half their bytes (MI355X_MICROARCH.md, HBM), so the
read side is doubled (an upper bound for the narrow reads this kernel has).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def pmc_avgs(d, kernel_pat="decode"):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel_pat in r["Kernel_Name"]:
                vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {c: sum(v.values()) / len(v) for c, v in vals.items() if v}


def main(src, name, kernel_pat="decode", precision="f32", root="."):
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(src, "stats", "**", "*kernel_stats.csv"), recursive=True)
    out = {"source": src, "precision": precision}
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{name}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            if kernel_pat in r["Name"]:
                out["kernel"] = r["Name"]
                out["calls"] = int(r["Calls"])
                out["avg_ns"] = float(r["AverageNs"])
    pmc = {}
    for sub in ("fetch", "write", "sq", "sq2"):
        pmc.update(pmc_avgs(os.path.join(src, sub), kernel_pat))
    out["pmc_per_dispatch"] = pmc
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        out["hbm_bytes_per_launch"] = (2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024
        out["fetch_bytes_raw"] = pmc["FETCH_SIZE"] * 1024
        out["write_bytes"] = pmc["WRITE_SIZE"] * 1024
    if "GRBM_GUI_ACTIVE" in pmc and "avg_ns" in out:
        out["effective_clock_ghz"] = pmc["GRBM_GUI_ACTIVE"] / 8 / out["avg_ns"]
    json.dump(out, open(os.path.join(prof, f"{name}_pmc.json"), "w"), indent=1)
    if "hbm_bytes_per_launch" in out:
        tl = os.path.join(prof, "traffic_latest.json")
        try:
            latest = json.load(open(tl))
        except (OSError, ValueError):
            latest = {}
        if "hbm_bytes_per_launch" in latest:   # pre-round-2 single-entry form (fp32)
            latest = {latest.get("precision", "f32"): latest}
        latest[precision] = {"hbm_bytes_per_launch": out["hbm_bytes_per_launch"], "source": f"profiles/{name}_pmc.json",
                             "kernel": out.get("kernel"), "precision": precision}
        json.dump(latest, open(tl, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
