#!/usr/bin/env python3
"""Summarise scripts/pmc_config3.sh output for one schedule: per decode launch, the
counters summed over every dispatch of the decoder's kernels (the flooding path is
several phase kernels per launch: init, T x (check, bit), finish, accounting), the
kernel-trace time per launch, and the fractions against the fp64 byte models.

Byte models per codeword-iteration (DVB-S2 R1/2: N = 64800, E = 226799):
  flooding, SURVEY 8(d)'s message model at fp64: the check phase reads E v2c and
    writes E c2v, the bit phase reads N y + E c2v and writes E v2c:
    32 E + 8 N bytes (2 x the fp32 16 E + 4 N);
  measured: FETCH_SIZE x 2 + WRITE_SIZE (KiB; gfx950 counts wide reads at half,
    MI355X_MICROARCH HBM section), i.e. the bytes between L2 and the fabric
    (Infinity Cache hits included: the MALL sits behind the fabric).

usage: summarize_config3.py DIR SCHED OUT_JSON [LAUNCHES] [BATCH]
  DIR/SCHED/{stats,p1..p5}: LAUNCHES decode launches each (default 2: warm-up + 1)."""
import collections
import csv
import glob
import json
import os
import sys

N, E, T = 64800, 226799, 50
HBM_PEAK = 8.0e12


def main(src, sched, out, launches=2, batch=2048):
    launches, batch = int(launches), int(batch)
    d = os.path.join(src, sched)
    tot = collections.defaultdict(float)
    names = set()
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_flood" in k or "k_decode_layered" in k or "k_decode_flood" in k or "k_decode_global" in k:
                names.add(k.split("(")[0])
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    pmc = {k: v / launches for k, v in tot.items()}
    stats = []
    ns = 0.0
    for f in glob.glob(os.path.join(d, "stats", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_flood" in r["Name"] or "k_decode_" in r["Name"]:
                stats.append({"name": r["Name"].split("(")[0], "calls": int(r["Calls"]),
                              "avg_ns": float(r["AverageNs"]), "total_ns": float(r["TotalDurationNs"])})
                ns += float(r["TotalDurationNs"])
    t_launch = ns / launches / 1e9 if ns else None
    der = {}
    if t_launch:
        der["kernel_s_per_launch"] = t_launch
        der["mbit_s_kernel_time"] = batch * N / t_launch / 1e6
    model = (32 * E + 8 * N) * T * batch
    der["model_bytes_per_launch_fp64"] = model
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        meas = (2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024
        der["measured_bytes_per_launch"] = meas
        der["measured_over_model"] = meas / model
        if t_launch:
            der["measured_gbs"] = meas / t_launch / 1e9
            der["measured_frac_hbm_peak"] = meas / t_launch / HBM_PEAK
            der["model_gbs"] = model / t_launch / 1e9
            der["model_frac_hbm_peak"] = model / t_launch / HBM_PEAK
    if "TCC_HIT_sum" in pmc and "TCC_MISS_sum" in pmc:
        der["l2_hit_rate"] = pmc["TCC_HIT_sum"] / max(1.0, pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"])
    if "SQ_WAIT_ANY" in pmc and "SQ_WAVE_CYCLES" in pmc:
        der["wait_any_frac"] = pmc["SQ_WAIT_ANY"] / pmc["SQ_WAVE_CYCLES"]
    if "SQ_ACTIVE_INST_VALU" in pmc and "SQ_WAVE_CYCLES" in pmc:
        der["active_valu_frac_of_wave_cycles"] = pmc["SQ_ACTIVE_INST_VALU"] / pmc["SQ_WAVE_CYCLES"]
    if "GRBM_GUI_ACTIVE" in pmc:
        der["gpu_cycles_per_launch"] = pmc["GRBM_GUI_ACTIVE"] / 8   # summed over the 8 XCDs
        if "SQ_INSTS_VALU" in pmc:
            der["valu_per_cu_cycle"] = pmc["SQ_INSTS_VALU"] / 256 / der["gpu_cycles_per_launch"]
    res = {"source": d, "schedule": sched, "precision": "f64", "batch": batch, "T": T,
           "launches_profiled": launches, "kernels": sorted(names), "kernel_trace": stats,
           "pmc_per_launch": pmc, "derived": der,
           "note": "DVB-S2 N=64800 R1/2 NMS alpha=1.25 T=50 fp64, 1.0 dB; counters summed over all decoder "
                   "dispatches of a launch; FETCH_SIZE/WRITE_SIZE in KiB"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(der, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
