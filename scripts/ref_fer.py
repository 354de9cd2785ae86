#!/usr/bin/env python3
"""Pin the reference's FER tightly: run the reference's own
decodeNMS (oracle/_ref, built from the unmodified sources by oracle/Makefile.ref)
on the 802.11n N=1944 R1/2 code, NMS alpha=1.25, T=50, at the SURVEY §8(d) SNR
points, over many REF_SEEDs. Each run ends by the reference's stop rule
(decodeMinSum.cpp:189: >= 200 bit errors and >= 40 frame errors), so every seed
contributes >= 40 frame errors; 10 seeds give >= 400 per point.

Writes tests/golden/reference_fer.json: per point the per-seed
(frame errors, frames, bit errors, uncoded errors) and the totals.
Build container only (needs oracle/_ref); the result is a committed fixture.

    python scripts/ref_fer.py [--seeds 10] [--jobs 8]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
POINTS = [1.0, 1.25, 1.5, 1.75]


def run_one(ref, alist, snr, seed, T, alpha):
    with tempfile.TemporaryDirectory() as td:
        t0 = time.perf_counter()
        out = subprocess.run([ref, alist, "0.5", str(snr), str(T), str(alpha), os.path.join(td, "log.txt")],
                             env=dict(os.environ, REF_SEED=str(seed)), capture_output=True, text=True,
                             check=True).stdout
        wall = time.perf_counter() - t0
    final = [l for l in out.splitlines() if l.startswith("Final result:")][0]
    m = re.match(r"Final result: (\d+) bit errs in (\d+) words.*Uncoded errors = (\d+)", final)
    bits, words, unc = (int(x) for x in m.groups())
    ferr = sum(1 for l in out.splitlines() if re.match(r"Ferr with \d+ errors", l))
    return {"seed": seed, "frame_err": ferr, "frames": words, "bit_err": bits, "uncoded_bit_err": unc,
            "wall_s": round(wall, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=10)
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "reference_fer.json"))
    args = ap.parse_args()
    from ldpcsimulation_amd import codes
    alist = codes.ensure_80211n_1944()
    ref = os.path.join(ROOT, "oracle", "_ref", "decodeNMS")
    if not os.path.exists(ref):
        sys.exit("oracle/_ref/decodeNMS missing: make ref")
    T, alpha = 50, 1.25
    jobs = [(snr, 1000 + 17 * k + int(snr * 100)) for snr in POINTS for k in range(args.seeds)]
    with ThreadPoolExecutor(args.jobs) as ex:
        res = list(ex.map(lambda j: (j[0], run_one(ref, alist, j[0], j[1], T, alpha)), jobs))
    out = {"binary": "oracle/_ref/decodeNMS (unmodified reference sources, g++ -O2, REF_SEED via --wrap=time)",
           "code": "80211n_1944_r12.alist", "R": 0.5, "T": T, "alpha": alpha,
           "stop_rule": "decodeMinSum.cpp:189 (>= 200 bit errors and >= 40 frame errors per run)",
           "points": []}
    for snr in POINTS:
        runs = [r for s, r in res if s == snr]
        tot = {k: sum(r[k] for r in runs) for k in ("frame_err", "frames", "bit_err", "uncoded_bit_err")}
        out["points"].append({"ebn0_db": snr, "runs": runs, **tot, "fer": tot["frame_err"] / tot["frames"]})
        print(f"{snr} dB: {tot['frame_err']}/{tot['frames']} = {tot['frame_err'] / tot['frames']:.4e}", flush=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
