#!/usr/bin/env python3
"""BASELINE config 3 measured as a config: the DVB-S2 N=64800
R1/2 SNR sweep with the layered NMS decoder on one GPU, as the reference runs it
(one point after the other to its stop rule, scripts/minsum_example_*.sh:23-26,
decodeMinSum.cpp:189), in fp64 and fp32.

Per point: the sweep's own wall-clock rates (sweep.py --json, over the whole point,
rounds, host reduction and launches included): frames_decoded*N/seconds (every frame
the GPUs decoded, the rounds past the stop included) and frames*N/seconds (the
frames the stop rule counts), the kernel
rate of the same decoder on full 2,048-codeword batches (best of 3), the driver
overhead between the two, and the layered kernel's algorithmic traffic rate
against the Infinity-Cache gather rate of MI355X_MICROARCH (8.6 TB/s, 38 MB table
of random rows): per codeword-iteration every row gathers and scatters its dc
posteriors and reads and writes its packed state (m1, m2, meta):
fp64 16 E + 40 M bytes, fp32 8 E + 24 M bytes.
usage: config3_sweep.py [OUT.jsonl]"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import code_path  # noqa: E402

SNRS = [0.9, 1.0, 1.1, 1.2, 1.3]
IC_GATHER = 8.6e12


def kernel_rate(prec, snr, batch=2048, T=50, reps=3):
    import torch  # noqa: F401  (one HIP runtime)
    from ldpcsimulation_amd import native
    g = native.Graph.from_alist(code_path("dvbs2_1_2.alist"))
    ctx = native.Context(g, 0, batch)
    cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=T, schedule=native.LAYERED,
                               precision=native.F64 if prec == "f64" else native.F32)
    ctx.sim_batch(snr, 0.5, cfg, seed=1, stream_id=9, first_cw=0, batch=batch, want_frames=False)
    best = 1e30
    for r in range(reps):
        t0 = time.perf_counter()
        ctx.sim_batch(snr, 0.5, cfg, seed=1, stream_id=9, first_cw=(r + 1) * batch, batch=batch, want_frames=False)
        best = min(best, time.perf_counter() - t0)
    bpci = (16 * g.E + 40 * g.M) if prec == "f64" else (8 * g.E + 24 * g.M)
    return {"kernel": ctx.kernel_info(cfg), "ms_per_batch": best * 1e3, "kernel_mbit_s": g.N * batch / best / 1e6,
            "bytes_per_codeword_iter": bpci, "achieved_tb_s": bpci * batch * T / best / 1e12,
            "frac_of_ic_gather": bpci * batch * T / best / IC_GATHER, "N": g.N, "E": g.E, "M": g.M}


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "config3.jsonl")
    lines = []
    for prec in ("f64", "f32"):
        t0 = time.perf_counter()
        p = subprocess.run([sys.executable, "-m", "ldpcsimulation_amd.sweep", code_path("dvbs2_1_2.alist"),
                            "--rate", "0.5", "--snr"] + [str(s) for s in SNRS] +
                           ["-T", "50", "--variant", "nms", "--alpha", "1.25", "--schedule", "layered",
                            "--batch", "2048", "--precision", prec, "--seed", "7", "--json"],
                           cwd=ROOT, capture_output=True, text=True, timeout=1200)
        if p.returncode:
            sys.exit(p.stderr[-2000:])
        wall = time.perf_counter() - t0
        pts = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
        logl = [l for l in p.stdout.splitlines() if l and not l.startswith("{")]
        for pt in pts:
            kr = kernel_rate(prec, pt["ebn0_db"])
            rec = {"config": 3, "code": "dvbs2_1_2 (N=64800, R=1/2)", "decoder": "layered NMS alpha=1.25, T=50",
                   "precision": prec, "ebn0_db": pt["ebn0_db"], "frames": pt["frames"],
                   "frame_err": pt["frame_err"], "bit_err": pt["bit_err"], "fer": pt["fer"], "ber": pt["ber"],
                   "rounds": pt["rounds"], "frames_decoded": pt["frames_decoded"], "seconds": pt["seconds"],
                   "sweep_mbit_s_stop_rule_frames": pt["mbit_s"],
                   "sweep_mbit_s_decoded": pt["frames_decoded"] * kr["N"] / pt["seconds"] / 1e6, **kr,
                   "driver_overhead": 1 - pt["frames_decoded"] * kr["N"] / pt["seconds"] / 1e6 / kr["kernel_mbit_s"]}
            lines.append(rec)
            print(json.dumps(rec), flush=True)
        print(f"{prec}: sweep of {len(pts)} points in {wall:.1f} s; log lines:", *logl, sep="\n", flush=True)
    with open(out, "w") as f:
        for r in lines:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
