#!/usr/bin/env python3
"""Benchmark of the hot path: fused AWGN -> flooding NMS decode -> error count.

Workload (BASELINE.json configs[1]): 802.11n N=1944 rate-1/2 QC-LDPC,
normalized min-sum (divide by alpha=1.25), T=50 iterations (fixed, as the
reference), a 65,536-codeword all-zero-codeword BPSK/AWGN batch per step at
Eb/N0 = 1.5 dB, noise from on-device Philox4x32-10 keyed by global frame
index. One step = one ldpc_sim_launch over one batch per GPU; inputs are
generated on the device (nothing crosses PCIe in the timed region).

The headline decodes in fp64, the reference's own arithmetic
(decodeMinSum.cpp:39-40,410-476 hold every message in `double`), with the
fast fp64 row kernel whose decisions equal the reference's bit for bit
(tests/test_rows_fast.py). The fp32 throughput path is timed after it over
the same steps and reported under "f32".

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

`--gpus N` without torchrun's environment starts torchrun itself (a child
process, before anything touches the GPU) and exits with its status.

Prints ONE JSON line (rank 0). value = decoded coded bits per second over all
ranks (Mbit/s), max-over-ranks wall time of the K timed steps. With N > 1 each
step also all-reduces that round's per-frame counter sums over the ranks (RCCL,
on the launch stream), the exchange the sharded SNR driver makes per round.

roofline: the resource that bounds the row kernel is the LDS
pipe. `achieved` = the ALGORITHMIC LDS-array cycles per launch -- per
codeword-iteration E gathers of app, E scatters of c2v, E bit-side reads of
c2v and N app writes, in 64-lane wave-instructions at their conflict-free
costs (ds_read_b64 2, ds_write_b64 6 cycles, MI355X_MICROARCH.md LDS table),
no padding -- divided by the average launch time (HIP events on the launch
stream), in G LDS-cycles/s; `peak` = CUs x 2.4 GHz. Companions in
`lds_model_alt`: `issued` (the wave-instructions the kernel issues, padding
edges of its row slots included; the library reports its slot degrees) and
`padded` (every row slot at the padded degree, the rounds 2-4 model). The SURVEY §8(d) flooding HBM
message model (16E+4N bytes per codeword-iteration) is kept as `hbm_model`;
it does not bound this kernel (messages never leave LDS), so its "fraction"
exceeds 1. `traffic` = HBM bytes per launch of the headline kernel, measured
live after the timed steps: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE;
separate passes, MI355X_MICROARCH's counter limits) over a child run of this
same workload (1 warm-up + 1 step), FETCH_SIZE doubled (the guide's gfx950
correction); `traffic_gbs` = those bytes over this run's average launch time,
against the 8 TB/s HBM peak. --live-pmc off (or running under a profiler)
falls back to the committed PMC summary (profiles/traffic_latest.json).

cpu_baseline: the reference's own decodeNMS (oracle/_ref, compiled from the
unmodified sources) on this box's host cores, same code/variant/T/SNR.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time
from typing import Optional

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded Mbit/s + FER match vs CPU, N=1944 rate-1/2 min-sum @ 1/2/4/8 MI355X"
HBM_PEAK = 8.0e12   # B/s, MI355X HBM3E (MI355X_MICROARCH.md)
CLOCK_HZ = 2.4e9    # MI355X peak engine clock: one LDS-array cycle per clock per CU
LDS_CYC = {"ds_read_b64": 2, "ds_write_b64": 6}   # cycles per wave-instruction, conflict-free
REF_FER = {1.0: (40, 96), 1.25: (40, 362), 1.5: (40, 2212), 1.75: (40, 41745)}   # SURVEY §6 (one seed each)
REF_FER_JSON = os.path.join(ROOT, "tests", "golden", "reference_fer.json")


def reference_fer() -> dict:
    """Reference FER per SNR: the multi-seed fixture (scripts/ref_fer.py) when present,
    else SURVEY §6's single-seed points."""
    try:
        d = json.load(open(REF_FER_JSON))
        return {float(p["ebn0_db"]): (int(p["frame_err"]), int(p["frames"])) for p in d["points"]}
    except (OSError, ValueError, KeyError):
        return dict(REF_FER)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=65536)
    p.add_argument("--ebn0", type=float, default=1.5)
    p.add_argument("--T", type=int, default=50)
    p.add_argument("--alpha", type=float, default=1.25)
    p.add_argument("--precision", choices=["f32", "f64"], default="f64")
    p.add_argument("--no-secondary", action="store_true", help="skip the fp32 run after the fp64 headline")
    p.add_argument("--seed", type=int, default=20261015)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-procs", type=int, default=0, help="0 = the box's CPU share (see cpu_share())")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    p.add_argument("--live-pmc", choices=["auto", "off"], default="auto",
                   help="auto: measure the headline kernel's HBM bytes with rocprofv3 --pmc child runs (N=1, rank 0)")
    p.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                   help="collective backend for N>1 (gloo + --share-device: rehearse N ranks on one GPU)")
    p.add_argument("--share-device", action="store_true", help="every rank on device 0 (rehearsal only)")
    p.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                   help="A/B only: a kernel-choice option of the context (native.OPTIONS, e.g. rows64=fast)")
    p.add_argument("--lib", default=None, help="A/B only: another build of the decoder library (make ppvariant ...)")
    return p.parse_args(argv)


def parse_options(items) -> dict:
    """--option NAME=VALUE items -> {name: value} (values: ints or native.OPTION_VALUES names)."""
    out = {}
    for it in items:
        k, _, v = it.partition("=")
        out[k.strip()] = int(v) if v.strip().lstrip("-").isdigit() else v.strip()
    return out


def cpu_share() -> int:
    """Cores this process may use: its CPU affinity, capped by OMP_NUM_THREADS when
    that is set (the GPU box sets it to its per-GPU share, 16, while its affinity
    shows the whole host)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS", "")
    cap = int(env) if env.strip().isdigit() and int(env) > 0 else aff
    return max(1, min(aff, cap))


def host_cores() -> int:
    """All cores this process's affinity shows (the whole host on the GPU box)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


KERNEL_SYMBOL = {"rows_pp": "k_rows_pp", "rows_fast": "k_rows_fast", "rows": "k_decode_rows"}


def pmc_kernel_average(out_dir: str, pattern: str, counter: str):
    """Average over the dispatches of kernels matching `pattern` of one counter in a
    rocprofv3 --output-format csv directory (per dispatch: the sum of its rows, the
    counter's per-XCD/instance values), or None."""
    vals = {}
    for f in glob.glob(os.path.join(out_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if pattern in r["Kernel_Name"] and r["Counter_Name"] == counter:
                    vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return sum(vals.values()) / len(vals) if vals else None


def live_traffic(args, kernel: str, precision: Optional[str] = None) -> dict:
    """HBM bytes per launch of `kernel` in this workload, measured now: one rocprofv3
    --pmc pass per counter (FETCH_SIZE, WRITE_SIZE) over a child bench run (1 warm-up
    + 1 step of the headline, nothing else), each under its own time limit. Per
    dispatch of the kernel: FETCH_SIZE x 2 (gfx950 counts wide reads at half,
    MI355X_MICROARCH HBM section) + WRITE_SIZE, in KiB from the counters."""
    exe = shutil.which("rocprofv3")
    if exe is None:
        return {"error": "rocprofv3 not on PATH"}
    pattern = KERNEL_SYMBOL.get(kernel, kernel)
    child = [sys.executable, os.path.abspath(__file__), "--steps", "1", "--warmup", "1", "--no-secondary",
             "--no-cpu-baseline", "--live-pmc", "off", "--precision", precision or args.precision, "--batch", str(args.batch),
             "--T", str(args.T), "--ebn0", str(args.ebn0), "--alpha", str(args.alpha), "--seed", str(args.seed)]
    child += [f"--option={o}" for o in args.option] + (["--lib", args.lib] if args.lib else [])
    env = dict(os.environ, TMPDIR="/tmp")
    kib = {}
    with tempfile.TemporaryDirectory(prefix="ldpc_pmc_", dir="/tmp") as d:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(d, ctr)
            cmd = ["timeout", "-s", "KILL", "150", exe, "--pmc", ctr, "-d", out, "-o", "pmc",
                   "--output-format", "csv", "--"] + child
            p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True)
            if p.returncode != 0:
                return {"error": f"{ctr} pass rc={p.returncode}: {(p.stderr or p.stdout)[-300:]}"}
            v = pmc_kernel_average(out, pattern, ctr)
            if v is None:
                return {"error": f"{ctr} pass: no {pattern} dispatch in the counter output"}
            kib[ctr] = v
    fetch, write = 2 * kib["FETCH_SIZE"] * 1024, kib["WRITE_SIZE"] * 1024
    return {"hbm_bytes_per_launch": fetch + write, "fetch_bytes_x2": fetch, "write_bytes": write,
            "kernel_pattern": pattern,
            "source": "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over a 1-step child run of this workload"}


def _final(out: str):
    line = [l for l in out.splitlines() if l.startswith("Final result:")][0]
    frames = int(line.split(" words")[0].split()[-1])
    ferr = sum(1 for l in out.splitlines() if l.startswith("Ferr with"))
    return frames, ferr


def physical_cores() -> int:
    """Distinct (package, core) pairs of /proc/cpuinfo: the host's physical cores (SMT
    siblings counted once); 0 when unknown."""
    pairs, phys = set(), None
    try:
        for l in open("/proc/cpuinfo"):
            if l.startswith("physical id"):
                phys = l.split(":", 1)[1].strip()
            elif l.startswith("core id"):
                pairs.add((phys, l.split(":", 1)[1].strip()))
    except OSError:
        return 0
    return len(pairs)


def _ref_runs(ref: str, alist: str, T: int, alpha: float, ebn0: float, procs: int, td: str, seed0: int):
    """`procs` concurrent runs of the reference binary to its stop rule: per-process
    (frames, wall seconds) and the wall time of the whole set."""
    def launch(k):
        env = dict(os.environ, REF_SEED=str(seed0 + k))
        f = open(f"{td}/out{seed0}_{k}.txt", "w")
        return subprocess.Popen([ref, alist, "0.5", str(ebn0), str(T), str(alpha), f"{td}/log{seed0}_{k}.txt"],
                                env=env, stdout=f), f, time.perf_counter()
    t0 = time.perf_counter()
    ps = [launch(k) for k in range(procs)]
    walls, frames = [], []
    for k, (p, f, ts) in enumerate(ps):
        rc = p.wait()
        walls.append(time.perf_counter() - ts)
        f.close()
        if rc:
            raise RuntimeError(f"reference CPU baseline process {k} failed ({rc})")
        frames.append(_final(open(f"{td}/out{seed0}_{k}.txt").read())[0])
    return frames, walls, time.perf_counter() - t0


def cpu_baseline(alist: str, T: int, alpha: float, ebn0: float, procs: int, scaling=(1, 4)) -> dict:
    """Time the reference CPU path on `procs` host cores, on the bench's own workload.

    Each process runs the unmodified reference decodeNMS once at the bench's
    Eb/N0, where its stop rule (decodeMinSum.cpp:189: >= 40 frame errors)
    ends the run after ~2,200 frames (1.5 dB) -- >= 500 frames per process.
    A process's rate is its frames x N over its own wall time; the
    aggregate is the sum over the concurrent processes. Process spawn and the
    alist parse are measured separately (a T=0 run of 40 frames) and are
    < 0.1 % of a run, so they are reported, not subtracted. The reference
    has no early stop, so its time per frame does not depend on the SNR.

    The box allots its GPU a `procs`-core share of a larger host, so the
    whole host is not run: the `procs`-process set is the largest measured
    point (host_measured_*), the same workload at `scaling` process counts
    shows how the per-process rate holds up to it, and the whole-host figure
    is an extrapolation of the per-process rate, bracketed by the host's
    physical cores (no SMT gain) and its logical CPUs (SMT siblings as full
    cores)."""
    ref = os.path.join(ROOT, "oracle", "_ref", "decodeNMS")
    if not os.path.exists(ref):
        return _cpu_baseline_port(alist, T, alpha, procs)
    N = 1944
    with tempfile.TemporaryDirectory() as td:
        frames, walls, wall_all = _ref_runs(ref, alist, T, alpha, ebn0, procs, td, 1000)
        curve = {}
        for n in scaling:
            if n < procs:
                fr, wa, _ = _ref_runs(ref, alist, T, alpha, ebn0, n, td, 2000 + 100 * n)
                curve[str(n)] = {"aggregate_mbit_s": float(sum(f * N / w / 1e6 for f, w in zip(fr, wa))),
                                 "per_process_mbit_s": float(np.median([f * N / w / 1e6 for f, w in zip(fr, wa)]))}
        # per-run fixed cost: spawn + alist parse + 40 frames of channel without decoding (T=0)
        ts = time.perf_counter()
        subprocess.run([ref, alist, "0.5", "0.0", "0", str(alpha), f"{td}/l0.txt"], env=dict(os.environ, REF_SEED="5"),
                       capture_output=True, text=True, check=True)
        t_fixed = time.perf_counter() - ts
        # the same workload built with the reference Makefile's own flags (-g, no -O): the "as shipped" rate,
        # one core, a 0.0 dB run (40 frames; time per frame does not depend on the SNR)
        single_g = None
        ref_g = os.path.join(ROOT, "oracle", "_ref", "decodeNMS_g")
        if os.path.exists(ref_g):
            ts = time.perf_counter()
            out = subprocess.run([ref_g, alist, "0.5", "0.0", str(T), str(alpha), f"{td}/lg.txt"],
                                 env=dict(os.environ, REF_SEED="7"), capture_output=True, text=True, check=True).stdout
            single_g = _final(out)[0] * N / (time.perf_counter() - ts) / 1e6
    rates = [f * N / w / 1e6 for f, w in zip(frames, walls)]
    agg = float(sum(rates))
    curve[str(procs)] = {"aggregate_mbit_s": agg, "per_process_mbit_s": float(np.median(rates))}
    hc, pc = host_cores(), physical_cores()
    per = float(np.median(rates))
    one = curve.get("1", {}).get("per_process_mbit_s")
    return {"value": agg, "unit": "Mbit/s", "cores": procs, "kind": "reference",
            "single_core_mbit_s": per,
            "host_measured_procs": procs, "host_measured_mbit_s": agg,
            "scaling_curve": curve,
            "efficiency_vs_one_process": (agg / (procs * one)) if one else None,
            # the whole host is not run here (the box allots its GPU a `procs`-core share):
            # the per-process rate measured at that share times the host's cores
            "host_cores": hc, "host_physical_cores": pc,
            "host_aggregate_mbit_s_extrapolated": per * hc,
            "host_aggregate_mbit_s_extrapolated_physical": per * pc if pc else None,
            "extrapolated_over_measured": per * hc / agg,
            "single_core_mbit_s_as_shipped_O0_g": single_g,
            "cpu_model": _cpu_model(),
            "frames_per_process_min": int(min(frames)), "frames_total": int(sum(frames)),
            "fixed_cost_per_run_s": round(t_fixed, 4),
            "sample": f"{procs} concurrent processes x 1 run of oracle/_ref/decodeNMS (unmodified reference, "
                      f"g++ -O2), 802.11n N=1944 NMS alpha={alpha} T={T} at {ebn0} dB until its stop rule "
                      f"(40 frame errors): {sum(frames)} frames, {min(frames)}..{max(frames)} per process, "
                      f"{wall_all:.1f} s wall; value = sum of per-process frames*N/wall; the same workload at "
                      f"{', '.join(str(n) for n in scaling if n < procs)} processes for the scaling curve"}


def _cpu_baseline_port(alist, T, alpha, procs):
    """Fallback when oracle/_ref was not shipped: the oracle restatement (fp64, ragged, find())."""
    import multiprocessing as mp
    n_frames = 100
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(procs) as pool:
        res = pool.starmap(_port_worker, [(alist, T, alpha, 1000 + k, n_frames) for k in range(procs)])
    wall = time.perf_counter() - t0
    frames = sum(res)
    return {"value": frames * 1944 / wall / 1e6, "unit": "Mbit/s", "cores": procs, "kind": "port",
            "cpu_model": _cpu_model(),
            "sample": f"{procs} processes x {n_frames} frames of the oracle restatement (fp64, ragged arrays, "
                      f"linear find(), gcc -O2), 802.11n N=1944 NMS alpha={alpha} T={T}; {wall:.2f} s wall"}


def _port_worker(alist, T, alpha, seed, n):
    from oracle import oracle as O
    A = O.Alist(alist)
    got, _, _ = A.minsum_run(0.5, 0.0, T, O.Cfg(variant=O.NMS, alpha=alpha), seed, max_frames=n)
    return got


def _cpu_model() -> str:
    try:
        for l in open("/proc/cpuinfo"):
            if l.startswith("model name"):
                return l.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def lds_model(si: dict, E: int, N: int) -> dict:
    """Algorithmic LDS-array cycles per codeword-group iteration of the flooding row
    kernels: E gathers of app and E scatters of c2v by the check rows,
    E reads of c2v and N writes of app by the bit nodes, in 64-lane wave-instructions
    at their conflict-free costs, no padding. One ds_*_b64 moves one fp64 value
    (C=1) or a codeword pair of fp32 (C=2), so a group is 1 or 2 codewords."""
    rd, wr = LDS_CYC["ds_read_b64"], LDS_CYC["ds_write_b64"]
    cyc = {"check_gather": E / 64 * rd, "check_scatter": E / 64 * wr, "bit_read": E / 64 * rd,
           "app_write": N / 64 * wr}
    return {"cycles_per_group_iter": sum(cyc.values()), "by_phase": cyc, "E": E, "N": N,
            "cw_per_group": si["cw_per_block"]}


def lds_models_alt(si: dict) -> dict:
    """Two companions of the algorithmic model: `issued` -- the wave-instructions the
    kernel issues (its row slots at the degree it compiles them with, padding edges
    included: the library reports the check-edge slots, `issued_check_edges`, e.g.
    768 x 7 + 256 x 8 for the ping-pong kernel's degree-aware slots, graph.h
    pp_row_slots), and `padded` -- every row slot at the padded degree dc (the model
    `frac` used in rounds 2-4)."""
    rd, wr = LDS_CYC["ds_read_b64"], LDS_CYC["ds_write_b64"]
    bit = si["e_pad"] / 64 * rd + si["threads"] * si["slots_per_thread"] / 64 * wr
    rows = si["threads"] * si["rows_per_thread"]
    return {"issued": {"cycles_per_group_iter": si["issued_check_edges"] / 64 * (rd + wr) + bit,
                       "check_edge_slots": si["issued_check_edges"], "degree_split": si["dc_low"] > 0},
            "padded": {"cycles_per_group_iter": rows * si["dc"] / 64 * (rd + wr) + bit}}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one rank per GPU: start torchrun as a child (nothing has touched the GPU yet)
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU")

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.share_device:
        local = 0
    # Under torchrun a process group always exists, one rank included (a one-rank RCCL
    # communicator): the per-step exchange and the max-over-ranks timing then run as they
    # do at 8 ranks. Without torchrun (the driver's N=1 run) there is no collective.
    distributed = "WORLD_SIZE" in os.environ
    if distributed:
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    coll_dev = "cuda" if args.backend == "nccl" else "cpu"

    from ldpcsimulation_amd import codes, native
    if args.lib:
        native.use_library(os.path.abspath(args.lib))
    alist = codes.ensure_80211n_1944()
    g = native.Graph.from_alist(alist)
    B = args.batch
    ctx = native.Context(g, local if world > 1 else 0, B)
    ctx.set_options(parse_options(args.option))
    # A dedicated (non-default) torch stream: the library launches on it, so the
    # torch events below bracket exactly the decode kernel on its own stream.
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    frames_dev = torch.empty((B, 4), dtype=torch.int32, device="cuda")

    def run(precision: str, stream_id: int) -> dict:
        cfg = native.DecoderConfig(variant=native.NMS, alpha=args.alpha, T=args.T,
                                   precision=native.F64 if precision == "f64" else native.F32)

        def step(k):
            first = (k * world + rank) * B
            ctx.sim_launch(args.ebn0, 0.5, cfg, args.seed, stream_id, first, B, frames_dev)
            if distributed and args.backend == "nccl":
                # the sharded driver's per-round exchange (sim.simulate_point): this round's
                # counters summed over ranks, RCCL on the launch stream
                part = frames_dev.sum(dim=0, dtype=torch.int64)
                dist.all_reduce(part)

        for k in range(args.warmup):
            step(k)
        torch.cuda.synchronize()
        ctx.read_counts(reset=True)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            ev[k][0].record(stream)
            step(args.warmup + k)
            ev[k][1].record(stream)
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        kern_ms = [a.elapsed_time(b) for a, b in ev]
        redo = ctx.redo_count()
        cnt = ctx.read_counts(reset=True).as_array()
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        c = torch.from_numpy(np.append(cnt, redo)).to(coll_dev)
        if distributed:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dist.all_reduce(c)
        tot = c.cpu().numpy()
        frames_total = int(tot[3])
        assert frames_total == args.steps * B * world, (frames_total, args.steps, B, world)
        elapsed = float(t.item())
        return {"cfg": cfg, "elapsed": elapsed, "kern_ms": kern_ms, "tot": tot,
                "value": frames_total * g.N / elapsed / 1e6}

    head = run(args.precision, 0)
    sec = None
    if not args.no_secondary and args.precision == "f64":
        sec = run("f32", 1)

    def roofline(r: dict) -> dict:
        avg_kernel_s = float(np.mean(r["kern_ms"])) / 1e3
        info = ctx.kernel_info(r["cfg"])
        B_cw = args.T * (16 * g.E + 4 * g.N)            # SURVEY §8(d) algorithmic HBM bytes / codeword
        hbm_achieved = B_cw * B / avg_kernel_s
        out = {"kernel": info["kernel"], "avg_kernel_ms": avg_kernel_s * 1e3,
               "hbm_model": {"achieved": hbm_achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                             "frac": hbm_achieved / HBM_PEAK, "bytes_per_codeword_model": B_cw,
                             "note": "SURVEY §8(d) flooding fp32 message model; messages stay in LDS, so > 1"}}
        try:
            si = ctx.row_sched_info(r["cfg"])
        except native.LdpcError:
            return out
        m = lds_model(si, g.E, g.N)
        groups = B / si["cw_per_block"]
        cycles = m["cycles_per_group_iter"] * args.T * groups          # whole launch, all CUs
        n_cu = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
        achieved = cycles / avg_kernel_s / 1e9
        peak = n_cu * CLOCK_HZ / 1e9
        alt = lds_models_alt(si)
        for k, v in alt.items():
            v["frac"] = v["cycles_per_group_iter"] * args.T * groups / avg_kernel_s / 1e9 / peak
        out.update({"bound": "lds", "achieved": achieved, "peak": peak, "unit": "G LDS-cycles/s",
                    "frac": achieved / peak, "lds_cycles_per_launch": cycles, "cus": n_cu,
                    "lds_model": m, "lds_model_alt": alt, "row_sched": si})
        return out

    if rank == 0:
        tot = head["tot"]
        rl = roofline(head)
        traffic, traffic_src, traffic_kernel, live = None, None, None, None
        nested = any(k.startswith("ROCPROF") for k in os.environ) or "rocprofiler" in os.environ.get("LD_PRELOAD", "")
        if args.live_pmc == "auto" and world == 1 and not nested:
            live = live_traffic(args, rl["kernel"])
            if "hbm_bytes_per_launch" in live:
                traffic, traffic_src, traffic_kernel = live["hbm_bytes_per_launch"], live["source"], live["kernel_pattern"]
        if traffic is None:   # the committed PMC summary of this round (scripts/profile_round.sh)
            try:
                tj = json.load(open(args.traffic_json))
                tj = tj.get(args.precision, {})
                traffic, traffic_kernel = tj.get("hbm_bytes_per_launch"), tj.get("kernel")
                traffic_src = f"committed: {tj.get('source')}" + (f" (live pass: {live['error']})" if live else "")
            except (OSError, ValueError):
                pass
        # the PMC bytes over this run's average launch time, against the HBM peak
        traffic_gbs = traffic / (rl["avg_kernel_ms"] / 1e3) / 1e9 if traffic else None
        k_fe, n_fe = int(tot[1]), int(tot[3])
        from ldpcsimulation_amd.sim import two_proportion_z, wilson_interval
        fer = {"ebn0_db": args.ebn0, "frame_err": k_fe, "frames": n_fe, "fer": k_fe / n_fe,
               "ber": float(tot[0]) / (n_fe * g.N), "wilson95": wilson_interval(k_fe, n_fe),
               "redecoded_exact_last_launch": int(tot[6])}
        ref = reference_fer()
        if args.ebn0 in ref and args.T == 50 and args.alpha == 1.25:
            kr, nr = ref[args.ebn0]
            fer.update(ref_frame_err=kr, ref_frames=nr, ref_fer=kr / nr,
                       ref_source=os.path.relpath(REF_FER_JSON, ROOT) if os.path.exists(REF_FER_JSON) else "SURVEY §6",
                       z_vs_reference=two_proportion_z(k_fe, n_fe, kr, nr))
        out = {
            "metric": METRIC, "value": head["value"], "unit": "Mbit/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": head["elapsed"] / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic: all-zero codeword, BPSK/AWGN from on-device Philox4x32-10 + Box-Muller (fp32 transform on the SIMD's v_log/v_sqrt/v_sin/v_cos_f32, samples widened to fp64 for the fp64 decoder)",
            "config": {"workload": f"802.11n N=1944 R1/2 QC-LDPC, NMS alpha={args.alpha}, T={args.T}, "
                                   f"{B}-codeword AWGN batch per GPU @ {args.ebn0} dB",
                       "code": "80211n_1944_r12 (N=1944, M=972, E=6966)", "batch_per_gpu": B,
                       "global_batch": B * world, "T": args.T, "ebn0_db": args.ebn0, "variant": "nms",
                       "parallelism": f"frame-sharded x{world}"},
            "roofline": {**{k: rl.get(k) for k in ("bound", "achieved", "peak", "unit", "frac")},
                         "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC)",
                         "traffic_gbs": traffic_gbs,
                         "traffic_frac_of_hbm_peak": traffic_gbs / (HBM_PEAK / 1e9) if traffic_gbs else None,
                         "traffic_source": traffic_src, "traffic_kernel": traffic_kernel,
                         "traffic_detail": {k: v for k, v in (live or {}).items() if k in ("fetch_bytes_x2", "write_bytes")},
                         **{k: v for k, v in rl.items() if k not in ("bound", "achieved", "peak", "unit", "frac")}},
            "fer": fer,
            "kernel_info": ctx.kernel_info(head["cfg"]),
            "collective_backend": dist.get_backend() if distributed else None,
        }
        if sec is not None:
            rs = roofline(sec)
            out["f32"] = {"value": sec["value"], "unit": "Mbit/s", "ms_per_step": sec["elapsed"] / args.steps * 1e3,
                          "avg_kernel_ms": rs["avg_kernel_ms"], "kernel": rs["kernel"],
                          "lds_frac": rs.get("frac"), "frame_err": int(sec["tot"][1]), "frames": int(sec["tot"][3]),
                          "note": "fp32 throughput path (same workload, Philox stream 1); not the reference's precision"}
            if args.live_pmc == "auto" and world == 1 and not nested:
                # the fp32 kernel's HBM bytes, measured the same way as the headline's
                lt = live_traffic(args, rs["kernel"], "f32")
                out["f32"]["traffic"] = lt.get("hbm_bytes_per_launch")
                out["f32"]["traffic_detail"] = {k: v for k, v in lt.items() if k != "hbm_bytes_per_launch"}
        if not args.no_cpu_baseline and world == 1:
            procs = args.cpu_procs or cpu_share()
            try:
                out["cpu_baseline"] = cpu_baseline(alist, args.T, args.alpha, args.ebn0, procs)
                out["speedup_vs_cpu"] = head["value"] / out["cpu_baseline"]["value"]
            except Exception as e:   # never lose the GPU line over the CPU leg
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
