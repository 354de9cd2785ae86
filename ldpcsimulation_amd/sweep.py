"""SNR sweep on one or more GPUs -- replacement of the reference's sweep scripts.

The reference launches one background process per SNR point, each appending
one line to a shared log (C_implementations/scripts/minsum_example_*.sh:23-27,
decodeMinSum.cpp:313-329). Here every SNR point runs on all ranks at once: the
frames of a point are sharded over the GPUs by global frame index (one process
per GPU, torch.distributed over RCCL, launched with torchrun), the six error
counters are all-reduced per round, and rank 0 appends the reference's log
line for each point.

    python -m ldpcsimulation_amd.sweep ALIST --rate 0.5 --snr 1.0 1.25 1.5 -T 50 \\
        --variant nms --alpha 1.25 --log results.txt
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m ldpcsimulation_amd.sweep ...
    # BASELINE config 3: DVB-S2 N=64800 R1/2, layered NMS, SNR sweep over 8 GPUs
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m ldpcsimulation_amd.sweep dvbs2_1_2.alist \\
        --rate 0.5 --snr 0.8 0.9 1.0 1.1 -T 50 --variant nms --alpha 1.25 --schedule layered --batch 2048
    # belief propagation (decodeBP: its stop rule 200 bit / 20|10|5 frame errors)
    python -m ldpcsimulation_amd.sweep ALIST --rate 0.5 --snr 1.5 2.0 -T 50 --variant bp
    # BASELINE config 5: GF(16) EMS on an NB alist (SystemC/NB-LDPC format), early stop
    python -m ldpcsimulation_amd.sweep codes/gf16_N1000_dv2_dc4.alist --ems --rate 0.5 --snr 1.5 2.0 -T 20
Log line: SNR BER avgIt FER T [Ymax] [alpha] [delta] alist (EMS: SNR BER avgIt FER T nm offset alist;
BER over coded bits, 4 per GF(16) symbol).

--checkpoint FILE appends each point's running totals after a round at most
every --checkpoint-interval seconds (default 10; 0 = every round; checkpoint.py); a sweep restarted with the same FILE and settings takes the
seed from it, skips finished points and resumes the others at their next
frame, with the totals an uninterrupted run gives.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

from . import checkpoint, native, sim

VARIANTS = {"ms": native.MS, "nms": native.NMS, "oms": native.OMS, "bp": native.BP}


def parse(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("alist")
    p.add_argument("--rate", type=float, required=True)
    p.add_argument("--snr", type=float, nargs="+", required=True, help="Eb/N0 points in dB")
    p.add_argument("-T", "--iterations", type=int, default=10)
    p.add_argument("--variant", choices=list(VARIANTS), default="ms")
    p.add_argument("--alpha", type=float, default=1.0)
    p.add_argument("--delta", type=float, default=0.0)
    p.add_argument("--quantize", nargs=2, metavar=("YMAX", "Q"), help="-D quantizeSamples front-end")
    p.add_argument("--saturate", type=float, metavar="YMAX", help="-D saturateSamples front-end")
    p.add_argument("--precision", choices=["f32", "f64"], default="f64",
                   help="f64 = the reference's double (default); f32 = the fp32 kernels (opt-in)")
    p.add_argument("--schedule", choices=["flooding", "layered"], default="flooding",
                   help="flooding = the reference's schedule; layered = row-serial (BASELINE config 3)")
    p.add_argument("--batch", type=int, default=65536, help="frames per GPU per round (the largest round)")
    p.add_argument("--first-round", type=int, default=None,
                   help="frames per GPU in the first round; rounds double up to --batch (default min(batch, 1024))")
    p.add_argument("--seed", type=int, default=None, help="noise seed (default: time)")
    p.add_argument("--min-bit-errors", type=int, default=200)
    p.add_argument("--min-frame-errors", type=int, default=None,
                   help="default 40 (decodeMinSum.cpp:189); BP: 20/10/5 by N (decodeBP.cpp:145-147); EMS: 40")
    p.add_argument("--ems", action="store_true", help="GF(q) Extended Min-Sum on an NB alist (BASELINE config 5)")
    p.add_argument("--nm", type=int, default=16, help="EMS message truncation")
    p.add_argument("--offset", type=float, default=0.0, help="EMS fill offset")
    p.add_argument("--no-early-stop", action="store_true", help="EMS: always run T iterations")
    p.add_argument("--max-frames", type=int, default=None)
    p.add_argument("--codewords", help="codeword file ('0'/'1' lines), as the reference's optional argument")
    p.add_argument("--log", "--log-file", dest="log",
                   help="append the reference's tab-separated result line per point (--log-file under torchrun, "
                        "whose parser takes --log for a prefix of its own --log-dir)")
    p.add_argument("--json", action="store_true", help="also print one JSON object per point")
    p.add_argument("--sync", action="store_true",
                   help="one blocking round at a time (default: the next round decodes while one is reduced)")
    p.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                   help="collective backend for world > 1 (nccl = RCCL over xGMI; gloo: CPU tensors)")
    p.add_argument("--share-device", action="store_true",
                   help="every rank on device 0 (rehearsal of N ranks on one GPU, with --backend gloo)")
    p.add_argument("--checkpoint", metavar="FILE",
                   help="per-round progress file (.partial); an existing one is resumed (same settings)")
    p.add_argument("--checkpoint-interval", type=float, default=10.0, metavar="S",
                   help="seconds between checkpoint records (0 = after every round); each record "
                        "all-reduces the point's error-weight histogram")
    return p.parse_args(argv)


def _checkpoint_config(a) -> dict:
    """Every setting that changes a point's result (not the batch or round sizes,
    the GPU count or the log options: exact_stop makes totals independent of them)."""
    return {"alist": os.path.basename(a.alist), "alist_md5": checkpoint.file_digest(a.alist), "rate": a.rate,
            "snr": list(a.snr), "T": a.iterations, "variant": a.variant, "alpha": a.alpha, "delta": a.delta,
            "quantize": a.quantize, "saturate": a.saturate, "precision": a.precision, "schedule": a.schedule,
            "min_bit_errors": a.min_bit_errors, "min_frame_errors": a.min_frame_errors, "max_frames": a.max_frames,
            "codewords_md5": checkpoint.file_digest(a.codewords), "ems": a.ems, "nm": a.nm, "offset": a.offset,
            "early_stop": not a.no_early_stop}


def _run_points(a, ck, rank, n_hist, run_point):
    """run_point(k, snr, resume, on_round) -> (result, log line, json dict) for each
    point not finished in the checkpoint; rank 0 logs and records each point.
    n_hist: the points' histogram length (bits per frame)."""
    for k, snr in enumerate(a.snr):
        done = ck.done_line(k, snr) if ck else None
        if done is not None:
            if rank == 0:
                print(done, flush=True)   # appended to the log by the run that finished it
            continue
        resume = ck.point_state(k, snr, n_hist) if ck else None
        on_round = (lambda st, k=k, snr=snr: ck.save_round(k, snr, st)) if ck else None
        res, line, js = run_point(k, snr, resume, on_round)
        if rank == 0:
            if a.log:
                with open(a.log, "a") as f:
                    f.write(line + "\n")
            print(line, flush=True)
            if a.json:
                js["resumed_from_frame"] = resume.next_frame if resume else 0
                print(json.dumps(js), flush=True)
        if ck:
            ck.save_done(k, snr, line)


def main(argv=None) -> int:
    a = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = local if world > 1 and not a.share_device else 0
    # under torchrun (WORLD_SIZE set) a process group always exists, one rank included:
    # the counters then go through the collective backend exactly as at 8 ranks
    distributed = "WORLD_SIZE" in os.environ
    if distributed:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(device)
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
    ck = checkpoint.SweepCheckpoint(a.checkpoint, _checkpoint_config(a), writer=rank == 0) if a.checkpoint else None
    if ck and ck.seed is not None:
        if a.seed is not None and a.seed != ck.seed:
            raise checkpoint.CheckpointMismatch(f"--seed {a.seed} != the checkpoint's seed {ck.seed}")
        a.seed = ck.seed          # every rank read the same file
    seed = a.seed if a.seed is not None else int(time.time())
    if distributed and a.seed is None:
        # every rank must key its noise with rank 0's seed (ranks may start in different seconds)
        import torch
        import torch.distributed as dist
        t = torch.tensor([seed], dtype=torch.int64, device=f"cuda:{device}" if a.backend == "nccl" else "cpu")
        dist.broadcast(t, src=0)
        seed = int(t.item())
    if os.environ.get("LDPC_SWEEP_REPORT_SEED"):   # tests: every rank reports the seed it keys its noise with
        print(json.dumps({"rank": rank, "seed": seed}), file=sys.stderr, flush=True)
    if ck:
        ck.start(seed)
    if a.ems:
        return _ems_sweep(a, seed, world, rank, device, ck)
    cfg = native.DecoderConfig(variant=VARIANTS[a.variant], T=a.iterations, alpha=a.alpha, delta=a.delta,
                               precision=native.F64 if a.precision == "f64" else native.F32,
                               schedule=native.LAYERED if a.schedule == "layered" else native.FLOODING)
    extra = []
    if a.quantize:
        cfg.quantize, cfg.ymax, cfg.qbits = True, float(a.quantize[0]), int(a.quantize[1])
        extra.append(cfg.ymax)
    elif a.saturate is not None:
        cfg.saturate, cfg.ymax = True, a.saturate
        extra.append(cfg.ymax)
    if a.variant == "nms":
        extra.append(a.alpha)
    elif a.variant == "oms":
        extra.append(a.delta)
    g = native.Graph.from_alist(a.alist)
    ctx = native.Context(g, device, a.batch)
    min_fe = a.min_frame_errors
    if min_fe is None:
        min_fe = (5 if g.N > 50000 else 10 if g.N > 10000 else 20) if a.variant == "bp" else 40
    if a.codewords:
        from .codes import read_codeword_file
        ctx.set_codewords(read_codeword_file(a.codewords, g.N))
    def run_point(k, snr, resume, on_round):
        def run_batch(first, n):
            fr, _ = ctx.sim_batch(snr, a.rate, cfg, seed, k, first, n)
            return fr

        launcher = None
        if not a.sync:
            # rounds run ahead: round k+1 decodes while round k is reduced (sim.AsyncLauncher)
            def run_launch(first, n, frames_dev):
                ctx.sim_launch(snr, a.rate, cfg, seed, k, first, n, frames_dev)
            launcher = sim.AsyncLauncher(ctx, a.batch, run_launch)
        t0 = time.perf_counter()
        res = sim.simulate_point(run_batch, g.N, a.iterations, snr, a.batch, a.min_bit_errors,
                                 min_fe, a.max_frames, device=device, launcher=launcher, first_round=a.first_round,
                                 resume=resume, on_round=on_round,
                                 on_round_interval=a.checkpoint_interval)
        dt = time.perf_counter() - t0
        c = res.counts
        ran = c["frames"] - (int(resume.acc[3]) if resume else 0)   # frames counted by this run
        return res, res.log_line(a.alist, extra), {
            "ebn0_db": snr, **c, "ber": res.ber, "fer": res.fer, "seconds": dt,
            "mbit_s": ran * g.N / dt / 1e6 if dt > 0 else None,
            "n_gpus": world, "wilson95": sim.wilson_interval(c["frame_err"], c["frames"]),
            "precision": a.precision, "schedule": a.schedule, "variant": a.variant,
            "kernel": ctx.kernel_info(cfg)["kernel"], "rounds": res.rounds, "frames_decoded": res.frames_decoded,
            "collectives": res.collectives}

    _run_points(a, ck, rank, g.N, run_point)
    if distributed:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


def _ems_sweep(a, seed, world, rank, device, ck=None) -> int:
    """One SNR point after the other on the GF(q) EMS decoder, frames sharded as above."""
    g = native.NbGraph.from_alist(a.alist)
    ctx = native.NbContext(g, device, a.batch)
    cfg = native.EmsConfig(T=a.iterations, nm=a.nm, offset=a.offset, early_stop=not a.no_early_stop)
    bits = g.N * g.m
    def run_point(k, snr, resume, on_round):
        def run_batch(first, n):
            fr, _ = ctx.sim_batch(snr, a.rate, cfg, seed, k, first, n)
            return fr
        t0 = time.perf_counter()
        res = sim.simulate_point(run_batch, bits, a.iterations, snr, a.batch, a.min_bit_errors,
                                 a.min_frame_errors if a.min_frame_errors is not None else 40, a.max_frames,
                                 device=device, iters_in_frames=True, first_round=a.first_round,
                                 resume=resume, on_round=on_round,
                                 on_round_interval=a.checkpoint_interval)
        dt = time.perf_counter() - t0
        c = res.counts
        ran = c["frames"] - (int(resume.acc[3]) if resume else 0)   # frames counted by this run
        return res, res.log_line(a.alist, [float(a.nm), a.offset]), {
            "ebn0_db": snr, **c, "ber": res.ber, "fer": res.fer, "avg_iters": res.avg_iters,
            "seconds": dt, "mbit_s": ran * bits / dt / 1e6 if dt > 0 else None,
            "n_gpus": world, "wilson95": sim.wilson_interval(c["frame_err"], c["frames"]),
            "precision": "f32", "rounds": res.rounds, "frames_decoded": res.frames_decoded}

    _run_points(a, ck, rank, bits, run_point)
    if "WORLD_SIZE" in os.environ:   # a process group exists only under torchrun (torch optional otherwise)
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
