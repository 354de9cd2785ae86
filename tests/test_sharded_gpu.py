"""The sharded SNR-point driver (sim.simulate_point, the replacement of the
reference's per-SNR process model scripts/minsum_example_PEGReg504x1008.sh:23-27
and the frame loop decodeMinSum.cpp:189-289) on the real HIP path.

Two gloo ranks, spawned processes with their own ldpc context on device 0 (one
box has one GPU; the data path has no collective beyond the 48-byte counter
all-reduce, so sharing the card changes nothing but speed), decode config 2
(802.11n N=1944, NMS alpha=1.25, T=50, fp64, on-device Philox noise) at
1.5 dB to the reference's stop rule. Their totals and error-weight
histogram must equal one rank's, for a different batch size too: the frames
are keyed by global index, and the exact-stop cut makes the result a
frame-by-frame run of the same noise.

Config 3's sweep (sweep.py --schedule layered: DVB-S2 N=64800, layered NMS,
the global layered kernel) is run the same way, two ranks against one, at one
SNR point of the sweep."""
import json
import os
import re
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import code_path

CODE = "80211n_1944_r12.alist"
EBN0, SEED, T = 1.5, 20261018, 50
# config 3: DVB-S2 layered, one point of the SNR sweep (fp64, the sweep's default precision)
DVB_CODE, DVB_EBN0, DVB_T = "dvbs2_1_2.alist", 1.0, 10


def _cfg(case="c2"):
    from ldpcsimulation_amd import native
    if case == "c3":
        return native.DecoderConfig(variant=native.NMS, alpha=1.25, T=DVB_T, precision=native.F64,
                                    schedule=native.LAYERED)
    return native.DecoderConfig(variant=native.NMS, alpha=1.25, T=T, precision=native.F64)


def _run(ctx, batch, case="c2"):
    from ldpcsimulation_amd import sim
    cfg = _cfg(case)
    ebn0, t = (DVB_EBN0, DVB_T) if case == "c3" else (EBN0, T)

    def run_batch(first, n):
        fr, _ = ctx.sim_batch(ebn0, 0.5, cfg, SEED, 0, first, n)
        return fr
    return sim.simulate_point(run_batch, ctx.graph.N, t, ebn0, batch, device=0)


def _run_async(ctx, batch):
    from ldpcsimulation_amd import sim
    cfg = _cfg()

    def run_launch(first, n, frames_dev):
        ctx.sim_launch(EBN0, 0.5, cfg, SEED, 0, first, n, frames_dev)
    launcher = sim.AsyncLauncher(ctx, batch, run_launch)
    try:
        return sim.simulate_point(None, ctx.graph.N, T, EBN0, batch, device=0, launcher=launcher)
    finally:
        ctx.set_stream(None)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, batch, path, q, case="c2"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ldpcsimulation_amd import native
        ctx = native.Context(native.Graph.from_alist(path), 0, batch)
        res = _run(ctx, batch, case)
        q.put((rank, res.counts, res.hist.tolist(), res.rounds))
    except Exception as e:   # report, never hang the parent
        q.put((rank, repr(e), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_on_the_hip_path_equal_one_rank(gpu_ctx_factory):
    import torch.multiprocessing as mp
    one = _run(gpu_ctx_factory(CODE, 2048), 2048)
    assert one.counts["frame_err"] >= 40 and one.counts["bit_err"] >= 200
    other_batch = _run(gpu_ctx_factory(CODE, 768), 768)
    assert other_batch.counts == one.counts and np.array_equal(other_batch.hist, one.hist)
    # rounds launched ahead (sim.AsyncLauncher: round k+1 decodes while round k is reduced)
    piped = _run_async(gpu_ctx_factory(CODE, 512), 512)
    assert piped.counts == one.counts and np.array_equal(piped.hist, one.hist)
    assert piped.rounds >= 4

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 1024, code_path(CODE), q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, counts, hist, rounds in out:
        assert isinstance(counts, dict), counts
        assert counts == one.counts, (rank, counts, one.counts)
        assert np.array_equal(np.array(hist), one.hist), rank


@pytest.mark.gpu
def test_dvbs2_layered_sweep_point_two_ranks_equal_one_rank(gpu_ctx_factory):
    """Config 3 on the HIP path: one SNR point of the DVB-S2 layered sweep, two gloo
    ranks (batch 48 each) against one rank at batch 96 and at batch 40."""
    import torch.multiprocessing as mp
    one = _run(gpu_ctx_factory(DVB_CODE, 96), 96, "c3")
    assert one.counts["frame_err"] >= 40 and one.counts["bit_err"] >= 200
    other = _run(gpu_ctx_factory(DVB_CODE, 40), 40, "c3")
    assert other.counts == one.counts and np.array_equal(other.hist, one.hist)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 48, code_path(DVB_CODE), q, "c3")) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, counts, hist, rounds in out:
        assert isinstance(counts, dict), counts
        assert counts == one.counts, (rank, counts, one.counts)
        assert np.array_equal(np.array(hist), one.hist), rank


@pytest.mark.gpu
def test_sweep_main_two_ranks(tmp_path):
    """sweep.main itself with two ranks (torch.distributed.run as a
    child process, gloo, both ranks on the box's one GPU) and no --seed: the ranks key
    their noise with rank 0's seed (broadcast), rank 0 alone appends one reference-format
    log line per point (decodeMinSum.cpp:313-329), and the counts equal a one-rank run
    with that seed."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    log2 = tmp_path / "two.txt"
    args = [code_path(CODE), "--rate", "0.5", "--snr", "1.25", "1.5", "-T", "50", "--variant", "nms",
            "--alpha", "1.25", "--batch", "2048", "--json"]
    env = dict(os.environ, LDPC_SWEEP_REPORT_SEED="1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        "-m", "ldpcsimulation_amd.sweep"] + args + ["--backend", "gloo", "--share-device",
                                                                    "--log-file", str(log2)],
                       cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    seeds = {}   # the two ranks' stderr lines may interleave without a newline between them
    for m in re.finditer(r'\{"rank": \d+, "seed": \d+\}', p.stderr):
        d = json.loads(m.group(0))
        seeds[d["rank"]] = d["seed"]
    assert set(seeds) == {0, 1} and seeds[0] == seeds[1], seeds
    lines = log2.read_text().splitlines()
    assert len(lines) == 2, lines                       # rank 0 only, one line per point
    assert [l.split("\t")[0] for l in lines] == ["1.25", "1.5"]
    two = [json.loads(l[l.index("{"):]) for l in p.stdout.splitlines() if '"ebn0_db"' in l]
    assert len(two) == 2 and all(d["n_gpus"] == 2 and d["precision"] == "f64" for d in two)
    log1 = tmp_path / "one.txt"
    q = subprocess.run([sys.executable, "-m", "ldpcsimulation_amd.sweep"] + args +
                       ["--seed", str(seeds[0]), "--log", str(log1)], cwd=root, capture_output=True, text=True,
                       timeout=600)
    assert q.returncode == 0, q.stderr[-3000:]
    one = [json.loads(l[l.index("{"):]) for l in q.stdout.splitlines() if '"ebn0_db"' in l]
    keys = ("bit_err", "frame_err", "uncoded_bit_err", "frames", "iters", "syndrome_fail")
    for a, b in zip(two, one):
        assert {k: a[k] for k in keys} == {k: b[k] for k in keys}, (a, b)
    assert log1.read_text().splitlines() == lines


@pytest.mark.gpu
def test_sweep_checkpoint_resume(tmp_path):
    """SURVEY §5 checkpoint/resume on the HIP path: `sweep.py --checkpoint` writes the
    uninterrupted run's log lines; with its .partial file cut back to mid-point
    states (a sweep killed during point 1), a restart resumes both points and appends
    the same lines; a restart of a finished sweep decodes and appends nothing. (The
    default --checkpoint-interval of 10 s records at most one round per 10 s; this
    test records every round.)"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = [code_path(CODE), "--rate", "0.5", "--snr", "1.5", "1.75", "-T", "50", "--variant", "nms",
            "--alpha", "1.25", "--batch", "2048", "--seed", "777", "--json"]

    def run(*extra):
        p = subprocess.run([sys.executable, "-m", "ldpcsimulation_amd.sweep"] + args + list(extra), cwd=root,
                           capture_output=True, text=True, timeout=600)
        assert p.returncode == 0, p.stderr[-3000:]
        return [json.loads(l[l.index("{"):]) for l in p.stdout.splitlines() if '"ebn0_db"' in l]

    run("--log", str(tmp_path / "full.txt"))
    want = (tmp_path / "full.txt").read_text().splitlines()
    ck = tmp_path / "ck.partial"
    run("--log", str(tmp_path / "a.txt"), "--checkpoint", str(ck), "--checkpoint-interval", "0")   # every round
    assert (tmp_path / "a.txt").read_text().splitlines() == want
    recs = [json.loads(l) for l in ck.read_text().splitlines()]
    r1 = [r for r in recs if r["kind"] == "round" and r["k"] == 1]
    assert len(r1) >= 4, len(r1)
    kept = [r for r in recs if r["kind"] == "header" or (r["kind"] == "round" and r["k"] == 0)] + r1[:3]
    ck.write_text("".join(json.dumps(r) + "\n" for r in kept))
    js = run("--log", str(tmp_path / "b.txt"), "--checkpoint", str(ck))
    assert (tmp_path / "b.txt").read_text().splitlines() == want
    assert js[1]["resumed_from_frame"] == r1[2]["next_frame"] > 0
    assert run("--log", str(tmp_path / "c.txt"), "--checkpoint", str(ck)) == []
    assert not (tmp_path / "c.txt").exists()


def _torchrun1(root, args, timeout=600):
    """One rank under torchrun (WORLD_SIZE=1): the process group exists, so every counter
    all-reduce and the cut round's all_gather go through the collective backend."""
    return subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                           "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args,
                          cwd=root, env=dict(os.environ), capture_output=True, text=True, timeout=timeout)


@pytest.mark.gpu
def test_sweep_one_rank_rccl_equals_no_dist(tmp_path):
    """the RCCL path executes on the MI355X. sweep.main under a one-rank
    torchrun with --backend nccl (init_process_group("nccl", device_id=...), the int64
    device all-reduce of every round, the device all_gather of the cut round where the
    stop rule is crossed) gives the totals and the log line of a run without
    torch.distributed -- the process-per-point model of
    scripts/minsum_example_PEGReg504x1008.sh:23-27 and the stop rule of
    decodeMinSum.cpp:189."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = [code_path(CODE), "--rate", "0.5", "--snr", "1.5", "-T", "50", "--variant", "nms", "--alpha", "1.25",
            "--batch", "2048", "--seed", "4242", "--json"]
    p = _torchrun1(root, ["-m", "ldpcsimulation_amd.sweep"] + args + ["--backend", "nccl",
                                                                       "--log-file", str(tmp_path / "nccl.txt")])
    assert p.returncode == 0, p.stderr[-3000:]
    d = [json.loads(l[l.index("{"):]) for l in p.stdout.splitlines() if '"ebn0_db"' in l]
    assert len(d) == 1
    col = d[0]["collectives"]
    assert col["backend"] == "nccl" and col["world"] == 1, col
    assert col["allreduce"] >= 2 and col["allgather"] >= 1, col     # rounds + the exact-stop cut round
    q = subprocess.run([sys.executable, "-m", "ldpcsimulation_amd.sweep"] + args + ["--log", str(tmp_path / "plain.txt")],
                       cwd=root, capture_output=True, text=True, timeout=600)
    assert q.returncode == 0, q.stderr[-3000:]
    e = [json.loads(l[l.index("{"):]) for l in q.stdout.splitlines() if '"ebn0_db"' in l]
    assert e[0]["collectives"]["backend"] is None
    keys = ("bit_err", "frame_err", "uncoded_bit_err", "frames", "iters", "syndrome_fail")
    assert {k: d[0][k] for k in keys} == {k: e[0][k] for k in keys}
    assert d[0]["frame_err"] >= 40 and d[0]["bit_err"] >= 200
    assert (tmp_path / "nccl.txt").read_text() == (tmp_path / "plain.txt").read_text()


@pytest.mark.gpu
def test_bench_one_rank_rccl_line():
    """bench.py --gpus 1 --backend nccl under a one-rank torchrun runs
    its per-step RCCL all-reduce, barrier and max-over-ranks timing and prints a valid
    line (the driver's 8-GPU launch is this command with --nproc-per-node 8)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = _torchrun1(root, ["bench.py", "--gpus", "1", "--backend", "nccl", "--steps", "2", "--warmup", "1",
                          "--batch", "8192", "--no-cpu-baseline", "--no-secondary", "--live-pmc", "off"])
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert line["collective_backend"] == "nccl" and line["n_gpus"] == 1 and line["steps"] == 2
    assert line["value"] > 0 and line["fer"]["frames"] == 2 * 8192
    assert line["kernel_info"]["kernel"] == "rows_pp"


@pytest.mark.gpu
def test_bench_two_ranks_share_device_line():
    """bench.py's world > 1 branches execute on the MI355X before the
    driver's 8-GPU run does -- the torchrun child it spawns itself (nothing touched the
    GPU before), the per-rank `first` offsets, global_batch, the max-over-ranks elapsed
    and the frames_total == steps * B * world assertion. Two ranks share device 0 and
    exchange over gloo (the frame sharding of scripts/minsum_example_PEGReg504x1008.sh:23-27
    replaced by frame-index shards; decodeMinSum.cpp:189's frame loop per shard)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--backend", "gloo", "--share-device",
                        "--steps", "2", "--warmup", "1", "--batch", "4096", "--no-cpu-baseline", "--no-secondary",
                        "--live-pmc", "off"], cwd=root, env=dict(os.environ), capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1   # rank 0 alone prints
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["steps"] == 2 and line["scaling"] == "weak"
    assert line["config"]["global_batch"] == 8192 and line["config"]["batch_per_gpu"] == 4096
    assert line["fer"]["frames"] == 2 * 2 * 4096
    assert line["kernel_info"]["kernel"] == "rows_pp"
    assert line["collective_backend"] == "gloo"
    assert line["value"] > 0 and line["ms_per_step"] > 0
