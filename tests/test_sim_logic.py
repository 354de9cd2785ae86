"""The SNR-point driver without a GPU: the reference's stop rule applied exactly,
independent of batch size and of the number of ranks (gloo, world_size 2).

Frame outcomes come from a deterministic fake keyed by the global frame index,
standing in for ldpc_sim_batch (which is keyed the same way on the device)."""
import os
import socket

import numpy as np
import pytest

from ldpcsimulation_amd import sim
from ldpcsimulation_amd.native import FRAME_DTYPE

N, T = 1944, 50


def fake_frames(first, n):
    f = np.arange(first, first + n, dtype=np.int64)
    h = (f * 2654435761) & 0xFFFFFFFF
    w = np.where((h >> 7) % 97 < 6, (h % 23) + 1, 0)
    out = np.zeros(n, dtype=FRAME_DTYPE)
    out["bit_err"] = w
    out["uncoded_bit_err"] = (h >> 3) % 211
    out["syndrome_fail"] = ((w > 0) & (f % 3 == 0)).astype(np.int32)
    return out


def sequential(min_bit=200, min_frame=40, max_frames=None):
    """Frame-by-frame loop of decodeMinSum.cpp:189-288 on the fake outcomes."""
    acc = np.zeros(6, dtype=np.int64)
    hist = np.zeros(N, dtype=np.int64)
    f = 0
    while acc[0] < min_bit or acc[1] < min_frame:
        if max_frames is not None and acc[3] >= max_frames:
            break
        r = fake_frames(f, 1)[0]
        w = int(r["bit_err"])
        acc += (w, w > 0, r["uncoded_bit_err"], 1, T, r["syndrome_fail"])
        if w:
            hist[w - 1] += 1
        f += 1
    return dict(zip(sim.COUNT_KEYS, (int(x) for x in acc))), hist


@pytest.mark.parametrize("batch", [1, 7, 64, 1000, 5000])
def test_exact_stop_independent_of_batch(batch):
    want, hist = sequential()
    res = sim.simulate_point(fake_frames, N, T, 1.5, batch)
    assert res.counts == want
    assert np.array_equal(res.hist, hist)


def test_stop_rule_needs_both_thresholds():
    assert not sim.stop_reached(199, 100)
    assert not sim.stop_reached(1000, 39)
    assert sim.stop_reached(200, 40)


def test_max_frames_cap():
    want, _ = sequential(min_bit=10 ** 9, min_frame=10 ** 9, max_frames=777)
    res = sim.simulate_point(fake_frames, N, T, 1.5, 100, min_bit_err=10 ** 9, min_frame_err=10 ** 9,
                             max_frames=777)
    assert res.counts == want and res.counts["frames"] == 777


def test_log_line_format():
    r = sim.PointResult(1.5, 1008, 10, {"bit_err": 1715, "frame_err": 40, "uncoded_bit_err": 0,
                                        "frames": 63, "iters": 630, "syndrome_fail": 0})
    # the reference's own line for this run: "2\t0.0270062\t10\t0.634921\t10\t<alist>"
    assert r.log_line("x.alist") == "1.5\t0.0270062\t10\t0.634921\t10\tx.alist"


def test_wilson_and_z():
    lo, hi = sim.wilson_interval(40, 2212)
    assert lo < 40 / 2212 < hi
    assert abs(sim.two_proportion_z(40, 2212, 40, 2212)) < 1e-12


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, batch, q, first_round=None, high_fer=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = sim.simulate_point(fake_frames_high_fer if high_fer else fake_frames, N, T, 1.0, batch,
                                 first_round=first_round)
        q.put((rank, res.counts, res.hist.tolist(), res.rounds, res.frames_decoded))
    finally:
        dist.destroy_process_group()


def _two_ranks(batch, first_round=None, high_fer=False):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, batch, q, first_round, high_fer)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("batch", [16, 300])
def test_two_ranks_gloo_identical_to_sequential(batch):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, batch, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want, hist = sequential()
    for rank, counts, h, rounds, _ in out:
        assert counts == want, rank
        assert np.array_equal(np.array(h), hist)


def fake_frames_high_fer(first, n):
    """A low-SNR point (FER ~0.4, as 802.11n N=1944 NMS at 1.0 dB): the stop rule is
    reached after ~100 frames."""
    out = fake_frames(first, n)
    f = np.arange(first, first + n, dtype=np.int64)
    h = (f * 2246822519) & 0xFFFFFFFF
    out["bit_err"] = np.where((h >> 9) % 5 < 2, (h % 37) + 3, 0)
    return out


def sequential_of(gen, min_bit=200, min_frame=40):
    acc = np.zeros(6, dtype=np.int64)
    f = 0
    while acc[0] < min_bit or acc[1] < min_frame:
        r = gen(f, 1)[0]
        w = int(r["bit_err"])
        acc += (w, w > 0, r["uncoded_bit_err"], 1, T, r["syndrome_fail"])
        f += 1
    return dict(zip(sim.COUNT_KEYS, (int(x) for x in acc)))


def test_round_sizes_double_up_to_batch():
    g = sim.round_sizes(65536)
    assert [next(g) for _ in range(9)] == [1024, 2048, 4096, 8192, 16384, 32768, 65536, 65536, 65536]
    g = sim.round_sizes(3000, first_round=1000)
    assert [next(g) for _ in range(4)] == [1000, 2000, 3000, 3000]
    g = sim.round_sizes(500)
    assert [next(g) for _ in range(2)] == [500, 500]


@pytest.mark.parametrize("first_round", [None, 1, 100, 65536])
def test_adaptive_rounds_same_totals(first_round):
    """Any first-round size gives the sequential totals and histogram (exact_stop)."""
    want, hist = sequential()
    res = sim.simulate_point(fake_frames, N, T, 1.5, 65536, first_round=first_round)
    assert res.counts == want and np.array_equal(res.hist, hist)
    L = _FakeLauncher()
    res = sim.simulate_point(fake_frames, N, T, 1.5, 65536, first_round=first_round, launcher=L)
    assert res.counts == want and np.array_equal(res.hist, hist) and not L.pending


def test_adaptive_rounds_decode_fewer_frames_at_high_fer():
    """at FER ~0.4 the default first round (1024) stops after one
    round, where fixed 65,536-frame rounds decode 65,536 frames for ~100 needed."""
    want = sequential_of(fake_frames_high_fer)
    assert want["frames"] < 200
    fixed = sim.simulate_point(fake_frames_high_fer, N, T, 1.0, 65536, first_round=65536)
    adapt = sim.simulate_point(fake_frames_high_fer, N, T, 1.0, 65536)
    assert fixed.counts == want and adapt.counts == want
    assert fixed.frames_decoded == 65536 and adapt.frames_decoded == 1024


def test_adaptive_rounds_two_ranks_gloo():
    """world 2 (gloo): the adaptive rounds give the sequential totals on both ranks and
    decode 2 x 1024 frames at the high-FER point (fixed rounds: 2 x 65,536)."""
    want = sequential_of(fake_frames_high_fer)
    for first_round, decoded in ((None, 2048), (65536, 131072)):
        for rank, counts, h, rounds, dec in _two_ranks(65536, first_round, high_fer=True):
            assert counts == want, (rank, first_round)
            assert dec == decoded, (rank, first_round, dec)


def fake_frames_early_stop(first, n):
    """As fake_frames, with a per-frame iteration count (early-stopping decoders: GDBF, EMS)."""
    out = fake_frames(first, n)
    f = np.arange(first, first + n, dtype=np.int64)
    out["iters"] = np.where(out["bit_err"] > 0, T, 1 + (f * 40503) % 17)
    return out


@pytest.mark.parametrize("batch", [1, 64, 5000])
def test_exact_stop_counts_reported_iterations(batch):
    """iters_in_frames: avgIt is the sum of the frames' own iteration counts up to the exact stop."""
    want, _ = sequential()
    frames = fake_frames_early_stop(0, want["frames"])
    res = sim.simulate_point(fake_frames_early_stop, N, T, 1.5, batch, iters_in_frames=True)
    assert res.counts["frames"] == want["frames"] and res.counts["bit_err"] == want["bit_err"]
    assert res.counts["iters"] == int(frames["iters"].sum())
    assert res.avg_iters < T


class _FakeLauncher:
    """Two-slot launcher over the fake frames, recording what was launched."""

    def __init__(self):
        self.pending = {}
        self.launched = []

    def launch(self, slot, first, n):
        assert slot not in self.pending, "slot reused before it was collected"
        self.pending[slot] = (first, n)
        self.launched.append(first)

    def collect(self, slot):
        first, n = self.pending.pop(slot)
        return fake_frames(first, n)


@pytest.mark.parametrize("batch", [7, 64, 1000])
def test_pipelined_rounds_identical_to_sequential(batch):
    """simulate_point with a launcher (round k+1 launched before round k is reduced)
    gives the sequential totals; every launched slot is collected; at most one round
    beyond the last needed one is launched."""
    want, hist = sequential()
    L = _FakeLauncher()
    res = sim.simulate_point(fake_frames, N, T, 1.5, batch, launcher=L)
    assert res.counts == want and np.array_equal(res.hist, hist)
    assert not L.pending
    assert len(L.launched) <= res.rounds + 1
    assert L.launched == sorted(set(L.launched))
    if res.rounds > 4:
        assert len(L.launched) == res.rounds + 1 or len(L.launched) == res.rounds


def test_pipelined_rounds_respect_max_frames():
    want, _ = sequential(min_bit=10 ** 9, min_frame=10 ** 9, max_frames=777)
    L = _FakeLauncher()
    res = sim.simulate_point(fake_frames, N, T, 1.5, 50, min_bit_err=10 ** 9, min_frame_err=10 ** 9,
                             max_frames=777, launcher=L)
    assert res.counts == want and not L.pending


def _states(gen=fake_frames, batch=100, launcher=None):
    st = []
    res = sim.simulate_point(gen, N, T, 1.5, batch, on_round=st.append, launcher=launcher)
    return res, st


@pytest.mark.parametrize("batch", [7, 100, 1000])
def test_resume_from_any_round_equals_uninterrupted(batch):
    """SURVEY §5 checkpoint/resume: the state after any fully counted round, fed back as
    `resume` (also with other round sizes and a launcher), gives the uninterrupted
    run's totals and histogram: the reference's frame-by-frame result."""
    want, hist = sequential()
    full, states = _states(batch=batch)
    assert full.counts == want and np.array_equal(full.hist, hist)
    assert len(states) == full.rounds - 1            # every round but the one the stop cuts
    for st in states:
        assert st.acc[3] == st.next_frame           # one rank: every frame before next_frame counted
        for b2, L in ((batch, None), (3 * batch + 1, None), (batch, _FakeLauncher())):
            res = sim.simulate_point(fake_frames, N, T, 1.5, b2, resume=st, launcher=L)
            assert res.counts == want and np.array_equal(res.hist, hist), (st.next_frame, b2)
            assert res.rounds >= st.rounds


def test_resume_state_histogram_matches_counters():
    _, states = _states(batch=64)
    for st in states:
        w = np.arange(1, N + 1)
        assert int((st.hist * w).sum()) == int(st.acc[0]) and int(st.hist.sum()) == int(st.acc[1])


def _resume_worker(rank, world, port, q, resume):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        st = []
        res = sim.simulate_point(fake_frames, N, T, 1.5, 50, resume=resume, on_round=st.append)
        q.put((rank, res.counts, res.hist.tolist(), [(s.next_frame, s.acc.tolist(), s.hist.tolist()) for s in st]))
    finally:
        dist.destroy_process_group()


def test_resume_two_ranks_gloo():
    """A one-rank checkpoint resumed on two ranks (and the two ranks' own per-round
    states, identical on both, all-reduced histogram) reproduce the sequential run."""
    import torch.multiprocessing as mp
    want, hist = sequential()
    _, states = _states(batch=100)
    mid = states[len(states) // 2]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_resume_worker, args=(r, 2, port, q, mid)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, counts, h, st in out:
        assert counts == want and np.array_equal(np.array(h), hist), rank
    assert out[0][3] == out[1][3]
    for nf, acc, h in out[0][3]:
        res = sim.simulate_point(fake_frames, N, T, 1.5, 77, resume=sim.PointState(nf, np.array(acc), np.array(h)))
        assert res.counts == want and np.array_equal(res.hist, hist)


# ---- world sizes 1, 2, 4 and 8 ----
# One spawned process group per world size runs a list of scenarios; every rank
# must report the sequential run's totals and histogram (decodeMinSum.cpp:189: the
# stop rule cuts at the same frame for any W), whatever the batch, the first round,
# the launcher or a resumed state.

def _run_scenario(sc, rank):
    gen = {"fake": fake_frames, "high": fake_frames_high_fer}[sc["gen"]]
    st = []
    interval = sc.get("interval", (0.0, 0.0))
    res = sim.simulate_point(gen, N, T, 1.5, sc["batch"], first_round=sc.get("first_round"),
                             launcher=_FakeLauncher() if sc.get("launcher") else None,
                             resume=sc.get("resume"), on_round=st.append if sc.get("collect") else None,
                             on_round_interval=interval[0] if rank == 0 else interval[1])
    return (res.counts, res.hist.tolist(), res.rounds, res.frames_decoded,
            [(s.next_frame, s.acc.tolist(), s.hist.tolist(), s.rounds, s.frames_decoded) for s in st])


def _scenario_worker(rank, world, port, q, scenarios):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, [_run_scenario(sc, rank) for sc in scenarios]))
    finally:
        dist.destroy_process_group()


def _ranks(world, scenarios):
    """Results per scenario, as a list over ranks (rank order)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scenario_worker, args=(r, world, port, q, scenarios)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [[out[r][i] for r in range(world)] for i in range(len(scenarios))]


SCENARIOS = [
    dict(gen="fake", batch=16),                              # many small rounds
    dict(gen="fake", batch=300),                             # uneven batch, adaptive first round min(300, 1024)
    dict(gen="fake", batch=1000, first_round=7),             # first round 7 per rank, doubling to 1000
    dict(gen="fake", batch=37, first_round=5, launcher=True),   # rounds launched ahead
    dict(gen="high", batch=65536),                           # high FER: stops inside the first round
    dict(gen="fake", batch=50, collect=True),                # per-round states (all-reduced histograms)
    dict(gen="fake", batch=50, collect=True, interval=(0.0, 1e9)),   # rank 0's clock decides for all
]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_world_sizes_identical_to_sequential(world):
    want, hist = sequential()
    want_high = sequential_of(fake_frames_high_fer)
    per = _ranks(world, SCENARIOS)
    for sc, ranks in zip(SCENARIOS, per):
        for rank, (counts, h, rounds, decoded, states) in enumerate(ranks):
            if sc["gen"] == "high":
                assert counts == want_high, (world, rank)
                assert decoded == min(1024, sc["batch"]) * world   # one adaptive round
                continue
            assert counts == want, (world, rank, sc)
            assert np.array_equal(np.array(h), hist), (world, rank, sc)
            if sc.get("collect"):
                assert states == ranks[0][4], (world, rank, sc)     # the same states on every rank
                assert len(states) == rounds - 1                    # every round but the cut one
                for nf, acc, sh, _, _ in states:
                    assert acc[3] == nf and int(np.sum(sh)) == acc[1]


def test_checkpoint_w2_resumed_at_w4_and_w1():
    """A state checkpointed by two ranks resumes on four ranks (and on one) with the
    uninterrupted run's totals and histogram."""
    want, hist = sequential()
    (ranks2,) = _ranks(2, [dict(gen="fake", batch=40, collect=True)])
    states = ranks2[0][4]
    assert len(states) >= 3
    resumes = [sim.PointState(nf, np.array(acc), np.array(h), r, d) for nf, acc, h, r, d in states[1::2]]
    scen = [dict(gen="fake", batch=b, resume=st) for st in resumes for b in (40, 23)]
    for world in (4, 1):
        for sc, ranks in zip(scen, _ranks(world, scen)):
            for rank, (counts, h, rounds, decoded, _) in enumerate(ranks):
                assert counts == want and np.array_equal(np.array(h), hist), (world, rank, sc["batch"])
                assert rounds >= sc["resume"].rounds
