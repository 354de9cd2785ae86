"""Monte-Carlo SNR driver: the reference's per-SNR frame loop, batched and sharded.

Reference: C_implementations/src/decodeMinSum.cpp:146-311 (one SNR point per
process; frames until errors >= 200 AND wordErrors >= 40) and the sweep
scripts (scripts/minsum_example_*.sh:23-27, one background process per SNR
point appending one line each to a shared log).

Here one SNR point is a sequence of rounds. In round k, rank r of W decodes
the global frames [k*B*W + r*B, k*B*W + (r+1)*B) on its own GPU with
counter-based noise keyed by the global frame index, so the frames -- and the
statistics for a given total -- do not depend on W or B. After each round the
six int64 counters are summed over ranks (one all-reduce of 48 bytes, RCCL
over xGMI with the nccl backend, gloo on CPU). With exact_stop (default) the
round that crosses the stop rule gathers its per-frame results and cuts at the
exact frame where the sequential reference would have stopped, so the
reported totals equal a frame-by-frame run of the same noise.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np

from .native import FRAME_DTYPE

COUNT_KEYS = ("bit_err", "frame_err", "uncoded_bit_err", "frames", "iters", "syndrome_fail")


@dataclass
class PointResult:
    ebn0_db: float
    N: int
    T: int
    counts: dict = field(default_factory=dict)
    rounds: int = 0
    frames_decoded: int = 0             # frames decoded over all ranks, incl. those past the stop
    hist: Optional[np.ndarray] = None   # error_weight_hist (:173), exact-stop frames only
    collectives: dict = field(default_factory=dict)   # backend and calls of the collective layer

    @property
    def ber(self) -> float:
        bits = self.counts["frames"] * self.N
        return self.counts["bit_err"] / bits if bits else float("nan")

    @property
    def fer(self) -> float:
        f = self.counts["frames"]
        return self.counts["frame_err"] / f if f else float("nan")

    @property
    def avg_iters(self) -> float:
        f = self.counts["frames"]
        return self.counts["iters"] / f if f else float("nan")

    def log_line(self, alist_name: str, extra=()) -> str:
        """The reference's log line (:313-329): SNR BER avgIt FER T [Ymax] [alpha] [delta] alist."""
        vals = [_cpp_double(self.ebn0_db), _cpp_double(self.ber), _cpp_double(self.avg_iters),
                _cpp_double(self.fer), str(self.T)] + [_cpp_double(x) for x in extra] + [alist_name]
        return "\t".join(vals)


def _cpp_double(x: float) -> str:
    """std::ostream default formatting of a double (%g, 6 significant digits)."""
    return f"{x:g}"


def stop_reached(bit_err: int, frame_err: int, min_bit_err: int = 200, min_frame_err: int = 40) -> bool:
    """Negation of the loop condition (errors < 200 || wordErrors < 40) at :189."""
    return not (bit_err < min_bit_err or frame_err < min_frame_err)


def exact_cut(prev: np.ndarray, frames: np.ndarray, T: int, min_bit_err=200, min_frame_err=40,
              iters_in_frames: bool = False):
    """Apply the stop rule frame by frame. prev = counters before this round;
    frames = this round's per-frame results in global frame order. Returns
    (counters after the last frame the reference would decode, frames used).
    iters_in_frames: decoders with early stop (GDBF, EMS) report each frame's
    iterations in its 4th field; otherwise every frame ran T."""
    acc = prev.copy()
    used = 0
    for w, unc, syn, its in frames:
        if stop_reached(acc[0], acc[1], min_bit_err, min_frame_err):
            break
        acc += (w, 1 if w > 0 else 0, unc, 1, its if iters_in_frames else T, syn)
        used += 1
    return acc, used


class _Comm:
    """Minimal collective layer: torch.distributed if initialised, else local. With a
    process group the collectives always run, at world size 1 too (a one-rank RCCL
    communicator under torchrun --nproc-per-node 1), so the path an 8-GPU run takes
    is the path a one-GPU run executes."""

    def __init__(self, device=None):
        self.dist = None
        self.rank, self.world = 0, 1
        self.device = device
        self.calls = {"allreduce": 0, "allgather": 0}
        try:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                self.dist = dist
                self.rank, self.world = dist.get_rank(), dist.get_world_size()
        except ImportError:
            pass

    def _tensor(self, arr: np.ndarray):
        import torch
        t = torch.from_numpy(np.array(arr, copy=True))   # a copy: the collective works in place
        if self.dist.get_backend() == "nccl":
            t = t.to(self.device if self.device is not None else "cuda")
        return t

    def allreduce_sum(self, arr: np.ndarray) -> np.ndarray:
        if self.dist is None:
            return arr
        self.calls["allreduce"] += 1
        t = self._tensor(arr)
        self.dist.all_reduce(t)
        return t.cpu().numpy()

    def allgather(self, arr: np.ndarray) -> np.ndarray:
        """Concatenate equal-shaped int arrays from all ranks, in rank order."""
        if self.dist is None:
            return arr
        self.calls["allgather"] += 1
        t = self._tensor(arr)
        out = [t.clone() for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return np.concatenate([o.cpu().numpy() for o in out])


@dataclass
class PointState:
    """An SNR point after its fully counted rounds: what a checkpoint holds
    (checkpoint.py). Frames are keyed by global index, so decoding on from
    next_frame with these totals reproduces the uninterrupted run exactly, for
    any number of ranks and round sizes."""
    next_frame: int                 # first global frame not yet counted
    acc: np.ndarray                 # the six counters (COUNT_KEYS order)
    hist: np.ndarray                # error-weight histogram over all ranks
    rounds: int = 0
    frames_decoded: int = 0


def round_sizes(batch: int, first_round: Optional[int] = None):
    """Frames per rank of rounds 0, 1, 2, ...: first_round (default min(batch, 1024)),
    doubling up to batch. A low-SNR point stops near its 40th frame error after a
    small first round instead of after batch x W frames; a high-SNR point reaches
    full rounds after a few doublings."""
    b = max(1, min(batch, first_round if first_round is not None else 1024))
    while True:
        yield b
        b = min(batch, 2 * b)


def simulate_point(run_batch: Callable[[int, int], np.ndarray], N: int, T: int, ebn0_db: float,
                   batch: int, min_bit_err: int = 200, min_frame_err: int = 40,
                   max_frames: Optional[int] = None, exact_stop: bool = True, device=None,
                   iters_in_frames: bool = False, launcher=None, first_round: Optional[int] = None,
                   resume: Optional[PointState] = None,
                   on_round: Optional[Callable[[PointState], None]] = None,
                   on_round_interval: float = 0.0) -> PointResult:
    """Run one SNR point to the reference's stop rule.

    run_batch(first_cw, n) must decode global frames first_cw..first_cw+n-1 on
    this rank and return their per-frame results (FRAME_DTYPE). All ranks of
    an initialised torch.distributed group must call this together.

    Round k decodes b_k frames per rank (round_sizes: first_round doubling up to
    batch). The global frames are still consumed in order -- round k covers
    [sum_{j<k} b_j W, sum_{j<=k} b_j W), rank r the r-th block of b_k -- so the
    totals (exact_stop) equal a frame-by-frame run for any W, batch and first_round.

    launcher (optional, e.g. AsyncLauncher): launch(slot, first_cw, n) starts a
    round without waiting and collect(slot) returns its frames. Then, once the
    counts show that at least two more rounds are needed, round k+1 is launched
    before round k is reduced, so the host-side reduction and the all-reduce
    overlap the next decode. The results are the same: frames are keyed by
    global index and a round launched ahead of the stop is discarded.

    resume: start from a checkpointed PointState (the same on every rank) instead
    of frame 0. on_round(state): called on every rank after a fully counted
    round with the point's state (its histogram all-reduced: a collective), for
    checkpoints -- after every round, or (on_round_interval > 0 s) after the first
    round that ends at least that long after the previous call. Rank 0's clock
    decides, and its decision rides in the round's counter all-reduce, so every
    rank makes the same call without another collective."""
    comm = _Comm(device)
    t_saved = time.monotonic()
    acc = np.zeros(6, dtype=np.int64)
    res = PointResult(ebn0_db, N, T)
    hist_local = np.zeros(N, dtype=np.int64)   # rounds fully counted: this rank's frames
    hist_cut = np.zeros(N, dtype=np.int64)     # the cut round: all ranks' frames (gathered)
    hist_base = np.zeros(N, dtype=np.int64)    # resumed rounds: all ranks' frames
    rnd = 0
    ahead = False          # round rnd already launched (into slot rnd % 2)
    last = None            # the previous round's all-reduced increments
    sizes, starts = [], [0]    # frames per rank of each round; global first frame of each round
    gen = round_sizes(batch, first_round)
    decoded = 0
    rounds0 = 0
    if resume is not None:
        acc = np.asarray(resume.acc, dtype=np.int64).copy()
        hist_base = np.asarray(resume.hist, dtype=np.int64).copy()
        starts = [int(resume.next_frame)]
        decoded, rounds0 = int(resume.frames_decoded), int(resume.rounds)

    def size_of(r):
        while len(sizes) <= r:
            sizes.append(next(gen))
            starts.append(starts[-1] + sizes[-1] * comm.world)
        return sizes[r]

    def first_of(r):
        b = size_of(r)
        return starts[r] + comm.rank * b

    while not stop_reached(acc[0], acc[1], min_bit_err, min_frame_err):
        if max_frames is not None and acc[3] >= max_frames:
            break
        first = first_of(rnd)
        if launcher is None:
            fr = np.ascontiguousarray(run_batch(first, size_of(rnd)))
        else:
            if not ahead:
                launcher.launch(rnd % 2, first, size_of(rnd))
            # launch the next round now when it is surely needed: this round, scaled from the
            # last one by its size, twice over stays below the stop rule and the frame cap
            # (the decision is the same on every rank)
            if last is not None:
                g = 2.0 * size_of(rnd) / size_of(rnd - 1)
                ahead = not stop_reached(acc[0] + g * last[0], acc[1] + g * last[1], min_bit_err, min_frame_err) \
                    and (max_frames is None or acc[3] + g * last[3] < max_frames)
            else:
                ahead = False
            if ahead:
                launcher.launch((rnd + 1) % 2, first_of(rnd + 1), size_of(rnd + 1))
            fr = np.ascontiguousarray(launcher.collect(rnd % 2))
        raw = fr.view(np.int32).reshape(-1, 4)
        want_save = on_round is not None and comm.rank == 0 and \
            (on_round_interval <= 0 or time.monotonic() - t_saved >= on_round_interval)
        local = np.array([raw[:, 0].sum(), (raw[:, 0] > 0).sum(), raw[:, 1].sum(), len(raw),
                          raw[:, 3].sum() if iters_in_frames else T * len(raw), raw[:, 2].sum(),
                          int(want_save)], dtype=np.int64)
        tot7 = comm.allreduce_sum(local)
        tot, save = tot7[:6], tot7[6] > 0
        decoded += int(tot[3])
        last = tot
        after = acc + tot
        crossed = stop_reached(after[0], after[1], min_bit_err, min_frame_err)
        limit_hit = max_frames is not None and after[3] > max_frames
        if exact_stop and (crossed or limit_hit):
            allf = comm.allgather(raw).reshape(-1, 4)
            if limit_hit:
                allf = allf[: max(0, max_frames - int(acc[3]))]
            acc, used = exact_cut(acc, allf, T, min_bit_err, min_frame_err, iters_in_frames)
            w = allf[:used, 0]
            np.add.at(hist_cut, w[w > 0] - 1, 1)
        else:
            acc = after
            w = raw[:, 0]
            np.add.at(hist_local, w[w > 0] - 1, 1)
            if on_round is not None and save:
                t_saved = time.monotonic()
                on_round(PointState(starts[rnd] + size_of(rnd) * comm.world, acc.copy(),
                                    comm.allreduce_sum(hist_local) + hist_base, rounds0 + rnd + 1, decoded))
        rnd += 1
    if launcher is not None and ahead:
        decoded += len(launcher.collect(rnd % 2)) * comm.world   # drain the round launched past the stop
    hist = comm.allreduce_sum(hist_local) + hist_cut + hist_base
    res.counts = dict(zip(COUNT_KEYS, (int(x) for x in acc)))
    res.rounds = rounds0 + rnd
    res.frames_decoded = decoded
    res.hist = hist
    res.collectives = {"backend": comm.dist.get_backend() if comm.dist else None, "world": comm.world, **comm.calls}
    return res


def wilson_interval(k: int, n: int, z: float = 1.96):
    if n == 0:
        return (float("nan"), float("nan"))
    p = k / n
    den = 1 + z * z / n
    c = (p + z * z / (2 * n)) / den
    h = z * math.sqrt(p * (1 - p) / n + z * z / (4 * n * n)) / den
    return (c - h, c + h)


def two_proportion_z(k1: int, n1: int, k2: int, n2: int) -> float:
    """z statistic of H0: p1 == p2 (pooled)."""
    p = (k1 + k2) / (n1 + n2)
    se = math.sqrt(p * (1 - p) * (1 / n1 + 1 / n2))
    return 0.0 if se == 0 else (k1 / n1 - k2 / n2) / se


class AsyncLauncher:
    """Two-slot asynchronous rounds on a native Context (ldpc_sim_launch): each slot
    has a device buffer of per-frame results, a pinned host copy and an event, all
    on the context's stream. launch() returns at once; collect() waits for the slot."""

    def __init__(self, ctx, batch: int, run_launch: Callable):
        import torch
        self.torch = torch
        self.stream = torch.cuda.Stream(device=torch.device("cuda", ctx.device))
        ctx.set_stream(self.stream.cuda_stream)
        self.run_launch = run_launch       # run_launch(first_cw, n, frames_dev_tensor)
        self.dev = [torch.empty((batch, 4), dtype=torch.int32, device=f"cuda:{ctx.device}") for _ in range(2)]
        self.host = [torch.empty((batch, 4), dtype=torch.int32).pin_memory() for _ in range(2)]
        self.ev = [torch.cuda.Event() for _ in range(2)]
        self.n = [0, 0]

    def launch(self, slot: int, first: int, n: int):
        with self.torch.cuda.stream(self.stream):
            self.run_launch(first, n, self.dev[slot][:n])
            self.host[slot][:n].copy_(self.dev[slot][:n], non_blocking=True)
            self.ev[slot].record(self.stream)
        self.n[slot] = n

    def collect(self, slot: int) -> np.ndarray:
        self.ev[slot].synchronize()
        return self.host[slot][: self.n[slot]].numpy().copy().view(FRAME_DTYPE).reshape(-1)
