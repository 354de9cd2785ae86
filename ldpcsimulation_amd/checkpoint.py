"""Per-round checkpoints of an SNR sweep, so a killed sweep resumes where it stopped.

The reference keeps nothing but the final log line of a point
(C_implementations/src/decodeMinSum.cpp:313-329): a process killed after hours
of frames loses the whole SNR point. Here every fully counted round
of a point appends its running state to a `.partial` file -- JSON lines:

    {"kind": "header", "version": 1, "seed": S, "config": {...}}
    {"kind": "round", "k": k, "snr": x, "next_frame": F, "acc": [6 counters],
     "hist": [[w, count], ...], "rounds": r, "frames_decoded": d}
    {"kind": "done", "k": k, "snr": x, "line": "<the point's log line>"}

Noise is keyed by (seed, point index k, global frame index), so decoding on from
next_frame with the stored counters gives exactly the uninterrupted run's totals
and histogram (sim.simulate_point's exact stop), whatever the number of GPUs or
round sizes of either run. The header pins the seed and every setting that
changes results; resuming with different settings is refused.
"""
from __future__ import annotations

import hashlib
import json
import os
from typing import Optional

import numpy as np

from .sim import PointState

VERSION = 1


def file_digest(path: Optional[str]) -> Optional[str]:
    """md5 of a file's bytes (the code or codeword file a result depends on)."""
    if not path:
        return None
    h = hashlib.md5()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


class CheckpointMismatch(RuntimeError):
    pass


class SweepCheckpoint:
    """A sweep's `.partial` file. Every rank loads it (read-only); only the writer
    (rank 0) appends. Records past a torn last line (a kill mid-write) are ignored."""

    def __init__(self, path: str, config: dict, writer: bool):
        self.path, self.config, self.writer = path, config, writer
        self.seed: Optional[int] = None
        self._rounds: dict = {}     # k -> last round record
        self._done: dict = {}       # k -> done record
        self._has_header = False
        self._repair = None         # (valid bytes, add a newline) when the file's tail needs fixing
        if os.path.exists(path):
            self._load()

    def _load(self):
        with open(self.path, "rb") as f:
            data = f.read()
        lines = data.split(b"\n")        # the last piece is b"" when the file ends with a newline
        end = 0                            # byte offset just past the last complete record
        for i, raw in enumerate(lines):
            last = i == len(lines) - 1
            if last and not raw:
                break
            try:
                rec = json.loads(raw)
            except (json.JSONDecodeError, UnicodeDecodeError):
                if last:
                    break           # torn last record: cut off before the next append
                raise CheckpointMismatch(f"{self.path}: line {i + 1} is not JSON")
            end += len(raw) + (0 if last else 1)
            kind = rec.get("kind")
            if kind == "header":
                if rec.get("version") != VERSION:
                    raise CheckpointMismatch(f"{self.path}: version {rec.get('version')} != {VERSION}")
                if rec.get("config") != self.config:
                    diff = sorted(k for k in set(rec.get("config", {})) | set(self.config)
                                  if rec.get("config", {}).get(k) != self.config.get(k))
                    raise CheckpointMismatch(f"{self.path}: settings differ from the checkpoint's: {diff}")
                self.seed = int(rec["seed"])
                self._has_header = True
            elif kind == "round":
                self._rounds[int(rec["k"])] = rec
            elif kind == "done":
                self._done[int(rec["k"])] = rec
        if not self._has_header and (self._rounds or self._done):
            raise CheckpointMismatch(f"{self.path}: records without a header")
        # what the writer repairs before its first append: the torn tail dropped, and a
        # complete last record that lost its newline terminated
        newline = end > 0 and not data[:end].endswith(b"\n")
        self._repair = (end, newline) if end != len(data) or newline else None

    def _append(self, rec: dict):
        if not self.writer:
            return
        if self._repair is not None:
            end, newline = self._repair
            with open(self.path, "r+b") as f:
                f.truncate(end)
                f.seek(end)
                if newline:
                    f.write(b"\n")
                f.flush()
                os.fsync(f.fileno())
            self._repair = None
        with open(self.path, "a") as f:
            f.write(json.dumps(rec, separators=(",", ":")) + "\n")
            f.flush()
            os.fsync(f.fileno())

    def start(self, seed: int):
        """Pin the seed (a new file gets its header)."""
        if self._has_header:
            if seed != self.seed:
                raise CheckpointMismatch(f"{self.path}: seed {seed} != the checkpoint's {self.seed}")
            return
        self.seed = seed
        self._has_header = True
        self._append({"kind": "header", "version": VERSION, "seed": int(seed), "config": self.config})

    def done_line(self, k: int, snr: float) -> Optional[str]:
        rec = self._done.get(k)
        if rec is None:
            return None
        if rec["snr"] != snr:
            raise CheckpointMismatch(f"{self.path}: point {k} was {rec['snr']} dB, now {snr}")
        return rec["line"]

    def point_state(self, k: int, snr: float, n_hist: int) -> Optional[PointState]:
        rec = self._rounds.get(k)
        if rec is None:
            return None
        if rec["snr"] != snr:
            raise CheckpointMismatch(f"{self.path}: point {k} was {rec['snr']} dB, now {snr}")
        hist = np.zeros(n_hist, dtype=np.int64)
        for w, c in rec["hist"]:
            hist[int(w) - 1] = int(c)
        return PointState(int(rec["next_frame"]), np.array(rec["acc"], dtype=np.int64), hist,
                          int(rec["rounds"]), int(rec["frames_decoded"]))

    def save_round(self, k: int, snr: float, st: PointState):
        nz = np.nonzero(st.hist)[0]
        self._append({"kind": "round", "k": k, "snr": snr, "next_frame": int(st.next_frame),
                      "acc": [int(x) for x in st.acc], "hist": [[int(i) + 1, int(st.hist[i])] for i in nz],
                      "rounds": int(st.rounds), "frames_decoded": int(st.frames_decoded)})

    def save_done(self, k: int, snr: float, line: str):
        self._append({"kind": "done", "k": k, "snr": snr, "line": line})
