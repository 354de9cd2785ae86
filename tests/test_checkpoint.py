"""Sweep checkpoints (ldpcsimulation_amd/checkpoint.py; SURVEY §5: the reference keeps
only the final log line of a point, decodeMinSum.cpp:313-329). CPU only: the file
format, the refusal of changed settings, and sweep._run_points killed mid-point and
restarted, with the fake frame source of test_sim_logic standing in for the GPU."""
import json

import numpy as np
import pytest

from conftest import code_path
from ldpcsimulation_amd import checkpoint, sim, sweep
from test_sim_logic import N, T, fake_frames, sequential


def _args(tmp_path, *extra):
    return sweep.parse([code_path("80211n_1944_r12.alist"), "--rate", "0.5", "--snr", "1.5", "1.75", "-T", str(T),
                        "--variant", "nms", "--alpha", "1.25", "--log", str(tmp_path / "log.txt"),
                        "--checkpoint", str(tmp_path / "ck.partial"), *extra])


class _Killed(Exception):
    pass


def _point_runner(kill_after_rounds=None):
    """run_point over fake frames (point k: frames offset by k), raising after
    kill_after_rounds checkpointed rounds of the whole sweep."""
    seen = [0]

    def run_point(k, snr, resume, on_round):
        def gen(first, n):
            return fake_frames(first + 100000 * k, n)

        def rec(st):
            on_round(st)
            seen[0] += 1
            if kill_after_rounds is not None and seen[0] >= kill_after_rounds:
                raise _Killed()
        res = sim.simulate_point(gen, N, T, snr, 97, resume=resume, on_round=rec)
        return res, res.log_line("x.alist", [1.25]), {"ebn0_db": snr, **res.counts}
    return run_point


def _sweep(a, runner):
    ck = checkpoint.SweepCheckpoint(a.checkpoint, sweep._checkpoint_config(a), writer=True)
    ck.start(ck.seed if ck.seed is not None else 1234)
    sweep._run_points(a, ck, 0, N, runner)


@pytest.mark.parametrize("kill_after", [1, 3, 9])
def test_killed_sweep_resumes_to_the_same_log(tmp_path, capsys, kill_after):
    ref_dir = tmp_path / "ref"
    ref_dir.mkdir()
    a_ref = _args(ref_dir)
    _sweep(a_ref, _point_runner())
    want = (ref_dir / "log.txt").read_text().splitlines()
    assert len(want) == 2
    a = _args(tmp_path)
    with pytest.raises(_Killed):
        _sweep(a, _point_runner(kill_after))
    recs = [json.loads(l) for l in (tmp_path / "ck.partial").read_text().splitlines()]
    assert recs[0]["kind"] == "header" and recs[0]["seed"] == 1234
    assert sum(r["kind"] == "round" for r in recs) == kill_after
    _sweep(_args(tmp_path), _point_runner())      # restart: same settings, same file
    assert (tmp_path / "log.txt").read_text().splitlines() == want
    # a third run finds both points done: nothing decoded, nothing appended
    _sweep(_args(tmp_path), _point_runner(kill_after_rounds=0))
    assert (tmp_path / "log.txt").read_text().splitlines() == want


def test_first_point_matches_sequential(tmp_path):
    a = _args(tmp_path)
    _sweep(a, _point_runner())
    want, _ = sequential()
    r = sim.PointResult(1.5, N, T, want)
    assert (tmp_path / "log.txt").read_text().splitlines()[0] == r.log_line("x.alist", [1.25])


def test_changed_settings_or_seed_are_refused(tmp_path):
    a = _args(tmp_path)
    _sweep(a, _point_runner())
    with pytest.raises(checkpoint.CheckpointMismatch, match="alpha"):
        checkpoint.SweepCheckpoint(a.checkpoint, sweep._checkpoint_config(_args(tmp_path, "--alpha", "1.5")), True)
    ck = checkpoint.SweepCheckpoint(a.checkpoint, sweep._checkpoint_config(a), True)
    assert ck.seed == 1234
    with pytest.raises(checkpoint.CheckpointMismatch, match="seed"):
        ck.start(99)
    # batch and round sizes do not change results: not part of the settings
    assert sweep._checkpoint_config(_args(tmp_path, "--batch", "7")) == sweep._checkpoint_config(a)


def test_torn_last_record_is_ignored(tmp_path):
    a = _args(tmp_path)
    with pytest.raises(_Killed):
        _sweep(a, _point_runner(2))
    p = tmp_path / "ck.partial"
    p.write_text(p.read_text() + '{"kind": "round", "k": 0, "snr": 1.5, "next_fr')
    ck = checkpoint.SweepCheckpoint(a.checkpoint, sweep._checkpoint_config(a), True)
    st = ck.point_state(0, 1.5, N)
    assert st is not None and st.rounds == 2 and st.next_frame == 2 * 97
    assert int((st.hist * np.arange(1, N + 1)).sum()) == int(st.acc[0])


@pytest.mark.parametrize("tail", ['{"kind": "round", "k": 0, "snr": 1.5, "next_fr', None])
def test_torn_tail_repaired_before_resume_appends(tmp_path, tail):
    """A sweep killed mid-write (torn last record), or one whose last complete record lost
    its newline, resumes, appends further rounds, can be killed and resumed again, and ends
    with the uninterrupted run's log (the first appended record was glued onto
    the fragment and the next load refused the file)."""
    ref_dir = tmp_path / "ref"
    ref_dir.mkdir()
    _sweep(_args(ref_dir), _point_runner())
    want = (ref_dir / "log.txt").read_text().splitlines()
    a = _args(tmp_path)
    with pytest.raises(_Killed):
        _sweep(a, _point_runner(2))
    p = tmp_path / "ck.partial"
    txt = p.read_text()
    p.write_text(txt + tail if tail is not None else txt.rstrip("\n"))
    with pytest.raises(_Killed):
        _sweep(_args(tmp_path), _point_runner(2))     # resume, append two rounds, killed again
    recs = [json.loads(l) for l in p.read_text().splitlines()]   # every line parses
    assert sum(r["kind"] == "round" for r in recs) == 4
    _sweep(_args(tmp_path), _point_runner())
    assert (tmp_path / "log.txt").read_text().splitlines() == want
