"""GDBF / NGDBF bit flipping (BASELINE config 4).

Oracle tier (CPU): oracle/gdbf_oracle.c restates src/decodeGDBF.cpp in its
parallel-flip mode and must reproduce every golden reference run
(tests/golden/reference_runs.json, decodeMNGDBF / decodeSMNGDBF /
decodeATGDBF / decodeSATGDBF / decodeSMGDBF compiled from the unmodified
sources by oracle/Makefile.ref): totals, per-frame error weights, average
iterations and the log line's smoothing count.
GPU tier: the HIP kernel through the C ABI, given the reference's own channel
samples and perturbations, gives the oracle's decisions and iteration counts
bit for bit (fp64 and fp32); on-device Philox noise matches statistically.
"""
import math

import numpy as np
import pytest

from conftest import code_path, golden_runs
from helpers import cw_lines, gdbf_config, gdbf_final_numbers
from oracle import oracle as O


@pytest.mark.parametrize("run", golden_runs("gdbf"), ids=lambda r: r["name"])
def test_oracle_reproduces_reference_gdbf_run(run):
    R, snr, c = gdbf_config(run)
    A = O.Alist(code_path(run["code"]))
    n, st, fw, fi = A.gdbf_run(R, snr, O.GdbfCfg(**c), run["seed"], cw_lines=cw_lines(run), cap=1000000)
    bit, words, avg_it, unc = gdbf_final_numbers(run["final"])
    assert (st["errors"], st["words"], st["uncoded"]) == (bit, words, unc)
    assert f"{st['iters'] / st['words']:g}" == f"{avg_it:g}"
    assert [int(w) for w in fw if w > 0] == run["ferr_weights"]
    if c["flags"] & O.GDBF_SMOOTH:   # log line: ... smoothingUsed, smoothingUsed/totalWords, windowsize ...
        fields = run["log_line"].split("\t")
        assert str(st["smoothing_used"]) in fields


def _reference_frames(A, run, nframes):
    """Channel samples and perturbation rows of the first frames of a golden run, drawn
    from the glibc restatement in the reference's order (:251-253, :318-333)."""
    R, snr, c = gdbf_config(run)
    cfg = O.GdbfCfg(**c)
    g = O.GlibcRandom(run["seed"])
    sigma = math.sqrt(10 ** (-snr / 10) / R / 2)
    frames = []
    for _ in range(nframes):
        y = np.array([1.0 * (1.0 + sigma * g.rann()) for _ in range(A.N)])
        state = O.GlibcRandom(0)
        state._s = type(g._s).from_buffer_copy(g._s)
        pert = None
        if cfg.flags & O.GDBF_NOISE:
            pert = np.array([sigma * cfg.noise_scale * state.rann() for _ in range(A.N * cfg.T)]).reshape(cfg.T, A.N)
        d, it, sat = A.gdbf_decode(y, pert, cfg)
        if cfg.flags & O.GDBF_NOISE:
            for _ in range(A.N * it):
                g.rann()
        frames.append((y, pert, d, it, sat))
    return cfg, frames


def test_oracle_frame_decode_matches_run():
    run = [r for r in golden_runs("gdbf") if r["name"] == "smngdbf_peg_3.5_T100_s5"][0]
    A = O.Alist(code_path(run["code"]))
    R, snr, c = gdbf_config(run)
    n, st, fw, fi = A.gdbf_run(R, snr, O.GdbfCfg(**c), run["seed"], max_frames=6, cap=6)
    _, frames = _reference_frames(A, run, 6)
    assert [int((f[2] != 1).sum()) for f in frames] == list(fw)
    assert [f[3] for f in frames] == list(fi)
