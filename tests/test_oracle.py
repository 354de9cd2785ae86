"""The CPU oracle against the reference's own outputs (golden fixtures) and KATs.

Pins the restatement: glibc random()/rann() known answers, Random123 Philox
known answers, and whole Monte-Carlo runs of the compiled reference
(tests/golden/reference_runs.json, made by tests/golden/make_golden.py from
oracle/_ref) reproduced frame by frame.
"""
import numpy as np
import pytest

from conftest import code_path, golden_runs
from helpers import cw_lines, final_numbers, run_config
from oracle import oracle as O


def test_glibc_random_kat():
    g = O.GlibcRandom(42)
    assert [g.random() for _ in range(4)] == [71876166, 708592740, 1483128881, 907283241]


def test_rann_kat():
    # rand.h:19-20 with the cos operand's ranf() drawn first (g++ order)
    g = O.GlibcRandom(42)
    got = [g.rann() for _ in range(3)]
    assert got == [0.87518550330287004, -0.38185485882140952, 0.20588689969294371]


def test_glibc_seed_zero_is_seed_one():
    a, b = O.GlibcRandom(0), O.GlibcRandom(1)
    assert [a.random() for _ in range(8)] == [b.random() for _ in range(8)]


@pytest.mark.parametrize("ctr,key,want", [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
])
def test_philox_random123_kat(ctr, key, want):
    assert O.philox4x32_10(ctr, key) == want


@pytest.mark.parametrize("run", golden_runs(), ids=lambda r: r["name"])
def test_oracle_reproduces_reference_run(run):
    R, snr, T, c = run_config(run)
    A = O.Alist(code_path(run["code"]))
    n, st, fw = A.minsum_run(R, snr, T, O.Cfg(**c), run["seed"], cw_lines=cw_lines(run), cap=200000)
    bit, words, unc = final_numbers(run["final"])
    assert (st["errors"], st["words"], st["uncoded"]) == (bit, words, unc)
    assert st["word_errors"] == len(run["ferr_weights"])
    assert [int(w) for w in fw if w > 0] == run["ferr_weights"]


def test_quantize_matches_reference_formula():
    # quantize() (decodeMinSum.cpp:480-489) on a few hand-checked points: Ymax=1.5, Q=4 -> step 0.2
    assert O.quantize(2.0, 1.5, 4) == 1.5
    assert O.quantize(-2.0, 1.5, 4) == -1.5
    assert O.quantize(0.05, 1.5, 4) == pytest.approx(0.2)       # zero level bumped to smallest
    assert O.quantize(-0.05, 1.5, 4) == pytest.approx(-0.2)
    assert O.quantize(0.45, 1.5, 4) == pytest.approx(0.4)
    assert O.quantize(0.0, 1.5, 4) == pytest.approx(0.2)        # sgn(0) = +1


def test_oracle_decode_matches_frame_loop():
    """orc_decode_f64 on the reference's own channel samples == the frame loop's weights."""
    A = O.Alist(code_path("PEGReg504x1008.alist"))
    n, st, fw = A.minsum_run(0.5, 2.0, 10, O.Cfg(), 42, max_frames=8, cap=8)
    g = O.GlibcRandom(42)
    sigma = np.sqrt(10 ** (-2.0 / 10) / 0.5 / 2)
    c = np.ones(A.N, dtype=np.int32)
    for f in range(8):
        y = g.channel(c, sigma)
        d = A.decode(y, 10, O.Cfg())
        assert int((d != 1).sum()) == fw[f]


@pytest.mark.parametrize("run", golden_runs("bp"), ids=lambda r: r["name"])
def test_oracle_reproduces_reference_bp_run(run):
    """decodeBP (tanh-rule belief propagation, src/decodeBP.cpp) restated in
    oracle/bp_oracle.c reproduces the reference's own runs frame by frame."""
    R, snr, T = float(run["args"][0]), float(run["args"][1]), int(run["args"][2])
    A = O.Alist(code_path(run["code"]))
    n, st, fw = A.bp_run(R, snr, T, run["seed"], cw_lines=cw_lines(run), cap=200000)
    bit, words, unc = final_numbers(run["final"])
    assert (st["errors"], st["words"], st["uncoded"]) == (bit, words, unc)
    assert [int(w) for w in fw if w > 0] == run["ferr_weights"]
