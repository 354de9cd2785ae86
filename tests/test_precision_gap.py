"""How far the fp32 throughput path is from the reference's fp64 arithmetic
(decodeMinSum.cpp:39-40,410-476 keep every message in `double`), measured on
identical channel samples.

The fp32 kernel's own Philox channel (sim_trace, F32) gives y as floats; the
same values, exactly representable in double, are decoded by the fp64 row
kernel (whose decisions equal the reference's, tests/test_rows_fast.py). Both
decode 802.11n N=1944, NMS alpha=1.25, T=50, 16,384 frames per Eb/N0 point.
Counted per point: frames whose 1944 decisions differ, and frames whose
outcome (decoded or not) differs. The measured table is written to
gpurun_out/precision_gap.json and recorded in DESIGN §7.

Bounds (the test's tolerance): decisions may differ only on frames that at
least one precision fails to decode, plus at most 0.1 % of the frames
(converged-in-both frames end on the same codeword, the all-zero word); and
the outcome may differ on at most max(8, 20 % of the failing frames) per
point, both directions counted."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT

CODE = "80211n_1944_r12.alist"
POINTS = [1.0, 1.25, 1.5, 1.75]
FRAMES = 16384


@pytest.mark.gpu
def test_f32_vs_f64_on_identical_y(gpu_ctx_factory):
    from ldpcsimulation_amd import native
    ctx = gpu_ctx_factory(CODE, 4096)
    c32 = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=50, precision=native.F32)
    c64 = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=50, precision=native.F64)
    table = []
    for k, ebn0 in enumerate(POINTS):
        n_diff_dec = n_diff_out = fe32 = fe64 = both_fail = diff_on_good = 0
        for part in range(FRAMES // 4096):
            y32, d32, fr32, _ = ctx.sim_trace(ebn0, 0.5, c32, seed=20261019, stream_id=k, first_cw=part * 4096,
                                              batch=4096)
            d64, fr64, _ = ctx.decode(y32.astype(np.float64), c64)
            assert ctx.redo_count() == 0
            w32, w64 = fr32["bit_err"], fr64["bit_err"]
            diff = (d32 != d64).any(axis=1)
            n_diff_dec += int(diff.sum())
            n_diff_out += int(((w32 > 0) != (w64 > 0)).sum())
            fe32 += int((w32 > 0).sum())
            fe64 += int((w64 > 0).sum())
            both_fail += int(((w32 > 0) & (w64 > 0)).sum())
            diff_on_good += int((diff & (w32 == 0) & (w64 == 0)).sum())
        table.append({"ebn0_db": ebn0, "frames": FRAMES, "frame_err_f32": fe32, "frame_err_f64": fe64,
                      "frames_decisions_differ": n_diff_dec, "frames_outcome_differs": n_diff_out,
                      "frames_fail_both": both_fail, "decisions_differ_on_decoded_frames": diff_on_good})
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "precision_gap.json"), "w") as f:
        json.dump(table, f, indent=1)
    print(json.dumps(table))
    for r in table:
        failing = r["frame_err_f32"] + r["frame_err_f64"] - r["frames_fail_both"]
        assert r["decisions_differ_on_decoded_frames"] <= FRAMES // 1000, r
        assert r["frames_decisions_differ"] <= failing + FRAMES // 1000, r
        assert r["frames_outcome_differs"] <= max(8, 0.2 * failing), r
