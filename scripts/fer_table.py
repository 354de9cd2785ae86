#!/usr/bin/env python3
"""FER of the bench workload (802.11n N=1944, NMS alpha=1.25, T=50, on-device
Philox channel) in fp64 (the reference's arithmetic) and fp32 at the four
SURVEY §8(d) points, beside the reference's own decodeNMS over 10 seeds per
point (tests/golden/reference_fer.json, scripts/ref_fer.py: 400 frame errors
each). Prints one JSON line per (precision, point): GPU frame errors / frames,
Wilson 95% interval, two-proportion z against the reference. Frames per
point are chosen so the GPU side holds >= ~250 frame errors."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ldpcsimulation_amd import codes, native  # noqa: E402
from ldpcsimulation_amd.sim import two_proportion_z, wilson_interval  # noqa: E402

ROUNDS = {1.0: 1, 1.25: 1, 1.5: 1, 1.75: 4}     # x 65536 frames


def main():
    with open(os.path.join(ROOT, "tests", "golden", "reference_fer.json")) as f:
        ref = {p["ebn0_db"]: (p["frame_err"], p["frames"]) for p in json.load(f)["points"]}
    g = native.Graph.from_alist(codes.ensure_80211n_1944())
    B = 65536
    ctx = native.Context(g, 0, B)
    for prec in ("f64", "f32"):
        cfg = native.DecoderConfig(variant=native.NMS, alpha=1.25, T=50,
                                   precision=native.F64 if prec == "f64" else native.F32)
        for ebn0, (k_ref, n_ref) in sorted(ref.items()):
            ferr = frames = bit_err = 0
            for r in range(ROUNDS[ebn0]):
                _, cnt = ctx.sim_batch(ebn0, 0.5, cfg, seed=20261015, stream_id=int(ebn0 * 100), first_cw=r * B,
                                       batch=B, want_frames=False)
                ferr += cnt.frame_err
                frames += cnt.frames
                bit_err += cnt.bit_err
            print(json.dumps({"precision": prec, "ebn0_db": ebn0, "frame_err": ferr, "frames": frames,
                              "fer": ferr / frames, "ber": bit_err / (frames * g.N),
                              "wilson95": wilson_interval(ferr, frames), "ref": [k_ref, n_ref],
                              "ref_fer": k_ref / n_ref, "z": two_proportion_z(ferr, frames, k_ref, n_ref)}),
                  flush=True)


if __name__ == "__main__":
    main()
