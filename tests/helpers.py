"""Shared helpers for the test-suite: map a golden reference run to decoder configs."""
import re

from conftest import code_path


def run_config(run):
    """(R, snr, T, dict(variant, alpha, delta, quantize, ymax, qbits)) of a golden reference run."""
    a = run["args"]
    R, snr, T = float(a[0]), float(a[1]), int(a[2])
    b = run["binary"].replace("_g", "")
    cfg = dict(variant=0, alpha=1.0, delta=0.0, quantize=False, ymax=0.0, qbits=0)
    if b == "decodeNMS":
        cfg.update(variant=1, alpha=float(a[3]))
    elif b == "decodeNormalizedMinSum":
        cfg.update(variant=1, quantize=True, ymax=float(a[3]), qbits=int(a[4]), alpha=float(a[5]))
    elif b == "decodeOffsetMinSum":
        cfg.update(variant=2, quantize=True, ymax=float(a[3]), qbits=int(a[4]), delta=float(a[5]))
    return R, snr, T, cfg


def cw_lines(run):
    if not run["cwfile"]:
        return None
    with open(code_path(run["cwfile"])) as f:
        return [l.rstrip("\n") for l in f if l.strip()]


def final_numbers(final_line):
    m = re.match(r"Final result: (\d+) bit errs in (\d+) words.*Uncoded errors = (\d+)", final_line)
    return tuple(int(x) for x in m.groups())
