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
    # the lines the reference cycles through (decodeMinSum.cpp:193-200): an unterminated
    # last line sets eof() as it is read, so the file is rewound instead of using it
    text = open(code_path(run["cwfile"])).read()
    lines = text.split("\n")
    if text.endswith("\n"):
        lines.pop()
    elif len(lines) > 1:
        lines.pop()
    return [l for l in lines if l.strip()]


def final_numbers(final_line):
    m = re.match(r"Final result: (\d+) bit errs in (\d+) words.*Uncoded errors = (\d+)", final_line)
    return tuple(int(x) for x in m.groups())


# decodeGDBF.cpp Makefile targets (C_implementations/Makefile:33-53) -> -D switches
GDBF_BINARIES = {
    "decodeMNGDBF": ("noise", "adapt", "weight", "saturate"),
    "decodeSMNGDBF": ("noise", "adapt", "weight", "smooth", "saturate"),
    "decodeATGDBF": ("adapt",),
    "decodeSATGDBF": ("adapt", "smooth"),
    "decodeSMGDBF": ("smooth",),
    "decodeSGDBF": ("sequential",),                                     # Makefile:27-28
    "decodeMGDBF": ("modeswitch",),                                     # Makefile:24-25
    "decodeStochasticNGDBF": ("quantize", "qprob", "weight", "saturate"),   # Makefile:30-31
}


def gdbf_config(run):
    """(R, snr, dict of oracle GdbfCfg fields) of a golden GDBF reference run. Positional
    arguments after the log file follow decodeGDBF.cpp:95-113: noiseScale, [NQ], lambda,
    alpha, windowsize, Ymax -- each present only with its switch."""
    from oracle import oracle as O
    a = run["args"]
    R, snr, T, theta = float(a[0]), float(a[1]), int(a[2]), float(a[3])
    rest = a[5:]
    sw = GDBF_BINARIES[run["binary"]]
    bits = {"noise": O.GDBF_NOISE, "adapt": O.GDBF_ADAPT, "weight": O.GDBF_WEIGHT,
            "smooth": O.GDBF_SMOOTH, "saturate": O.GDBF_SATURATE, "quantize": O.GDBF_QUANTIZE,
            "sequential": O.GDBF_SEQUENTIAL, "modeswitch": O.GDBF_MODESWITCH, "qprob": O.GDBF_QPROB}
    cfg = dict(flags=sum(bits[s] for s in sw), T=T, theta=theta, lambda_=0.991, alpha=2.25,
               noise_scale=1.0, ymax=2.25, windowsize=64, nq=16)   # the reference's defaults (:48-56)
    i = 0
    for names, key, conv in ((("noise", "qprob"), "noise_scale", float), (("quantize",), "nq", int),
                             (("adapt",), "lambda_", float), (("weight",), "alpha", float),
                             (("smooth",), "windowsize", int), (("saturate",), "ymax", float)):
        if any(n in sw for n in names):
            cfg[key] = conv(rest[i])
            i += 1
    return R, snr, cfg


def gdbf_final_numbers(final_line):
    """(bit errors, words, average iterations, uncoded errors) of a GDBF 'Final result' line."""
    m = re.match(r"Final result: (\d+) bit errs in (\d+) words.*Average iterations = ([0-9.e+-]+)\. "
                 r"Uncoded errors = (\d+)", final_line)
    return int(m.group(1)), int(m.group(2)), float(m.group(3)), int(m.group(4))
