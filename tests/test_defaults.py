"""Product defaults follow the reference's arithmetic (decodeMinSum.cpp:39-40,177-178:
every message is a `double`): fp64 wherever the product picks a precision, fp32 only
on request. CPU only: the CLIs stop before any device call
under LDPC_DRY_RUN, the sweep's defaults come from its parser."""
import os
import subprocess

import pytest

from conftest import code_path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")


def test_sweep_defaults_to_f64_and_adaptive_rounds():
    from ldpcsimulation_amd import sweep
    a = sweep.parse(["x.alist", "--rate", "0.5", "--snr", "1.0"])
    assert a.precision == "f64"
    assert a.first_round is None and a.batch == 65536     # rounds grow from min(batch, 1024)
    assert a.backend == "nccl" and not a.share_device
    assert sweep.parse(["x.alist", "--rate", "0.5", "--snr", "1.0", "--precision", "f32"]).precision == "f32"


@pytest.mark.parametrize("cli,args", [
    ("decodeNMS", ["0.5", "1.25", "50", "1.25"]),
    ("decodeMinSum", ["0.5", "1.25", "50"]),
    ("decodeSMNGDBF", None),
])
@pytest.mark.parametrize("rng", ["glibc", "philox"])
def test_cli_precision_defaults_to_f64(tmp_path, cli, args, rng):
    exe = os.path.join(BIN, cli)
    if not os.path.exists(exe):
        pytest.skip(f"{cli} not built")
    log = str(tmp_path / "l.txt")
    if args is None:   # the GDBF argument list from its usage line: alist R SNR T theta logfile ...
        names = subprocess.run([exe], capture_output=True, text=True).stdout.split()[2:-2]
        vals = {"R": "0.5", "SNR": "3.5", "T": "10", "theta": "-0.6", "logfilename": log}
        argv = [vals.get(n, "1.0") for n in names[1:]]
    else:
        argv = args + [log]
    env = dict(os.environ, LDPC_RNG=rng, LDPC_DRY_RUN="1", LDPC_SEED="1")
    env.pop("LDPC_PRECISION", None)
    p = subprocess.run([exe, code_path("80211n_1944_r12.alist")] + argv, env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    assert f"rng={rng} precision=f64" in p.stderr
    env["LDPC_PRECISION"] = "f32"
    p = subprocess.run([exe, code_path("80211n_1944_r12.alist")] + argv, env=env,
                       capture_output=True, text=True, timeout=60)
    assert "precision=f32" in p.stderr


def test_python_configs_default_to_f64():
    from ldpcsimulation_amd import native
    assert native.DecoderConfig().precision == native.F64
    assert native.GdbfConfig().precision == native.F64
