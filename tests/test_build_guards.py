"""The wrong-result experiment switches build only into A/B libraries (VERDICT r5 item 6;
the reference fixes its variants at build time, C_implementations/Makefile:58-65).

* `make` refuses VFLAGS on the product targets (the *variant targets build into ab/);
* each kernel source refuses its wrong-result switch unless LDPC_AB_BUILD is defined --
  checked by preprocessing the device side (hipcc -E stops at the #error).
No GPU is involved."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ldpcsimulation_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

SWITCHES = [("rows_pp.hip", "LDPC_PP_EXP"), ("rows_pp.hip", "LDPC_PP_TAILEXP"), ("rows_fast.hip", "LDPC_FAST_EXP"),
            ("nb.hip", "LDPC_EMS_EXP"), ("rows_pp.hip", "LDPC_BM_OCML"), ("rows_pp.hip", "LDPC_BM64")]


def test_make_refuses_vflags_on_the_product():
    p = subprocess.run(["make", "-n", "all", "VFLAGS=-DLDPC_PP_EXP=1"], cwd=ROOT, capture_output=True, text=True)
    assert p.returncode != 0 and "A/B targets" in p.stderr, p.stderr
    p = subprocess.run(["make", "-n", "ppvariant", "NAME=x", "VFLAGS=-DLDPC_PP_EXP=1"], cwd=ROOT,
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stderr


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("src,macro", SWITCHES)
def test_kernel_sources_refuse_wrong_result_switches(src, macro):
    base = [HIPCC, "--offload-arch=gfx950", "-std=c++17", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
            "--cuda-device-only", "-E", os.path.join(CSRC, src), "-o", os.devnull, f"-D{macro}=1"]
    refused = subprocess.run(base, capture_output=True, text=True)
    assert refused.returncode != 0 and macro in refused.stderr, refused.stderr[-500:]
    allowed = subprocess.run(base + ["-DLDPC_AB_BUILD"], capture_output=True, text=True)
    assert allowed.returncode == 0, allowed.stderr[-500:]
