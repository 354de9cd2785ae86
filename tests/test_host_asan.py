"""Host code under AddressSanitizer + UBSan: `make build/host_asan`
compiles graph.cpp (load_alist, build_graph, the row / flood / layer schedules)
and the CPU oracle with -fsanitize=address,undefined -fno-sanitize-recover=all;
tests/native/host_asan.cpp drives them over every code fixture (DVB-S2
included), the reference's own malformed 802.11n alists when the reference is
present, and malformed graphs. Any sanitizer report fails the run."""
import glob
import os
import shutil
import subprocess

import pytest

from conftest import REFERENCE, ROOT, code_path


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_graph_compiler_and_oracle_clean_under_asan_ubsan():
    subprocess.run(["make", "-C", ROOT, "build/host_asan"], check=True, capture_output=True, text=True)
    codes = [code_path(n) for n in ("4000.2000.4.244.alist", "80211n_1944_r12.alist", "PEGReg504x1008.alist",
                                    "dvbs2_1_2.alist")]
    codes += sorted(glob.glob(os.path.join(REFERENCE, "codes", "802.11n", "*.alist")))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([os.path.join(ROOT, "build", "host_asan")] + codes, capture_output=True, text=True,
                       env=env, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "ok (0 failures)" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
