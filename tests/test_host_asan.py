"""Host code under AddressSanitizer + UBSan: `make build/host_asan`
compiles graph.cpp (load_alist, build_graph, the row / flood / layer schedules),
nb_graph.cpp (the NB alist reader of SystemC/NB-LDPC/src/alist.cpp:29-53's format,
the GF tables, the message-slot swizzle search), cli_common.h (the CLIs' codeword
files and alist headers) and the CPU oracle with -fsanitize=address,undefined
-fno-sanitize-recover=all; tests/native/host_asan.cpp drives them over every code
fixture (DVB-S2 included), the reference's own malformed 802.11n alists and its
SystemC/NB-LDPC/codes/* files when the reference is present, the GF(q) fixtures,
the codeword-file fixtures, and generated malformed inputs (truncated files,
degree-0 and degree-1 checks, out-of-range indices and coefficients, disagreeing
views, empty / unterminated / binary / CRLF codeword files). Any sanitizer report
fails the run."""
import glob
import os
import shutil
import subprocess
import tempfile

import pytest

from conftest import REFERENCE, ROOT, code_path


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_graph_compiler_and_oracle_clean_under_asan_ubsan():
    subprocess.run(["make", "-C", ROOT, "build/host_asan"], check=True, capture_output=True, text=True)
    codes = [code_path(n) for n in ("4000.2000.4.244.alist", "80211n_1944_r12.alist", "PEGReg504x1008.alist",
                                    "dvbs2_1_2.alist")]
    codes += sorted(glob.glob(os.path.join(REFERENCE, "codes", "802.11n", "*.alist")))
    nb = [code_path(n) for n in ("gf16_N1000_dv2_dc4.alist", "q4.sp.9000.6000.4500.1.alist",
                                 "q8.sp.6000.4000.3000.1.alist")]
    nb += sorted(p for p in glob.glob(os.path.join(REFERENCE, "SystemC", "NB-LDPC", "codes", "*", "*"))
                 if os.path.isfile(p))
    cw = [code_path(n) for n in ("PEGReg504x1008_data20.enc", "PEGReg504x1008_data5_noeol.enc")]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    with tempfile.TemporaryDirectory() as td:
        p = subprocess.run([os.path.join(ROOT, "build", "host_asan")] + codes + ["--nb"] + nb + ["--cw"] + cw +
                           ["--tmp", td], capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "ok (0 failures)" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
    # the GF(16) code loads, with swizzles whose XOR over every check is 0 (checked inside)
    assert "gf16_N1000_dv2_dc4.alist: NB N=1000 M=500 q=16 E=2000" in p.stdout
    assert "q4.sp.9000.6000.4500.1.alist: NB N=9000 M=6000 q=4" in p.stdout
    assert p.stdout.count("bytes of invalid-symbol reports") >= 5 * 7 + 2
