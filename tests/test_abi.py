"""The C-ABI library: loads without a GPU, exports every symbol include/ldpc_hip.h
declares, and validates H matrices (graph functions need no device)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import REFERENCE, ROOT, code_path
from ldpcsimulation_amd import codes, native


def _declared_functions():
    txt = open(os.path.join(ROOT, "include", "ldpc_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ldpc_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = C.CDLL(native.LIB_PATH)
    declared = _declared_functions()
    assert len(declared) >= 19
    for name in declared:
        assert hasattr(L, name), name
    assert sorted(native.EXPORTED) == declared


def test_abi_version_and_errors():
    L = native.lib()
    assert L.ldpc_abi_version() == native.ABI_VERSION == 9
    with pytest.raises(native.LdpcError) as e:
        native.Graph.from_alist("/nonexistent/file.alist")
    assert e.value.code == -5
    assert b"cannot open" in L.ldpc_last_error()


@pytest.mark.parametrize("name,N,M,E", [
    ("PEGReg504x1008.alist", 1008, 504, 3024),
    ("4000.2000.4.244.alist", 4000, 2000, 16000),
    ("80211n_1944_r12.alist", 1944, 972, 6966),
])
def test_graph_from_alist(name, N, M, E):
    g = native.Graph.from_alist(code_path(name))
    assert (g.N, g.M, g.E) == (N, M, E)


def test_graph_from_lists_matches_alist():
    H = codes.ieee80211n_r12(81)
    g = native.Graph.from_lists(H.N, H.M, H.nlist(), H.mlist())
    assert (g.N, g.M, g.E, g.maxdv, g.maxdc) == (1944, 972, 6966, 11, 8)


def test_graph_validation_rejects_inconsistent_views():
    # bit 0 claims check 1, but check 1 does not list bit 0
    with pytest.raises(native.LdpcError) as e:
        native.Graph.from_lists(3, 2, [[1], [1, 2], [2]], [[2], [2, 3]])
    assert e.value.code == -6
    # out-of-range index
    with pytest.raises(native.LdpcError):
        native.Graph.from_lists(2, 1, [[1], [1]], [[1, 3]])
    # duplicate edge
    with pytest.raises(native.LdpcError):
        native.Graph.from_lists(2, 1, [[1, 1], []], [[1, 1]])


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference tree not present")
def test_broken_reference_80211n_file_is_an_error_not_a_crash():
    """codes/802.11n/802.11n.alist is transposed and unpadded; the reference loader
    reads garbage and decodeMinSum segfaults. Ours reports it."""
    with pytest.raises(native.LdpcError) as e:
        native.Graph.from_alist(os.path.join(REFERENCE, "codes", "802.11n", "802.11n.alist"))
    assert e.value.code == -6


def test_decoder_config_struct_layout():
    assert C.sizeof(native._Cfg) == 6 * 4 + 3 * 8 + 2 * 4 + 2 * 8   # ABI 2: + schedule, reserved; ABI 4: + n0, max_llr
    assert C.sizeof(native.Counts) == 48
    assert native.FRAME_DTYPE.itemsize == 16


def test_shipped_library_holds_only_the_kept_ping_pong_kernel():
    """the product library carries only the kept k_rows_pp -- two
    slots per block in barrier intervals, instantiated per precision, channel source,
    variant, division and row-slot layout (k_rows_pp<F, SRC, CPT, VAR, FDIV, SPLIT>) -- and no
    environment switch that swaps in a rejected schedule (the round-3 LDPC_PP_MODE
    1/2 instances: one row per thread, dataflow sync)."""
    import subprocess
    syms = subprocess.run(["nm", "-C", native.LIB_PATH], capture_output=True, text=True, check=True).stdout
    kern = sorted({m for m in re.findall(r"ldpc::k_rows_pp<([^>]*)>", syms)})
    # fp64: 2 sources x (MS, OMS, NMS, NMS Markstein) x 2 row-slot layouts;
    # fp32 pairs: 2 sources x (MS, NMS with the verified reciprocal) x 2 layouts
    assert len(kern) == 24, kern
    for k in kern:
        ft, src, cpt, var, fdiv, split = (x.strip() for x in k.split(","))
        assert ft in ("double", "float") and cpt == "4" and split in ("true", "false") and src in ("0", "1"), k
    assert sum(k.startswith("float") for k in kern) == 8
    with open(native.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"LDPC_PP_MODE" not in blob and b"pp_wait" not in blob
