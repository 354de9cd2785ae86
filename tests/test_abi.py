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
    assert L.ldpc_abi_version() == native.ABI_VERSION == 11
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


# Every environment variable that chose a kernel before ABI 10.
FORMER_KNOBS = ["LDPC_ROWS", "LDPC_ROWS32", "LDPC_PP_ROWS", "LDPC_KERNEL", "LDPC_FORCE_GLOBAL", "LDPC_FLOOD_MODE",
                "LDPC_FLOOD_MSG", "LDPC_FLOOD_SPS_CHECK", "LDPC_FLOOD_SPS_BIT", "LDPC_FLOOD_RESIDENT",
                "LDPC_FLOOD_STREAMS", "LDPC_FLOOD_BPC", "LDPC_LAYERED_BPC", "LDPC_LAYERED_LDS_POS",
                "LDPC_LAYERED_R64", "LDPC_LAYERED_THREADS", "LDPC_BLOCKS_PER_CU", "LDPC_FAST_BPC", "LDPC_RPT",
                "LDPC_BP_KERNEL", "LDPC_GDBF_KERNEL", "LDPC_EMS_THREADS", "LDPC_EMS_SWIZZLE", "LDPC_LIB"]
KNOB_VALUES = {"LDPC_ROWS": "old", "LDPC_ROWS32": "rows", "LDPC_PP_ROWS": "plain", "LDPC_KERNEL": "global",
               "LDPC_FORCE_GLOBAL": "1", "LDPC_FLOOD_MODE": "persistent", "LDPC_FLOOD_MSG": "c2v",
               "LDPC_BP_KERNEL": "generic", "LDPC_GDBF_KERNEL": "generic", "LDPC_LIB": "ppst"}


def test_shipped_library_reads_no_environment():
    """Kernel selection is an ABI option (ldpc_ctx_set_option), never the environment:
    the product library imports no getenv/secure_getenv and holds none of the former
    knobs' names, so no variable can reroute it (the reference fixes its algorithm per
    binary at build time, C_implementations/Makefile:58-65)."""
    import subprocess
    und = subprocess.run(["nm", "-D", "--undefined-only", native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert not re.search(r"\b(secure_)?getenv\b", und), und
    with open(native.LIB_PATH, "rb") as f:
        blob = f.read()
    for k in FORMER_KNOBS:
        assert k.encode() not in blob, k
    src = open(os.path.join(ROOT, "ldpcsimulation_amd", "native.py")).read()
    assert "LDPC_LIB" not in src and "os.environ" not in src and "getenv" not in src


def test_python_host_ignores_former_knobs(monkeypatch):
    """With every former knob set, the Python host still loads the product library and
    names the same defaults (the options are per-context ABI calls)."""
    import importlib
    for k in FORMER_KNOBS:
        monkeypatch.setenv(k, KNOB_VALUES.get(k, "1"))
    mod = importlib.reload(native)
    try:
        assert mod.LIB_PATH.endswith(os.path.join("lib", "libldpc_hip.so"))
        assert mod.option_id("rows64") == 1 and mod.option_value("rows64", "pp") == 0
    finally:
        monkeypatch.undo()
        importlib.reload(native)


def test_option_enum_matches_header():
    """native.OPTIONS mirrors include/ldpc_hip.h's ldpc_option enum."""
    txt = open(os.path.join(ROOT, "include", "ldpc_hip.h")).read()
    enum = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"LDPC_OPT_([A-Z0-9_]+)\s*=\s*(\d+)", txt)}
    assert enum == native.OPTIONS
    assert int(re.search(r"#define LDPC_OPT_COUNT (\d+)", txt).group(1)) == max(enum.values()) + 1


def test_set_option_validates_without_a_device():
    """Option validation happens before any device call: a NULL context is refused."""
    L = native.lib()
    assert L.ldpc_ctx_set_option(None, 1, 0) == -1
    assert L.ldpc_nb_ctx_set_option(None, 20, 512) == -1
    v = C.c_int(7)
    assert L.ldpc_ctx_get_option(None, 1, C.byref(v)) == -1
