"""The bounds-checked device build (SURVEY §5 "bounds-checked debug kernels"; VERDICT r5
item 5): `make checked` compiles every kernel with -DLDPC_CHECK (check.h), which tests
each schedule-derived LDS / global index on the device -- rows_pp's gathers, scatters,
bit slots and app writes, rows_fast's, the flood / layered global slots, the GDBF rows'
bit and check-term slots, the EMS message slots, the BP rows' columns and message slots
-- and fails the launching ABI call with LDPC_ERR_DEVICE on a violation. The reference
validates nothing (C_implementations/src/alist.cpp:22-95); here the host validates the
graph (graph.cpp, nb_graph.cpp) and the checked build re-proves the schedules on the
device.

GPU tier: small batches of the five BASELINE configs' codes (plus BP and the degree-1 /
heavy-column fixtures) decoded by the checked library and by the product library, each
in a child process of its own (one library per process): no violation, and identical
decisions, per-frame results and counters.
CPU tier: the checked library exists beside the product, exports the same symbols, and
the product library reports no compiled checks."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, code_path

CHECKED = os.path.join(ROOT, "ldpcsimulation_amd", "lib", "checked", "libldpc_hip_checked.so")

# name -> (kind, code, decoder settings); small batches, every kernel family of the configs
CASES = {
    "c1_rows_fast_f64": ("minsum", "PEGReg504x1008.alist", dict(variant="ms", prec="f64", T=10, batch=512)),
    "c2_rows_pp_f64": ("minsum", "80211n_1944_r12.alist", dict(variant="nms", prec="f64", T=50, batch=1024)),
    "c2_rows_pp_f32": ("minsum", "80211n_1944_r12.alist", dict(variant="nms", prec="f32", T=50, batch=1024)),
    "c3_flood_f64": ("minsum", "dvbs2_1_2.alist", dict(variant="nms", prec="f64", T=6, batch=4)),
    "c3_layered_f64": ("minsum", "dvbs2_1_2.alist", dict(variant="nms", prec="f64", T=6, batch=4, layered=True)),
    "c4_gdbf_f32": ("gdbf", "80211n_1944_r12.alist", dict(prec="f32", T=60, batch=1024)),
    "c4_gdbf_f64": ("gdbf", "80211n_1944_r12.alist", dict(prec="f64", T=60, batch=1024)),
    "c5_ems": ("ems", "gf16", dict(T=10, batch=512)),
    "bp_rows_f64": ("minsum", "80211n_1944_r12.alist", dict(variant="bp", prec="f64", T=10, batch=256)),
    "deg1_f64": ("minsum", "deg1", dict(variant="nms", prec="f64", T=12, batch=64)),
    "deg1_f32": ("minsum", "deg1", dict(variant="ms", prec="f32", T=12, batch=64)),
    "heavy_flood_f64": ("minsum", "heavy", dict(variant="nms", prec="f64", T=7, batch=64, kernel="flood")),
}


def _fixtures(tmp):
    """The degree-1-check and heavy-column codes of tests/test_gpu_parity.py."""
    from ldpcsimulation_amd import codes
    H = codes.read_alist(code_path("PEGReg504x1008.alist"))
    deg1 = os.path.join(tmp, "peg_deg1.alist")
    codes.write_alist(codes.ParityCheck.from_rows(H.N, H.rows + [[5], [17, 900]]), deg1)
    rng = np.random.default_rng(40)
    N, M = 600, 300
    rows = [sorted(set(rng.choice(np.arange(1, N), size=6, replace=False).tolist())) for _ in range(M)]
    for j in range(40):
        rows[j] = sorted(set(rows[j]) | {0})
    heavy = os.path.join(tmp, "heavy_col.alist")
    codes.write_alist(codes.ParityCheck.from_rows(N, rows), heavy)
    return {"deg1": deg1, "heavy": heavy}


def run_cases(lib, out, fixtures):
    """Child process: decode every case with library `lib`, save the results to `out` (npz)."""
    from ldpcsimulation_amd import codes, native
    native.use_library(lib)
    res, kern = {}, {}
    for name, (kind, code, s) in CASES.items():
        if kind == "ems":
            g = native.NbGraph.from_alist(codes.ensure_gf16_code())
            ctx = native.NbContext(g, 0, s["batch"])
            cfg = native.EmsConfig(T=s["T"], nm=16, offset=0.0, early_stop=True)
            _, d, fr, cnt = ctx.sim_trace(2.0, 0.5, cfg, seed=9, stream_id=1, first_cw=100, batch=s["batch"])
            kern[name] = ctx.kernel_info()["kernel"]
        else:
            path = fixtures.get(code) or code_path(code)
            ctx = native.Context(native.Graph.from_alist(path), 0, s["batch"])
            prec = native.F64 if s["prec"] == "f64" else native.F32
            if s.get("kernel"):
                ctx.set_option("kernel", s["kernel"])
            if kind == "gdbf":
                cfg = native.GdbfConfig(T=s["T"], precision=prec)
                fr, cnt = ctx.gdbf_sim_batch(3.5, 0.5, cfg, seed=9, stream_id=1, first_cw=100, batch=s["batch"])
                d = None
                kern[name] = ctx.gdbf_kernel_info(cfg)["kernel"]
            else:
                v = {"ms": dict(variant=native.MS), "nms": dict(variant=native.NMS, alpha=1.25),
                     "bp": dict(variant=native.BP)}[s["variant"]]
                sched = native.LAYERED if s.get("layered") else native.FLOODING
                cfg = native.DecoderConfig(T=s["T"], precision=prec, schedule=sched, **v)
                snr = 1.0 if code == "dvbs2_1_2.alist" else 2.0
                _, d, fr, cnt = ctx.sim_trace(snr, 0.5, cfg, seed=9, stream_id=1, first_cw=100, batch=s["batch"])
                kern[name] = ctx.kernel_info(cfg)["kernel"]
        res[name + "__counts"] = np.array([int(v) for v in cnt.as_dict().values()], dtype=np.int64)
        res[name + "__frames"] = np.asarray(fr).view(np.int32).reshape(len(fr), -1) if fr is not None else np.zeros(0)
        if d is not None:
            res[name + "__d"] = np.asarray(d)
    np.savez(out, **res)
    with open(out + ".json", "w") as f:
        json.dump(kern, f)


def _child(lib, out, fixtures):
    code = ("import sys, json; sys.path.insert(0, %r); sys.path.insert(0, %r); import test_checked_build as t; "
            "t.run_cases(%r, %r, json.loads(%r))" % (ROOT, os.path.join(ROOT, "tests"), lib, out,
                                                     json.dumps(fixtures)))
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=600)


def test_checked_library_built_beside_the_product():
    """`make checked` (also run by __graft_entry__.build) puts the checked library beside the
    product; it exports the same ABI, and the product compiles no checks."""
    from ldpcsimulation_amd import native
    assert os.path.exists(CHECKED), "run `make checked`"
    L = C.CDLL(CHECKED)
    for name in native.EXPORTED:
        assert hasattr(L, name), name
    P = native.lib()
    assert P.ldpc_check_selftest(0) == -4   # LDPC_ERR_UNSUPPORTED, no device call
    assert b"make checked" in P.ldpc_last_error()


@pytest.mark.gpu
def test_checked_build_reports_a_violation(tmp_path):
    """The mechanism end to end on the device: a kernel of the checked build indexes past a
    bound on purpose; the record reaches the host and the ABI call fails naming it."""
    code = ("import sys, ctypes as C; sys.path.insert(0, %r); from ldpcsimulation_amd import native; "
            "native.use_library(%r); L = native.lib(); rc = L.ldpc_check_selftest(0); "
            "print(rc, L.ldpc_last_error().decode())" % (ROOT, CHECKED))
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    rc, msg = p.stdout.strip().split(" ", 1)
    assert int(rc) == -3, msg                                   # LDPC_ERR_DEVICE
    assert "LDPC_CHECK: bp_rows bit index 7 >= bound 3" in msg, msg


@pytest.mark.gpu
def test_checked_build_equals_product_on_the_config_codes(tmp_path):
    """Every case decoded by the checked library raises no violation (an LdpcError in the
    child would fail it) and gives the product library's decisions, per-frame results and
    counters, on the same kernels."""
    from ldpcsimulation_amd import native
    fx = _fixtures(str(tmp_path))
    a, b = str(tmp_path / "product.npz"), str(tmp_path / "checked.npz")
    pa = _child(native.LIB_PATH, a, fx)
    assert pa.returncode == 0, pa.stderr[-3000:]
    pb = _child(CHECKED, b, fx)
    assert pb.returncode == 0, pb.stderr[-3000:]
    ka, kb = json.load(open(a + ".json")), json.load(open(b + ".json"))
    assert ka == kb
    assert {ka["c1_rows_fast_f64"], ka["c2_rows_pp_f64"], ka["c3_flood_f64"], ka["c3_layered_f64"][:7],
            ka["c4_gdbf_f32"], ka["bp_rows_f64"]} == {"rows_fast", "rows_pp", "flood", "layered", "gdbf_rows",
                                                        "bp_rows"}
    ra, rb = np.load(a), np.load(b)
    assert sorted(ra.files) == sorted(rb.files)
    for k in ra.files:
        assert np.array_equal(ra[k], rb[k]), k
