import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLD = os.path.join(ROOT, "tests", "golden")
CODES = os.path.join(GOLD, "codes")
REFERENCE = "/root/reference/C_implementations"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libldpc_hip.so on the device)")


def code_path(name: str) -> str:
    """Path of a code fixture; *.alist stored as *.alist.xz is decompressed once into .cache/."""
    p = os.path.join(CODES, name)
    if not os.path.exists(p) and os.path.exists(p + ".xz"):
        import lzma
        cache = os.path.join(CODES, ".cache")
        os.makedirs(cache, exist_ok=True)
        p = os.path.join(cache, name)
        if not os.path.exists(p):
            tmp = p + f".{os.getpid()}.tmp"
            with lzma.open(os.path.join(CODES, name + ".xz"), "rb") as fi, open(tmp, "wb") as fo:
                fo.write(fi.read())
            os.replace(tmp, p)
    return p


def golden_runs(kind: str = "minsum"):
    """Reference runs of tests/golden/reference_runs.json: kind "minsum" (decodeMinSum
    family), "gdbf" (decodeGDBF family) or "bp" (decodeBP)."""
    with open(os.path.join(GOLD, "reference_runs.json")) as f:
        runs = json.load(f)["runs"]

    def kind_of(r):
        return "gdbf" if "GDBF" in r["binary"] else ("bp" if r["binary"] == "decodeBP" else "minsum")
    return [r for r in runs if kind_of(r) == kind]


@pytest.fixture(scope="session")
def gpu_ctx_factory():
    """Device contexts, cached per (code, max_batch); fails loudly without the HIP library."""
    from ldpcsimulation_amd import native
    assert native.device_count() > 0, "no HIP device visible"
    cache = {}

    def make(code: str, max_batch: int = 4096):
        key = (code, max_batch)
        if key not in cache:
            g = native.Graph.from_alist(code_path(code) if not os.path.isabs(code) else code)
            cache[key] = native.Context(g, 0, max_batch)
        cache[key].reset_options()   # kernel-choice options a previous test set stay with that test
        return cache[key]

    return make
