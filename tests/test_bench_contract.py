"""bench.py's command-line contract (no GPU): defaults are N=1 and a short
K/W, and the driver's flags parse."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_defaults(monkeypatch):
    b = _bench()
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = b.parse()
    assert (a.gpus, a.steps, a.warmup) == (1, 5, 2)
    assert (a.batch, a.T, a.alpha, a.ebn0, a.precision) == (65536, 50, 1.25, 1.5, "f32")


def test_driver_flags(monkeypatch):
    b = _bench()
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "20", "--warmup", "3"])
    a = b.parse()
    assert (a.gpus, a.steps, a.warmup) == (8, 20, 3)


def test_reference_fer_table_matches_survey():
    b = _bench()
    assert b.REF_FER == {1.0: (40, 96), 1.25: (40, 362), 1.5: (40, 2212), 1.75: (40, 41745)}
    assert b.HBM_PEAK == 8.0e12
