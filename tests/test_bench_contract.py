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
    assert (a.batch, a.T, a.alpha, a.ebn0, a.precision) == (65536, 50, 1.25, 1.5, "f64")


def test_driver_flags(monkeypatch):
    b = _bench()
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "20", "--warmup", "3"])
    a = b.parse()
    assert (a.gpus, a.steps, a.warmup) == (8, 20, 3)


def test_reference_fer_table_matches_survey():
    b = _bench()
    assert b.REF_FER == {1.0: (40, 96), 1.25: (40, 362), 1.5: (40, 2212), 1.75: (40, 41745)}
    assert b.HBM_PEAK == 8.0e12


def test_gpus_mismatch_is_rejected(monkeypatch):
    """--gpus N under a torchrun of another size exits non-zero before any GPU call."""
    import pytest
    b = _bench()
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.setenv("WORLD_SIZE", "4")
    with pytest.raises(SystemExit) as e:
        b.main()
    assert e.value.code not in (0, None)


def test_gpus_without_torchrun_spawns_ranks(monkeypatch):
    """--gpus N with no WORLD_SIZE starts torchrun with N ranks as a child and exits with its status."""
    import pytest
    b = _bench()
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 0
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(b.subprocess, "call", fake_call)
    with pytest.raises(SystemExit) as e:
        b.main()
    assert e.value.code == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=2" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "2", "--steps", "3"]


def test_lds_model_of_the_n1944_row_schedule():
    """The LDS roofline models for the N=1944 code (E = 6966): the headline
    `frac` is the algorithmic one -- E gathers + E scatters + E bit reads + N app writes,
    no padding: 1270.7 LDS-array cycles per codeword-iteration; the
    companions are the kernel's issued slots (768 x 7 + 256 x 8 check edges with the
    degree-aware slots, as the library reports them: 1346) and the padded rows-2..4
    model (1024 row slots x 8, e_pad 7232, 512 x 4 bit slots: 1442)."""
    b = _bench()
    si = {"threads": 512, "rows_per_thread": 2, "slots_per_thread": 4, "dc": 8, "e_pad": 7232,
          "cw_per_block": 1, "lds_bytes": 148520, "blocks_per_cu": 1, "dc_low": 7,
          "issued_check_edges": 768 * 7 + 256 * 8}
    m = b.lds_model(si, 6966, 1944)
    assert m["by_phase"] == {"check_gather": 6966 / 32, "check_scatter": 6966 * 6 / 64, "bit_read": 6966 / 32,
                             "app_write": 1944 * 6 / 64}
    assert abs(m["cycles_per_group_iter"] - 1270.6875) < 1e-9
    alt = b.lds_models_alt(si)
    assert alt["issued"]["cycles_per_group_iter"] == 116 * 8 + 226 + 192 == 1346
    assert alt["padded"]["cycles_per_group_iter"] == 1442 and alt["issued"]["degree_split"]


def test_cpu_share_is_capped(monkeypatch):
    b = _bench()
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert 1 <= b.cpu_share() <= 3


def test_cpu_share_is_the_affinity_without_omp(monkeypatch):
    """with OMP_NUM_THREADS unset the share is the whole affinity."""
    b = _bench()
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    assert b.cpu_share() == len(os.sched_getaffinity(0)) == b.host_cores()


def test_reference_fer_fixture():
    """tests/golden/reference_fer.json (scripts/ref_fer.py, the reference's own decodeNMS
    over 10 seeds per point): every seed ends by the stop rule (>= 40 frame errors,
    >= 200 bit errors), totals add up, and each point agrees with SURVEY §6's single-seed
    run (|z| < 3). bench.py reads it for its FER comparison."""
    import json
    from ldpcsimulation_amd.sim import two_proportion_z
    b = _bench()
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_fer.json")))
    assert d["T"] == 50 and d["alpha"] == 1.25 and d["code"] == "80211n_1944_r12.alist"
    for p in d["points"]:
        runs = p["runs"]
        assert len(runs) == 10 and len({r["seed"] for r in runs}) == 10
        assert all(r["frame_err"] >= 40 and r["bit_err"] >= 200 for r in runs)
        for k in ("frame_err", "frames", "bit_err"):
            assert p[k] == sum(r[k] for r in runs)
        k1, n1 = b.REF_FER[p["ebn0_db"]]
        assert abs(two_proportion_z(p["frame_err"], p["frames"], k1, n1)) < 3
    assert b.reference_fer()[1.5] == (400, 27816)


def test_pmc_kernel_average_parses_rocprof_csv(tmp_path):
    """bench.py's live HBM traffic: per-dispatch sums of one counter over the matching
    kernel's dispatches, averaged (other kernels and counters ignored)."""
    import bench
    d = tmp_path / "FETCH_SIZE" / "host" / "123"
    d.mkdir(parents=True)
    rows = [("1", "void ldpc::k_rows_pp<1, 8, 4, 1, true, 0>(...)", "FETCH_SIZE", "100"),
            ("1", "void ldpc::k_rows_pp<1, 8, 4, 1, true, 0>(...)", "FETCH_SIZE", "20"),
            ("2", "void ldpc::k_redo<...>(...)", "FETCH_SIZE", "999"),
            ("3", "void ldpc::k_rows_pp<1, 8, 4, 1, true, 0>(...)", "FETCH_SIZE", "140"),
            ("3", "void ldpc::k_rows_pp<1, 8, 4, 1, true, 0>(...)", "WRITE_SIZE", "5")]
    with open(d / "pmc_counter_collection.csv", "w") as f:
        f.write("Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value\n")
        for r in rows:
            f.write(",".join(f'"{x}"' for x in r) + "\n")
    assert bench.pmc_kernel_average(str(tmp_path / "FETCH_SIZE"), "k_rows_pp", "FETCH_SIZE") == 130.0
    assert bench.pmc_kernel_average(str(tmp_path / "FETCH_SIZE"), "k_rows_fast", "FETCH_SIZE") is None
    assert bench.KERNEL_SYMBOL["rows_pp"] == "k_rows_pp"
