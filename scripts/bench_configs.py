#!/usr/bin/env python3
"""One measured line per BASELINE config and decoder, each with a named roofline
(VERDICT r5 item 2). Run on the GPU box:

    python scripts/bench_configs.py [--only NAME ...] [--pmc on|off] [--out FILE] [--pmc-dir DIR]

Per config it (1) times the fused on-device simulation (HIP events around the
library's launch: `ldpc_ctx_last_kernel_ms` / `ldpc_nb_ctx_last_kernel_ms`; inputs
are generated on the device, nothing crosses PCIe), then (2) runs four rocprofv3
`--pmc` passes, one counter set each, over a child process that makes exactly one
launch of the same workload (`--child NAME`), and sums the counters of that
launch's dispatches (`ldpc::k_*`, the once-per-context `k_verify_div` excluded).

Every line carries `roofline = {bound, achieved, peak, unit, frac}` for the resource
the counters show busiest, and the other resources' fractions beside it:

* `lds`   -- `SQ_LDS_IDX_ACTIVE` (LDS-array cycles, bank conflicts included) over
             256 CUs x kernel cycles (2.4 GHz); for the two min-sum row kernels
             (configs 1 and 2) the achieved figure is the algorithmic model of
             bench.py (E gathers + E scatters + E bit reads + N app writes at the
             LDS table's conflict-free costs), as in the headline line;
* `valu`  -- VALU issue cycles per SIMD from the instruction mix
             (`SQ_INSTS_VALU_{ADD,MUL,FMA}_F64` 4 cycles per wave64 instruction,
             `SQ_INSTS_VALU_TRANS_F32` and `_F64` 8, every other VALU instruction 2
             -- MI355X_MICROARCH: a wave64 VALU instruction issues over 2 cycles on a
             SIMD-32; fp64 at half that rate) over 1 024 SIMDs x kernel cycles;
             `fp64_flops` (`SQ_INSTS_VALU_FLOPS_FP64` against the 78.6 TFLOP/s fp64
             vector peak) beside it for the fp64 decoders;
* `hbm`   -- memory-side bytes, FETCH_SIZE x 2 + WRITE_SIZE (MI355X_MICROARCH's
             gfx950 correction) per second against 8.0 TB/s (6.29 TB/s achievable).

Which of these binds is a reading of the counters, not a proof: a kernel whose
largest fraction is well below 1 is latency-bound, and the line says so.
Reference paths: src/decodeMinSum.cpp:247-263 (configs 1-3), src/decodeGDBF.cpp:517-621
(config 4), SystemC/NB-LDPC/inc/nodes.h:195-293 (config 5), src/decodeBP.cpp:353-409.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

CLOCK = 2.4e9            # MI355X max shader clock (MI355X_MICROARCH chip table)
CUS = 256
HBM_PEAK = 8.0e12        # spec; 6.29 TB/s measured achievable
HBM_ACHIEVABLE = 6.29e12
FP64_PEAK = 78.6e12      # fp64 vector FLOP/s (half the fp32 vector 157.3 TF)
LDS_CYC = {"ds_read_b64": 2, "ds_write_b64": 6}

# name -> workload (BASELINE.json configs; the headline is config 2, measured by bench.py)
CONFIGS = {
    "c1_peg1008_ms_f64": dict(kind="minsum", code="PEGReg504x1008.alist", variant="ms", prec="f64", T=10,
                              batch=65536, snr=2.0,
                              what="config 1: smallest H (PEG 504x1008), min-sum 10 iterations, fp64"),
    "c2_80211n_nms_f64": dict(kind="minsum", code="80211n_1944_r12.alist", variant="nms", prec="f64", T=50,
                              batch=65536, snr=1.5,
                              what="config 2 (headline): 802.11n N=1944 R1/2, NMS alpha=1.25, T=50, fp64"),
    "c3_dvbs2_flood_f64": dict(kind="minsum", code="dvbs2_1_2.alist", variant="nms", prec="f64", T=50, batch=2048,
                               snr=1.0, what="config 3: DVB-S2 N=64800 R1/2, flooding NMS, T=50, fp64"),
    "c3_dvbs2_layered_f64": dict(kind="minsum", code="dvbs2_1_2.alist", variant="nms", prec="f64", T=50,
                                 batch=2048, snr=1.0, schedule="layered",
                                 what="config 3: DVB-S2 N=64800 R1/2, layered NMS, T=50, fp64"),
    "c4_smngdbf_f32": dict(kind="gdbf", code="80211n_1944_r12.alist", prec="f32", T=100, batch=65536, snr=3.5,
                           what="config 4: SMNGDBF on 802.11n N=1944, T<=100, fp32"),
    "c4_smngdbf_f64": dict(kind="gdbf", code="80211n_1944_r12.alist", prec="f64", T=100, batch=65536, snr=3.5,
                           what="config 4: SMNGDBF on 802.11n N=1944, T<=100, fp64"),
    "c5_ems_gf16": dict(kind="ems", T=20, nm=16, batch=16384, snr=2.0,
                        what="config 5: GF(16) EMS, N=1000 symbols (4000 bits), nm=16, T<=20"),
    "bp_80211n_f64": dict(kind="minsum", code="80211n_1944_r12.alist", variant="bp", prec="f64", T=50,
                          batch=16384, snr=1.5, what="BP (tanh rule) on 802.11n N=1944, T=50, fp64"),
    "bp_80211n_f32": dict(kind="minsum", code="80211n_1944_r12.alist", variant="bp", prec="f32", T=50,
                          batch=16384, snr=1.5, what="BP (tanh rule) on 802.11n N=1944, T=50, fp32"),
}

PMC_PASSES = [
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY "
    "GRBM_GUI_ACTIVE",
    "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 "
    "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE",
    "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS "
    "GRBM_GUI_ACTIVE",
    "FETCH_SIZE GRBM_GUI_ACTIVE",
    "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE",
]


# --latency: the memory pipeline's occupancy and latencies (Little's law per CU)
LATENCY_PASSES = [
    "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum "
    "GRBM_GUI_ACTIVE",
    "TCC_REQ_sum TCC_BUSY_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum GRBM_GUI_ACTIVE",
    "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES "
    "TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE",
]


class Workload:
    """One config's context and launch, through the C ABI (native.py)."""

    def __init__(self, name, lib=None):
        from ldpcsimulation_amd import codes, native
        if lib:
            native.use_library(os.path.abspath(lib))
        from conftest import code_path
        self.native, self.name, self.c = native, name, CONFIGS[name]
        c = self.c
        if c["kind"] == "ems":
            self.g = native.NbGraph.from_alist(codes.ensure_gf16_code())
            self.ctx = native.NbContext(self.g, 0, c["batch"])
            self.cfg = native.EmsConfig(T=c["T"], nm=c["nm"], offset=0.0, early_stop=True)
            self.bits = self.g.N * self.g.m
            self.launch_fn = self.ctx.sim_launch
            self.kernel = self.ctx.kernel_info()["kernel"]
            return
        self.g = native.Graph.from_alist(code_path(c["code"]))
        self.ctx = native.Context(self.g, 0, c["batch"])
        prec = native.F64 if c["prec"] == "f64" else native.F32
        self.bits = self.g.N
        if c["kind"] == "gdbf":
            self.cfg = native.GdbfConfig(T=c["T"], precision=prec)
            self.launch_fn = self.ctx.gdbf_sim_launch
            self.kernel = self.ctx.gdbf_kernel_info(self.cfg)["kernel"]
        else:
            v = {"ms": dict(variant=native.MS), "nms": dict(variant=native.NMS, alpha=1.25),
                 "bp": dict(variant=native.BP)}[c["variant"]]
            sched = native.LAYERED if c.get("schedule") == "layered" else native.FLOODING
            self.cfg = native.DecoderConfig(T=c["T"], precision=prec, schedule=sched, **v)
            self.launch_fn = self.ctx.sim_launch
            self.kernel = self.ctx.kernel_info(self.cfg)["kernel"]

    def launch(self, k, batch=None):
        b = batch or self.c["batch"]
        self.launch_fn(self.c["snr"], 0.5, self.cfg, seed=1, stream_id=0, first_cw=k * self.c["batch"], batch=b)
        return self.ctx.last_kernel_ms()

    def counts(self):
        return self.ctx.read_counts(reset=True)


def lds_edges_cycles(w):
    """bench.py's algorithmic LDS model per launch for the two min-sum row kernels (None otherwise)."""
    if w.c["kind"] != "minsum":
        return None
    try:
        si = w.ctx.row_sched_info(w.cfg)
    except w.native.LdpcError:
        return None
    g = w.g
    per = (2 * g.E * LDS_CYC["ds_read_b64"] + g.E * LDS_CYC["ds_write_b64"] + g.N * LDS_CYC["ds_write_b64"]) / 64
    return per * w.c["T"] * w.c["batch"], si


def timed(name, reps, lib):
    w = Workload(name, lib)
    w.launch(reps + 1, batch=min(w.c["batch"], 1024))   # warm-up (code objects, verify_div)
    w.counts()
    kms = []
    t0 = time.perf_counter()
    for k in range(reps):
        kms.append(w.launch(k))
    wall = time.perf_counter() - t0
    cnt = w.counts()
    d = {k: int(v) for k, v in cnt.as_dict().items()}
    frames = d.get("frames")
    kms_best = min(kms)
    out = {"name": name, "what": w.c["what"], "kernel": w.kernel, "batch": w.c["batch"], "T": w.c["T"],
           "ebn0_db": w.c["snr"], "reps": reps, "kernel_ms": kms, "kernel_ms_best": kms_best,
           "value": w.bits * w.c["batch"] / (kms_best / 1e3) / 1e6, "unit": "Mbit/s (coded bits, kernel time)",
           "wall_mbit_s": w.bits * frames / wall / 1e6 if frames else None,
           "fer": d.get("frame_err", 0) / frames if frames else None,
           "avg_iters": d.get("iters", 0) / frames if frames else None, "frames": frames}
    m = lds_edges_cycles(w)
    if m:
        out["lds_model_cycles_per_launch"], out["row_sched"] = m
    return out


def child(name, lib):
    """One launch of the workload (under rocprofv3 --pmc)."""
    w = Workload(name, lib)
    w.launch(0)
    w.counts()


def read_pmc(d):
    """Counters of the launch's decode dispatches, summed (k_verify_div excluded)."""
    tot = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "ldpc::k_" not in k or "k_verify_div" in k:
                continue
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return tot


def pmc(name, lib, outdir, passes=None):
    tot = {}
    for i, cs in enumerate(passes or PMC_PASSES):
        d = os.path.join(outdir, name, f"p{i + 1}")
        shutil.rmtree(d, ignore_errors=True)
        cmd = ["rocprofv3", "--pmc"] + cs.split() + ["-d", d, "-o", "pmc", "--output-format", "csv", "--",
                                                      sys.executable, os.path.abspath(__file__), "--child", name]
        if lib:
            cmd += ["--lib", lib]
        p = subprocess.run(["timeout", "-s", "KILL", "120"] + cmd, capture_output=True, text=True,
                           env=dict(os.environ, TMPDIR="/tmp"))
        if p.returncode != 0:
            raise RuntimeError(f"pmc pass {i + 1} of {name}: rc {p.returncode}: {p.stderr[-800:]}")
        got = read_pmc(d)
        grbm = got.pop("GRBM_GUI_ACTIVE", None)
        if grbm:
            tot.setdefault("GRBM_GUI_ACTIVE_passes", []).append(grbm)
        tot.update(got)
    return tot


def fractions(line, c):
    """Resource fractions of one launch from its counters and the timed kernel time."""
    t = line["kernel_ms_best"] / 1e3
    cyc = t * CLOCK
    f = {}
    if "SQ_LDS_IDX_ACTIVE" in c:
        f["lds"] = {"achieved": c["SQ_LDS_IDX_ACTIVE"] / t / 1e9, "peak": CUS * CLOCK / 1e9,
                    "unit": "G LDS-array cycles/s (SQ_LDS_IDX_ACTIVE, conflicts included)",
                    "frac": c["SQ_LDS_IDX_ACTIVE"] / (CUS * cyc),
                    "bank_conflict_share": c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c["SQ_LDS_IDX_ACTIVE"], 1)}
        if "lds_model_cycles_per_launch" in line:
            m = line["lds_model_cycles_per_launch"]
            f["lds_algorithmic"] = {"achieved": m / t / 1e9, "peak": CUS * CLOCK / 1e9,
                                    "unit": "G LDS-cycles/s (E gathers + E scatters + E bit reads + N app writes)",
                                    "frac": m / (CUS * cyc)}
    if "SQ_INSTS_VALU" in c:
        f64 = sum(c.get(k, 0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64"))
        tr = c.get("SQ_INSTS_VALU_TRANS_F32", 0) + c.get("SQ_INSTS_VALU_TRANS_F64", 0)
        other = c["SQ_INSTS_VALU"] - f64 - tr
        issue = 2 * other + 4 * f64 + 8 * tr
        f["valu"] = {"achieved": issue / t / 1e9, "peak": CUS * 4 * CLOCK / 1e9,
                     "unit": "G SIMD issue-cycles/s (instruction mix: 2 / fp64 add-mul-fma 4 / transcendental 8)",
                     "frac": issue / (CUS * 4 * cyc),
                     "valu_instr_per_cu_cycle": c["SQ_INSTS_VALU"] / (CUS * cyc),
                     "mix": {"fp64_add_mul_fma": f64, "transcendental": tr, "other": other}}
    if c.get("SQ_INSTS_VALU_FLOPS_FP64"):
        f["fp64_flops"] = {"achieved": c["SQ_INSTS_VALU_FLOPS_FP64"] / t / 1e12, "peak": FP64_PEAK / 1e12,
                           "unit": "TFLOP/s fp64 (SQ_INSTS_VALU_FLOPS_FP64)",
                           "frac": c["SQ_INSTS_VALU_FLOPS_FP64"] / t / FP64_PEAK}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        b = 2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024   # rocprofv3 reports KB
        f["hbm"] = {"achieved": b / t / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s (FETCH_SIZE x 2 + WRITE_SIZE)",
                    "frac": b / t / HBM_PEAK, "frac_of_achievable": b / t / HBM_ACHIEVABLE, "bytes_per_launch": b}
    if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
        f["wait_any_share"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    g = c.get("GRBM_GUI_ACTIVE_passes")
    if g:
        f["profiled_clock_ghz"] = sum(g) / len(g) / 8 / t / 1e9   # approximate: profiled launch vs timed launch
    return f


def latency(line, c):
    """Little's law per CU from the latency passes: average TCP->TCC read requests in
    flight = sum of their latencies / kernel cycles; bytes per cycle = in flight x 64 B /
    latency (the measured rate, restated); and the occupancy of the units in between."""
    g = c.get("GRBM_GUI_ACTIVE_passes")
    cyc = (sum(g) / len(g) / 8) if g else line["kernel_ms_best"] / 1e3 * CLOCK   # per-XCD cycles of the launch
    out = {"kernel_cycles": cyc}
    rq, lat = c.get("TCP_TCC_READ_REQ_sum"), c.get("TCP_TCC_READ_REQ_LATENCY_sum")
    if rq and lat:
        out["tcp_tcc_read_latency_cycles"] = lat / rq
        out["tcp_tcc_reads_in_flight_per_cu"] = lat / (CUS * cyc)
        out["tcp_tcc_read_req_per_cu_cycle"] = rq / (CUS * cyc)
        out["littles_law_read_bytes_per_cu_cycle_64B"] = out["tcp_tcc_reads_in_flight_per_cu"] * 64 / out[
            "tcp_tcc_read_latency_cycles"]
    if c.get("TCP_TCC_WRITE_REQ_sum"):
        out["tcp_tcc_write_req_per_cu_cycle"] = c["TCP_TCC_WRITE_REQ_sum"] / (CUS * cyc)
    if c.get("TCP_PENDING_STALL_CYCLES_sum") is not None:
        out["tcp_pending_stall_share"] = c["TCP_PENDING_STALL_CYCLES_sum"] / (CUS * cyc)
    if c.get("TCC_EA0_RDREQ_sum") and c.get("TCC_EA0_RDREQ_LEVEL_sum"):
        out["fabric_read_latency_cycles"] = c["TCC_EA0_RDREQ_LEVEL_sum"] / c["TCC_EA0_RDREQ_sum"]
        out["fabric_reads_in_flight_per_xcd"] = c["TCC_EA0_RDREQ_LEVEL_sum"] / (8 * cyc)
    if c.get("TCC_BUSY_sum"):
        out["tcc_busy_share"] = c["TCC_BUSY_sum"] / (128 * cyc)   # 16 channels x 8 XCDs
    if c.get("TCC_REQ_sum"):
        out["tcc_req_per_channel_cycle"] = c["TCC_REQ_sum"] / (128 * cyc)
    if c.get("TA_BUSY_sum"):
        out["ta_busy_share"] = c["TA_BUSY_sum"] / (CUS * cyc)
        out["ta_addr_stalled_by_tc_share"] = c.get("TA_ADDR_STALLED_BY_TC_CYCLES_sum", 0) / (CUS * cyc)
    if c.get("SQ_INSTS_VMEM_RD"):
        out["vmem_rd_instr_per_cu_cycle"] = c["SQ_INSTS_VMEM_RD"] / (CUS * cyc)
        out["vmem_wr_instr_per_cu_cycle"] = c.get("SQ_INSTS_VMEM_WR", 0) / (CUS * cyc)
    if c.get("SQ_WAIT_ANY") and c.get("SQ_WAVE_CYCLES"):
        out["wait_any_share"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    return out


def roofline(line, f):
    """The binding resource: the largest fraction (LDS kernels keep the algorithmic model)."""
    cand = {k: v for k, v in f.items() if k in ("lds", "valu", "hbm")}
    if not cand:
        return None
    k = max(cand, key=lambda x: cand[x]["frac"])
    r = cand[k]
    if k == "lds" and "lds_algorithmic" in f:
        r = f["lds_algorithmic"]
    out = {"bound": k, "achieved": r["achieved"], "peak": r["peak"], "unit": r["unit"], "frac": r["frac"]}
    if cand[k]["frac"] < 0.7:
        out["note"] = ("no resource above 0.7 of its peak: latency-bound (wait_any_share %.2f)"
                       % f.get("wait_any_share", float("nan")))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pmc", choices=["on", "off"], default="on")
    ap.add_argument("--pmc-dir", default=os.path.join(ROOT, "gpurun_out", "bench_configs_pmc"))
    ap.add_argument("--out", default=None, help="append the JSON lines here too")
    ap.add_argument("--child", default=None)
    ap.add_argument("--lib", default=None, help="A/B only: another build of the decoder library")
    ap.add_argument("--latency", action="store_true", help="also the memory-latency passes (Little's law)")
    a = ap.parse_args()
    if a.child:
        child(a.child, a.lib)
        return 0
    names = a.only or list(CONFIGS)
    for n in names:
        if n not in CONFIGS:
            sys.exit(f"unknown config {n}; known: {', '.join(CONFIGS)}")
    for n in names:
        # the timed run in a child process of its own (one context, one device state per config)
        p = subprocess.run([sys.executable, "-c",
                            "import json,sys; sys.argv=['x']; sys.path.insert(0, %r); import bench_configs as b; "
                            "print(json.dumps(b.timed(%r, %d, %r)))" % (os.path.dirname(os.path.abspath(__file__)),
                                                                         n, a.reps, a.lib)],
                           capture_output=True, text=True, timeout=600)
        if p.returncode != 0:
            raise RuntimeError(f"timed run of {n}: {p.stderr[-1500:]}")
        line = json.loads(p.stdout.strip().splitlines()[-1])
        if a.pmc == "on":
            c = pmc(n, a.lib, a.pmc_dir)
            f = fractions(line, c)
            line["fractions"] = f
            line["roofline"] = roofline(line, f)
            line["pmc"] = {k: v for k, v in c.items()}
            line["pmc_source"] = "rocprofv3 --pmc, %d passes over one launch (%s)" % (
                len(PMC_PASSES), os.path.relpath(os.path.join(a.pmc_dir, n), ROOT))
        if a.latency:
            cl = pmc(n, a.lib, os.path.join(a.pmc_dir, "latency"), LATENCY_PASSES)
            line["latency"] = latency(line, cl)
            line["latency_pmc"] = cl
        s = json.dumps(line)
        print(s, flush=True)
        if a.out:
            with open(a.out, "a") as fo:
                fo.write(s + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
