"""ctypes binding of the C ABI in include/ldpc_hip.h (libldpc_hip.so).

This is the only way the Python side reaches the decoder: there is no CPU
fallback. If the HIP library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "lib", "libldpc_hip.so")

LDPC_OK = 0
MS, NMS, OMS, BP = 0, 1, 2, 3
F32, F64 = 0, 1
FLOODING, LAYERED = 0, 1
ABI_VERSION = 11
# Kernel-selection options (include/ldpc_hip.h ldpc_option): tests and A/B runs set
# them per context through the ABI; the library never reads the environment.
OPTIONS = {"rows64": 1, "rows32": 2, "pp_slots": 3, "kernel": 4, "flood_mode": 5, "flood_msg": 6,
           "flood_sps_check": 7, "flood_sps_bit": 8, "flood_resident": 9, "flood_streams": 10, "flood_bpc": 11,
           "layered_bpc": 12, "layered_lds_pos": 13, "layered_rows64": 14, "layered_threads": 15,
           "rows_bpc": 16, "fast_bpc": 17, "bp_kernel": 18, "gdbf_kernel": 19, "ems_threads": 20,
           "ems_swizzle": 21}
# options of the GF(q) EMS context only (ldpc_nb_ctx_set_option); the binary context refuses them
EMS_OPTIONS = ("ems_threads", "ems_swizzle")
# symbolic values of the kernel-choice options
OPTION_VALUES = {"rows64": {"pp": 0, "fast": 1, "rows": 2}, "rows32": {"pp": 0, "fast": 1, "rows": 2},
                 "pp_slots": {"split": 0, "plain": 1}, "kernel": {"auto": 0, "lds": 1, "flood": 2, "global": 3},
                 "flood_mode": {"phase": 0, "persistent": 1}, "flood_msg": {"packed": 0, "c2v": 1},
                 "bp_kernel": {"rows": 0, "generic": 1}, "gdbf_kernel": {"rows": 0, "generic": 1},
                 "ems_swizzle": {"on": 0, "off": 1}}


def option_id(name) -> int:
    return name if isinstance(name, int) else OPTIONS[name]


def option_value(name, value) -> int:
    if isinstance(value, str) and not isinstance(name, int):
        return OPTION_VALUES[name][value]
    return int(value)


def use_library(path: str):
    """Load another build of the library (A/B variants; `bench.py --lib`). Only before
    the first call into the library; the product path is LIB_PATH."""
    global LIB_PATH
    if _lib is not None and os.path.abspath(path) != os.path.abspath(LIB_PATH):
        raise RuntimeError("the decoder library is already loaded")
    LIB_PATH = path
_STATUS = {0: "OK", -1: "INVALID", -2: "NOMEM", -3: "DEVICE", -4: "UNSUPPORTED", -5: "IO", -6: "GRAPH"}


class LdpcError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ldpc error {code} ({_STATUS.get(code, '?')}): {msg}")
        self.code = code


class Counts(C.Structure):
    _fields_ = [("bit_err", C.c_int64), ("frame_err", C.c_int64), ("uncoded_bit_err", C.c_int64),
                ("frames", C.c_int64), ("iters", C.c_int64), ("syndrome_fail", C.c_int64)]

    def as_dict(self) -> dict:
        return {k: int(getattr(self, k)) for k, _ in self._fields_}

    def as_array(self) -> np.ndarray:
        return np.array([getattr(self, k) for k, _ in self._fields_], dtype=np.int64)


FRAME_DTYPE = np.dtype([("bit_err", np.int32), ("uncoded_bit_err", np.int32),
                        ("syndrome_fail", np.int32), ("iters", np.int32)])


class _Cfg(C.Structure):
    _fields_ = [("variant", C.c_int32), ("precision", C.c_int32), ("T", C.c_int32),
                ("quantize", C.c_int32), ("saturate", C.c_int32), ("qbits", C.c_int32),
                ("ymax", C.c_double), ("alpha", C.c_double), ("delta", C.c_double),
                ("schedule", C.c_int32), ("reserved", C.c_int32), ("n0", C.c_double), ("max_llr", C.c_double)]


GDBF_NOISE, GDBF_ADAPT, GDBF_WEIGHT, GDBF_SMOOTH, GDBF_SATURATE, GDBF_QUANTIZE = 1, 2, 4, 8, 16, 32
GDBF_SEQUENTIAL, GDBF_MODESWITCH, GDBF_QPROB = 64, 128, 256
# the reference's decodeGDBF.cpp Makefile targets (C_implementations/Makefile:33-53)
GDBF_VARIANTS = {
    "MNGDBF": GDBF_NOISE | GDBF_ADAPT | GDBF_WEIGHT | GDBF_SATURATE,
    "SMNGDBF": GDBF_NOISE | GDBF_ADAPT | GDBF_WEIGHT | GDBF_SMOOTH | GDBF_SATURATE,
    "ATGDBF": GDBF_ADAPT,
    "SATGDBF": GDBF_ADAPT | GDBF_SMOOTH,
    "SMGDBF": GDBF_SMOOTH,
    "SGDBF": GDBF_SEQUENTIAL,
    "MGDBF": GDBF_MODESWITCH,
    "StochasticNGDBF": GDBF_QUANTIZE | GDBF_QPROB | GDBF_WEIGHT | GDBF_SATURATE,
}


class _GdbfCfg(C.Structure):
    _fields_ = [("flags", C.c_int32), ("precision", C.c_int32), ("T", C.c_int32), ("windowsize", C.c_int32),
                ("nq", C.c_int32), ("tswitch", C.c_int32), ("theta", C.c_double), ("lambda_", C.c_double),
                ("alpha", C.c_double), ("noise_scale", C.c_double), ("ymax", C.c_double), ("qsigma", C.c_double)]


@dataclass
class GdbfConfig:
    """GDBF / NGDBF bit flipping (src/decodeGDBF.cpp parallel mode); flags = the -D switches."""
    flags: int = GDBF_VARIANTS["SMNGDBF"]
    T: int = 100
    theta: float = -0.6
    lambda_: float = 0.99
    alpha: float = 0.8
    noise_scale: float = 0.75
    ymax: float = 2.5
    windowsize: int = 16
    nq: int = 16
    precision: int = 1   # F64, the reference's double (decodeGDBF.cpp); F32 = 0 opt-in
    tswitch: int = 0     # MODESWITCH: Tswitch (:51)
    qsigma: float = 0.0  # QPROB, gdbf_decode only: the normalCDF sigma

    def _c(self) -> _GdbfCfg:
        return _GdbfCfg(self.flags, self.precision, self.T, self.windowsize, self.nq, self.tswitch, self.theta,
                        self.lambda_, self.alpha, self.noise_scale, self.ymax, self.qsigma)


@dataclass
class DecoderConfig:
    """Runtime form of the reference's compile-time decoder switches."""
    variant: int = MS            # MS | NMS (-D normalizedMS) | OMS (-D offsetMS)
    T: int = 10                  # iterations (fixed, no early termination)
    precision: int = F64         # F64 = the reference's double (default) | F32 throughput path (opt-in)
    alpha: float = 1.0           # NMS divisor
    delta: float = 0.0           # OMS offset
    quantize: bool = False       # -D quantizeSamples
    saturate: bool = False       # -D saturateSamples
    ymax: float = 0.0
    qbits: int = 0
    schedule: int = FLOODING     # FLOODING (the reference's) | LAYERED (row-serial, config 3)
    n0: float = 0.0              # BP (variant BP): N0 of the LLR front-end 4*y/N0 (decode only)
    max_llr: float = 0.0         # BP: MAXLLR (0 = the reference's 20)

    def _c(self) -> _Cfg:
        return _Cfg(self.variant, self.precision, self.T, int(self.quantize), int(self.saturate),
                    self.qbits, self.ymax, self.alpha, self.delta, self.schedule, 0, self.n0, self.max_llr)


class _EmsCfg(C.Structure):
    _fields_ = [("T", C.c_int32), ("nm", C.c_int32), ("early_stop", C.c_int32), ("reserved", C.c_int32),
                ("offset", C.c_double)]


class NbCounts(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("bit_err", "frame_err", "uncoded_bit_err", "frames", "iters",
                                         "syndrome_fail", "symbol_err")]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


@dataclass
class EmsConfig:
    """Extended Min-Sum over GF(q) (include/ldpc_hip.h ldpc_ems_cfg)."""
    T: int = 20
    nm: int = 16                 # message truncation (>= q: full vectors)
    offset: float = 0.0          # fill offset for truncated symbols
    early_stop: bool = True      # stop when H d = 0

    def _c(self) -> _EmsCfg:
        return _EmsCfg(self.T, self.nm, int(self.early_stop), 0, self.offset)


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"HIP decoder library not built: {LIB_PATH} (run __graft_entry__.build() or `make`)")
    # One HIP runtime per process: torch ships its own libamdhip64 (soname
    # libamdhip64.so.7, DT_NEEDED by file name), and loading this library first
    # would map /opt/rocm's copy as well -- two runtimes, and torch.cuda then finds
    # no GPU. Imported first, torch's copy satisfies this library's soname.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, u32, u64, dbl = C.c_void_p, C.c_int, C.c_int64, C.c_uint32, C.c_uint64, C.c_double
    sig = {
        "ldpc_abi_version": ([], i32),
        "ldpc_f64_nms_fast_division": ([dbl], i32),
        "ldpc_bp_math_probe": ([i32, vp, i32, vp, vp], i32),
        "ldpc_check_selftest": ([i32], i32),
        "ldpc_last_error": ([], C.c_char_p),
        "ldpc_graph_create": ([i32, i32, vp, vp, vp, vp, C.POINTER(vp)], i32),
        "ldpc_graph_load_alist": ([C.c_char_p, C.POINTER(vp)], i32),
        "ldpc_graph_info": ([vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), C.POINTER(i32),
                             C.POINTER(i32)], i32),
        "ldpc_graph_destroy": ([vp], None),
        "ldpc_graph_layers": ([vp, vp, vp, C.POINTER(i32)], i32),
        "ldpc_device_count": ([C.POINTER(i32)], i32),
        "ldpc_ctx_create": ([i32, vp, i32, C.POINTER(vp)], i32),
        "ldpc_ctx_set_stream": ([vp, vp], i32),
        "ldpc_ctx_synchronize": ([vp], i32),
        "ldpc_ctx_destroy": ([vp], None),
        "ldpc_decode_batch": ([vp, vp, i32, C.POINTER(_Cfg), vp, vp, vp, C.POINTER(Counts)], i32),
        "ldpc_sim_set_codewords": ([vp, vp, i32], i32),
        "ldpc_sim_launch": ([vp, dbl, dbl, C.POINTER(_Cfg), u64, u32, u64, i32, vp], i32),
        "ldpc_ctx_read_counts": ([vp, C.POINTER(Counts), i32], i32),
        "ldpc_ctx_read_histogram": ([vp, vp, i32], i32),
        "ldpc_sim_batch": ([vp, dbl, dbl, C.POINTER(_Cfg), u64, u32, u64, i32, vp, C.POINTER(Counts)], i32),
        "ldpc_sim_trace": ([vp, dbl, dbl, C.POINTER(_Cfg), u64, u32, u64, i32, vp, vp, vp, C.POINTER(Counts)],
                           i32),
        "ldpc_ctx_last_kernel_ms": ([vp, C.POINTER(C.c_float)], i32),
        "ldpc_ctx_kernel_info": ([vp, C.POINTER(_Cfg), C.c_char_p, i32, C.POINTER(i32), C.POINTER(i32)], i32),
        "ldpc_ctx_redo_count": ([vp, C.POINTER(C.c_int64)], i32),
        "ldpc_ctx_row_sched_info": ([vp, C.POINTER(_Cfg), vp], i32),
        "ldpc_ctx_set_option": ([vp, i32, i32], i32),
        "ldpc_ctx_get_option": ([vp, i32, C.POINTER(i32)], i32),
        "ldpc_nb_ctx_set_option": ([vp, i32, i32], i32),
        "ldpc_gdbf_decode_batch": ([vp, vp, vp, i32, C.POINTER(_GdbfCfg), vp, vp, vp, C.POINTER(Counts)], i32),
        "ldpc_gdbf_sim_launch": ([vp, dbl, dbl, C.POINTER(_GdbfCfg), u64, u32, u64, i32, vp], i32),
        "ldpc_gdbf_sim_batch": ([vp, dbl, dbl, C.POINTER(_GdbfCfg), u64, u32, u64, i32, vp, C.POINTER(Counts)],
                                i32),
        "ldpc_gdbf_kernel_info": ([vp, C.POINTER(_GdbfCfg), C.c_char_p, i32, C.POINTER(i32)], i32),
        "ldpc_nb_graph_create": ([i32, i32, i32, vp, vp, vp, vp, vp, vp, C.POINTER(vp)], i32),
        "ldpc_nb_graph_load_alist": ([C.c_char_p, C.POINTER(vp)], i32),
        "ldpc_nb_graph_info": ([vp] + [C.POINTER(i32)] * 6, i32),
        "ldpc_nb_graph_destroy": ([vp], None),
        "ldpc_nb_ctx_create": ([i32, vp, i32, C.POINTER(vp)], i32),
        "ldpc_nb_ctx_set_stream": ([vp, vp], i32),
        "ldpc_nb_ctx_destroy": ([vp], None),
        "ldpc_nb_ctx_read_counts": ([vp, C.POINTER(NbCounts), i32], i32),
        "ldpc_nb_ctx_last_kernel_ms": ([vp, C.POINTER(C.c_float)], i32),
        "ldpc_ems_kernel_info": ([vp, C.c_char_p, i32, C.POINTER(i32)], i32),
        "ldpc_ems_decode_batch": ([vp, vp, i32, dbl, C.POINTER(_EmsCfg), vp, vp, vp, C.POINTER(NbCounts)], i32),
        "ldpc_ems_sim_launch": ([vp, dbl, dbl, C.POINTER(_EmsCfg), u64, u32, u64, i32, vp], i32),
        "ldpc_ems_sim_batch": ([vp, dbl, dbl, C.POINTER(_EmsCfg), u64, u32, u64, i32, vp, C.POINTER(NbCounts)],
                               i32),
        "ldpc_ems_sim_trace": ([vp, dbl, dbl, C.POINTER(_EmsCfg), u64, u32, u64, i32, vp, vp, vp,
                                C.POINTER(NbCounts)], i32),
    }
    for name, (argt, rest) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = argt
        fn.restype = rest
    if L.ldpc_abi_version() != ABI_VERSION:
        raise ImportError(f"{LIB_PATH}: ABI version {L.ldpc_abi_version()}, this binding needs {ABI_VERSION}")
    _lib = L
    return L


# Every symbol include/ldpc_hip.h declares (checked by tests/test_abi.py).
EXPORTED = ["ldpc_abi_version", "ldpc_f64_nms_fast_division", "ldpc_bp_math_probe", "ldpc_check_selftest", "ldpc_last_error", "ldpc_graph_create", "ldpc_graph_load_alist",
            "ldpc_graph_info", "ldpc_graph_destroy", "ldpc_graph_layers", "ldpc_device_count", "ldpc_ctx_create",
            "ldpc_ctx_set_stream", "ldpc_ctx_synchronize", "ldpc_ctx_destroy", "ldpc_decode_batch",
            "ldpc_sim_set_codewords", "ldpc_sim_launch", "ldpc_ctx_read_counts", "ldpc_ctx_read_histogram",
            "ldpc_sim_batch", "ldpc_sim_trace", "ldpc_ctx_last_kernel_ms", "ldpc_ctx_kernel_info", "ldpc_ctx_redo_count",
            "ldpc_ctx_row_sched_info", "ldpc_ctx_set_option", "ldpc_ctx_get_option", "ldpc_nb_ctx_set_option",
            "ldpc_gdbf_decode_batch", "ldpc_gdbf_sim_launch", "ldpc_gdbf_sim_batch", "ldpc_gdbf_kernel_info",
            "ldpc_nb_graph_create", "ldpc_nb_graph_load_alist", "ldpc_nb_graph_info", "ldpc_nb_graph_destroy",
            "ldpc_nb_ctx_create", "ldpc_nb_ctx_set_stream", "ldpc_nb_ctx_destroy", "ldpc_nb_ctx_read_counts",
            "ldpc_nb_ctx_last_kernel_ms", "ldpc_ems_kernel_info", "ldpc_ems_decode_batch", "ldpc_ems_sim_launch",
            "ldpc_ems_sim_batch", "ldpc_ems_sim_trace"]


def _check(rc: int):
    if rc != LDPC_OK:
        raise LdpcError(rc, lib().ldpc_last_error().decode(errors="replace"))


def device_count() -> int:
    n = C.c_int(0)
    rc = lib().ldpc_device_count(C.byref(n))
    return n.value if rc == LDPC_OK else 0


class Graph:
    """Immutable Tanner graph (H matrix) on the host side of the ABI."""

    def __init__(self, handle):
        self._h = handle
        N, M, E, dv, dc = (C.c_int() for _ in range(5))
        _check(lib().ldpc_graph_info(self._h, C.byref(N), C.byref(M), C.byref(E), C.byref(dv), C.byref(dc)))
        self.N, self.M, self.E, self.maxdv, self.maxdc = N.value, M.value, E.value, dv.value, dc.value

    @classmethod
    def from_alist(cls, path: str) -> "Graph":
        h = C.c_void_p()
        _check(lib().ldpc_graph_load_alist(os.fspath(path).encode(), C.byref(h)))
        return cls(h)

    @classmethod
    def from_lists(cls, N: int, M: int, nlist, mlist) -> "Graph":
        """nlist[i]: 1-based checks of bit i; mlist[j]: 1-based bits of check j (alist_struct form)."""
        num_n = (C.c_int * N)(*[len(x) for x in nlist])
        num_m = (C.c_int * M)(*[len(x) for x in mlist])
        keep = [(C.c_int * max(len(x), 1))(*x) for x in nlist] + [(C.c_int * max(len(x), 1))(*x) for x in mlist]
        np_ = (C.c_void_p * N)(*[C.cast(a, C.c_void_p) for a in keep[:N]])
        mp_ = (C.c_void_p * M)(*[C.cast(a, C.c_void_p) for a in keep[N:]])
        h = C.c_void_p()
        _check(lib().ldpc_graph_create(N, M, num_n, np_, num_m, mp_, C.byref(h)))
        return cls(h)

    def layers(self):
        """(row_order [M] int32, layer_ptr [nlayers+1] int32) of the LAYERED schedule."""
        n = C.c_int()
        _check(lib().ldpc_graph_layers(self._h, None, None, C.byref(n)))
        order = np.empty(self.M, dtype=np.int32)
        ptr = np.empty(n.value + 1, dtype=np.int32)
        _check(lib().ldpc_graph_layers(self._h, order.ctypes.data, ptr.ctypes.data, C.byref(n)))
        return order, ptr

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.ldpc_graph_destroy(h)
            self._h = None


def _ptr(a) -> Optional[int]:
    """Address of a numpy array or a torch tensor (host or device)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        if not a.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        if not a.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return a.data_ptr()
    raise TypeError(type(a))


class Context:
    """One device context (stream, counters, scratch) bound to a graph."""

    def __init__(self, graph: Graph, device: int = 0, max_batch: int = 65536):
        self.graph = graph
        self.device = device
        self.max_batch = max_batch
        h = C.c_void_p()
        _check(lib().ldpc_ctx_create(device, graph._h, max_batch, C.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.ldpc_ctx_destroy(h)
            self._h = None

    def set_stream(self, stream_handle: Optional[int]):
        _check(lib().ldpc_ctx_set_stream(self._h, stream_handle))

    def set_option(self, name, value):
        """Override the kernel choice (ldpc_ctx_set_option): name from OPTIONS, value an int
        or a symbolic value from OPTION_VALUES (e.g. set_option("rows64", "fast"))."""
        _check(lib().ldpc_ctx_set_option(self._h, option_id(name), option_value(name, value)))

    def get_option(self, name) -> int:
        v = C.c_int()
        _check(lib().ldpc_ctx_get_option(self._h, option_id(name), C.byref(v)))
        return int(v.value)

    def set_options(self, opts: Optional[dict]):
        for k, v in (opts or {}).items():
            self.set_option(k, v)

    def reset_options(self):
        """Every option back to 0, the library's own kernel choice."""
        for name, k in OPTIONS.items():
            if name not in EMS_OPTIONS:   # those belong to the nb context (NbContext.set_options)
                _check(lib().ldpc_ctx_set_option(self._h, k, 0))

    def synchronize(self):
        _check(lib().ldpc_ctx_synchronize(self._h))

    def decode(self, y, cfg: DecoderConfig, c=None, want_decisions: bool = True, want_frames: bool = True):
        """Decode y[batch, N] (float32 for F32, float64 for F64; numpy or torch, host or device).

        Returns (d [batch,N] int8 or None, frames structured array or None, Counts)."""
        N = self.graph.N
        if isinstance(y, np.ndarray):
            want = np.float64 if cfg.precision == F64 else np.float32
            if y.dtype != want:
                raise TypeError(f"y must be {np.dtype(want)} for this precision, got {y.dtype}")
            y = np.ascontiguousarray(y)
            size = y.size
        else:   # torch tensor: the kernel reads batch*N elements of the precision's width
            want = "torch.float64" if cfg.precision == F64 else "torch.float32"
            if str(y.dtype) != want:
                raise TypeError(f"y must be {want} for this precision, got {y.dtype}")
            size = y.numel()
        if size % N:
            raise ValueError(f"y has {size} elements, not a multiple of N={N}")
        batch = size // N
        if c is not None:
            if isinstance(c, np.ndarray):
                c = np.ascontiguousarray(c, dtype=np.int8)
            elif str(c.dtype) != "torch.int8":
                raise TypeError(f"c must be torch.int8 (bipolar +1/-1), got {c.dtype}")
            csize = c.size if isinstance(c, np.ndarray) else c.numel()
            if csize != batch * N:
                raise ValueError(f"c has {csize} elements, y {batch * N}")
        d = np.empty((batch, N), dtype=np.int8) if want_decisions else None
        fr = np.empty(batch, dtype=FRAME_DTYPE) if want_frames else None
        cnt = Counts()
        _check(lib().ldpc_decode_batch(self._h, _ptr(y), batch, C.byref(cfg._c()), _ptr(c), _ptr(d), _ptr(fr),
                                       C.byref(cnt)))
        return d, fr, cnt

    def set_codewords(self, bits: Optional[np.ndarray]):
        if bits is None:
            _check(lib().ldpc_sim_set_codewords(self._h, None, 0))
            return
        bits = np.ascontiguousarray(bits, dtype=np.uint8).reshape(-1, self.graph.N)
        _check(lib().ldpc_sim_set_codewords(self._h, bits.ctypes.data, bits.shape[0]))

    def sim_launch(self, ebn0_db: float, R: float, cfg: DecoderConfig, seed: int, stream_id: int, first_cw: int,
                   batch: int, frames_dev=None):
        _check(lib().ldpc_sim_launch(self._h, ebn0_db, R, C.byref(cfg._c()), seed, stream_id, first_cw, batch,
                                     _ptr(frames_dev)))

    def sim_batch(self, ebn0_db: float, R: float, cfg: DecoderConfig, seed: int, stream_id: int, first_cw: int,
                  batch: int, want_frames: bool = True):
        fr = np.empty(batch, dtype=FRAME_DTYPE) if want_frames else None
        cnt = Counts()
        _check(lib().ldpc_sim_batch(self._h, ebn0_db, R, C.byref(cfg._c()), seed, stream_id, first_cw, batch,
                                    _ptr(fr), C.byref(cnt)))
        return fr, cnt

    def sim_trace(self, ebn0_db: float, R: float, cfg: DecoderConfig, seed: int, stream_id: int, first_cw: int,
                  batch: int):
        """sim_batch that also returns the generated channel samples and decisions."""
        N = self.graph.N
        y = np.empty((batch, N), dtype=np.float64 if cfg.precision == F64 else np.float32)
        d = np.empty((batch, N), dtype=np.int8)
        fr = np.empty(batch, dtype=FRAME_DTYPE)
        cnt = Counts()
        _check(lib().ldpc_sim_trace(self._h, ebn0_db, R, C.byref(cfg._c()), seed, stream_id, first_cw, batch,
                                    y.ctypes.data, d.ctypes.data, fr.ctypes.data, C.byref(cnt)))
        return y, d, fr, cnt

    def read_counts(self, reset: bool = False) -> Counts:
        cnt = Counts()
        _check(lib().ldpc_ctx_read_counts(self._h, C.byref(cnt), int(reset)))
        return cnt

    def read_histogram(self, reset: bool = False) -> np.ndarray:
        h = np.zeros(self.graph.N, dtype=np.int64)
        _check(lib().ldpc_ctx_read_histogram(self._h, h.ctypes.data, int(reset)))
        return h

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        _check(lib().ldpc_ctx_last_kernel_ms(self._h, C.byref(ms)))
        return float(ms.value)

    def redo_count(self) -> int:
        """Codewords of the last launch the fast fp64 row kernel re-decoded on the exact path."""
        n = C.c_int64()
        _check(lib().ldpc_ctx_redo_count(self._h, C.byref(n)))
        return int(n.value)

    def row_sched_info(self, cfg: DecoderConfig) -> dict:
        """Shape of the row kernel that decodes cfg (raises LdpcError UNSUPPORTED for other kernels)."""
        info = np.zeros(10, dtype=np.int32)
        _check(lib().ldpc_ctx_row_sched_info(self._h, C.byref(cfg._c()), info.ctypes.data))
        keys = ("threads", "rows_per_thread", "slots_per_thread", "dc", "e_pad", "cw_per_block", "lds_bytes",
                "blocks_per_cu", "dc_low", "issued_check_edges")
        return {k: int(v) for k, v in zip(keys, info)}

    def kernel_info(self, cfg: DecoderConfig) -> dict:
        name = C.create_string_buffer(32)
        lds, bpc = C.c_int(), C.c_int()
        _check(lib().ldpc_ctx_kernel_info(self._h, C.byref(cfg._c()), name, 32, C.byref(lds), C.byref(bpc)))
        return {"kernel": name.value.decode(), "lds_bytes": lds.value, "blocks_per_cu": bpc.value}

    # ---- GDBF / NGDBF (src/decodeGDBF.cpp) ----
    def gdbf_decode(self, y, pert, cfg: GdbfConfig, c=None, want_decisions: bool = True):
        """Decode raw channel samples y[batch, N] with perturbations pert[batch, T, N] (or None
        without GDBF_NOISE). Returns (d, frames (iters = iterations run), Counts)."""
        N = self.graph.N
        want = np.float64 if cfg.precision == F64 else np.float32
        y = np.ascontiguousarray(y, dtype=want).reshape(-1, N)
        batch = y.shape[0]
        if pert is not None:
            pert = np.ascontiguousarray(pert, dtype=want).reshape(batch, cfg.T, N)
        if c is not None:
            c = np.ascontiguousarray(c, dtype=np.int8)
        d = np.empty((batch, N), dtype=np.int8) if want_decisions else None
        fr = np.empty(batch, dtype=FRAME_DTYPE)
        cnt = Counts()
        _check(lib().ldpc_gdbf_decode_batch(self._h, _ptr(y), _ptr(pert), batch, C.byref(cfg._c()), _ptr(c),
                                            _ptr(d), _ptr(fr), C.byref(cnt)))
        return d, fr, cnt

    def gdbf_sim_launch(self, ebn0_db: float, R: float, cfg: GdbfConfig, seed: int, stream_id: int, first_cw: int,
                        batch: int, frames_dev=None):
        _check(lib().ldpc_gdbf_sim_launch(self._h, ebn0_db, R, C.byref(cfg._c()), seed, stream_id, first_cw, batch,
                                          _ptr(frames_dev)))

    def gdbf_sim_batch(self, ebn0_db: float, R: float, cfg: GdbfConfig, seed: int, stream_id: int, first_cw: int,
                       batch: int, want_frames: bool = True):
        fr = np.empty(batch, dtype=FRAME_DTYPE) if want_frames else None
        cnt = Counts()
        _check(lib().ldpc_gdbf_sim_batch(self._h, ebn0_db, R, C.byref(cfg._c()), seed, stream_id, first_cw, batch,
                                         _ptr(fr), C.byref(cnt)))
        return fr, cnt

    def gdbf_kernel_info(self, cfg: GdbfConfig) -> dict:
        name = C.create_string_buffer(32)
        lds = C.c_int()
        _check(lib().ldpc_gdbf_kernel_info(self._h, C.byref(cfg._c()), name, 32, C.byref(lds)))
        return {"kernel": name.value.decode(), "lds_bytes": lds.value}


# ---- non-binary GF(q) codes, Extended Min-Sum (BASELINE config 5) ----
class NbGraph:
    """GF(q) Tanner graph (NB alist of SystemC/NB-LDPC/src/alist.cpp)."""

    def __init__(self, handle):
        self._h = handle
        N, M, q, E, dv, dc = (C.c_int() for _ in range(6))
        _check(lib().ldpc_nb_graph_info(handle, C.byref(N), C.byref(M), C.byref(q), C.byref(E), C.byref(dv),
                                        C.byref(dc)))
        self.N, self.M, self.q, self.E, self.maxdv, self.maxdc = N.value, M.value, q.value, E.value, dv.value, dc.value
        self.m = self.q.bit_length() - 1

    @classmethod
    def from_alist(cls, path: str) -> "NbGraph":
        h = C.c_void_p()
        _check(lib().ldpc_nb_graph_load_alist(path.encode(), C.byref(h)))
        return cls(h)

    @classmethod
    def from_lists(cls, N: int, M: int, q: int, cols, rows) -> "NbGraph":
        """cols[i] = [(row, h), ...], rows[j] = [(col, h), ...], 0-based (as codes.NbParityCheck)."""
        def arrs(lists, one_based):
            n = (C.c_int * len(lists))(*[len(l) for l in lists])
            idx = [(C.c_int * max(len(l), 1))(*[a + 1 for a, _ in l]) for l in lists]
            val = [(C.c_int * max(len(l), 1))(*[h for _, h in l]) for l in lists]
            pi = (C.POINTER(C.c_int) * len(lists))(*[C.cast(a, C.POINTER(C.c_int)) for a in idx])
            pv = (C.POINTER(C.c_int) * len(lists))(*[C.cast(a, C.POINTER(C.c_int)) for a in val])
            return n, pi, pv, (idx, val)
        nn, ni, nv, keep1 = arrs(cols, True)
        mn, mi, mv, keep2 = arrs(rows, True)
        h = C.c_void_p()
        _check(lib().ldpc_nb_graph_create(N, M, q, nn, ni, nv, mn, mi, mv, C.byref(h)))
        return cls(h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.ldpc_nb_graph_destroy(h)
            self._h = None


class NbContext:
    """Device context of the EMS decoder (GF(16))."""

    def __init__(self, graph: NbGraph, device: int = 0, max_batch: int = 65536):
        self.graph = graph
        self.max_batch = max_batch
        h = C.c_void_p()
        _check(lib().ldpc_nb_ctx_create(device, graph._h, max_batch, C.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.ldpc_nb_ctx_destroy(h)
            self._h = None

    def set_stream(self, stream_handle: Optional[int]):
        _check(lib().ldpc_nb_ctx_set_stream(self._h, stream_handle))

    def set_option(self, name, value):
        """EMS options (ems_threads, ems_swizzle) of ldpc_nb_ctx_set_option."""
        _check(lib().ldpc_nb_ctx_set_option(self._h, option_id(name), option_value(name, value)))

    def decode(self, y, n0: float, cfg: EmsConfig, c=None, want_decisions: bool = True):
        """Decode y[batch, N*m] float32 (numpy or torch, host or device). Returns (d [batch,N] uint8, frames, NbCounts)."""
        g = self.graph
        if isinstance(y, np.ndarray):
            if y.dtype != np.float32:
                raise TypeError(f"y must be float32, got {y.dtype}")
            y = np.ascontiguousarray(y)
            batch = y.size // (g.N * g.m)
        else:
            batch = y.numel() // (g.N * g.m)
        if c is not None and isinstance(c, np.ndarray):
            c = np.ascontiguousarray(c, dtype=np.uint8)
        d = np.empty((batch, g.N), dtype=np.uint8) if want_decisions else None
        fr = np.empty(batch, dtype=FRAME_DTYPE)
        cnt = NbCounts()
        _check(lib().ldpc_ems_decode_batch(self._h, _ptr(y), batch, n0, C.byref(cfg._c()), _ptr(c), _ptr(d),
                                           _ptr(fr), C.byref(cnt)))
        return d, fr, cnt

    def sim_launch(self, ebn0_db: float, R: float, cfg: EmsConfig, seed: int, stream_id: int, first_cw: int,
                   batch: int, frames_dev=None):
        _check(lib().ldpc_ems_sim_launch(self._h, ebn0_db, R, C.byref(cfg._c()), seed, stream_id, first_cw, batch,
                                         _ptr(frames_dev)))

    def sim_batch(self, ebn0_db: float, R: float, cfg: EmsConfig, seed: int, stream_id: int, first_cw: int,
                  batch: int):
        fr = np.empty(batch, dtype=FRAME_DTYPE)
        cnt = NbCounts()
        _check(lib().ldpc_ems_sim_batch(self._h, ebn0_db, R, C.byref(cfg._c()), seed, stream_id, first_cw, batch,
                                        fr.ctypes.data, C.byref(cnt)))
        return fr, cnt

    def sim_trace(self, ebn0_db: float, R: float, cfg: EmsConfig, seed: int, stream_id: int, first_cw: int,
                  batch: int):
        g = self.graph
        y = np.empty((batch, g.N * g.m), dtype=np.float32)
        d = np.empty((batch, g.N), dtype=np.uint8)
        fr = np.empty(batch, dtype=FRAME_DTYPE)
        cnt = NbCounts()
        _check(lib().ldpc_ems_sim_trace(self._h, ebn0_db, R, C.byref(cfg._c()), seed, stream_id, first_cw, batch,
                                        y.ctypes.data, d.ctypes.data, fr.ctypes.data, C.byref(cnt)))
        return y, d, fr, cnt

    def read_counts(self, reset: bool = False) -> NbCounts:
        cnt = NbCounts()
        _check(lib().ldpc_nb_ctx_read_counts(self._h, C.byref(cnt), int(reset)))
        return cnt

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        _check(lib().ldpc_nb_ctx_last_kernel_ms(self._h, C.byref(ms)))
        return float(ms.value)

    def kernel_info(self) -> dict:
        name = C.create_string_buffer(32)
        lds = C.c_int()
        _check(lib().ldpc_ems_kernel_info(self._h, name, 32, C.byref(lds)))
        return {"kernel": name.value.decode(), "lds_bytes": lds.value}
