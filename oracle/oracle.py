"""ctypes wrapper of the CPU ORACLE (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package
(ldpcsimulation_amd/), which must fail loudly without its HIP library instead
of falling back here. See oracle/ldpc_oracle.h for the reference file:line
each routine restates.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

MS, NMS, OMS = 0, 1, 2


class _Rng(C.Structure):
    _fields_ = [("tbl", C.c_int32 * 31), ("front", C.c_int), ("rear", C.c_int)]


class _Alist(C.Structure):
    _fields_ = [("N", C.c_int), ("M", C.c_int), ("maxdv", C.c_int), ("maxdc", C.c_int),
                ("deg_n", C.POINTER(C.c_int)), ("deg_m", C.POINTER(C.c_int)),
                ("nlist", C.POINTER(C.c_int)), ("mlist", C.POINTER(C.c_int))]


class _Cfg(C.Structure):
    _fields_ = [("variant", C.c_int), ("alpha", C.c_double), ("delta", C.c_double),
                ("quantize", C.c_int), ("saturate", C.c_int), ("ymax", C.c_double),
                ("qbits", C.c_int)]


class _GdbfCfg(C.Structure):
    _fields_ = [("flags", C.c_int), ("T", C.c_int), ("windowsize", C.c_int), ("nq", C.c_int),
                ("theta", C.c_double), ("lambda_", C.c_double), ("alpha", C.c_double),
                ("noise_scale", C.c_double), ("ymax", C.c_double), ("tswitch", C.c_int),
                ("qsigma", C.c_double)]


class _Stats(C.Structure):
    _fields_ = [("errors", C.c_int64), ("uncoded", C.c_int64), ("bits", C.c_int64),
                ("words", C.c_int64), ("word_errors", C.c_int64), ("iters", C.c_int64)]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: {path} (run `make -f oracle/Makefile`)")
        L = C.CDLL(path)
        L.orc_srandom.argtypes = [C.POINTER(_Rng), C.c_uint32]
        L.orc_random.argtypes = [C.POINTER(_Rng)]
        L.orc_random.restype = C.c_int32
        L.orc_ranf.argtypes = [C.POINTER(_Rng)]
        L.orc_ranf.restype = C.c_double
        L.orc_ranu.argtypes = [C.POINTER(_Rng)]
        L.orc_ranu.restype = C.c_double
        L.orc_rann.argtypes = [C.POINTER(_Rng)]
        L.orc_rann.restype = C.c_double
        L.orc_rann_fill.argtypes = [C.POINTER(_Rng), C.c_long, C.c_double, C.c_void_p]
        L.orc_alist_load.argtypes = [C.c_char_p, C.POINTER(_Alist)]
        L.orc_alist_free.argtypes = [C.POINTER(_Alist)]
        L.orc_minsum_run.argtypes = [C.POINTER(_Alist), C.c_double, C.c_double, C.c_int,
                                     C.POINTER(_Cfg), C.c_uint32, C.c_void_p, C.c_int,
                                     C.c_int64, C.c_void_p, C.c_int64, C.POINTER(_Stats)]
        L.orc_minsum_run.restype = C.c_int64
        L.orc_channel.argtypes = [C.POINTER(_Rng), C.c_int, C.c_double, C.c_void_p, C.c_void_p]
        L.orc_quantize.argtypes = [C.c_double, C.c_double, C.c_double]
        L.orc_quantize.restype = C.c_double
        L.orc_quantize_f32.argtypes = [C.c_float, C.c_float, C.c_float]
        L.orc_quantize_f32.restype = C.c_float
        for name in ("orc_decode_f64", "orc_decode_f32"):
            getattr(L, name).argtypes = [C.POINTER(_Alist), C.c_void_p, C.c_int,
                                         C.POINTER(_Cfg), C.c_void_p]
        L.orc_decode_f64_snap.argtypes = [C.POINTER(_Alist), C.c_void_p, C.c_int, C.POINTER(_Cfg),
                                          C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        for name in ("orc_decode_layered_f64", "orc_decode_layered_f32"):
            getattr(L, name).argtypes = [C.POINTER(_Alist), C.c_void_p, C.c_int,
                                         C.POINTER(_Cfg), C.c_void_p, C.c_void_p]
        L.orc_philox4x32_10.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_markstein_mismatch.argtypes = [C.c_double, C.c_long, C.c_uint64]
        L.orc_markstein_mismatch.restype = C.c_long
        L.orc_gdbf_front.argtypes = [C.c_double, C.POINTER(_GdbfCfg), C.POINTER(C.c_int)]
        L.orc_gdbf_front.restype = C.c_double
        L.orc_gdbf_front_f32.argtypes = [C.c_float, C.POINTER(_GdbfCfg), C.POINTER(C.c_int)]
        L.orc_gdbf_front_f32.restype = C.c_float
        for name in ("orc_gdbf_decode_f64", "orc_gdbf_decode_f32"):
            getattr(L, name).argtypes = [C.POINTER(_Alist), C.c_void_p, C.c_void_p, C.POINTER(_GdbfCfg),
                                         C.c_void_p, C.POINTER(C.c_int)]
            getattr(L, name).restype = C.c_int
        L.orc_gdbf_run.argtypes = [C.POINTER(_Alist), C.c_double, C.c_double, C.POINTER(_GdbfCfg), C.c_uint32,
                                   C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                   C.POINTER(_Stats), C.POINTER(C.c_int64)]
        L.orc_gdbf_run.restype = C.c_int64
        L.orc_bp_front.argtypes = [C.c_double, C.c_double, C.c_double, C.POINTER(C.c_int)]
        L.orc_bp_front.restype = C.c_double
        for name in ("orc_bp_decode_f64", "orc_bp_decode_f32"):
            getattr(L, name).argtypes = [C.POINTER(_Alist), C.c_void_p, C.c_int, C.c_double, C.c_void_p,
                                         C.c_void_p]
        L.orc_bp_run.argtypes = [C.POINTER(_Alist), C.c_double, C.c_double, C.c_int, C.c_uint32, C.c_void_p,
                                 C.c_int, C.c_int64, C.c_void_p, C.c_int64, C.POINTER(_Stats)]
        L.orc_bp_run.restype = C.c_int64
        _LIB = L
    return _LIB


class GlibcRandom:
    """glibc srandom()/random() TYPE_3 restatement + rand.h ranf/rann."""

    def __init__(self, seed: int):
        self._s = _Rng()
        lib().orc_srandom(C.byref(self._s), seed & 0xFFFFFFFF)

    def random(self) -> int:
        return lib().orc_random(C.byref(self._s))

    def ranf(self) -> float:
        return lib().orc_ranf(C.byref(self._s))

    def rann(self) -> float:
        return lib().orc_rann(C.byref(self._s))

    def ranu_fill(self, n: int) -> np.ndarray:
        """n draws of rand.h's ranu() = (1 + random()) / (2 + 0x7fffffff)."""
        f = lib().orc_ranu
        return np.array([f(C.byref(self._s)) for _ in range(n)], dtype=np.float64)

    def rann_fill(self, n: int, scale: float = 1.0) -> np.ndarray:
        out = np.empty(n, dtype=np.float64)
        lib().orc_rann_fill(C.byref(self._s), n, scale, out.ctypes.data)
        return out

    def copy(self) -> "GlibcRandom":
        g = GlibcRandom.__new__(GlibcRandom)
        g._s = _Rng.from_buffer_copy(self._s)
        return g

    def channel(self, c: np.ndarray, sigma: float) -> np.ndarray:
        c = np.ascontiguousarray(c, dtype=np.int32)
        y = np.empty(c.shape[0], dtype=np.float64)
        lib().orc_channel(C.byref(self._s), c.shape[0], sigma, c.ctypes.data, y.ctypes.data)
        return y


@dataclass
class Cfg:
    variant: int = MS
    alpha: float = 1.0
    delta: float = 0.0
    quantize: bool = False
    saturate: bool = False
    ymax: float = 0.0
    qbits: int = 0

    def c(self) -> _Cfg:
        return _Cfg(self.variant, self.alpha, self.delta, int(self.quantize),
                    int(self.saturate), self.ymax, self.qbits)


GDBF_NOISE, GDBF_ADAPT, GDBF_WEIGHT, GDBF_SMOOTH, GDBF_SATURATE, GDBF_QUANTIZE = 1, 2, 4, 8, 16, 32
GDBF_SEQUENTIAL, GDBF_MODESWITCH, GDBF_QPROB = 64, 128, 256


@dataclass
class GdbfCfg:
    """decodeGDBF.cpp parallel mode; flags = the -D switches (GDBF_*)."""
    flags: int = 0
    T: int = 100
    theta: float = -0.9
    lambda_: float = 1.0
    alpha: float = 1.0
    noise_scale: float = 0.0
    ymax: float = 0.0
    windowsize: int = 64
    nq: int = 16
    tswitch: int = 0        # modeswitching: Tswitch (:51)
    qsigma: float = 0.0     # quantizeProbabilities (gdbf_decode): the sigma of normalCDF

    def c(self) -> _GdbfCfg:
        return _GdbfCfg(self.flags, self.T, self.windowsize, self.nq, self.theta, self.lambda_, self.alpha,
                        self.noise_scale, self.ymax, self.tswitch, self.qsigma)


class Alist:
    def __init__(self, path: str):
        self._a = _Alist()
        if lib().orc_alist_load(path.encode(), C.byref(self._a)) != 0:
            raise IOError(path)
        self.N, self.M = self._a.N, self._a.M

    def __del__(self):
        try:
            lib().orc_alist_free(C.byref(self._a))
        except Exception:
            pass

    def minsum_run(self, R, snr, T, cfg: Cfg, seed, cw_lines=None, max_frames=-1, cap=0):
        st = _Stats()
        fw = np.zeros(max(cap, 1), dtype=np.int32)
        if cw_lines:
            arr = (C.c_char_p * len(cw_lines))(*[s.encode() for s in cw_lines])
            cwp, ncw = C.cast(arr, C.c_void_p), len(cw_lines)
        else:
            arr, cwp, ncw = None, None, 0
        n = lib().orc_minsum_run(C.byref(self._a), R, snr, T, C.byref(cfg.c()), seed & 0xFFFFFFFF,
                                 cwp, ncw, max_frames, fw.ctypes.data if cap else None, cap,
                                 C.byref(st))
        return n, {k: getattr(st, k) for k, _ in _Stats._fields_}, fw[:min(n, cap)]

    def decode(self, yq: np.ndarray, T: int, cfg: Cfg, workers: int = 1) -> np.ndarray:
        """Decode a [B, N] or [N] batch; dtype float64 or float32 selects precision.
        workers > 1 decodes frames on that many threads (the C call releases the GIL;
        every call allocates its own state)."""
        yq = np.ascontiguousarray(yq)
        single = yq.ndim == 1
        yq2 = yq.reshape(-1, self.N)
        d = np.empty(yq2.shape, dtype=np.int8)
        fn = lib().orc_decode_f64 if yq2.dtype == np.float64 else lib().orc_decode_f32
        assert yq2.dtype in (np.float64, np.float32)
        cc = cfg.c()

        def run(lo, hi):
            for b in range(lo, hi):
                fn(C.byref(self._a), yq2[b].ctypes.data, T, C.byref(cc), d[b].ctypes.data)
        B = yq2.shape[0]
        if workers <= 1 or B < 2:
            run(0, B)
        else:
            from concurrent.futures import ThreadPoolExecutor
            step = (B + workers - 1) // workers
            with ThreadPoolExecutor(workers) as ex:
                list(ex.map(lambda lo: run(lo, min(B, lo + step)), range(0, B, step)))
        return d[0] if single else d

    def decode_layered(self, yq: np.ndarray, T: int, cfg: Cfg, order=None) -> np.ndarray:
        """Layered (row-serial) decode of a [B, N] or [N] batch in row order `order`."""
        yq = np.ascontiguousarray(yq)
        single = yq.ndim == 1
        yq2 = yq.reshape(-1, self.N)
        d = np.empty(yq2.shape, dtype=np.int8)
        assert yq2.dtype in (np.float64, np.float32)
        fn = lib().orc_decode_layered_f64 if yq2.dtype == np.float64 else lib().orc_decode_layered_f32
        o = None if order is None else np.ascontiguousarray(order, dtype=np.int32)
        assert o is None or o.shape == (self.M,)
        cc = cfg.c()
        for b in range(yq2.shape[0]):
            fn(C.byref(self._a), yq2[b].ctypes.data, T, C.byref(cc),
               None if o is None else o.ctypes.data, d[b].ctypes.data)
        return d[0] if single else d

    def gdbf_decode(self, y: np.ndarray, pert, cfg: GdbfCfg):
        """One GDBF/NGDBF frame from RAW channel samples y [N] (front-end applied here)
        and perturbations pert [T][N] (or None). Returns (d, iterations, satisfied)."""
        f32 = y.dtype == np.float32
        front = lib().orc_gdbf_front_f32 if f32 else lib().orc_gdbf_front
        cc = cfg.c()
        r = C.c_int()
        yq = np.empty(self.N, dtype=y.dtype)
        d = np.empty(self.N, dtype=np.int8)
        for i in range(self.N):
            yq[i] = front(float(y[i]), C.byref(cc), C.byref(r))
            d[i] = r.value
        p = None if pert is None else np.ascontiguousarray(pert, dtype=y.dtype)
        sat = C.c_int()
        fn = lib().orc_gdbf_decode_f32 if f32 else lib().orc_gdbf_decode_f64
        it = fn(C.byref(self._a), yq.ctypes.data, None if p is None else p.ctypes.data, C.byref(cc),
                d.ctypes.data, C.byref(sat))
        return d, it, bool(sat.value)

    def gdbf_run(self, R, snr, cfg: GdbfCfg, seed, cw_lines=None, max_frames=-1, cap=0):
        st = _Stats()
        su = C.c_int64()
        fw = np.zeros(max(cap, 1), dtype=np.int32)
        fi = np.zeros(max(cap, 1), dtype=np.int32)
        if cw_lines:
            arr = (C.c_char_p * len(cw_lines))(*[s.encode() for s in cw_lines])
            cwp, ncw = C.cast(arr, C.c_void_p), len(cw_lines)
        else:
            arr, cwp, ncw = None, None, 0
        n = lib().orc_gdbf_run(C.byref(self._a), R, snr, C.byref(cfg.c()), seed & 0xFFFFFFFF, cwp, ncw,
                               max_frames, fw.ctypes.data if cap else None, fi.ctypes.data if cap else None,
                               cap, C.byref(st), C.byref(su))
        k = min(n, cap)
        return n, {**{k2: getattr(st, k2) for k2, _ in _Stats._fields_}, "smoothing_used": su.value}, \
            fw[:k], fi[:k]

    def bp_front(self, y: np.ndarray, N0: float, maxllr: float = 20.0) -> np.ndarray:
        r = C.c_int()
        return np.array([lib().orc_bp_front(float(v), N0, maxllr, C.byref(r)) for v in np.ravel(y)]).reshape(
            np.shape(y))

    def bp_decode(self, yq: np.ndarray, T: int, maxllr: float = 20.0, want_c2v: bool = False):
        """BP decode of a [B, N] or [N] batch of front-end outputs (float64 or float32)."""
        yq = np.ascontiguousarray(yq)
        single = yq.ndim == 1
        yq2 = yq.reshape(-1, self.N)
        d = np.empty(yq2.shape, dtype=np.int8)
        fn = lib().orc_bp_decode_f64 if yq2.dtype == np.float64 else lib().orc_bp_decode_f32
        c2v = np.zeros((yq2.shape[0], self.M * max(self._a.maxdc, 1)), dtype=yq2.dtype) if want_c2v else None
        for b in range(yq2.shape[0]):
            fn(C.byref(self._a), yq2[b].ctypes.data, T, maxllr, d[b].ctypes.data,
               c2v[b].ctypes.data if want_c2v else None)
        d = d[0] if single else d
        return (d, c2v) if want_c2v else d

    def bp_run(self, R, snr, T, seed, cw_lines=None, max_frames=-1, cap=0):
        st = _Stats()
        fw = np.zeros(max(cap, 1), dtype=np.int32)
        if cw_lines:
            arr = (C.c_char_p * len(cw_lines))(*[s.encode() for s in cw_lines])
            cwp, ncw = C.cast(arr, C.c_void_p), len(cw_lines)
        else:
            arr, cwp, ncw = None, None, 0
        n = lib().orc_bp_run(C.byref(self._a), R, snr, T, seed & 0xFFFFFFFF, cwp, ncw, max_frames,
                             fw.ctypes.data if cap else None, cap, C.byref(st))
        return n, {k: getattr(st, k) for k, _ in _Stats._fields_}, fw[:min(n, cap)]

    def decode_snap(self, yq: np.ndarray, T: int, cfg: Cfg, snap_it: int):
        yq = np.ascontiguousarray(yq, dtype=np.float64)
        E = int(sum(self._a.deg_m[j] for j in range(self.M)))
        c2v = np.empty(E, dtype=np.float64)
        app = np.empty(self.N, dtype=np.float64)
        d = np.empty(self.N, dtype=np.int8)
        lib().orc_decode_f64_snap(C.byref(self._a), yq.ctypes.data, T, C.byref(cfg.c()),
                                  d.ctypes.data, snap_it, c2v.ctypes.data, app.ctypes.data)
        return d, c2v, app


def markstein_mismatch(alpha: float, n: int, seed: int = 1) -> int:
    """Count of sampled x where the fast fp64 NMS division differs from IEEE x/alpha."""
    return int(lib().orc_markstein_mismatch(alpha, n, seed))


def quantize(x: float, ymax: float, qbits: int) -> float:
    return lib().orc_quantize(x, ymax, 2.0 ** qbits)


def quantize_f32(x: float, ymax: float, qbits: int) -> float:
    return lib().orc_quantize_f32(x, ymax, 2.0 ** qbits)


def philox4x32_10(ctr, key) -> list:
    c = np.ascontiguousarray(np.array(ctr, dtype=np.uint32))
    k = np.ascontiguousarray(np.array(key, dtype=np.uint32))
    o = np.empty(4, dtype=np.uint32)
    lib().orc_philox4x32_10(c.ctypes.data, k.ctypes.data, o.ctypes.data)
    return [int(x) for x in o]


class NbCode:
    """GF(q) code (ldpcsimulation_amd.codes.NbParityCheck) bound to the EMS oracle (ems_oracle.c)."""

    def __init__(self, H):
        self.H = H
        self.N, self.M, self.q = H.N, H.M, H.q
        self.m = q_bits = int(H.q).bit_length() - 1
        assert 1 << q_bits == H.q
        self._csr = [np.ascontiguousarray(a, dtype=np.int32) for a in H.csr()]
        L = lib()
        if not getattr(L, "_ems_set", False):
            L.orc_gf_mul.argtypes = [C.c_int, C.c_int, C.c_int]
            L.orc_gf_mul.restype = C.c_int
            L.orc_nb_front.argtypes = [C.c_void_p, C.c_int, C.c_float, C.c_void_p]
            L.orc_ems_decode.argtypes = [C.c_int, C.c_int, C.c_int] + [C.c_void_p] * 6 + [
                C.c_int, C.c_int, C.c_float, C.c_int, C.c_void_p, C.POINTER(C.c_int)]
            L.orc_ems_decode.restype = C.c_int
            L._ems_set = True

    def front(self, y: np.ndarray, n0: float) -> np.ndarray:
        y = np.ascontiguousarray(y, dtype=np.float32)
        lam = np.empty_like(y)
        lib().orc_nb_front(y.ctypes.data, y.size, n0, lam.ctypes.data)
        return lam

    def decode(self, y: np.ndarray, n0: float, T: int, nm: int = 16, offset: float = 0.0, early_stop: bool = True):
        """EMS decode of y[B, N*m] (fp32 channel samples). Returns (d [B,N] uint8, iters [B], syndrome_fail [B])."""
        y2 = np.ascontiguousarray(y, dtype=np.float32).reshape(-1, self.N * self.m)
        B = y2.shape[0]
        d = np.empty((B, self.N), dtype=np.uint8)
        its = np.empty(B, dtype=np.int32)
        sf = np.empty(B, dtype=np.int32)
        rp, rc, rh, cp, cs = self._csr
        for b in range(B):
            lam = self.front(y2[b], n0)
            f = C.c_int()
            its[b] = lib().orc_ems_decode(self.N, self.M, self.q, rp.ctypes.data, rc.ctypes.data, rh.ctypes.data,
                                          cp.ctypes.data, cs.ctypes.data, lam.ctypes.data, T, nm, offset,
                                          int(early_stop), d[b].ctypes.data, C.byref(f))
            sf[b] = f.value
        return d, its, sf
