"""H-matrix data formats on either side of the decode path.

* MacKay alist read/write with the reference loader's semantics
  (C_implementations/src/alist.cpp:70-93: fixed-width zero-padded lines).
* Tolerant import of unpadded / transposed alists, e.g. the reference's
  codes/802.11n/*.alist, which store row lists first and omit padding, so the
  reference loader reads them with N and M swapped and segfaults.
* Quasi-cyclic expansion of the IEEE 802.11n rate-1/2 base matrices
  (Z = 27 and Z = 81). The N = 1944 code (BASELINE config 2) exists nowhere in
  the reference; it is generated here and pinned by the SURVEY's md5 of the
  zero-padded alist (tests/test_codes.py).
"""
from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass
from typing import List, Sequence

# IEEE 802.11n R=1/2 base matrices (-1 = zero block).
BASE_R12_Z81 = [
    [57, -1, -1, -1, 50, -1, 11, -1, 50, -1, 79, -1, 1, 0, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1],
    [3, -1, 28, -1, 0, -1, -1, -1, 55, 7, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1, -1, -1],
    [30, -1, -1, -1, 24, 37, -1, -1, 56, 14, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1, -1],
    [62, 53, -1, -1, 53, -1, -1, 3, 35, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1],
    [40, -1, -1, 20, 66, -1, -1, 22, 28, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1],
    [0, -1, -1, -1, 8, -1, 42, -1, 50, -1, -1, 8, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1],
    [69, 79, 79, -1, -1, -1, 56, -1, 52, -1, -1, -1, 0, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1],
    [65, -1, -1, -1, 38, 57, -1, -1, 72, -1, 27, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1],
    [64, -1, -1, -1, 14, 52, -1, -1, 30, -1, -1, 32, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1],
    [-1, 45, -1, 70, 0, -1, -1, -1, 77, 9, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1],
    [2, 56, -1, 57, 35, -1, -1, -1, -1, -1, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0],
    [24, -1, 61, -1, 60, -1, -1, 27, 51, -1, -1, 16, 1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0],
]
BASE_R12_Z27 = [
    [0, -1, -1, -1, 0, 0, -1, -1, 0, -1, -1, 0, 1, 0, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1],
    [22, 0, -1, -1, 17, -1, 0, 0, 12, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1, -1, -1],
    [6, -1, 0, -1, 10, -1, -1, -1, 24, -1, 0, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1, -1],
    [2, -1, -1, 0, 20, -1, -1, -1, 25, 0, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1, -1],
    [23, -1, -1, -1, 3, -1, -1, -1, 0, -1, 9, 11, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1, -1],
    [24, -1, 23, 1, 17, -1, 3, -1, 10, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1, -1],
    [25, -1, -1, -1, 8, -1, -1, -1, 7, 18, -1, -1, 0, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1, -1],
    [13, 24, -1, -1, 0, -1, 8, -1, 6, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1, -1],
    [7, 20, -1, 16, 22, 10, -1, -1, 23, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1, -1],
    [11, -1, -1, -1, 19, -1, -1, -1, 13, -1, 3, 17, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0, -1],
    [25, -1, 8, -1, 23, 18, -1, 14, 9, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, 0],
    [3, -1, -1, -1, 16, -1, -1, 2, 25, 5, -1, -1, 1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0],
]
# md5 of the zero-padded alist of the N=1944 code.
MD5_80211N_1944 = "6e7b47f79e731d594830a1ba2096f419"


@dataclass
class ParityCheck:
    """H as row lists (0-based bit indices per check) and column lists."""
    N: int
    M: int
    rows: List[List[int]]
    cols: List[List[int]]

    @classmethod
    def from_rows(cls, N: int, rows: Sequence[Sequence[int]]) -> "ParityCheck":
        rows = [list(r) for r in rows]
        cols: List[List[int]] = [[] for _ in range(N)]
        for j, r in enumerate(rows):
            for i in r:
                cols[i].append(j)
        return cls(N, len(rows), rows, cols)

    @property
    def E(self) -> int:
        return sum(len(r) for r in self.rows)

    def nlist(self):   # 1-based, alist_struct form
        return [[j + 1 for j in c] for c in self.cols]

    def mlist(self):
        return [[i + 1 for i in r] for r in self.rows]

    def syndrome(self, bits) -> List[int]:
        return [sum(int(bits[i]) for i in r) & 1 for r in self.rows]


def expand_qc(base: Sequence[Sequence[int]], Z: int, shift: str = "right") -> ParityCheck:
    """Lift a base matrix: block (r, c) with shift s puts row r*Z+t on column
    c*Z + (t+s) mod Z ("right", the IEEE convention) or (t-s) mod Z ("left",
    the convention of the reference's codes/802.11n files)."""
    mb, nb = len(base), len(base[0])
    rows: List[List[int]] = [[] for _ in range(mb * Z)]
    for r in range(mb):
        for c in range(nb):
            s = base[r][c]
            if s < 0:
                continue
            for t in range(Z):
                off = (t + s) % Z if shift == "right" else (t - s) % Z
                rows[r * Z + t].append(c * Z + off)
    return ParityCheck.from_rows(nb * Z, [sorted(x) for x in rows])


def ieee80211n_r12(Z: int = 81, shift: str = "right") -> ParityCheck:
    base = {81: BASE_R12_Z81, 27: BASE_R12_Z27}.get(Z)
    if base is None:
        raise ValueError("Z must be 27 or 81")
    return expand_qc(base, Z, shift)


def alist_text(H: ParityCheck) -> str:
    """Zero-padded MacKay alist, the layout loadFile() expects."""
    dv = max(len(c) for c in H.cols)
    dc = max(len(r) for r in H.rows)
    out = [f"{H.N} {H.M}", f"{dv} {dc}",
           " ".join(str(len(c)) for c in H.cols), " ".join(str(len(r)) for r in H.rows)]
    for c in H.cols:
        out.append(" ".join([str(j + 1) for j in c] + ["0"] * (dv - len(c))))
    for r in H.rows:
        out.append(" ".join([str(i + 1) for i in r] + ["0"] * (dc - len(r))))
    return "\n".join(out) + "\n"


def write_alist(H: ParityCheck, path: str) -> str:
    txt = alist_text(H)
    with open(path, "w") as f:
        f.write(txt)
    return hashlib.md5(txt.encode()).hexdigest()


def read_alist(path: str) -> ParityCheck:
    """Reference semantics: token stream, fixed widths from the header."""
    with open(path) as f:
        tok = [int(x) for x in f.read().split()]
    N, M, dv, dc = tok[:4]
    p = 4
    wn, p = tok[p:p + N], p + N
    wm, p = tok[p:p + M], p + M
    cols = []
    for i in range(N):
        cols.append([x - 1 for x in tok[p:p + wn[i]]])
        p += dv
    rows = []
    for j in range(M):
        rows.append([x - 1 for x in tok[p:p + wm[j]]])
        p += dc
    return ParityCheck(N, M, rows, cols)


def read_alist_tolerant(path: str, transposed: bool = False) -> ParityCheck:
    """Line-based reader for unpadded alists; transposed=True for files that
    store row lists before column lists (the SystemC / codes/802.11n layout).
    Column lists are rebuilt from the row lists, so missing column lines (the
    reference's 802.11n files lack 12) do not matter."""
    with open(path) as f:
        lines = [ln.split() for ln in f if ln.strip()]
    a, b = int(lines[0][0]), int(lines[0][1])
    N, M = (b, a) if transposed else (a, b)
    w = [int(x) for x in lines[2]] if not transposed else [int(x) for x in lines[3]]
    start = 4 + (0 if transposed else N)
    rows = []
    for j in range(M):
        ent = [int(x) - 1 for x in lines[start + j] if int(x) > 0]
        rows.append(sorted(ent))
    del w
    return ParityCheck.from_rows(N, rows)


def codes_dir() -> str:
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "codes")
    os.makedirs(d, exist_ok=True)
    return d


def ensure_80211n_1944() -> str:
    """Path of the generated N=1944 R1/2 alist (codes/80211n_1944_r12.alist)."""
    path = os.path.join(codes_dir(), "80211n_1944_r12.alist")
    txt = alist_text(ieee80211n_r12(81))
    if not os.path.exists(path) or open(path).read() != txt:
        # write-then-rename: ranks of a multi-GPU run may get here together
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            f.write(txt)
        os.replace(tmp, path)
    return path


def gf2_rank(H: ParityCheck) -> int:
    """Rank over GF(2) (bitset Gaussian elimination)."""
    rows = [sum(1 << i for i in r) for r in H.rows]
    rank = 0
    for bit in range(H.N):
        piv = next((k for k in range(rank, len(rows)) if (rows[k] >> bit) & 1), None)
        if piv is None:
            continue
        rows[rank], rows[piv] = rows[piv], rows[rank]
        for k in range(len(rows)):
            if k != rank and (rows[k] >> bit) & 1:
                rows[k] ^= rows[rank]
        rank += 1
    return rank


def has_4cycle(H: ParityCheck) -> bool:
    seen = set()
    for r in H.rows:
        for a in range(len(r)):
            for b in range(a + 1, len(r)):
                key = (r[a], r[b])
                if key in seen:
                    return True
                seen.add(key)
    return False


# --------------------------------------------------------------------------
# Non-binary (GF(q)) codes: the NB alist of SystemC/NB-LDPC/src/alist.cpp:23-56
# ("N M q", "maxdv maxdc", column weights, row weights, then per column
# maxdv (row, value) pairs and per row maxdc (column, value) pairs, 1-based,
# zero-padded with "0 0"), and the GF(16) code of BASELINE config 5, which the
# reference does not hold (its NB codes are GF(2/4/8), N = 6000-9000).
# --------------------------------------------------------------------------
GF_POLY = {2: 0x3, 4: 0x7, 8: 0xB, 16: 0x13, 32: 0x25, 64: 0x43}   # primitive polynomials


def gf_mul(q: int, a: int, b: int) -> int:
    """a*b in GF(q), q = 2^m, polynomial basis over GF_POLY[q]."""
    poly, r = GF_POLY[q], 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & q:
            a ^= poly
    return r


def gf_inv(q: int, a: int) -> int:
    return next(b for b in range(1, q) if gf_mul(q, a, b) == 1)


@dataclass
class NbParityCheck:
    """H over GF(q): rows[j] = [(col, h), ...] in mlist order, cols[i] = [(row, h), ...] in nlist order."""
    N: int
    M: int
    q: int
    rows: List[List[tuple]]
    cols: List[List[tuple]]

    @property
    def E(self) -> int:
        return sum(len(r) for r in self.rows)

    def csr(self):
        """Device/oracle layout: row_ptr[M+1], row_col[E], row_h[E] (edge slot = row_ptr[j] + k),
        col_ptr[N+1], col_slot[E] (each symbol's edge slots in nlist order)."""
        import numpy as np
        row_ptr = np.zeros(self.M + 1, dtype=np.int32)
        for j, r in enumerate(self.rows):
            row_ptr[j + 1] = row_ptr[j] + len(r)
        row_col = np.array([c for r in self.rows for c, _ in r], dtype=np.int32)
        row_h = np.array([h for r in self.rows for _, h in r], dtype=np.int32)
        col_ptr = np.zeros(self.N + 1, dtype=np.int32)
        slots = []
        for i, c in enumerate(self.cols):
            col_ptr[i + 1] = col_ptr[i] + len(c)
            for j, _ in c:
                k = max(k for k, (cc, _) in enumerate(self.rows[j]) if cc == i)
                slots.append(int(row_ptr[j]) + k)
        return row_ptr, row_col, row_h, col_ptr, np.array(slots, dtype=np.int32)

    def syndrome(self, d) -> List[int]:
        out = []
        for r in self.rows:
            s = 0
            for c, h in r:
                s ^= gf_mul(self.q, h, int(d[c]))
            out.append(s)
        return out


def nb_alist_text(H: NbParityCheck) -> str:
    dv = max(len(c) for c in H.cols)
    dc = max(len(r) for r in H.rows)
    out = [f"{H.N} {H.M} {H.q}", f"{dv} {dc}",
           " ".join(str(len(c)) for c in H.cols), " ".join(str(len(r)) for r in H.rows)]
    for c in H.cols:
        out.append(" ".join(f"{j + 1} {h}" for j, h in c) + " 0 0" * (dv - len(c)))
    for r in H.rows:
        out.append(" ".join(f"{i + 1} {h}" for i, h in r) + " 0 0" * (dc - len(r)))
    return "\n".join(out) + "\n"


def read_nb_alist(path: str) -> NbParityCheck:
    """NB alist with loadFile's semantics (SystemC/NB-LDPC/src/alist.cpp:29-53): whitespace-separated
    integers, fixed maxdv / maxdc pairs per line, (0, 0) padding; validated (both views agree)."""
    with open(path) as f:
        tok = [int(x) for x in f.read().split()]
    N, M, q, dv, dc = tok[:5]
    p = 5
    wn, p = tok[p:p + N], p + N
    wm, p = tok[p:p + M], p + M
    cols, rows = [], []
    for i in range(N):
        pr = tok[p:p + 2 * dv]
        p += 2 * dv
        cols.append([(pr[2 * k] - 1, pr[2 * k + 1]) for k in range(wn[i])])
    for j in range(M):
        pr = tok[p:p + 2 * dc]
        p += 2 * dc
        rows.append([(pr[2 * k] - 1, pr[2 * k + 1]) for k in range(wm[j])])
    H = NbParityCheck(N, M, q, rows, cols)
    a = sorted((j, i, h) for i, c in enumerate(cols) for j, h in c)
    b = sorted((j, i, h) for j, r in enumerate(rows) for i, h in r)
    if a != b:
        raise ValueError(f"{path}: column and row views disagree")
    if any(not (0 < h < q) for _, _, h in a):
        raise ValueError(f"{path}: coefficient outside 1..q-1")
    return H


def peg_nb_code(N: int, M: int, dv: int, q: int, seed: int) -> NbParityCheck:
    """Progressive-edge-growth (Hu, Eleftheriou, Arnold 2005) Tanner graph with
    column weight dv and row weight capped at ceil(N*dv/M) (so a dv*N = dc*M
    code comes out regular): each new edge of a symbol goes to a check of the
    greatest graph distance from it (unreachable first), then lowest degree,
    ties broken by a seeded RNG; nonzero GF(q) coefficients are drawn
    uniformly from the same RNG."""
    import numpy as np
    rng = np.random.default_rng(seed)
    cap = -(-N * dv // M)
    chk = [[] for _ in range(M)]
    var = [[] for _ in range(N)]
    deg = np.zeros(M, dtype=np.int64)
    big = 1 << 30
    for v in range(N):
        for _ in range(dv):
            depth = np.full(M, big, dtype=np.int64)   # distance in check layers from v
            seen_v = np.zeros(N, dtype=bool)
            seen_v[v] = True
            frontier, lvl = [v], 0
            while frontier:
                nc = [c for u in frontier for c in var[u] if depth[c] == big]
                nc = list(dict.fromkeys(nc))
                if not nc:
                    break
                depth[nc] = lvl
                nv = list(dict.fromkeys(u for c in nc for u in chk[c] if not seen_v[u]))
                seen_v[nv] = True
                frontier, lvl = nv, lvl + 1
            ok = np.flatnonzero((deg < cap) & ~np.isin(np.arange(M), var[v]))
            pool = ok[depth[ok] == depth[ok].max()]
            pool = pool[deg[pool] == deg[pool].min()]
            c = int(rng.choice(pool))
            chk[c].append(v)
            var[v].append(c)
            deg[c] += 1
    h = {}
    for v in range(N):
        for c in var[v]:
            h[(c, v)] = int(rng.integers(1, q))
    rows = [[(v, h[(c, v)]) for v in sorted(chk[c])] for c in range(M)]
    cols = [[(c, h[(c, v)]) for c in sorted(var[v])] for v in range(N)]
    return NbParityCheck(N, M, q, rows, cols)


GF16_CODE = "gf16_N1000_dv2_dc4.alist"   # BASELINE config 5: N = 1000 GF(16) symbols, rate 1/2


def ensure_gf16_code() -> str:
    """Path of the config-5 code (codes/gf16_N1000_dv2_dc4.alist), generated by peg_nb_code(seed=16)."""
    path = os.path.join(codes_dir(), GF16_CODE)
    if not os.path.exists(path):
        txt = nb_alist_text(peg_nb_code(1000, 500, 2, 16, seed=16))
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            f.write(txt)
        os.replace(tmp, path)
    return path


def nb_girth_at_least_6(H: NbParityCheck) -> bool:
    """No two checks share two symbols (no 4-cycles)."""
    seen = set()
    for r in H.rows:
        cs = sorted(c for c, _ in r)
        for a in range(len(cs)):
            for b in range(a + 1, len(cs)):
                if (cs[a], cs[b]) in seen:
                    return False
                seen.add((cs[a], cs[b]))
    return True


def read_codeword_file(path: str, N: int) -> np.ndarray:
    """The codewords (0/1 bits, [rows, N] uint8) a reference run with this codeword
    file cycles through (decodeMinSum.cpp:193-211): one line per frame, the file
    rewound when getline() sets eof() -- so a last line without a trailing newline
    is never used (unless it is the only line). A symbol other than '0'/'1' (short
    lines included) keeps the previous frame's bit, as the reference leaves c[i]
    unchanged; the table holds the values of the first pass through the file."""
    with open(path, "rb") as f:
        text = f.read().decode("latin-1")
    lines = text.split("\n")
    if text.endswith("\n") or len(lines) > 1:
        lines.pop()
    if not lines:
        lines = [""]
    import numpy as np
    out = np.zeros((len(lines), N), dtype=np.uint8)
    cur = np.zeros(N, dtype=np.uint8)
    bad = 0
    for r, l in enumerate(lines):
        for i in range(N):
            ch = l[i] if i < len(l) else "\0"
            if ch == "1":
                cur[i] = 1
            elif ch == "0":
                cur[i] = 0
            else:
                bad += 1
        out[r] = cur
    if bad:
        import warnings
        warnings.warn(f"{path}: {bad} invalid symbols (kept the previous frame's bits, as the reference does)")
    return out
