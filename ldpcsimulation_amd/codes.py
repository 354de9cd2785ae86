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
        with open(path, "w") as f:
            f.write(txt)
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
