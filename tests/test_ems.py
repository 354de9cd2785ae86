"""Non-binary GF(16) Extended Min-Sum (BASELINE config 5).

PARITY UNPINNED against the reference: its NB-LDPC model
(SystemC/NB-LDPC/inc/nodes.h) is a q^dc-LUT BP that does not compile, holds
no EMS and no GF(16) code. The oracle (oracle/ems_oracle.c) restates the EMS
of Declercq & Fossorier (2007) as DESIGN.md §11 defines it, and is anchored
where the reference does pin something:
  - the NB alist format of SystemC/NB-LDPC/src/alist.cpp:23-56 (round trip,
    validation);
  - q = 2: GF(2) EMS is binary min-sum, so the EMS oracle must give exactly
    the decisions of the min-sum oracle, which reproduces the reference's
    decodeMinSum runs frame by frame (tests/test_oracle.py).
GPU tier: the HIP kernel (nb.hip) against the oracle, bit for bit: same
decided symbols, iteration counts, syndrome flags and error counts.
"""
import hashlib
import math
import os

import numpy as np
import pytest

from conftest import code_path
from oracle import oracle as O

GF16 = "gf16_N1000_dv2_dc4.alist"
GF16_MD5 = "2e1fc43f5e523c3b86fbe09a64aefb40"


def _codes():
    from ldpcsimulation_amd import codes
    return codes


def _frames(nb, nframes, ebn0, seed, R=0.5, c=None):
    """BPSK per bit (bit i of the symbol value, 0 -> +1), y = x(1 + sigma n), float32."""
    rng = np.random.default_rng(seed)
    n0 = 10 ** (-ebn0 / 10) / R
    sigma = math.sqrt(n0 / 2)
    x = np.ones((nframes, nb), dtype=np.float64)
    if c is not None:
        bits = (c[:, :, None] >> np.arange(4)) & 1
        x = 1.0 - 2.0 * bits.reshape(nframes, nb)
    y = (x * (1 + sigma * rng.standard_normal((nframes, nb)))).astype(np.float32)
    return y, n0


# ------------------------------------------------------------------ CPU tier
def test_gf16_field_axioms():
    codes = _codes()
    q = 16
    mul = np.array([[codes.gf_mul(q, a, b) for b in range(q)] for a in range(q)])
    L = O.lib()
    O.NbCode(codes.read_nb_alist(code_path(GF16)))     # sets the oracle signatures
    assert all(L.orc_gf_mul(q, a, b) == mul[a, b] for a in range(q) for b in range(q))
    assert (mul == mul.T).all() and (mul[1] == np.arange(q)).all() and (mul[0] == 0).all()
    for a in range(1, q):
        assert sorted(mul[a, 1:]) == list(range(1, q))          # nonzero row is a permutation
    for a in range(q):
        for b in range(q):
            for c in range(q):
                assert mul[mul[a, b], c] == mul[a, mul[b, c]]
                assert mul[a, b ^ c] == mul[a, b] ^ mul[a, c]
    # x^4 + x + 1 is primitive: alpha = 2 has order 15
    p, order = 1, 0
    while True:
        p, order = mul[p, 2], order + 1
        if p == 1:
            break
    assert order == 15


def test_gf16_code_fixture_pinned_and_regular():
    codes = _codes()
    path = code_path(GF16)
    assert hashlib.md5(open(path, "rb").read()).hexdigest() == GF16_MD5
    H = codes.read_nb_alist(path)
    assert (H.N, H.M, H.q, H.E) == (1000, 500, 16, 2000)
    assert {len(r) for r in H.rows} == {4} and {len(c) for c in H.cols} == {2}
    assert codes.nb_girth_at_least_6(H)
    assert codes.nb_alist_text(H) == open(path).read()
    # the generator reproduces the fixture
    assert codes.nb_alist_text(codes.peg_nb_code(1000, 500, 2, 16, seed=16)) == open(path).read()


def test_nb_alist_loader_rejects_inconsistent_views(tmp_path):
    codes = _codes()
    H = codes.read_nb_alist(code_path(GF16))
    txt = codes.nb_alist_text(H).splitlines()
    head = 4
    row0 = txt[head + H.N].split()
    row0[1] = str(int(row0[1]) % 15 + 1)                 # change one coefficient in the row view
    txt[head + H.N] = " ".join(row0)
    p = tmp_path / "bad.alist"
    p.write_text("\n".join(txt) + "\n")
    with pytest.raises(ValueError):
        codes.read_nb_alist(str(p))
    from ldpcsimulation_amd import native
    with pytest.raises(native.LdpcError) as e:
        native.NbGraph.from_alist(str(p))
    assert e.value.code == -6
    g = native.NbGraph.from_alist(code_path(GF16))
    assert (g.N, g.M, g.q, g.E, g.maxdv, g.maxdc) == (1000, 500, 16, 2000, 2, 4)


def test_nb_graph_rejects_degree_one_check():
    """A GF(q) check of degree 1 (or 0) is refused at graph creation (LDPC_ERR_GRAPH),
    before a context's slot-swizzle search could pick two slots of it."""
    from ldpcsimulation_amd import native
    cols = [[(0, 3)], [(0, 5), (1, 7)], [(1, 2)]]
    rows = [[(1, 5), (0, 3)], [(1, 7), (2, 2)]]
    g = native.NbGraph.from_lists(3, 2, 16, cols, rows)
    assert (g.N, g.M, g.maxdc) == (3, 2, 2)
    bad_cols = [[(0, 3)], [(1, 7)], [(1, 2)]]
    bad_rows = [[(0, 3)], [(1, 7), (2, 2)]]           # check 0 has one edge
    with pytest.raises(native.LdpcError) as e:
        native.NbGraph.from_lists(3, 2, 16, bad_cols, bad_rows)
    assert e.value.code == -6 and "degree" in str(e.value)


def test_ems_q2_equals_binary_min_sum_oracle():
    """GF(2) EMS (nm = 2, no offset, no early stop) is binary min-sum: identical decisions to the
    reference-pinned min-sum oracle on the same bit LLRs (PEGReg504x1008, glibc noise)."""
    codes = _codes()
    P = codes.read_alist(code_path("PEGReg504x1008.alist"))
    H = codes.NbParityCheck(P.N, P.M, 2, [[(i, 1) for i in r] for r in P.rows], [[(j, 1) for j in c] for c in P.cols])
    A, B = O.NbCode(H), O.Alist(code_path("PEGReg504x1008.alist"))
    n0 = 10 ** (-2.0 / 10) / 0.5
    g = O.GlibcRandom(5)
    y = np.stack([g.channel(np.ones(P.N, dtype=np.int32), math.sqrt(n0 / 2)) for _ in range(30)]).astype(np.float32)
    lam = np.stack([A.front(r, n0) for r in y]).astype(np.float64)
    for T in (1, 5, 10):
        d, its, _ = A.decode(y, n0, T, nm=2, early_stop=False)
        want = (B.decode(lam, T, O.Cfg()) == -1).astype(np.uint8)
        assert np.array_equal(d, want), f"T={T}"
        assert (its == T).all()


def test_ems_oracle_properties():
    codes = _codes()
    H = codes.read_nb_alist(code_path(GF16))
    A = O.NbCode(H)
    y, n0 = _frames(H.N * 4, 6, 1.8, seed=3)
    lam = np.stack([A.front(r, n0) for r in y])
    hard = ((lam.reshape(6, H.N, 4) < 0) << np.arange(4)).sum(axis=2)
    d0, its0, _ = A.decode(y, n0, 0)
    assert np.array_equal(d0, hard) and (its0 == 0).all()       # T = 0: the channel's hard decisions
    d, its, sf = A.decode(y, n0, 30, nm=16, early_stop=True)
    for b in range(6):
        synd = H.syndrome(d[b])
        assert (sf[b] == 0) == (not any(synd))
        if its[b] < 30:
            assert sf[b] == 0                                    # early stop only on a codeword
    # a high-SNR frame decodes within a couple of iterations
    yc, n0c = _frames(H.N * 4, 1, 8.0, seed=4)
    dc, itc, sfc = A.decode(yc, n0c, 10)
    assert (dc == 0).all() and itc[0] <= 2 and sfc[0] == 0


# ------------------------------------------------------------------ GPU tier
def _native():
    from ldpcsimulation_amd import native
    return native


@pytest.fixture(scope="module")
def nbctx():
    native = _native()
    g = native.NbGraph.from_alist(code_path(GF16))
    return native.NbContext(g, 0, 4096)


EMS_CFGS = [dict(nm=16, offset=0.0, early_stop=True), dict(nm=16, offset=0.0, early_stop=False),
            dict(nm=8, offset=0.5, early_stop=True), dict(nm=4, offset=1.0, early_stop=False),
            dict(nm=12, offset=0.25, early_stop=True)]


@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(len(EMS_CFGS)))
def test_ems_decisions_bit_exact_vs_oracle(nbctx, ci):
    native = _native()
    c = EMS_CFGS[ci]
    H = _codes().read_nb_alist(code_path(GF16))
    A = O.NbCode(H)
    y, n0 = _frames(H.N * 4, 8, 1.6, seed=100 + ci)
    for T in (0, 1, 3, 15):
        d, fr, cnt = nbctx.decode(y, n0, native.EmsConfig(T=T, **c))
        want, its, sf = A.decode(y, n0, T, **c)
        assert int((d != want).sum()) == 0, f"T={T}: {(d != want).sum()} symbols differ"
        assert np.array_equal(fr["iters"], its) and np.array_equal(fr["syndrome_fail"], sf)
        be = np.array([sum(bin(int(s)).count("1") for s in row) for row in want])
        assert np.array_equal(fr["bit_err"], be)
        assert cnt.frames == 8 and cnt.iters == int(its.sum()) and cnt.bit_err == int(be.sum())
        assert cnt.symbol_err == int((want != 0).sum()) and cnt.frame_err == int((want != 0).any(axis=1).sum())


@pytest.mark.gpu
def test_ems_given_codeword_accounting(nbctx):
    native = _native()
    H = _codes().read_nb_alist(code_path(GF16))
    A = O.NbCode(H)
    rng = np.random.default_rng(9)
    c = rng.integers(0, 16, size=(4, H.N), dtype=np.uint8)      # accounting only: any symbols
    y, n0 = _frames(H.N * 4, 4, 2.0, seed=11, c=c)
    d, fr, cnt = nbctx.decode(y, n0, native.EmsConfig(T=5), c=c)
    want, _, _ = A.decode(y, n0, 5)
    assert np.array_equal(d, want)
    be = np.array([sum(bin(int(a) ^ int(b)).count("1") for a, b in zip(dr, cr)) for dr, cr in zip(want, c)])
    assert np.array_equal(fr["bit_err"], be)
    lam = np.stack([A.front(r, n0) for r in y]).reshape(4, H.N, 4)
    unc = ((lam < 0) != ((c[:, :, None] >> np.arange(4)) & 1)).sum(axis=(1, 2))
    assert np.array_equal(fr["uncoded_bit_err"], unc)


@pytest.mark.gpu
def test_ems_sim_on_device_noise_matches_oracle(nbctx):
    native = _native()
    H = _codes().read_nb_alist(code_path(GF16))
    A = O.NbCode(H)
    cfg = native.EmsConfig(T=20, nm=16)
    y, d, fr, cnt = nbctx.sim_trace(1.5, 0.5, cfg, seed=7, stream_id=1, first_cw=300, batch=16)
    n0 = 10 ** (-1.5 / 10) / 0.5
    want, its, sf = A.decode(y, n0, 20)
    assert np.array_equal(d, want) and np.array_equal(fr["iters"], its)
    assert abs(float(y.mean()) - 1.0) < 0.02 and abs(float(y.std()) - math.sqrt(n0 / 2)) < 0.02


@pytest.mark.gpu
def test_ems_sim_independent_of_batch_split(nbctx):
    native = _native()
    cfg = native.EmsConfig(T=10)
    full, _ = nbctx.sim_batch(1.5, 0.5, cfg, seed=5, stream_id=0, first_cw=0, batch=300)
    a, _ = nbctx.sim_batch(1.5, 0.5, cfg, seed=5, stream_id=0, first_cw=0, batch=100)
    b, _ = nbctx.sim_batch(1.5, 0.5, cfg, seed=5, stream_id=0, first_cw=100, batch=200)
    assert np.array_equal(full, np.concatenate([a, b]))


@pytest.mark.gpu
def test_ems_ticketed_codewords_independent_of_batch_split():
    """More codewords than blocks (256): past the first grid they come from the ticket
    counter in completion order (nb.hip k_ems); the per-frame records must not depend on it."""
    native = _native()
    from ldpcsimulation_amd import codes
    g = native.NbGraph.from_alist(codes.ensure_gf16_code())
    ctx = native.NbContext(g, 0, 2048)
    cfg = native.EmsConfig(T=12)
    full, cf = ctx.sim_batch(2.0, 0.5, cfg, seed=8, stream_id=2, first_cw=0, batch=2048)
    a, ca = ctx.sim_batch(2.0, 0.5, cfg, seed=8, stream_id=2, first_cw=0, batch=700)
    b, cb = ctx.sim_batch(2.0, 0.5, cfg, seed=8, stream_id=2, first_cw=700, batch=1348)
    assert np.array_equal(full, np.concatenate([a, b]))
    assert cf.frames == 2048 and cf.iters == ca.iters + cb.iters
    assert len(set(full["iters"].tolist())) > 3


@pytest.mark.gpu
def test_ems_waterfall(nbctx):
    """FER falls with Eb/N0, early-stopped frames are codewords (parity unpinned: no reference FER)."""
    native = _native()
    cfg = native.EmsConfig(T=30, nm=16)
    fer = []
    for ebn0 in (1.0, 1.5, 2.0):
        fr, cnt = nbctx.sim_batch(ebn0, 0.5, cfg, seed=13, stream_id=2, first_cw=0, batch=4096)
        assert ((fr["iters"] < 30) <= (fr["syndrome_fail"] == 0)).all()
        fer.append(cnt.frame_err / cnt.frames)
    assert fer[0] > fer[1] > fer[2] and fer[0] > 0.5 and fer[2] < 0.05, fer


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2000, 1000, 2), (400, 200, 4), (300, 200, 3), (600, 260, 2)],
                         ids=["global_state_N2000", "dc8_kernel", "irregular_dc", "padded_stride_more_symbols"])
def test_ems_other_kernels_bit_exact(shape):
    """The global-memory message slot (codes beyond LDS, more symbols than threads), the
    DC=8 build (row degree 5..8), irregular row degrees, and a code whose position-major
    slot count (maxdc*M = 1 300) pads to a 2 048-slot chunk stride with more symbols (600)
    than the DC=8 build's 512 threads, against the oracle."""
    native = _native()
    codes = _codes()
    N, M, dv = shape
    H = codes.peg_nb_code(N, M, dv, 16, seed=N + M)
    g = native.NbGraph.from_lists(H.N, H.M, H.q, H.cols, H.rows)
    ctx = native.NbContext(g, 0, 64)
    info = ctx.kernel_info()
    assert info["kernel"] == ("ems_global" if N == 2000 else "ems_lds")
    A = O.NbCode(H)
    y, n0 = _frames(H.N * 4, 6, 2.2, seed=N)
    for c in (dict(nm=16, offset=0.0, early_stop=True), dict(nm=6, offset=0.5, early_stop=False)):
        for T in (1, 8):
            d, fr, _ = ctx.decode(y, n0, native.EmsConfig(T=T, **c))
            want, its, sf = A.decode(y, n0, T, **c)
            assert int((d != want).sum()) == 0, (c, T)
            assert np.array_equal(fr["iters"], its) and np.array_equal(fr["syndrome_fail"], sf)


def _random_nb_code(col_deg, row_deg, q, seed):
    """A random GF(q) code with the given column and row degrees (sum equal; no edge
    twice), fast at any size (PEG is not)."""
    codes = _codes()
    rng = np.random.default_rng(seed)
    col_deg, row_deg = list(col_deg), list(row_deg)
    assert sum(col_deg) == sum(row_deg) and min(row_deg) >= 2
    N, M = len(col_deg), len(row_deg)
    rsock = np.repeat(np.arange(M), row_deg)
    for _ in range(1000):
        perm = rng.permutation(len(rsock))
        cols, at = [], 0
        for d in col_deg:
            cols.append(sorted(int(r) for r in rsock[perm[at:at + d]]))
            at += d
        if all(len(set(c)) == len(c) for c in cols):
            break
    else:
        raise RuntimeError("no simple graph found")
    cols = [[(c, int(rng.integers(1, q))) for c in r] for r in cols]
    rows = [[] for _ in range(M)]
    for v, r in enumerate(cols):
        for c, h in r:
            rows[c].append((v, h))
    return codes.NbParityCheck(N, M, q, rows, cols)


@pytest.mark.gpu
def test_ems_chunk_stride_65536_accepted_bit_exact():
    """maxdc * M just above 32 768 (one row of degree 8 among 4 097: 32 776
    slots) rounds the chunk stride up to 65 536 slots; such a code is decoded -- the
    16-bit entries are the slot indices, below 65 536 -- on the global-state kernel
    (4 MB of messages per codeword), equal to the oracle."""
    native = _native()
    H = _random_nb_code([3] * 4096 + [2] * 4, [8] + [3] * 4096, 16, seed=65)
    assert max(len(r) for r in H.rows) * H.M == 32776
    g = native.NbGraph.from_lists(H.N, H.M, H.q, H.cols, H.rows)
    ctx = native.NbContext(g, 0, 8)
    assert ctx.kernel_info()["kernel"] == "ems_global"
    A = O.NbCode(H)
    y, n0 = _frames(H.N * 4, 3, 2.2, seed=65)
    for T in (1, 4):
        c = dict(nm=16, offset=0.0, early_stop=True)
        d, fr, _ = ctx.decode(y, n0, native.EmsConfig(T=T, **c))
        want, its, sf = A.decode(y, n0, T, **c)
        assert int((d != want).sum()) == 0, T
        assert np.array_equal(fr["iters"], its) and np.array_equal(fr["syndrome_fail"], sf)


def test_nb_graph_above_the_16_bit_slot_bound_is_refused_at_context_creation_only():
    """maxdc * M = 65 540 exceeds the 16-bit slot indices: the graph itself is valid
    (host-side checks pass; the context refuses it with LDPC_ERR_UNSUPPORTED on a GPU box)."""
    native = _native()
    H = _random_nb_code([2] * 32770, [4] * 16385, 16, seed=66)
    g = native.NbGraph.from_lists(H.N, H.M, H.q, H.cols, H.rows)
    assert (g.N, g.M) == (32770, 16385) and max(len(r) for r in H.rows) * H.M > 65535


@pytest.mark.parametrize("name,q", [("q4.sp.9000.6000.4500.1.alist", 4), ("q8.sp.6000.4000.3000.1.alist", 8)])
def test_reference_nb_codes_load_and_decode(name, q):
    """The reference's own GF(4) / GF(8) codes (SystemC/NB-LDPC/codes/GF4, GF8; fixtures
    compressed under tests/golden/codes) load through both NB alist readers with
    consistent column and row views, and the EMS oracle (any q = 2^m) decodes
    them at 3 dB. The GPU kernels are built for GF(16) only."""
    codes = _codes()
    from ldpcsimulation_amd import native
    H = codes.read_nb_alist(code_path(name))
    g = native.NbGraph.from_alist(code_path(name))
    assert (g.N, g.M, g.q, g.E) == (H.N, H.M, H.q, H.E) and H.q == q
    A = O.NbCode(H)
    R = 1 - H.M / H.N
    rng = np.random.default_rng(q)
    n0 = 10 ** (-3.0 / 10) / R
    y = (1 + math.sqrt(n0 / 2) * rng.standard_normal((2, H.N * A.m))).astype(np.float32)
    d, its, sf = A.decode(y, n0, 20)
    assert (d == 0).all() and (sf == 0).all() and (its < 20).all()
