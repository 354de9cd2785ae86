"""H-matrix generation and I/O: the 802.11n QC expansion pinned against the
reference's own file and the SURVEY's md5, alist round trips."""
import hashlib
import os

import pytest

from conftest import REFERENCE, code_path
from ldpcsimulation_amd import codes


def test_80211n_1944_md5_and_structure(tmp_path):
    H = codes.ieee80211n_r12(81)
    assert (H.N, H.M, H.E) == (1944, 972, 6966)
    md5 = codes.write_alist(H, str(tmp_path / "h.alist"))
    assert md5 == codes.MD5_80211N_1944
    dv = sorted({len(c) for c in H.cols})
    dc = sorted({len(r) for r in H.rows})
    assert dv == [2, 3, 4, 11] and dc == [7, 8]
    assert not codes.has_4cycle(H)


def test_80211n_1944_full_rank():
    assert codes.gf2_rank(codes.ieee80211n_r12(81)) == 972


def test_committed_fixture_is_the_generated_code():
    with open(code_path("80211n_1944_r12.alist"), "rb") as f:
        assert hashlib.md5(f.read()).hexdigest() == codes.MD5_80211N_1944


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference tree not present")
@pytest.mark.parametrize("fname", ["802.11n.alist", "ldpc_802.11n.alist"])
def test_z27_left_shift_matches_reference_file(fname):
    """The reference's 802.11n files hold the Z=27 R1/2 code with left-shift circulants."""
    R = codes.read_alist_tolerant(os.path.join(REFERENCE, "codes", "802.11n", fname), transposed=True)
    H = codes.ieee80211n_r12(27, "left")
    assert (R.N, R.M) == (648, 324)
    assert R.rows == H.rows


def test_alist_roundtrip(tmp_path):
    H = codes.read_alist(code_path("PEGReg504x1008.alist"))
    p = tmp_path / "peg.alist"
    codes.write_alist(H, str(p))
    H2 = codes.read_alist(str(p))
    assert H2.rows == H.rows and H2.cols == H.cols
    # the committed PEG file is zero padded exactly like the writer's output
    assert open(p).read().split() == open(code_path("PEGReg504x1008.alist")).read().split()


@pytest.mark.parametrize("name,data,n", [("PEGReg504x1008.alist", "PEGReg504x1008_data20.enc", 20),
                                         ("4000.2000.4.244.alist", "4000.2000.4.244_data10.enc", 10)])
def test_codeword_fixtures_satisfy_parity(name, data, n):
    H = codes.read_alist(code_path(name))
    lines = [l.strip() for l in open(code_path(data)) if l.strip()]
    assert len(lines) == n
    for l in lines:
        assert len(l) == H.N and sum(H.syndrome(l)) == 0


def test_read_codeword_file_follows_the_reference_eof_rule(tmp_path):
    """decodeMinSum.cpp:193-211: an unterminated last line is never used; invalid
    symbols keep the previous frame's bit; a terminated file cycles all its lines."""
    from ldpcsimulation_amd.codes import read_codeword_file
    import warnings
    p = tmp_path / "a.enc"
    p.write_text("0101\n1100\n0011")
    assert read_codeword_file(str(p), 4).tolist() == [[0, 1, 0, 1], [1, 1, 0, 0]]
    p.write_text("0101\n1100\n0011\n")
    assert read_codeword_file(str(p), 4).tolist() == [[0, 1, 0, 1], [1, 1, 0, 0], [0, 0, 1, 1]]
    p.write_text("0111")
    assert read_codeword_file(str(p), 4).tolist() == [[0, 1, 1, 1]]
    p.write_text("1111\n0x0\n")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        got = read_codeword_file(str(p), 4).tolist()
    assert got == [[1, 1, 1, 1], [0, 1, 0, 1]] and w
