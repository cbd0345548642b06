"""CPU: the oracle's per-NAM site checks (ora_nam_site) on hand-derived cases of
reverse_nam_if_needed (src/aln.cpp:60-93) and extend_seed_part's ungapped test
(src/aln.cpp:374-395).  aln.cpp cannot be compiled here (it includes a CUDA
header, src/include/gasal.h:9), so these fixtures are derived by hand from its
text; k_sites is then checked against this oracle on the GPU (test_seed_gpu)."""
import numpy as np

import oracle_lib

K = 20
ACGT = np.frombuffer(b"ACGT", np.uint8)


def _nam(qs, qe, rs, re_, is_rc=0, ref_id=0):
    n = np.zeros(1, dtype=oracle_lib.NAM_DTYPE)[0]
    n["query_start"], n["query_end"], n["ref_start"], n["ref_end"], n["is_rc"], n["ref_id"] = qs, qe, rs, re_, is_rc, ref_id
    return n


def _contig(seed=1, n=2000):
    return ACGT[np.random.default_rng(seed).integers(0, 4, n)].tobytes()


def test_revcomp_table():
    # revcomp.hpp:11-28: upper-case complement, U -> A, everything else N, reversed
    assert oracle_lib.reverse_complement(b"ACGTU") == b"AACGT"
    assert oracle_lib.reverse_complement(b"acgtn*") == b"NNACGT"


def test_forward_consistent_exact():
    c = _contig()
    read = c[500:650]
    f, n_mm, pos = oracle_lib.nam_site(_nam(10, 140, 510, 640), read, c, K)
    # both end k-mers match as is (orientation 0); projection [500, 650) is read-length;
    # Hamming 0 < 5 % -> accepted with no positions
    assert (f, n_mm, pos) == (0 | 4 | 8, 0, [])


def test_false_reverse_is_flipped():
    c = _contig()
    read = c[500:650]
    # a NAM that claims reverse orientation but whose k-mers match the forward read:
    # query coordinates become L - qe, L - qs (aln.cpp:80-89)
    L = len(read)
    f, n_mm, _ = oracle_lib.nam_site(_nam(L - 140, L - 10, 510, 640, is_rc=1), read, c, K)
    assert f == 1 | 4 | 8 and n_mm == 0


def test_reverse_read():
    c = _contig()
    read = oracle_lib.reverse_complement(c[700:850])
    f, n_mm, _ = oracle_lib.nam_site(_nam(5, 120, 705, 820, is_rc=1), read, c, K)
    assert f == 0 | 4 | 8 and n_mm == 0


def test_inconsistent():
    c = _contig()
    read = bytearray(c[500:650])
    read[12] = ord("A") if read[12] != ord("A") else ord("C")       # breaks the start k-mer
    f, n_mm, pos = oracle_lib.nam_site(_nam(10, 140, 510, 640), bytes(read), c, K)
    assert (f, n_mm, pos) == (2, 0, [])


def test_mismatches_below_and_at_five_percent():
    c = _contig()
    base = bytearray(c[500:650])
    def mutate(idx):
        r = bytearray(base)
        for i in idx:
            r[i] = ord("A") if r[i] != ord("A") else ord("G")
        return bytes(r)
    # 7 / 150 = 0.0467 < 0.05: accepted, positions in query coordinates
    mm = [30, 31, 60, 70, 80, 90, 100]
    f, n_mm, pos = oracle_lib.nam_site(_nam(10, 140, 510, 640), mutate(mm), c, K)
    assert (f, n_mm, pos) == (4 | 8, 7, mm)
    # 8 / 150 = 0.0533: Hamming computed, not accepted (no positions)
    f, n_mm, pos = oracle_lib.nam_site(_nam(10, 140, 510, 640), mutate(mm + [110]), c, K)
    assert (f, n_mm, pos) == (4, 8, [])


def test_projection_clamped_at_contig_ends():
    c = _contig(n=600)
    # read starting 10 bases before the contig: projected start clamps to 0 -> window of L - 10
    read = b"ACGTACGTAC" + c[0:140]
    f, _, _ = oracle_lib.nam_site(_nam(15, 130, 5, 120), read, c, K)
    assert f == 0            # consistent, but the window is not read-length: no Hamming test
    # read running 10 bases past the contig end: projected end clamps to |contig|
    read = c[460:600] + b"ACGTACGTAC"
    f, _, _ = oracle_lib.nam_site(_nam(0, 120, 460, 580), read, c, K)
    assert f == 0
