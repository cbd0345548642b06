"""GPU parity: rsa_randstrobes / rsa_seed (HIP) vs the oracle (pinned to the reference)."""
import os

import numpy as np
import pytest

import oracle_lib
from helpers import GOLDEN, build_sti


def _reads(name):
    with open(os.path.join(GOLDEN, f"{name}_reads.txt"), "rb") as f:
        return [l.rstrip(b"\n") for l in f]


@pytest.fixture(scope="module", params=["small", "rep"])
def setup(request, tmp_path_factory):
    from rabbitsalign_amd import native
    d = tmp_path_factory.mktemp(request.param)
    fa, sti = build_sti(d, request.param)
    idx = native.load_index(fa, sti)
    ctx = native.GpuContext(idx)
    yield request.param, idx, ctx, oracle_lib.OracleIndex(idx)
    ctx.close()


@pytest.mark.gpu
def test_randstrobes(setup):
    name, idx, ctx, ora = setup
    reads = _reads(name)
    got = ctx.randstrobes(reads)
    for r, g in zip(reads, got):
        w = ora.randstrobes(r)
        assert len(g) == len(w)
        assert np.array_equal(g["hash"], w["hash"]) and np.array_equal(g["start"], w["start"])
        assert np.array_equal(g["end"], w["end"]) and np.array_equal(g["is_reverse"], w["is_reverse"])


def _nam_equal(g, w):
    if len(g) != len(w):
        return False
    for f in ("nam_id", "query_start", "query_end", "query_prev_hit_startpos", "ref_start", "ref_end",
              "ref_prev_hit_startpos", "n_hits", "ref_id", "is_rc"):
        if not np.array_equal(g[f], w[f]):
            return False
    return np.array_equal(g["score"].view(np.uint32), w["score"].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("rescue_level", [2, 1])
def test_seed(setup, rescue_level):
    name, idx, ctx, ora = setup
    reads = _reads(name)
    nams, nonrep, resc = ctx.seed(reads, rescue_level=rescue_level)
    bad = []
    for i, r in enumerate(reads):
        w, wn, wr = ora.seed(r, rescue_level=rescue_level)
        if not _nam_equal(nams[i], w) or np.float32(nonrep[i]).view(np.uint32) != np.float32(wn).view(np.uint32) \
                or bool(resc[i]) != wr:
            bad.append(i)
    assert not bad, f"{len(bad)} reads differ, first {bad[:5]}"


@pytest.mark.gpu
def test_seed_batch_independent(setup):
    name, idx, ctx, ora = setup
    reads = _reads(name)
    a, _, _ = ctx.seed(reads)
    b, _, _ = ctx.seed(reads[::-1])
    for x, y in zip(a, b[::-1]):
        assert _nam_equal(x, y)


_COMP = bytes.maketrans(b"ACGTUacgtu", b"TGCAATGCAA")


def _revcomp(r):
    out = bytes(c if c in b"ACGTUacgtu" else ord("N") for c in r).translate(_COMP)
    return out[::-1]


def _sub(s, pos, n):
    if pos < 0 or pos > len(s):          # a negative int cast to size_t clamps to the end
        pos = len(s)
    return s[pos:pos + n]


def _site_ref(nam, read, ref, coff, k):
    """reverse_nam_if_needed (src/aln.cpp:60-93) then extend_seed_part's Hamming
    test (aln.cpp:374-431), restated; returns (flags, n_mm, positions)."""
    L = len(read)
    rc = _revcomp(read)
    contig = ref[int(coff[nam["ref_id"]]):int(coff[nam["ref_id"] + 1])]
    is_rc, qs, qe, rs, re_ = bool(nam["is_rc"]), int(nam["query_start"]), int(nam["query_end"]), \
        int(nam["ref_start"]), int(nam["ref_end"])
    seq, seq_rc = (rc, read) if is_rc else (read, rc)
    if _sub(contig, rs, k) == _sub(seq, qs, k) and _sub(contig, re_ - k, k) == _sub(seq, qe - k, k):
        flags = 0
    elif _sub(contig, rs, k) == _sub(seq_rc, L - qe, k) and _sub(contig, re_ - k, k) == _sub(seq_rc, L - qs - k, k):
        flags, is_rc, qs, qe = 1, not is_rc, L - qe, L - qs
    else:
        return 2, 0, []
    q = rc if is_rc else read
    ps, pe = max(0, rs - qs), min(re_ + L - qe, len(contig))
    if pe - ps != L:
        return flags, 0, []
    pos = [i for i in range(L) if contig[ps + i] != q[i]]
    flags |= 4
    if np.float32(len(pos)) / np.float32(L) < 0.05:
        return flags | 8, len(pos), pos
    return flags, len(pos), []


@pytest.mark.gpu
@pytest.mark.parametrize("mm_capacity", [None, 8])
def test_sites(setup, mm_capacity):
    """k_sites against the restated host checks, for every NAM of
    every golden read; a tiny position pool must flag POOL_FULL instead of writing."""
    name, idx, ctx, ora = setup
    reads = _reads(name)
    ref = idx.ref_seq.tobytes()
    nams, _, _, sites, pool = ctx.seed(reads, sites=True, mm_capacity=mm_capacity)
    n_pos = n_checked = 0
    for r, ns, ss in zip(reads, nams, sites):
        for nam, st in zip(ns, ss):
            flags, n_mm, pos = _site_ref(nam, r, ref, idx.contig_offsets, idx.k)
            got = int(st["flags"])
            if got & 16:                       # pool full: positions withheld, everything else equal
                assert flags & 8 and mm_capacity is not None
                got = (got & ~16) | 8
            else:
                if flags & 8:
                    o = int(st["mm_offset"])
                    assert [int(x) for x in pool[o:o + int(st["n_mm"])]] == pos
                    n_pos += 1
            assert got == flags, (r, nam, got, flags)
            if flags & 4:
                assert int(st["n_mm"]) == n_mm
                n_checked += 1
    assert n_checked > 0 and (n_pos > 0 or mm_capacity is not None)
