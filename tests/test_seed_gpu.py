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
def test_seed_bucket_lines_equal_table(setup, monkeypatch):
    """k_lookup through the bucket lines (bounds and up to 7 entries in one 128-byte
    line; the default) and through the .sti bucket table + entries (RSA_BUCKET_LINES=0)
    give the same NAMs.  The "rep" index holds buckets past the line's capacity, so
    both of the line path's branches run there."""
    from rabbitsalign_amd import native
    name, idx, ctx, ora = setup
    reads = _reads(name)
    sizes = np.diff(idx.bucket_starts.astype(np.int64))
    assert (sizes <= 7).any()
    if name == "rep":
        assert (sizes > 7).any()
    bits = int(idx.bits)
    monkeypatch.setenv("RSA_BUCKET_LINES", "0")
    plain = native.GpuContext(idx)
    try:
        assert ctx.resident_bytes() - plain.resident_bytes() == 128 << bits
        for level in (2, 1):
            a, an, ar = ctx.seed(reads, rescue_level=level)
            b, bn, br = plain.seed(reads, rescue_level=level)
            assert all(_nam_equal(x, y) for x, y in zip(a, b))
            assert np.array_equal(np.asarray(an, np.float32).view(np.uint32), np.asarray(bn, np.float32).view(np.uint32))
            assert list(ar) == list(br)
    finally:
        plain.close()


@pytest.mark.gpu
def test_seed_by_score_order(setup):
    """order=RSA_NAMS_BY_SCORE: each list of 2..16 NAMs comes as libstdc++'s
    std::sort(by_score) leaves it (insertion sort: stable, descending score), longer
    lists as found; the site checks stay at each NAM's nam_id and carry its query span
    and strand as found (what the host reverses from)."""
    from rabbitsalign_amd import native
    name, idx, ctx, ora = setup
    reads = _reads(name)
    found, _, _, s_found, p_found = ctx.seed(reads, sites=True)
    srt, _, _, s_srt, p_srt = ctx.seed(reads, sites=True, order=native.NAMS_BY_SCORE)
    n_sorted = 0
    for f, s, sf, ss in zip(found, srt, s_found, s_srt):
        if 2 <= len(f) <= 16:
            perm = sorted(range(len(f)), key=lambda i: (-float(f["score"][i]), i))
            want = f[perm]
            n_sorted += int(perm != list(range(len(f))))
        else:
            want = f
        assert _nam_equal(s, want)
        assert list(f["nam_id"]) == list(range(len(f)))
        for fld in ("flags", "n_mm"):
            assert np.array_equal(sf[fld], ss[fld])
        assert np.array_equal(ss["orig_query_start"], f["query_start"])
        assert np.array_equal(ss["orig_query_end"], f["query_end"])
        assert np.array_equal(ss["orig_is_rc"], f["is_rc"].astype(np.uint8))
        for a, b in zip(sf, ss):                 # the same mismatch positions wherever they were pooled
            if a["flags"] & 8:
                assert list(p_found[a["mm_offset"]:a["mm_offset"] + a["n_mm"]]) == \
                    list(p_srt[b["mm_offset"]:b["mm_offset"] + b["n_mm"]])
    if name == "small":                          # (the repetitive reads' short lists happen to come in order)
        assert n_sorted > 0


@pytest.mark.gpu
@pytest.mark.parametrize("qw", ["0", "2"])
def test_seed_query_write_modes(setup, monkeypatch, qw):
    """k_seed_query (randstrobes + lookup fused) writes a read's query randstrobes and
    QrsInfo only when it predicts the global-map or rescue pass will read them; the
    passes make them themselves (query_lane) for a read it did not.  RSA_SEED_QW=0
    (never written: every rescued / global-map read goes through query_lane) and 2
    (always written) must both give the oracle's NAMs.  Reads of 520-840 bases (joined
    golden reads) take the lane path (k_randstrobes + k_lookup) beside the fused one."""
    name, idx, ctx, ora = setup
    reads = _reads(name)
    joined = [b"".join(reads[i:i + 6])[:520 + 40 * (i % 9)] for i in range(0, min(len(reads), 60), 6)]
    reads = reads + [r for r in joined if len(r) > 512]
    monkeypatch.setenv("RSA_SEED_QW", qw)
    for rescue_level in (2, 1):
        ctx.reset_stats()
        nams, nonrep, resc = ctx.seed(reads, rescue_level=rescue_level)
        st = ctx.stats()
        if rescue_level == 2:
            # 0: every rescued read's randstrobes were made by query_lane; 2: none were needed
            assert (st["query_fixed_reads"] > 0) == (qw == "0"), st["query_fixed_reads"]
            assert (st["query_written"] > 0) == (qw == "2") or qw == "0", st["query_written"]
        bad = []
        for i, r in enumerate(reads):
            w, wn, wr = ora.seed(r, rescue_level=rescue_level)
            if not _nam_equal(nams[i], w) or np.float32(nonrep[i]).view(np.uint32) != np.float32(wn).view(np.uint32) \
                    or bool(resc[i]) != wr:
                bad.append(i)
        assert not bad, f"RSA_SEED_QW={qw} rescue_level={rescue_level}: {len(bad)} reads differ, first {bad[:5]}"
        if rescue_level == 2:
            assert any(resc), "no rescued read: the fallback did not run"


@pytest.mark.gpu
def test_seed_batch_independent(setup):
    name, idx, ctx, ora = setup
    reads = _reads(name)
    a, _, _ = ctx.seed(reads)
    b, _, _ = ctx.seed(reads[::-1])
    for x, y in zip(a, b[::-1]):
        assert _nam_equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", ["8", "16"])
@pytest.mark.parametrize("mm_capacity", [None, 8])
def test_sites(setup, mm_capacity, lanes, monkeypatch):
    """k_sites against the oracle's ora_nam_site (reverse_nam_if_needed
    aln.cpp:60-93 + extend_seed_part's Hamming test aln.cpp:374-395), for every NAM of
    every golden read; a tiny position pool must flag POOL_FULL instead of writing.  Both
    kernel shapes: 8 and 16 lanes a NAM (RSA_SITES_G; the call's default follows the mean
    read length)."""
    monkeypatch.setenv("RSA_SITES_G", lanes)
    name, idx, ctx, ora = setup
    reads = _reads(name)
    ref = idx.ref_seq.tobytes()
    coff = idx.contig_offsets
    nams, _, _, sites, pool = ctx.seed(reads, sites=True, mm_capacity=mm_capacity)
    n_pos = n_checked = 0
    for r, ns, ss in zip(reads, nams, sites):
        for nam, st in zip(ns, ss):
            c = int(nam["ref_id"])
            flags, n_mm, pos = oracle_lib.nam_site(nam, r, ref[int(coff[c]):int(coff[c + 1])], idx.k)
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


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", ["8", "16"])
def test_sites_hamming_align(setup, lanes, monkeypatch):
    """k_sites with hamming_align on (rsa_nam_batch.hamming_align, RSA_SITE_ALIGNED): every
    accepted site's score, segment, mismatch count and CIGAR equal the oracle's literal
    restatement of aligner.cpp:219-302 on the same oriented read and projected window;
    everything else equals the positions mode.  Both kernel shapes (RSA_SITES_G 8 / 16)."""
    monkeypatch.setenv("RSA_SITES_G", lanes)
    from rabbitsalign_amd.native import GpuContext
    name, idx, ctx, ora = setup
    reads = _reads(name)
    ref = idx.ref_seq.tobytes()
    coff = idx.contig_offsets
    # a pool large enough for every result (the pool-full flag is covered by the positions test)
    nams, _, _, sites, pool = ctx.seed(reads, sites=True, hamming=(2, 8, 10), mm_capacity=1 << 24)
    n_aln = 0
    for r, ns, ss in zip(reads, nams, sites):
        rc = oracle_lib.reverse_complement(r)
        for nam, st in zip(ns, ss):
            c = int(nam["ref_id"])
            contig = ref[int(coff[c]):int(coff[c + 1])]
            flags, n_mm, pos = oracle_lib.nam_site(nam, r, contig, idx.k)
            got = int(st["flags"])
            assert not got & 16, "pool full at 2^24 words"
            assert (got & ~32) == flags, (r, nam, got, flags)
            if not flags & 8:
                assert not got & 32
                continue
            assert got & 32
            # the oriented read and its projected window (aln.cpp:374-395)
            rev = (flags & 3) == 1
            is_rc = bool(nam["is_rc"]) != rev
            qs = len(r) - int(nam["query_end"]) if rev else int(nam["query_start"])
            q = rc if is_rc else r
            ps = max(0, int(nam["ref_start"]) - qs)
            want = oracle_lib.hamming_align(q, contig[ps:ps + len(r)])
            assert GpuContext.decode_hamming(pool, int(st["mm_offset"])) == want, (r, nam)
            n_aln += 1
    assert n_aln > 0


def _adversarial_reads(rng):
    acgt = np.frombuffer(b"ACGT", np.uint8)

    def rnd(n):
        return acgt[rng.integers(0, 4, n)].tobytes()

    reads = [b"", b"A", rnd(10), rnd(149), rnd(150), rnd(250), rnd(511), rnd(512), rnd(513), rnd(1000),
             b"A" * 150, b"AC" * 75, b"ACG" * 50, b"ACGT" * 40, b"AAAAC" * 30, b"N" * 150,
             rnd(60) + b"N" + rnd(89), rnd(40) + b"NNNNN" + rnd(40) + b"A" * 30 + rnd(35),
             rnd(150).lower(), rnd(70).replace(b"T", b"U") + rnd(80), rnd(100) + b"A" * 600,
             (rnd(7) * 30)[:200], rnd(30) + b"CACACACACACACACACACACACACA" + rnd(100)]
    for _ in range(200):                  # random tandem repeats (ties in the syncmer window)
        unit = rnd(int(rng.integers(1, 7)))
        body = (unit * 200)[:int(rng.integers(20, 300))]
        reads.append(rnd(int(rng.integers(0, 40))) + body + rnd(int(rng.integers(0, 40))))
    for _ in range(300):
        r = bytearray(rnd(int(rng.choice([100, 150, 250, 400, 600]))))
        for i in rng.integers(0, len(r), int(rng.integers(0, 4))):
            r[i] = ord("N")
        reads.append(bytes(r))
    return reads


@pytest.mark.gpu
@pytest.mark.parametrize("kslu", [(20, 16, 1, 7), (22, 18, 2, 12), (18, 14, -2, 3), (24, 18, 2, 12),
                                  (30, 12, 1, 4), (32, 30, 1, 8), (20, 20, 1, 4)])
def test_randstrobes_adversarial(kslu):
    """k_rs_wave (one wave a read) and the one-lane kernel it hands long reads and
    wide windows to, vs the oracle: empty, short, max-length (512/513) and long reads;
    tandem repeats whose equal s-mer hashes make the syncmer window's tie rules
    matter (the wave kernel's serial walk); N runs, lowercase, U; window widths
    k-s+1 = 1, 2, 5, 7 (wave kernel) and 19 (one-lane kernel)."""
    from rabbitsalign_amd import native
    k, s, l, u = kslu
    rng = np.random.default_rng(k * 100 + s)
    ref, offs = np.frombuffer(b"ACGT" * 64, np.uint8).copy(), np.array([0, 256], np.uint64)
    idx = native.empty_index(ref, offs)
    idx.k, idx.s, idx.l, idx.u = k, s, l, u
    ctx = native.GpuContext(idx)
    try:
        ora = oracle_lib.OracleIndex(idx)
        reads = _adversarial_reads(rng)
        got = ctx.randstrobes(reads)
        bad = []
        for i, (r, g) in enumerate(zip(reads, got)):
            w = ora.randstrobes(r)
            if len(g) != len(w) or not all(np.array_equal(g[f], w[f]) for f in ("hash", "start", "end", "is_reverse")):
                bad.append(i)
        assert not bad, f"{len(bad)} reads differ, first {[reads[i][:40] for i in bad[:3]]}"
        assert sum(len(g) for g in got) > 1000
    finally:
        ctx.close()
