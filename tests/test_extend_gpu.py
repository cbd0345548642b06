"""GPU parity: rsa_extend (HIP) vs the oracle's Aligner::align restatement."""
import numpy as np
import pytest

import oracle_lib
from jobgen import make_jobs, random_reference


def _compare(ctx, ref, offs, seed, n, qlens=(150,)):
    rng = np.random.default_rng(seed)
    queries, jobs, pairs = make_jobs(rng, ref, offs, n, qlens)
    alns, pool = ctx.extend(queries, jobs)
    bad = []
    for i, (q, r) in enumerate(pairs):
        o = oracle_lib.align(q, r)
        a = alns[i]
        cig = [int(x) for x in pool[int(a["cigar_offset"]):int(a["cigar_offset"]) + int(a["cigar_len"])]]
        got = dict(sw_score=int(a["sw_score"]), edit_distance=int(a["edit_distance"]), ref_start=int(a["ref_start"]),
                   ref_end=int(a["ref_end"]), query_start=int(a["query_start"]), query_end=int(a["query_end"]),
                   cigar=cig)
        if got["sw_score"] < -1000:   # sentinel: only score/ed/ref_start are defined
            for k in ("ref_end", "query_start", "query_end"):
                got[k] = o[k]
        if got != o:
            bad.append((i, q, r, o, got))
    return bad


@pytest.fixture(scope="module")
def ctx():
    from rabbitsalign_amd import native
    rng = np.random.default_rng(7)
    ref, offs = random_reference(rng)
    c = native.GpuContext(native.empty_index(ref, offs))
    yield c, ref, offs
    c.close()


@pytest.mark.gpu
def test_extend_150(ctx):
    c, ref, offs = ctx
    bad = _compare(c, ref, offs, 1, 4000)
    assert not bad, f"{len(bad)} mismatches, first: {bad[0]}"


@pytest.mark.gpu
def test_extend_mixed_lengths(ctx):
    c, ref, offs = ctx
    bad = _compare(c, ref, offs, 2, 3000, qlens=(100, 150, 250, 300, 500, 64, 65, 128, 129))
    assert not bad, f"{len(bad)} mismatches, first: {bad[0]}"


@pytest.mark.gpu
def test_extend_order_independent(ctx):
    c, ref, offs = ctx
    rng = np.random.default_rng(3)
    queries, jobs, pairs = make_jobs(rng, ref, offs, 500)
    a1, p1 = c.extend(queries, jobs)
    perm = rng.permutation(len(jobs))
    a2, p2 = c.extend(queries, jobs[perm])
    for k, i in enumerate(perm):
        x, y = a1[i], a2[k]
        assert x["sw_score"] == y["sw_score"] and x["ref_start"] == y["ref_start"]
        assert list(p1[x["cigar_offset"]:x["cigar_offset"] + x["cigar_len"]]) == \
            list(p2[y["cigar_offset"]:y["cigar_offset"] + y["cigar_len"]])


@pytest.mark.gpu
def test_extend_band_paths_exercised(ctx):
    """Jobs whose bands the 16-lane kernel cannot hold go through the 64-lane
    queue kernel, and bands wider than 64 cells through the panel kernel;
    all three must agree with the oracle."""
    c, ref, offs = ctx
    c.reset_stats()
    bad = _compare(c, ref, offs, 5, 3000, qlens=(150, 250, 400))
    assert not bad, f"{len(bad)} mismatches, first: {bad[0]}"
    st = c.stats()
    assert st["band_deferred"] > 0, st
    assert st["band_overflow"] > 0, st
    k = st["kernels"]
    assert k["ext_band_wide"]["launches"] > 0 and k["ext_band_panel"]["launches"] > 0


@pytest.mark.gpu
def test_extend_band16_capacity_classes(ctx, monkeypatch):
    """k_ext_band16 comes in three direction capacities (4096 / 8192 / 16384; a call
    with queries over 200 bp takes 8192).  250-bp jobs with indels (bands of 3-15 cells)
    give the oracle's results in each, and a larger capacity defers fewer jobs to the
    one-wave kernel."""
    c, ref, offs = ctx
    deferred = {}
    for cap in ("4096", "8192", "16384"):
        monkeypatch.setenv("RSA_BAND16_DIRCAP", cap)
        c.reset_stats()
        bad = _compare(c, ref, offs, 11, 2500, qlens=(250, 240, 300))
        assert not bad, f"RSA_BAND16_DIRCAP={cap}: {len(bad)} mismatches, first: {bad[0]}"
        deferred[cap] = c.stats()["band_deferred"]
    assert deferred["4096"] > deferred["8192"] >= deferred["16384"], deferred


def _has_shared_substring(q: bytes, w: bytes, k: int) -> bool:
    """has_shared_substring (src/aln.cpp:1000-1013) restated: some (2k/3)-mer of the query
    starting at a multiple of k/3, with i + sub < len(query), occurs in the window."""
    sub, step = 2 * k // 3, k // 3
    i = 0
    while i + sub < len(q):
        if w.find(q[i:i + sub]) >= 0:
            return True
        i += step
    return False


@pytest.mark.gpu
def test_extend_shared_check(ctx):
    """RSA_JOB_SHARED_CHECK jobs: k_shared_check's RSA_ALN_NO_SHARED equals the host
    function on every job (related and unrelated query/window pairs, N bytes, k 3-36,
    queries up to 1024 bp, windows up to 4096), and unflagged jobs never carry it."""
    from jobgen import JOB_DTYPE, ACGT, mutate
    c, ref, offs = ctx
    rng = np.random.default_rng(21)
    queries = bytearray()
    jobs = np.zeros(1500, dtype=JOB_DTYPE)
    want = []
    for i in range(len(jobs)):
        ci = int(rng.integers(0, len(offs) - 1))
        clen = int(offs[ci + 1] - offs[ci])
        L = int(rng.choice([20, 100, 150, 250, 1024]))
        W = int(rng.choice([30, 300, 525, 2000, 2500, 4096]))
        rs = int(rng.integers(0, clen - W - 1))
        win = ref[int(offs[ci]) + rs:int(offs[ci]) + rs + W]
        kind = int(rng.integers(0, 4))
        if kind == 0 and W > L:                      # the mate inside the window, with errors
            a = int(rng.integers(0, W - L))
            q = mutate(rng, win[a:a + L], sub=float(rng.choice([0.01, 0.1, 0.3])), ind=0.01)[:L]
        elif kind == 1:                              # unrelated
            q = ACGT[rng.integers(0, 4, L)]
        else:                                        # unrelated with one planted piece of the window
            q = ACGT[rng.integers(0, 4, L)].copy()
            n = int(rng.integers(5, 25))
            a, b = int(rng.integers(0, max(1, W - n))), int(rng.integers(0, max(1, L - n)))
            q[b:b + n] = win[a:a + n][:len(q[b:b + n])]
        if rng.random() < 0.1:
            q = q.copy(); q[rng.integers(0, len(q), 3)] = ord("N")
        k = int(rng.choice([3, 10, 15, 20, 24, 32, 36]))
        flag = i % 5 != 0
        qb = bytes(q)
        qlen = len(qb) | ((0x80000000 | (k << 24)) if flag else 0)
        jobs[i] = (len(queries), qlen, ci, rs, W)
        queries += qb
        want.append(flag and not _has_shared_substring(qb, bytes(win), k))
    alns, _ = c.extend(bytes(queries), jobs)
    got = [(int(a["flags"]) & 1) == 1 for a in alns]
    bad = [i for i in range(len(jobs)) if got[i] != want[i]]
    assert not bad, f"{len(bad)} jobs differ, first {bad[:5]}"
    assert 50 < sum(want) < len(jobs) - 300, sum(want)


def _wide_band_jobs(rng, ref, offs, n):
    """Queries that bridge a long deletion (or carry a long insertion) of the
    window: |ref span - query span| of 65-1200 bp, so banded_sw needs bands far
    wider than one wave (2 x 1200 + 1 cells at most): k_ext_band_panel's panels."""
    from jobgen import JOB_DTYPE, ACGT, mutate
    queries = bytearray()
    jobs = np.zeros(n, dtype=JOB_DTYPE)
    pairs = []
    for i in range(n):
        c = int(rng.integers(0, len(offs) - 1))
        clen = int(offs[c + 1] - offs[c])
        gap = int(rng.choice([65, 100, 180, 300, 500, 800, 1200]))
        flank = int(rng.integers(160, 420))
        deletion = rng.random() < 0.7
        span = 2 * flank + (gap if deletion else 0) + 60
        rs = int(rng.integers(0, clen - span - 1))
        win = ref[int(offs[c]) + rs:int(offs[c]) + rs + span]
        left, right = win[30:30 + flank], win[30 + flank + (gap if deletion else 0):30 + 2 * flank + (gap if deletion else 0)]
        mid = np.zeros(0, np.uint8) if deletion else ACGT[rng.integers(0, 4, min(gap, 1000 - 2 * flank))]
        q = mutate(rng, np.concatenate([left, mid, right]), sub=float(rng.choice([0.0, 0.01, 0.03])), ind=0.005)[:1000]
        if rng.random() < 0.3 and span > 2000:
            win = win[:2000]
        qb = bytes(q)
        jobs[i] = (len(queries), len(qb), c, rs, len(win))
        queries += qb
        pairs.append((qb, bytes(win)))
    return bytes(queries), jobs, pairs


@pytest.mark.gpu
def test_extend_wide_bands_panel_kernel(ctx):
    """Bands 65-2401 cells wide: every job through k_ext_band_panel, == the oracle."""
    c, ref, offs = ctx
    rng = np.random.default_rng(23)
    queries, jobs, pairs = _wide_band_jobs(rng, ref, offs, 120)
    c.reset_stats()
    alns, pool = c.extend(queries, jobs)
    bad = []
    for i, (q, r) in enumerate(pairs):
        o = oracle_lib.align(q, r)
        a = alns[i]
        cig = [int(x) for x in pool[int(a["cigar_offset"]):int(a["cigar_offset"]) + int(a["cigar_len"])]]
        got = dict(sw_score=int(a["sw_score"]), edit_distance=int(a["edit_distance"]), ref_start=int(a["ref_start"]),
                   ref_end=int(a["ref_end"]), query_start=int(a["query_start"]), query_end=int(a["query_end"]),
                   cigar=cig)
        if got["sw_score"] < -1000:
            for k in ("ref_end", "query_start", "query_end"):
                got[k] = o[k]
        if got != o:
            bad.append((i, len(q), len(r), o, got))
    assert not bad, f"{len(bad)} mismatches, first: {bad[0]}"
    st = c.stats()
    assert st["band_overflow"] >= 60, st
    assert st["kernels"]["ext_band_panel"]["launches"] > 0


@pytest.mark.gpu
def test_extend_hand_derived_cases():
    """The GPU path on the hand-derived Aligner::align cases (tests/wrapper_cases.py)."""
    from rabbitsalign_amd import native
    from wrapper_cases import cases
    from jobgen import JOB_DTYPE
    cs = cases()
    ref = b"".join(r for _, _, r, _ in cs)
    offs = np.zeros(len(cs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(r) for _, _, r, _ in cs])
    ctx = native.GpuContext(native.empty_index(np.frombuffer(ref, np.uint8).copy(), offs))
    try:
        queries = b"".join(q for _, q, _, _ in cs)
        jobs = np.zeros(len(cs), dtype=JOB_DTYPE)
        qo = 0
        for i, (_, q, r, _) in enumerate(cs):
            jobs[i] = (qo, len(q), i, 0, len(r))
            qo += len(q)
        alns, pool = ctx.extend(queries, jobs)
        for i, (name, q, r, want) in enumerate(cs):
            a = alns[i]
            got = dict(sw_score=int(a["sw_score"]), edit_distance=int(a["edit_distance"]), ref_start=int(a["ref_start"]),
                       ref_end=int(a["ref_end"]), query_start=int(a["query_start"]), query_end=int(a["query_end"]),
                       cigar=[int(x) for x in pool[int(a["cigar_offset"]):int(a["cigar_offset"]) + int(a["cigar_len"])]])
            for k, v in want.items():
                assert got[k] == v, (name, k, got[k], v)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_extend_async_equals_sync(ctx):
    """rsa_extend_async / rsa_ready / rsa_wait (the split of the boundary the reference
    uses to overlap chunks, gasal2_ssw.cpp:114-249): several calls pending at once,
    waited out of order, give rsa_extend's results; past RSA_MAX_PENDING the call
    returns RSA_ERR_BUSY instead of blocking."""
    c, ref, offs = ctx
    batches = []
    for seed in range(4):
        rng = np.random.default_rng(100 + seed)
        queries, jobs, _ = make_jobs(rng, ref, offs, 700 + 300 * seed, (100, 150, 250, 400))
        batches.append((queries, jobs))
    want = [c.extend(q, j) for q, j in batches]
    pend = [c.extend_async(q, j) for q, j in batches]
    for k in (2, 0, 3, 1):
        alns, pool = pend[k].wait()
        wa, wp = want[k]
        assert (alns == wa).all()
        for x, y in zip(alns, wa):
            assert list(pool[x["cigar_offset"]:x["cigar_offset"] + x["cigar_len"]]) == \
                list(wp[y["cigar_offset"]:y["cigar_offset"] + y["cigar_len"]])
    # the pending limit
    q, j = batches[0]
    many = []
    try:
        for _ in range(12):
            many.append(c.extend_async(q, j[:50]))
        with pytest.raises(RuntimeError, match=r"\(-5\)"):
            c.extend_async(q, j[:50])
        assert c.extend(q, j[:50])[0].shape == (50,)      # synchronous calls still get a lane
    finally:
        for p in many:
            p.wait()
    empty = c.extend_async(q, j[:0])
    assert empty.ready()
    assert empty.wait()[0].shape == (0,)


@pytest.mark.gpu
def test_extend_grouped_and_wave_scans(ctx):
    """The grouped scan (k_ext_scan_g, queries <= 256 bp and windows <= 1 KB) and the
    one-job-per-wave scan (k_ext_scan, the rest) on one mixed batch: Aligner::align's results."""
    c, ref, offs = ctx
    bad = _compare(c, ref, offs, 11, 3000, qlens=(150, 100, 250, 64, 129, 300))
    assert not bad, f"{len(bad)} mismatches, first: {bad[0]}"


def _block_replacement_jobs(rng, ref, offs, n, L=250):
    """Queries copied from their window with one block replaced (d bases deleted, e
    random bases inserted at the same place, 1-25 each) and light substitutions:
    the best path often has an insertion next to a deletion, which is where the
    byte and word layouts of SSW may differ (k_ext_scan_v's certificate fails and
    the job takes the two-layout re-run)."""
    from jobgen import JOB_DTYPE, ACGT
    queries = bytearray()
    jobs = np.zeros(n, dtype=JOB_DTYPE)
    pairs = []
    for i in range(n):
        c = int(rng.integers(0, len(offs) - 1))
        clen = int(offs[c + 1] - offs[c])
        rl = L + int(rng.integers(20, 150))
        rs = int(rng.integers(0, clen - rl - 1))
        win = ref[int(offs[c]) + rs:int(offs[c]) + rs + rl].copy()
        a = int(rng.integers(0, 30))
        cut = int(rng.integers(L // 4, 3 * L // 4))
        d, e = int(rng.integers(1, 26)), int(rng.integers(1, 26))
        q = np.concatenate([win[a:a + cut], ACGT[rng.integers(0, 4, e)], win[a + cut + d:]])[:L].copy()
        subs = rng.random(len(q)) < 0.005
        q[subs] = ACGT[rng.integers(0, 4, int(subs.sum()))]
        if len(q) < L:
            q = np.concatenate([q, ACGT[rng.integers(0, 4, L - len(q))]])
        qb = bytes(q)
        jobs[i] = (len(queries), len(qb), c, rs, rl)
        queries += qb
        pairs.append((qb, bytes(win)))
    return bytes(queries), jobs, pairs


@pytest.mark.gpu
@pytest.mark.parametrize("redo_dev", [None, "0", "1"], ids=["in_stream", "host", "cap_exceeded"])
def test_extend_scan_certificate_and_redo(ctx, redo_dev, monkeypatch):
    """k_ext_scan_v takes the word layout on the word score alone and the band path
    certifies it; jobs whose path puts an insertion next to a deletion are re-run
    through the two-layout scan.  Both outcomes occur here and every result is
    Aligner::align's -- with the re-run in the call's stream (default), from the host
    (RSA_REDO_DEV=0), and from the host after an in-stream pass whose cap the list
    exceeds (RSA_REDO_DEV=1)."""
    if redo_dev is not None:
        monkeypatch.setenv("RSA_REDO_DEV", redo_dev)
    c, ref, offs = ctx
    rng = np.random.default_rng(31)
    queries, jobs, pairs = _block_replacement_jobs(rng, ref, offs, 1500)
    c.reset_stats()
    alns, pool = c.extend(queries, jobs)
    bad = []
    for i, (q, r) in enumerate(pairs):
        o = oracle_lib.align(q, r)
        a = alns[i]
        got = dict(sw_score=int(a["sw_score"]), edit_distance=int(a["edit_distance"]), ref_start=int(a["ref_start"]),
                   ref_end=int(a["ref_end"]), query_start=int(a["query_start"]), query_end=int(a["query_end"]),
                   cigar=[int(x) for x in pool[int(a["cigar_offset"]):int(a["cigar_offset"]) + int(a["cigar_len"])]])
        if got["sw_score"] < -1000:
            for k in ("ref_end", "query_start", "query_end"):
                got[k] = o[k]
        if got != o:
            bad.append((i, o, got))
    assert not bad, f"{len(bad)} mismatches, first: {bad[0]}"
    st = c.stats()
    assert st["scan_certified"] > 1000 and st["scan_redo"] > 1, st


@pytest.mark.gpu
def test_extend_scan_v_equals_scan_g(ctx, monkeypatch):
    """The virtual-lane scan (default) and the two-layout grouped scan (RSA_SCAN_V=0,
    read when a context opens) give identical results on one mixed batch."""
    from rabbitsalign_amd import native
    c, ref, offs = ctx
    rng = np.random.default_rng(41)
    queries, jobs, _ = make_jobs(rng, ref, offs, 3000, (150, 100, 250, 64, 33, 129, 200))
    q2, j2, _ = _block_replacement_jobs(rng, ref, offs, 300)
    j2 = j2.copy()
    j2["query_offset"] += len(queries)
    queries, jobs = queries + q2, np.concatenate([jobs, j2])
    a1, p1 = c.extend(queries, jobs)
    monkeypatch.setenv("RSA_SCAN_V", "0")
    c2 = native.GpuContext(native.empty_index(ref, offs))
    try:
        a2, p2 = c2.extend(queries, jobs)
    finally:
        c2.close()
    assert (a1[["sw_score", "edit_distance", "ref_start", "ref_end", "query_start", "query_end", "cigar_len"]] ==
            a2[["sw_score", "edit_distance", "ref_start", "ref_end", "query_start", "query_end", "cigar_len"]]).all()
    for x, y in zip(a1, a2):
        assert list(p1[x["cigar_offset"]:x["cigar_offset"] + x["cigar_len"]]) == \
            list(p2[y["cigar_offset"]:y["cigar_offset"] + y["cigar_len"]])
