"""GPU: hand-derived jobs through rsa_extend (HIP) and the host's window and
store code (src/pc.cpp:177-242, 291-368).  The reads are exact copies of the
contig, so every expectation follows from the windows (tests/host_cases.py
arithmetic) and Aligner::align's end bonus: an exact 150-mer scores 2 x 150 +
10 + 10 = 320 with both ends reached (src/aligner.cpp:138-207), CIGAR 150=."""
import random

import numpy as np
import pytest

from host_cases import EQ, op
from test_host_cases_cpu import nam_args, parse_aln, run_cases

CONTIG_LEN = 20000


def _contig():
    rnd = random.Random(29)
    return bytes(rnd.choice(b"ACGT") for _ in range(CONTIG_LEN))


def _rc(s):
    return s[::-1].translate(bytes.maketrans(b"ACGT", b"TGCA"))


def _cases(C):
    # (name, kind, nam, read seq, mu, sigma, expected alignment, expected window)
    return [
        # read = contig[3000:3150]; NAM q[10,140) r[3010,3140): projected 3000, window
        # (2950, 250); the read sits 50 into it -> stored ref_start 2950 + 50 = 3000
        ("ext_fwd", "ext", (10, 140, 3010, 3140, 0), C[3000:3150], None, None,
         (3000, 150, 0, 0, 320, 0, 0, 1, [op(150, EQ)]), (2950, 250)),
        # read = rc(contig[5000:5150]): an rc NAM on the read's rc coordinates q[20,150)
        # r[5020,5150); the job aligns read.rc = contig[5000:5150] in (4950, 250)
        ("ext_rc", "ext", (20, 150, 5020, 5150, 1), _rc(C[5000:5150]), None, None,
         (5000, 150, 0, 0, 320, 1, 0, 1, [op(150, EQ)]), (4950, 250)),
        # mate rescue, forward anchor q[0,150) r[7000,7150), mu 300 sigma 100: window
        # a = 7150 - 75 = 7075, b = 7150 + 800 = 7950; the mate read is rc(contig[7300:7450])
        # and the job aligns its rc, found 225 into the window -> ref_start 7300, is_rc 1
        ("rescue_fwd", "rescue", (0, 150, 7000, 7150, 0), _rc(C[7300:7450]), "300", "100",
         (7300, 150, 0, 0, 320, 1, 0, 0, [op(150, EQ)]), (7075, 875)),
        # rc anchor q[0,150) r[9000,9150), mu 301.25 sigma 29.5: a = 9000 - 448.75 = 8551.25 ->
        # 8551, b = 9075; the mate read is contig[8700:8850] (aligned as is), 149 into the
        # window -> ref_start 8700, is_rc 0
        ("rescue_rc", "rescue", (0, 150, 9000, 9150, 1), C[8700:8850], "301.25", "29.5",
         (8700, 150, 0, 0, 320, 0, 0, 0, [op(150, EQ)]), (8551, 524)),
    ]


@pytest.mark.gpu
def test_host_cases_through_rsa_extend():
    from rabbitsalign_amd import native
    from jobgen import JOB_DTYPE
    C = _contig()
    cases = _cases(C)
    lines = []
    for name, kind, nam, read, mu, sigma, _, _ in cases:
        if kind == "ext":
            lines.append(f"ext_window {nam_args(nam)} {len(read)} {CONTIG_LEN}")
        else:
            lines.append(f"rescue_window {nam_args(nam)} {len(read)} {CONTIG_LEN} {mu} {sigma}")
    windows = [tuple(int(x) for x in l.split()[1:]) for l in run_cases(lines)]
    assert windows == [c[7] for c in cases]
    # the query of each job: the read's rc for an rc extension NAM, the read for a forward
    # one (pc.cpp:225); for a rescue, the read for an rc anchor and its rc for a forward one
    queries, jobs = b"", np.zeros(len(cases), dtype=JOB_DTYPE)
    for i, ((name, kind, nam, read, mu, sigma, _, _), (ws, wl)) in enumerate(zip(cases, windows)):
        rc = nam[4] == 1
        q = (_rc(read) if rc else read) if kind == "ext" else (read if rc else _rc(read))
        jobs[i] = (len(queries), len(q), 0, ws, wl)
        queries += q
    ref = np.frombuffer(C, dtype=np.uint8).copy()
    offs = np.array([0, CONTIG_LEN], dtype=np.uint64)
    ctx = native.GpuContext(native.empty_index(ref, offs))
    try:
        alns, pool = ctx.extend(queries, jobs)
    finally:
        ctx.close()
    stores = []
    for i, (name, kind, nam, read, mu, sigma, _, _) in enumerate(cases):
        a = alns[i]
        ops = [int(x) for x in pool[int(a["cigar_offset"]):int(a["cigar_offset"]) + int(a["cigar_len"])]]
        info = f"{int(a['ref_start'])} {int(a['ref_end'])} {int(a['query_start'])} {int(a['query_end'])} " \
               f"{int(a['edit_distance'])} {int(a['sw_score'])} {len(ops)} " + " ".join(str(x) for x in ops)
        if kind == "ext":
            stores.append(f"ext_store {nam_args(nam)} {len(read)} {info}")
        else:
            stores.append(f"rescue_store {nam_args(nam)} {len(read)} {CONTIG_LEN} {mu} {sigma} {info}")
    got = [parse_aln(l) for l in run_cases(stores)]
    for (name, *_, want, _), g in zip(cases, got):
        assert g == want, (name, g, want)
