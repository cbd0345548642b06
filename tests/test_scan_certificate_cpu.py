"""The word-result certificate of the scan kernel, checked on the oracle (CPU).

k_ext_scan_v runs SSW's word layout first and, when the word score reaches the byte
layout's saturation bound (score + bias >= 255, /root/reference/ext/ssw/ssw.c:838-850),
takes the word result without running the byte layout -- provided the job's band path
(banded_sw's traceback of that result, ssw.c:590-774) has no insertion next to a
deletion.  The argument: the two striped layouts differ only where an F
value that crossed a stripe boundary would open an E gap, i.e. an I directly followed
by a D; a path without one scores at least its own score in the byte layout, whose max
then saturates, so SSW itself would have taken the word result.

Here the implication is tested on 30 000 adversarial jobs with the oracle's restated
striped scans (oracle/rsa_oracle.c ora_scan_certificate: word scan, forced-word
ssw_align for the path, byte scan), which are themselves pinned against the reference's
own ssw.c (tests/test_oracle_golden.py).  Jobs: 150 and 250 bp queries (100 bp cannot
reach the bound at match 2) from their windows with up to 8 % substitutions, up to 3 %
indels, and block replacements (d bases deleted and e random bases inserted at one
place, which puts I next to D on the best path).  Every certified job must saturate
the byte layout; both outcomes (certified, and re-run for an I next to a D) must occur.
"""
import ctypes as C

import numpy as np

import oracle_lib
from jobgen import ACGT, mutate


def _translate(b: np.ndarray) -> np.ndarray:
    t = np.full(256, 4, dtype=np.int8)
    for ch, v in ((b"A", 0), (b"a", 0), (b"U", 0), (b"u", 0), (b"C", 1), (b"c", 1), (b"G", 2), (b"g", 2),
                  (b"T", 3), (b"t", 3)):
        t[ch[0]] = v
    return t[b]


def _jobs(rng, n):
    ref = ACGT[rng.integers(0, 4, 2_000_000)]
    for _ in range(n):
        L = int(rng.choice((150, 250)))
        rl = L + int(rng.integers(20, 160))
        rs = int(rng.integers(0, len(ref) - rl - 1))
        win = ref[rs:rs + rl]
        a = int(rng.integers(0, rl - L + 1))
        kind = int(rng.integers(0, 3))
        if kind == 0:                                      # substitutions + indels at random rates
            q = mutate(rng, win[a:a + L + 20], sub=float(rng.uniform(0, 0.08)), ind=float(rng.uniform(0, 0.03)))
        elif kind == 1:                                    # block replacement (I next to D on the best path)
            cut = int(rng.integers(L // 4, 3 * L // 4))
            d, e = int(rng.integers(1, 26)), int(rng.integers(1, 26))
            q = np.concatenate([win[a:a + cut], ACGT[rng.integers(0, 4, e)], win[a + cut + d:]])
            subs = rng.random(len(q)) < float(rng.uniform(0, 0.02))
            q = q.copy()
            q[subs] = ACGT[rng.integers(0, 4, int(subs.sum()))]
        else:                                              # two blocks, substitutions
            q = win[a:a + L + 30].copy()
            for _ in range(2):
                c = int(rng.integers(10, max(11, len(q) - 40)))
                d, e = int(rng.integers(0, 12)), int(rng.integers(0, 12))
                q = np.concatenate([q[:c], ACGT[rng.integers(0, 4, e)], q[c + d:]])
            subs = rng.random(len(q)) < float(rng.uniform(0, 0.05))
            q[subs] = ACGT[rng.integers(0, 4, int(subs.sum()))]
        q = q[:L]
        if len(q) < L:
            q = np.concatenate([q, ACGT[rng.integers(0, 4, L - len(q))]])
        yield _translate(q), _translate(win)


def test_word_result_certificate_30k():
    from concurrent.futures import ThreadPoolExecutor
    L = oracle_lib.lib()
    L.ora_scan_certificate.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    L.ora_scan_certificate.restype = C.c_int
    rng = np.random.default_rng(2024)
    jobs = [(np.ascontiguousarray(q), np.ascontiguousarray(r)) for q, r in _jobs(rng, 30_000)]

    def check(lo_hi):                                      # ctypes drops the GIL: one slice a thread
        return [L.ora_scan_certificate(q.ctypes.data, len(q), r.ctypes.data, len(r), 2, 8, 12, 1)
                for q, r in jobs[lo_hi[0]:lo_hi[1]]]
    cuts = np.linspace(0, len(jobs), 9).astype(int)
    with ThreadPoolExecutor(8) as ex:
        res = [v for part in ex.map(check, zip(cuts[:-1], cuts[1:])) for v in part]
    counts = {v: res.count(v) for v in (0, 1, 2, -1)}
    bad = [i for i, v in enumerate(res) if v < 0][:5]
    assert counts[-1] == 0, f"certified jobs whose byte layout does not saturate: {bad} ({counts})"
    assert counts[2] > 5000 and counts[1] > 100, counts      # both outcomes exercised
