"""CPU: the C restatement (oracle/) reproduces the reference's golden vectors."""
import os
import subprocess

import numpy as np
import pytest

import oracle_lib
from helpers import GOLDEN, build_sti, read_lines


@pytest.fixture(scope="module")
def cli():
    if not os.path.exists(oracle_lib.ORACLE_CLI):
        subprocess.run(["make", "-s", "-C", oracle_lib.ORACLE_DIR, "oracle"], check=True)
    return oracle_lib.ORACLE_CLI


@pytest.mark.parametrize("name", ["small", "rep"])
def test_seeds_golden(cli, tmp_path, name):
    fa, sti = build_sti(tmp_path, name)
    out = tmp_path / "seeds.txt"
    subprocess.run([cli, "seeds", sti, os.path.join(GOLDEN, f"{name}_reads.txt"), str(out), "2"], check=True)
    want = read_lines(os.path.join(GOLDEN, f"{name}_seeds.golden.gz"))
    got = out.read_text()
    assert got == want


def test_ssw_golden(cli, tmp_path):
    want = read_lines(os.path.join(GOLDEN, "ssw.golden.gz"))
    jobs = tmp_path / "jobs.txt"
    jobs.write_text("".join(" ".join(l.split()[:2]) + "\n" for l in want.splitlines()))
    out = tmp_path / "ssw.txt"
    subprocess.run([cli, "ssw", str(jobs), str(out)], check=True)
    assert out.read_text() == want


@pytest.mark.skipif(not os.path.exists(oracle_lib.REFGEN), reason="reference build absent")
@pytest.mark.parametrize("seed", [1001, 1002])
def test_ssw_live_reference(cli, tmp_path, seed):
    """Fresh random jobs every seed, compared with the reference's ssw.c run here."""
    ref = tmp_path / "ref.txt"
    subprocess.run([oracle_lib.REFGEN, "sswrand", str(seed), "20000", str(ref)], check=True)
    jobs = tmp_path / "jobs.txt"
    jobs.write_text("".join(" ".join(l.split()[:2]) + "\n" for l in ref.read_text().splitlines()))
    out = tmp_path / "ora.txt"
    subprocess.run([cli, "ssw", str(jobs), str(out)], check=True)
    assert out.read_text() == ref.read_text()


def test_aligner_wrapper_basic():
    """Aligner::align wrapper semantics on hand-made cases (end bonus, soft clips, sentinels)."""
    q = b"ACGTACGTAC" * 15
    r = b"TTTTT" + q + b"GGGGG"
    a = oracle_lib.align(q, r)
    assert a["sw_score"] == 2 * len(q) + 20 and a["edit_distance"] == 0
    assert a["query_start"] == 0 and a["query_end"] == len(q) and a["ref_start"] == 5
    assert a["cigar"] == [(len(q) << 4) | 7]
    long_ref = b"A" * 2001
    s = oracle_lib.align(q, long_ref)
    assert s["sw_score"] == -1000000 and s["edit_distance"] == 100000
    # mismatch near the start: soft clip replaced by end-bonus extension when it pays
    q2 = b"T" + q[1:]
    a2 = oracle_lib.align(q2, r)
    assert a2["query_start"] == 0 and a2["cigar"][0] == (1 << 4) | 8


def test_aligner_wrapper_hand_derived():
    """The oracle's Aligner::align restatement on hand-derived cases (tests/wrapper_cases.py):
    end bonus at both ends, front/back extension replacing a soft clip, the equal-score
    case that keeps it, N == N as '=', a clip at reference start, the >2000 sentinel."""
    from wrapper_cases import cases
    for name, q, r, want in cases():
        got = oracle_lib.align(q, r)
        if want is None:
            continue
        for k, v in want.items():
            assert got[k] == v, (name, k, got[k], v)


@pytest.mark.skipif(not os.path.exists(oracle_lib.REFGEN), reason="reference build (oracle/_ref/refgen) absent")
def test_wrapper_cases_ssw_core_live(tmp_path):
    """The SSW part of each hand derivation in tests/wrapper_cases.py (score1, begins,
    ends, the M/I/D CIGAR) against the reference's own ssw.c (oracle/_ref/refgen ssw),
    so only the Aligner::align wrapper above it stays restated-only."""
    from wrapper_cases import cases, ssw_core
    core = ssw_core()
    sel = [(n, q, r) for n, q, r, _ in cases() if n in core]
    assert len(sel) == len(core)
    jobs = tmp_path / "jobs.txt"
    jobs.write_text("".join(f"{q.decode()} {r.decode()}\n" for _, q, r in sel))
    out = tmp_path / "out.txt"
    subprocess.run([oracle_lib.REFGEN, "ssw", str(jobs), str(out)], check=True)
    lines = out.read_text().splitlines()
    assert len(lines) == len(sel)
    for (name, _, _), line in zip(sel, lines):
        f = line.split()[2:]
        score1, rb, re_, qb, qe, flag, n = (int(x) for x in f[:7])
        cig = [int(x) for x in f[7:7 + n]]
        assert flag == 0, name
        assert (score1, rb, re_, qb, qe, cig) == core[name], (name, (score1, rb, re_, qb, qe, cig), core[name])
