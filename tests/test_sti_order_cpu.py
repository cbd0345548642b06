"""The .sti entry order under (hash, position) ties.

populate() sorts with pdqsort_branchless under RefRandstrobe::operator<, which
compares (hash, position) only (/root/reference/src/index.cpp:168,
src/randstrobes.hpp:32-35), so entries equal in both keep the order that sort's
element moves leave.  The product replays those moves (csrc/host/sti_order.hpp,
single- and multi-threaded); here the replay is compared byte for byte with the
reference's own pdqsort_branchless (oracle/_ref/refgen pdqsort: ext/pdqsort
compiled where it lies) on inputs that drive every branch: the small-range
insertion sort, median-of-3 and ninther pivots, block partitioning, partition-left
on runs equal to the previous pivot, the pattern-breaking swaps after unbalanced
splits, the bounded insertion sort on already-partitioned ranges, and the task
split of the multi-threaded replay.
"""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from helpers import GOLDEN, INDEXER, ROOT, golden_sha

import oracle_lib

HOSTCASES = os.path.join(ROOT, "rabbitsalign_amd", "bin", "rsa_host_cases")
DT = np.dtype([("hash", "<u8"), ("position", "<u4"), ("packed", "<u4")])


def entries(hashes, positions, packed=None):
    a = np.zeros(len(hashes), dtype=DT)
    a["hash"] = hashes
    a["position"] = positions
    a["packed"] = np.arange(len(hashes), dtype=np.uint32) if packed is None else packed
    return a


def cases():
    rng = np.random.default_rng(11)
    out = []
    for n in (0, 1, 2, 5, 23, 24, 25, 100, 128, 129, 130, 1000, 4097):
        h = rng.integers(0, 8, n, dtype=np.uint64)            # few hashes: ties everywhere
        out.append((f"few_{n}", entries(h, rng.integers(0, 4, n))))
    n = 300_000
    h = rng.integers(0, 1 << 62, n, dtype=np.uint64)
    dup = rng.integers(0, n, n // 5)                             # 20 % of entries copy another's key
    p = rng.integers(0, 1 << 31, n)
    h[dup] = h[rng.integers(0, n, n // 5)]
    p[dup] = p[rng.integers(0, n, n // 5)]
    out.append(("random_ties", entries(h, p)))
    out.append(("all_equal", entries(np.full(5000, 7, np.uint64), np.full(5000, 3))))
    s = np.sort(rng.integers(0, 1000, 20_000).astype(np.uint64))
    out.append(("sorted", entries(s, np.zeros(len(s)))))
    out.append(("reversed", entries(s[::-1].copy(), np.zeros(len(s)))))
    organ = np.concatenate([s[::2], s[1::2][::-1]])
    out.append(("organ_pipe", entries(organ, np.zeros(len(organ)))))
    saw = np.tile(np.arange(64, dtype=np.uint64), 300)
    out.append(("sawtooth", entries(saw, np.tile(np.arange(3), 6400))))
    # an index's generation order (contig, position) where contigs 3-5 repeat contigs 0-2
    base_p = np.sort(rng.choice(10_000_000, 40_000, replace=False)).astype(np.uint32)
    hs, ps, pk = [], [], []
    for c in range(6):
        hs.append(rng.integers(0, 1 << 60, 40_000, dtype=np.uint64) if c < 3 else hs[c - 3])
        ps.append(base_p)
        pk.append((np.uint32(c) << np.uint32(8)) + rng.integers(0, 80, 40_000).astype(np.uint32))
    out.append(("dup_contigs", entries(np.concatenate(hs), np.concatenate(ps), np.concatenate(pk))))
    big = 1_500_000                                               # large enough for the task split
    h = rng.integers(0, 1 << 20, big, dtype=np.uint64)
    out.append(("big_ties", entries(h, rng.integers(0, 2, big))))
    return out


@pytest.mark.skipif(not os.path.exists(oracle_lib.REFGEN), reason="oracle/_ref/refgen not built")
@pytest.mark.parametrize("name,arr", cases(), ids=[c[0] for c in cases()])
def test_pdqsort_replay_equals_reference(tmp_path, name, arr):
    src = tmp_path / "in.bin"
    arr.tofile(src)
    ref = tmp_path / "ref.bin"
    subprocess.run([oracle_lib.REFGEN, "pdqsort", str(src), str(ref)], check=True)
    want = np.fromfile(ref, dtype=DT)
    keys = np.lexsort((arr["position"], arr["hash"]))
    assert np.array_equal(want[["hash", "position"]], arr[keys][["hash", "position"]])   # a sort at all
    for threads in (1, 8):
        got_path = tmp_path / f"ours{threads}.bin"
        subprocess.run([HOSTCASES, "pdqsort", str(src), str(got_path), str(threads)], check=True)
        got = np.fromfile(got_path, dtype=DT)
        assert got.tobytes() == want.tobytes(), f"{name}: {threads} threads"


def _host_index(fa, out, *opts):
    subprocess.run([INDEXER, "index", *opts, "--cpu-index", "-t", "8", "-o", str(out), str(fa)], check=True,
                   capture_output=True, text=True)
    with open(out, "rb") as f:
        return f.read()


def test_host_index_repetitive_reference_equals_reference_sti(tmp_path):
    """rep.fa's tie groups: the host build (StiIndex::build) writes the reference's .sti
    bytes (tests/golden/sti.sha256, from the reference's own populate())."""
    data = _host_index(os.path.join(GOLDEN, "rep.fa"), tmp_path / "c.sti", "-r", "150")
    assert hashlib.sha256(data).hexdigest() == golden_sha("rep")


@pytest.mark.skipif(not os.path.exists(oracle_lib.REFGEN), reason="oracle/_ref/refgen not built")
@pytest.mark.parametrize("read_len", [100, 150, 250])
def test_host_index_duplicated_contigs_equals_reference(tmp_path, read_len):
    """The adversarial reference of test_index_gpu.py (a duplicated contig prefix: equal
    (hash, position) keys in two contigs, plus repeats, N runs, lowercase, tiny contigs):
    host build == the reference's populate() byte for byte, for the three profiles."""
    from test_index_gpu import adversarial_fasta
    fa = adversarial_fasta(tmp_path / "adv.fa", 5)
    ours = _host_index(fa, tmp_path / "c.sti", "-r", str(read_len))
    subprocess.run([oracle_lib.REFGEN, "index", str(fa), str(read_len), str(tmp_path / "r.sti"), "4"], check=True,
                   capture_output=True)
    with open(tmp_path / "r.sti", "rb") as f:
        ref = f.read()
    assert ours == ref
