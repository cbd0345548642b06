"""GPU index construction (rsa_index_build_run) against the
host build and the reference's own .sti bytes.

- golden: `rsalign index` (GPU build) on the golden FASTAs hashes to the sha256
  of the .sti the reference's populate() wrote (tests/golden/sti.sha256);
- adversarial references: the GPU .sti equals the host build's (`--cpu-index`,
  itself pinned by the golden sha) byte for byte, for the three read-length
  profiles and a k-s+1 != 5 parameter set.  The contigs carry what the segment
  warm-up must survive: poly-A and di/tri-nucleotide repeats far longer than a
  segment (replayed segments), N runs, lowercase bases, contigs shorter than k
  or w_max, contigs of exactly one/two segments, and duplicated contigs (equal
  (hash, position) keys in two contigs).
"""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from helpers import GOLDEN, ROOT, golden_sha

RSALIGN = os.path.join(ROOT, "rabbitsalign_amd", "bin", "rsalign")


def _index(fa, out, *opts):
    subprocess.run([RSALIGN, "index", *opts, "-t", "4", "-o", str(out), str(fa)], check=True,
                   capture_output=True, text=True)
    with open(out, "rb") as f:
        return f.read()


def adversarial_fasta(path, seed):
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)

    def rnd(n):
        return acgt[rng.integers(0, 4, n)].tobytes()

    contigs = []
    a = rnd(30_000) + b"A" * 20_000 + rnd(9_000) + b"AC" * 9_000 + rnd(5_000) + b"ACG" * 4_000 + rnd(7_000)
    contigs.append(a)
    b = bytearray(rnd(50_000))
    for st in (1_000, 4_090, 17_000, 33_333):      # N runs, one across a segment boundary
        n = int(rng.integers(1, 40))
        b[st:st + n] = b"N" * n
    lower = rng.integers(0, len(b), 2_000)
    for i in lower:
        b[i] = b[i] | 0x20
    contigs.append(bytes(b))
    contigs += [rnd(5), rnd(15), rnd(25), rnd(4096), rnd(8192), rnd(4097)]
    contigs.append(contigs[0][:40_000])             # duplicated content: equal (hash, position) keys
    contigs.append(b"T" * 9_000 + rnd(3_000) + b"GT" * 5_000)
    contigs.append(rnd(120_000))
    with open(path, "w") as f:
        for i, c in enumerate(contigs):
            f.write(f">c{i} desc\n")
            s = c.decode()
            for j in range(0, len(s), 70):
                f.write(s[j:j + 70] + "\n")
    return path


@pytest.mark.gpu
def test_gpu_index_matches_reference_sti(tmp_path):
    """No (hash, position) ties across contigs: the GPU .sti is the reference's, byte for byte."""
    data = _index(os.path.join(GOLDEN, "small.fa"), tmp_path / "g.sti", "-r", "150")
    assert hashlib.sha256(data).hexdigest() == golden_sha("small")


@pytest.mark.gpu
def test_gpu_index_repetitive_reference(tmp_path):
    """rep.fa (140 contigs copied from each other) has thousands of entries with equal
    (hash, position) in several contigs.  Their order is what pdqsort_branchless's element
    moves leave (index.cpp:168); the GPU build counts them on the device and replays that
    sort on the host (sti_order.hpp).  The GPU .sti is the reference's, byte for byte,
    and so is the host build's."""
    from rabbitsalign_amd import native
    fa = os.path.join(GOLDEN, "rep.fa")
    g = _index(fa, tmp_path / "g.sti", "-r", "150")
    assert hashlib.sha256(g).hexdigest() == golden_sha("rep")
    c = _index(fa, tmp_path / "c.sti", "-r", "150", "--cpu-index")
    assert g == c
    ra = native.read_sti(str(tmp_path / "g.sti"))["randstrobes"]
    tie = (ra["hash"][1:] == ra["hash"][:-1]) & (ra["position"][1:] == ra["position"][:-1])
    assert tie.sum() > 0                                   # the fixture does exercise ties


@pytest.mark.gpu
@pytest.mark.parametrize("opts", [["-r", "100"], ["-r", "150"], ["-r", "250"], ["-r", "150", "-k", "24", "-s", "18"]],
                         ids=["r100", "r150", "r250", "k24s18"])
def test_gpu_index_equals_host_build(tmp_path, opts):
    fa = adversarial_fasta(tmp_path / "adv.fa", 5)
    g = _index(fa, tmp_path / "g.sti", *opts)
    c = _index(fa, tmp_path / "c.sti", *opts, "--cpu-index")
    assert len(g) == len(c)
    assert g == c


@pytest.mark.gpu
def test_gpu_index_replays_unconverged_segments(tmp_path):
    """The poly-A / tandem-repeat contigs must force replays, and the replayed
    result must still equal the host build (checked above); here the API view."""
    from rabbitsalign_amd import native
    fa = adversarial_fasta(tmp_path / "adv.fa", 9)
    names, ref, offs = native.read_fasta(str(fa))
    _index(fa, tmp_path / "c.sti", "-r", "150", "--cpu-index")
    d = native.read_sti(str(tmp_path / "c.sti"))
    k, s = d["k"], d["s"]
    w = k // (k - s + 1)
    rs, st, fc, info = native.build_index(ref, offs, k=k, s=s, w_min=max(0, w + d["l"]), w_max=w + d["u"],
                                          max_dist=d["max_dist"], q=d["q"])
    assert info["replayed_segments"] > 0
    assert info["n_randstrobes"] == len(rs) > 0
    assert d["filter_cutoff"] == fc and d["bits"] == info["bits"]
    assert np.array_equal(d["randstrobes"], rs)
    assert np.array_equal(d["bucket_starts"], st)


@pytest.mark.gpu
def test_gpu_index_medium_random(tmp_path):
    """30 Mb, 3 contigs (bits 21): GPU build == host build."""
    rng = np.random.default_rng(3)
    fa = tmp_path / "m.fa"
    with open(fa, "w") as f:
        for i, n in enumerate((12_000_000, 10_000_000, 8_000_000)):
            s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, n)].tobytes().decode()
            f.write(f">m{i}\n")
            for j in range(0, n, 100):
                f.write(s[j:j + 100] + "\n")
    g = _index(fa, tmp_path / "g.sti", "-r", "150")
    c = _index(fa, tmp_path / "c.sti", "-r", "150", "--cpu-index")
    assert g == c


@pytest.mark.gpu
def test_open_built_failure_leaves_build_valid():
    """rsa_open_built with a view whose bits differ from the build's fails and leaves
    the build owned by the caller (rsa_gpu.h): it can still be downloaded and freed,
    and a matching view then adopts it (the failure path freed it)."""
    import ctypes as C
    from rabbitsalign_amd import native
    lib = native.load()
    rng = np.random.default_rng(5)
    ref = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 200_000)].copy()
    offs = np.array([0, 120_000, 200_000], dtype=np.uint64)
    p = native.IndexBuildParams(20, 16, 3, 5, 11, 80, 255, -1, 0.0002)
    info = native.IndexBuildInfo()
    err = C.create_string_buffer(512)
    h = lib.rsa_index_build_run(0, ref.ctypes.data, offs.ctypes.data, 2, C.byref(p), C.byref(info), err, 512)
    assert h, err.value
    v = native.IndexView()
    v.bits = info.bits + 1
    v.filter_cutoff = info.filter_cutoff
    v.k, v.s, v.t_syncmer, v.w_min, v.w_max, v.max_dist, v.q = 20, 16, 3, 5, 11, 80, 255
    v.contig_offsets = offs.ctypes.data
    v.n_contigs = 2
    assert not lib.rsa_open_built(h, C.byref(v), err, 512)
    assert b"bits" in err.value
    rs = np.zeros(info.n_randstrobes, dtype=native.RS_DTYPE)
    st = np.zeros((1 << info.bits) + 1, dtype=np.uint64)
    assert lib.rsa_index_build_download(h, rs.ctypes.data, st.ctypes.data) == 0
    assert st[-1] == info.n_randstrobes and np.all(np.diff(rs["hash"].astype(np.float64)) >= 0)
    v.bits = info.bits
    ctx = lib.rsa_open_built(h, C.byref(v), err, 512)
    assert ctx, err.value
    back = np.zeros_like(rs)
    lib.rsa_index_download.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    assert lib.rsa_index_download(ctx, back.ctypes.data, 0) == 0
    assert back.tobytes() == rs.tobytes()
    lib.rsa_close(ctx)
