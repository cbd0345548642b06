"""GPU end to end: `rsalign` (HIP engine) writes SAM byte-identical (minus @PG)
to the CPU path (the reference's own hot-path code, oracle/_ref/rsalign_ref)."""
import os

import pytest

from e2e import CPU_PORT, CPU_REF, RSALIGN, make_dataset, map_reads, sam_body


def _cpu():
    return CPU_REF if os.path.exists(CPU_REF) else CPU_PORT


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [
    dict(name="pe150", pairs=6000, L=150),
    dict(name="pe250", pairs=3000, L=250, mu=500, sigma=50),
    dict(name="pe100_many", pairs=3000, L=100, contigs=40, repeat_frac=0.1, n_rate=0.01),
    dict(name="se100", pairs=5000, L=100, se=True),
])
def test_sam_identical(tmp_path, cfg):
    fa, reads = make_dataset(str(tmp_path), **cfg)
    opts = ["-t", "4", "--chunk-size", "1000"]
    map_reads(RSALIGN, fa, reads, str(tmp_path / "gpu.sam"), *opts)
    map_reads(_cpu(), fa, reads, str(tmp_path / "cpu.sam"), *opts)
    g, c = sam_body(tmp_path / "gpu.sam"), sam_body(tmp_path / "cpu.sam")
    assert len(g) == len(c)
    diff = [i for i, (x, y) in enumerate(zip(g, c)) if x != y]
    assert not diff, f"{len(diff)} SAM lines differ, first:\n{g[diff[0]]}{c[diff[0]]}"


@pytest.mark.gpu
def test_sam_identical_eqx_details(tmp_path):
    fa, reads = make_dataset(str(tmp_path), name="eqx", pairs=2000)
    opts = ["-t", "2", "--eqx", "--details", "--rg-id", "grp1", "--rg", "SM:x", "-N", "2"]
    map_reads(RSALIGN, fa, reads, str(tmp_path / "gpu.sam"), *opts)
    map_reads(_cpu(), fa, reads, str(tmp_path / "cpu.sam"), *opts)
    assert sam_body(tmp_path / "gpu.sam") == sam_body(tmp_path / "cpu.sam")


@pytest.mark.gpu
def test_sam_identical_unrelated_mates(tmp_path):
    """A third of the second mates replaced by random sequence: their mate rescues find no
    shared substring, which the GPU engine learns from k_shared_check (RSA_ALN_NO_SHARED)
    once the insert-size estimate is frozen.  The SAM equals the CPU path's, with the
    test --details counts (tried alignments, mate rescues) included."""
    import random
    fa, reads = make_dataset(str(tmp_path), name="um", pairs=4000)
    rnd = random.Random(9)
    with open(reads[1]) as f:
        lines = f.read().split("\n")
    for r in range(0, len(lines) - 3, 4):
        if (r // 4) % 3 == 1:
            lines[r + 1] = "".join(rnd.choice("ACGT") for _ in lines[r + 1])
    with open(reads[1], "w") as f:
        f.write("\n".join(lines))
    opts = ["-t", "4", "--chunk-size", "500", "--details"]
    map_reads(RSALIGN, fa, reads, str(tmp_path / "gpu.sam"), *opts)
    map_reads(_cpu(), fa, reads, str(tmp_path / "cpu.sam"), *opts)
    g, c = sam_body(tmp_path / "gpu.sam"), sam_body(tmp_path / "cpu.sam")
    assert len(g) == len(c)
    diff = [i for i, (x, y) in enumerate(zip(g, c)) if x != y]
    assert not diff, f"{len(diff)} SAM lines differ, first:\n{g[diff[0]]}{c[diff[0]]}"
