"""GPU: rsam_add_devices spreads the mapping calls over several device contexts
(here two contexts on the one GPU of the box, each with its own index replica):
the SAM equals the single-context SAM and the CPU path's."""
import os

import pytest

from helpers import ROOT

REF_LIB = os.path.join(ROOT, "oracle", "_ref", "librsalign_ref.so")


def _first_diffs(d, k=4):
    """the first k differing SAM body lines of one.sam / multi.sam (the failure message)"""
    with open(d / "one.sam", "rb") as f1, open(d / "multi.sam", "rb") as f2:
        x = [ln for ln in f1 if not ln.startswith(b"@")]
        y = [ln for ln in f2 if not ln.startswith(b"@")]
    out = [f"{len(x)} / {len(y)} lines"]
    for i, (p, q) in enumerate(zip(x, y)):
        if p != q:
            out.append(f"line {i}:\n one   {p[:300]!r}\n multi {q[:300]!r}")
            if len(out) > k:
                break
    return "\n".join(out)


@pytest.mark.gpu
def test_add_devices_same_sam(tmp_path):
    import torch  # noqa: F401
    from rabbitsalign_amd import mapper as M
    m = M.Mapper.synthetic(3, 20_000_000, 4, 150, device=0, threads=8)
    try:
        reads = m.synthetic_reads(9, 0, 40_000, 150, 300.0, 30.0, True)
        a = m.map(reads, threads=8, sam_path=tmp_path / "one.sam")
        m.add_devices([0])
        m.reset_kernel_stats()
        b = m.map(reads, threads=8, sam_path=tmp_path / "multi.sam")
        assert (a.sam_hash, a.sam_bytes) == (b.sam_hash, b.sam_bytes), _first_diffs(tmp_path)
        assert m.engine.endswith("x2")
        assert m.kernel_stats()["kernels"]["ext_scan"]["launches"] > 0
        if os.path.exists(REF_LIB):
            c = m.like(device=0, threads=8, lib_path=REF_LIB)
            try:
                s = c.map(reads, threads=8)
            finally:
                c.close()
            assert (s.sam_hash, s.sam_bytes) == (a.sam_hash, a.sam_bytes)
        reads.close()
    finally:
        m.close()
