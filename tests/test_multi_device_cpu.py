"""CPU: one input mapped over several engines ("devices") gives the 1-device SAM.

The pipeline keeps one chunk queue with the global chunk_index seeding
minstd_rand (src/pc.cpp:1583, 1750), one insert-size freeze and one ordered writer
(pc.cpp:119-135); the multi-device engine (csrc/host/multi.cpp) only decides which
device serves each seeding / extension call.  Here the devices are
CPU engines: the C restatement (rsalign_cpu --devices) and the reference-code
library (librsalign_ref.so, rsam_add_devices)."""
import os

import pytest

from e2e import CPU_PORT, make_dataset, map_reads, sam_body
from helpers import ROOT

REF_LIB = os.path.join(ROOT, "oracle", "_ref", "librsalign_ref.so")


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    d = tmp_path_factory.mktemp("multi")
    fa, reads = make_dataset(str(d), pairs=3000, ref_len=200_000, cpu_index=True)
    one = d / "one.sam"
    map_reads(CPU_PORT, fa, reads, str(one), "-t", "4", "--chunk-size", "250")
    return d, fa, reads, sam_body(one)


@pytest.mark.parametrize("devices", ["0,1", "0,1,2,3", "3,3"])
def test_cli_devices_same_sam(data, devices):
    d, fa, reads, want = data
    out = d / f"multi_{devices.replace(',', '_')}.sam"
    map_reads(CPU_PORT, fa, reads, str(out), "-t", "6", "--chunk-size", "250", "--devices", devices)
    assert sam_body(out) == want


def test_cli_devices_bad_list(data):
    import subprocess
    d, fa, reads, _ = data
    r = subprocess.run([CPU_PORT, "--use-index", "--devices", "0,,1", "-o", str(d / "x.sam"), fa, *reads],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "device list" in r.stderr


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="reference build absent")
def test_library_add_devices_same_sam():
    from rabbitsalign_amd import mapper as M
    m = M.Mapper.synthetic(3, 2_000_000, 3, 150, device=0, threads=4, lib_path=REF_LIB)
    try:
        reads = m.synthetic_reads(5, 0, 6000, 150, 300.0, 30.0, True)
        a = m.map(reads, threads=4, chunk_size=500)
        m.add_devices([1, 2])
        b = m.map(reads, threads=6, chunk_size=500)
        assert (a.sam_hash, a.sam_bytes, a.n_reads) == (b.sam_hash, b.sam_bytes, b.n_reads)
        assert "x3" in m.engine
        reads.close()
    finally:
        m.close()
