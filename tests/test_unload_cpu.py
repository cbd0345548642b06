"""Load, map, close and unload the mapping library twice in one process.

rsam_close of the last open mapper joins every thread the host pipeline keeps
between calls (the worker pool, the SAM writer and the FASTQ readers end with their
call) and frees its pooled buffers, so after it nothing of the library runs: the
library can be dlclose'd and opened again, and the process exits without a static
destructor reaching into a torn-down runtime.  Run on the CPU-path build (same host
pipeline; the engine does not matter here) in a child process, so a crash at
unload or exit fails the test instead of the runner."""
import os
import subprocess
import sys

import pytest

from helpers import ROOT

REF_CPU_LIB = os.path.join(ROOT, "oracle", "_ref", "librsalign_ref.so")

SCRIPT = r"""
import os, sys
sys.path.insert(0, sys.argv[1])
from rabbitsalign_amd import mapper
lib, d = sys.argv[2], sys.argv[3]
base = len(os.listdir("/proc/self/task"))      # numpy's own threads included
hashes = []
for rep in range(2):
    m = mapper.Mapper.synthetic(3, 1_000_000, 2, 150, threads=4, lib_path=lib)
    reads = m.synthetic_reads(7, 0, 3000, 150, 300.0, 30.0, True)
    fq1, fq2 = os.path.join(d, "r1.fq"), os.path.join(d, "r2.fq")
    reads.write_fastq(fq1, fq2)
    a = m.map(reads, threads=4, chunk_size=500)
    b = m.map_files(fq1, fq2, threads=4, chunk_size=500, sam_path=os.path.join(d, f"o{rep}.sam"))
    reads.close()
    m.close()
    mapper.unload(lib)
    hashes.append((a.sam_hash, b.sam_bytes))
    # only the threads from before the first mapper are left: the pipeline's were joined
    assert len(os.listdir("/proc/self/task")) == base, os.listdir("/proc/self/task")
assert hashes[0] == hashes[1], hashes
print("unload ok", hashes[0])
"""


@pytest.mark.skipif(not os.path.exists(REF_CPU_LIB), reason="CPU-path library not built")
def test_load_map_unload_twice(tmp_path):
    r = subprocess.run([sys.executable, "-c", SCRIPT, ROOT, REF_CPU_LIB, str(tmp_path)], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "unload ok" in r.stdout
