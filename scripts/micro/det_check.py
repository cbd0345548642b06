import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch  # noqa
from rabbitsalign_amd import mapper as M
m = M.Mapper.synthetic(3, 20_000_000, 4, 150, device=0, threads=8)
reads = m.synthetic_reads(9, 0, 40_000, 150, 300.0, 30.0, True)
hs = []
for i in range(3):
    m.reset_kernel_stats()
    a = m.map(reads, threads=8)
    ks = m.kernel_stats()
    print("run", i, a.sam_hash, a.sam_bytes, {k: ks.get(k) for k in ("band_deferred", "band_overflow", "scan_redo", "scan_certified", "jobs")}, flush=True)
    hs.append(a.sam_hash)
print("deterministic", len(set(hs)) == 1)
reads.close(); m.close()
