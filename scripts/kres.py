#!/usr/bin/env python3
"""Register / scratch / occupancy of the kernels of one HIP source whose names
match a pattern (hipcc -Rpass-analysis=kernel-resource-usage).

    python scripts/kres.py rabbitsalign_amd/csrc/gpu/index_build.hip k_seg
"""
import re
import subprocess
import sys

src, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src,
                    "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                   capture_output=True, text=True)
cur, rows = None, {}
for line in r.stderr.splitlines():
    m = re.search(r"remark:\s+Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for name, v in rows.items():
    if pat in name:
        print(f"{name[:90]:90s} vgpr {v.get('VGPRs')} agpr {v.get('AGPRs')} sgpr {v.get('TotalSGPRs')} "
              f"scratch {v.get('ScratchSize [bytes/lane]')} lds {v.get('LDS Size [bytes/block]')} "
              f"occ {v.get('Occupancy [waves/SIMD]')}")
if r.returncode:
    print(r.stderr[-2000:])
    sys.exit(r.returncode)
