#!/usr/bin/env python3
"""GPU busy time from a rocprofv3 kernel trace: union of kernel intervals per
timed step (the bench's warmup + steps show up as bursts separated by idle gaps),
plus per-kernel totals.   python scripts/busy.py <dir with run_results.db>"""
import os
import sqlite3
import sys

db = sys.argv[1]
if os.path.isdir(db):
    db = os.path.join(db, "run_results.db")
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
iv = [(s, e, n.split("(")[0]) for n, s, e in rows]
segs = []
cs, ce = iv[0][0], iv[0][1]
for s, e, _ in iv[1:]:
    if s > ce:
        segs.append((cs, ce))
        cs, ce = s, e
    else:
        ce = max(ce, e)
segs.append((cs, ce))
# bursts: split where the GPU idles > 50 ms (between map() calls)
bursts, cur = [], [segs[0]]
for a, b in segs[1:]:
    if a - cur[-1][1] > 50e6:
        bursts.append(cur)
        cur = [(a, b)]
    else:
        cur.append((a, b))
bursts.append(cur)
for i, bsegs in enumerate(bursts):
    span = bsegs[-1][1] - bsegs[0][0]
    busy = sum(b - a for a, b in bsegs)
    print(f"burst {i}: span {span/1e6:.1f} ms, busy {busy/1e6:.1f} ms ({100*busy/span:.0f}%)")
tot = {}
for s, e, n in iv:
    tot[n] = tot.get(n, 0) + (e - s)
print("kernel-time sum (overlapping):", {k: round(v / 1e6, 1) for k, v in sorted(tot.items(), key=lambda x: -x[1])})
