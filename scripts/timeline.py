#!/usr/bin/env python3
"""Where a bench step's wall time goes on the device, from a rocprofv3 trace.

    python scripts/timeline.py <run_results.db> [gap_ms]

reads the kernel (and, if traced, memory-copy) intervals of a `rocprofv3
--kernel-trace [--memory-copy-trace]` run, splits them into bursts separated by
more than gap_ms (default 3) of device silence -- a bench step is one burst --
and prints per burst: wall span, union of kernel intervals, union of copies,
union of both, the busy union of each hardware queue, and the summed kernel time
of the kernel families (seeding / extension / other).
"""
import sqlite3
import sys
from collections import defaultdict


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        tot += ce - cs
    return tot


def family(n):
    n = n.replace("void ", "")
    if n.startswith(("k_ext", "k_cig", "k_shared_check")):
        return "extend"
    if n.startswith(("k_seed", "k_lookup", "k_find_nams", "k_rescue", "k_compact", "k_sites", "k_query_fix")):
        return "seed"
    if n.startswith("__amd_rocclr"):
        return "blit"
    return "other"


def main():
    db = sys.argv[1]
    gap = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 3e6
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    qcol = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
    ks = c.execute(f"select name, start, \"end\", {qcol or 0} from kernels order by start").fetchall()
    try:
        cps = c.execute("select start, \"end\", size from memory_copies order by start").fetchall()
    except sqlite3.Error:
        cps = []
    ev = [(s, e, "k", n, q) for n, s, e, q in ks] + [(s, e, "c", sz, None) for s, e, sz in cps]
    ev.sort()
    bursts, cur, cur_end = [], [], None
    for x in ev:
        if cur and x[0] > cur_end + gap:
            bursts.append(cur)
            cur = []
        cur.append(x)
        cur_end = x[1] if len(cur) == 1 else max(cur_end, x[1])
    if cur:
        bursts.append(cur)
    print(f"queue column: {qcol}; kernels {len(ks)}, copies {len(cps)}, bursts {len(bursts)}")
    for b in bursts:
        lo, hi = min(x[0] for x in b), max(x[1] for x in b)
        span = hi - lo
        if span < 20e6:
            continue
        kiv = [(x[0], x[1]) for x in b if x[2] == "k"]
        civ = [(x[0], x[1]) for x in b if x[2] == "c"]
        fam, perq = defaultdict(float), defaultdict(list)
        for x in b:
            if x[2] == "k":
                fam[family(x[3])] += x[1] - x[0]
                perq[x[4]].append((x[0], x[1]))
        cbytes = sum(x[3] or 0 for x in b if x[2] == "c")
        nseed = sum(1 for x in b if x[2] == "k" and "k_lookup" in x[3])
        print(f"burst {span / 1e6:8.1f} ms  k_lookup {nseed:4d}  kernels-union {union(kiv) / span:5.1%}  "
              f"copies-union {union(civ) / span:5.1%} ({len(civ)} copies, {cbytes / 1e6:.0f} MB)  "
              f"any {union(kiv + civ) / span:5.1%}  sum-ms " +
              " ".join(f"{k} {v / 1e6:.1f}" for k, v in sorted(fam.items())) +
              "  per-queue-busy " + " ".join(f"{union(v) / span:.0%}" for _, v in sorted(perq.items())))


if __name__ == "__main__":
    main()
