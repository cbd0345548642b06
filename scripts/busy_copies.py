#!/usr/bin/env python3
"""GPU activity over the mapping span from a rocprofv3 database taken with
--kernel-trace --memory-copy-trace: the union of kernel intervals, of copy
intervals, of both, and the copy bytes per direction.

    python scripts/busy_copies.py <run_results.db>
"""
import sqlite3
import sys


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


def main():
    c = sqlite3.connect(sys.argv[1])
    names = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    print("tables:", ", ".join(n for n in names if not n.startswith("rocpd_") or "copy" in n))
    ks = c.execute("select name, start, \"end\" from kernels").fetchall()
    look = [(s, e) for n, s, e in ks if "k_lookup" in n]
    lo, hi = min(s for s, _ in look), max(e for _, e in look)
    kiv = [(max(s, lo), min(e, hi)) for _, s, e in ks if e > lo and s < hi]
    ctab = next((n for n in names if n in ("memory_copies", "memory_copy")), None)
    civ, by = [], {}
    if ctab:
        cols = [r[1] for r in c.execute(f"pragma table_info({ctab})")]
        print("copy columns:", cols)
        dcol = next((x for x in ("direction", "kind", "name", "operation") if x in cols), None)
        scol = next((x for x in ("size", "bytes") if x in cols), None)
        q = f"select start, \"end\"{', ' + dcol if dcol else ''}{', ' + scol if scol else ''} from {ctab}"
        for row in c.execute(q):
            s, e = row[0], row[1]
            if e <= lo or s >= hi:
                continue
            civ.append((max(s, lo), min(e, hi)))
            d = row[2] if dcol else "?"
            b = row[3] if scol and dcol else (row[2] if scol else 0)
            x = by.setdefault(str(d), [0, 0, 0])
            x[0] += 1
            x[1] += b or 0
            x[2] += min(e, hi) - max(s, lo)
    span = hi - lo
    ku, cu, bu = union(kiv), union(civ), union(kiv + civ)
    print(f"span {span / 1e6:.1f} ms: kernels busy {100 * ku / span:.1f} %, copies busy {100 * cu / span:.1f} %, "
          f"either {100 * bu / span:.1f} %")
    for d, (n, b, t) in sorted(by.items()):
        print(f"  copies {d}: {n} calls, {b / 1e6:.1f} MB, summed {t / 1e6:.1f} ms, "
              f"{b / (t if t else 1):.2f} GB/s while running")


if __name__ == "__main__":
    main()
