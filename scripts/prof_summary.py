#!/usr/bin/env python3
"""Summarise rocprofv3 databases of a bench run into profiles/.

    python scripts/prof_summary.py gpurun_out/prof_r01 profiles/r01

reads <dir>/trace/run_results.db (--kernel-trace --stats), and, when present,
<dir>/pmc_fetch/run_results.db and <dir>/pmc_write/run_results.db (one PMC
counter per pass).  Writes <out>_rocprof.md (per-kernel table) and
<out>_traffic.json (HBM bytes per launch per kernel: FETCH_SIZE doubled, the
gfx950 correction of MI355X_MICROARCH.md "HBM", plus WRITE_SIZE, both KB->B).
"""
import json
import os
import sqlite3
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0]


def kernel_times(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name").fetchall()
    return {short(r[0]): {"calls": r[1], "total_ms": r[2] / 1e6, "avg_us": r[3] / 1e3, "min_us": r[4] / 1e3,
                          "max_us": r[5] / 1e3} for r in rows}


def busy(db):
    """GPU busy time over the mapping span (first to last seeding kernel): the union
    of all kernel intervals, their summed durations (concurrency = sum / union), and
    the union per 100 ms window."""
    c = sqlite3.connect(db)
    try:
        rows = c.execute("select name, start, \"end\" from kernels order by start").fetchall()
    except sqlite3.Error:
        return None
    base = lambda n: short(n).split("<")[0].split()[-1]      # "void k_seed_query<256, 6>" -> k_seed_query
    seed = [r for r in rows if base(r[0]) in ("k_lookup", "k_seed_query")]
    if not seed:
        return None
    lo, hi = seed[0][1], max(r[2] for r in seed)
    iv = [(max(s, lo), min(e, hi)) for _, s, e in rows if e > lo and s < hi]

    def union_of(ivs):
        union, cur_s, cur_e, tot = 0, None, None, 0
        for s, e in sorted(ivs):
            tot += e - s
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    union += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            union += cur_e - cur_s
        return union, tot

    union, tot = union_of(iv)
    span = hi - lo
    out = {"span_ms": span / 1e6, "busy_union_ms": union / 1e6, "busy_frac": union / span if span else None,
           "kernel_sum_ms": tot / 1e6, "mean_concurrency": tot / union if union else None}
    # the score scan's launches: their own union (two combined extension calls can overlap)
    sc = [(max(s, lo), min(e, hi)) for n, s, e in rows if short(n).startswith("void k_ext_scan_v") and e > lo and s < hi]
    if sc:
        su, st = union_of(sc)
        out["scan_v"] = {"launches": len(sc), "sum_ms": st / 1e6, "union_ms": su / 1e6,
                         "self_concurrency": st / su if su else None}
    return out


def counter(db, cname):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, count(*), avg(value), sum(value) from counters_collection "
                     "where counter_name = ? group by kernel_name", (cname,)).fetchall()
    return {short(r[0]): {"dispatches": r[1], "avg_kb": r[2], "sum_kb": r[3]} for r in rows}


def main():
    src, out = sys.argv[1], sys.argv[2]
    tdb = os.path.join(src, "trace", "run_results.db")
    if not os.path.exists(tdb):
        import glob
        tdb = (glob.glob(os.path.join(src, "t*", "**", "*.db"), recursive=True) or [tdb])[0]
    kt = kernel_times(tdb)
    fetch = write = {}
    fdb = os.path.join(src, "pmc_fetch", "run_results.db")
    wdb = os.path.join(src, "pmc_write", "run_results.db")
    if os.path.exists(fdb):
        fetch = counter(fdb, "FETCH_SIZE")
    if os.path.exists(wdb):
        write = counter(wdb, "WRITE_SIZE")
    total = sum(v["total_ms"] for v in kt.values())
    lines = [f"# rocprofv3 summary: {src}", "",
             "Kernel trace (`rocprofv3 --kernel-trace --stats`), PMC in separate passes "
             "(`--pmc FETCH_SIZE`, `--pmc WRITE_SIZE`). HBM read bytes = 2 x FETCH_SIZE (gfx950 correction).", "",
             "| kernel | calls | total ms | % | avg us | min us | max us | HBM read B/launch | HBM write B/launch |",
             "|---|---:|---:|---:|---:|---:|---:|---:|---:|"]
    traffic = {}
    for k, v in sorted(kt.items(), key=lambda kv: -kv[1]["total_ms"]):
        rd = 2 * 1024 * fetch[k]["avg_kb"] if k in fetch else None
        wr = 1024 * write[k]["avg_kb"] if k in write else None
        if rd is not None or wr is not None:
            traffic[k] = {"read_bytes": rd, "write_bytes": wr,
                          "bytes": (rd or 0) + (wr or 0) if rd is not None and wr is not None else None}
        lines.append(f"| {k} | {v['calls']} | {v['total_ms']:.2f} | {100 * v['total_ms'] / total:.1f} | "
                     f"{v['avg_us']:.1f} | {v['min_us']:.1f} | {v['max_us']:.1f} | "
                     f"{'' if rd is None else f'{rd:.0f}'} | {'' if wr is None else f'{wr:.0f}'} |")
    b = busy(tdb)
    if b:
        lines += ["", f"GPU busy over the mapping span (first to last seeding kernel, warm-up included): "
                      f"{b['busy_union_ms']:.1f} ms of {b['span_ms']:.1f} ms = {100 * b['busy_frac']:.1f} % "
                      f"(union of kernel intervals); summed kernel time {b['kernel_sum_ms']:.1f} ms, mean "
                      f"concurrency while busy {b['mean_concurrency']:.2f}."]
        if b.get("scan_v"):
            v = b["scan_v"]
            lines += ["", f"`k_ext_scan_v` launches: {v['launches']}, summed duration {v['sum_ms']:.1f} ms, union "
                          f"{v['union_ms']:.1f} ms (launches overlapping each other: {v['self_concurrency']:.2f}x)."]
    with open(out + "_rocprof.md", "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(out + "_traffic.json", "w") as f:
        json.dump({"source": src, "kernels": kt, "traffic_per_launch": traffic, "busy": b}, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
