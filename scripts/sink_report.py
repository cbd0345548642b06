#!/usr/bin/env python3
"""Summarise an RSA_SINK_TRACE file (one line a SAM write: seconds since the writer
started at the call and at the return, bytes, bytes queued; "end T" a mapping call).

    python scripts/sink_report.py sink.txt [bench.json]

Per mapping call: the first write, the writer's idle time between writes (and the
largest gaps, by chunk), its busy time and rate, and the call's end; the timed steps
are the last ones.  With the bench line, its value and host core-us a read."""
import json
import sys


def calls(path):
    out, cur = [], []
    for line in open(path):
        f = line.split()
        if not f:
            continue
        if f[0] == "end":
            out.append((cur, float(f[1])))
            cur = []
        else:
            cur.append((float(f[0]), float(f[1]), int(f[2]), int(f[3])) + ((f[4],) if len(f) > 4 else ("W",)))
    return out


def main():
    segs = calls(sys.argv[1])
    for cur, end in segs:
        if not cur:
            continue
        gaps = [(cur[i][0] - cur[i - 1][1]) * 1e3 for i in range(1, len(cur))]
        busy = sum(x[1] - x[0] for x in cur)
        nbytes = sum(x[2] for x in cur)
        for kind in ("W", "D"):                       # writer thread / direct hand-off (RSA_SINK_DIRECT)
            k = [x for x in cur if x[4] == kind]
            if k:
                kb, kn = sum(x[1] - x[0] for x in k), sum(x[2] for x in k)
                print(f"    {kind}: {len(k)} writes, {kn / 1e6:.0f} MB, {kn / max(kb, 1e-9) / 1e9:.2f} GB/s")
        big = [(i, round(g, 1)) for i, g in enumerate(gaps, 1) if g > 2.0]
        print(f"  first {cur[0][0] * 1e3:5.1f} ms  idle {sum(g for g in gaps if g > 0):5.1f} ms  busy {busy * 1e3:5.1f} ms "
              f"({nbytes / busy / 1e9:.2f} GB/s)  end {end * 1e3:5.1f} ms  gaps>2ms {big}")
    tail = [c for c in segs if c[0]][-5:]          # the bench's timed steps (5 by default)
    if tail:
        def mean(f):
            return sum(f(c) for c in tail) / len(tail)
        first = mean(lambda c: c[0][0][0] * 1e3)
        head = mean(lambda c: sum(max(0.0, c[0][i][0] - c[0][i - 1][1]) for i in range(1, min(5, len(c[0])))) * 1e3)
        idle = mean(lambda c: sum(max(0.0, c[0][i][0] - c[0][i - 1][1]) for i in range(1, len(c[0]))) * 1e3)
        end = mean(lambda c: c[1] * 1e3)
        print(f"  last {len(tail)} calls: first write {first:.1f} ms, idle at chunks 1-4 {head:.1f} ms, idle {idle:.1f} ms, "
              f"end {end:.1f} ms")
    if len(sys.argv) > 2:
        try:
            d = json.load(open(sys.argv[2]))
            print(f"  value {d['value']:.3f} Mreads/s, {d['host_cpu']['core_us_per_read']} core-us a read, "
                  f"in memory {d['in_memory']['value']:.3f}")
        except (OSError, ValueError, KeyError):
            pass


if __name__ == "__main__":
    main()
