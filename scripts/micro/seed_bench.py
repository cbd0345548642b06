#!/usr/bin/env python3
"""Isolated timing of the seeding kernels (rsa_seed) on headline-shaped batches.

A random reference (default 3 Gb in 24 contigs, r150 index parameters, built on the
GPU), batches of 2 x 10000 reads of 150 bp sampled from it with 1 % substitutions and
random orientation, mapped with site checks and hamming_align (as the pipeline asks),
every launch timed with HIP events (RSA_KTIMER_EVERY=1).  Prints the mean launch time
of each kernel over the timed calls.

    python scripts/micro/seed_bench.py [--ref-len 3e9] [--calls 30] [--reads 20000]
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("RSA_KTIMER_EVERY", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref-len", type=float, default=3e9)
    ap.add_argument("--contigs", type=int, default=24)
    ap.add_argument("--reads", type=int, default=20000)
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--out", default="")
    ap.add_argument("--ab", default="", help="'VAR=a|VAR=b': settings alternated (--rounds times), per-setting means")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    from rabbitsalign_amd import native
    rng = np.random.default_rng(3)
    n = int(a.ref_len)
    t = time.time()
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    ref = acgt[rng.integers(0, 4, n, dtype=np.uint8)]
    offs = np.linspace(0, n, a.contigs + 1).astype(np.uint64)
    rs, st, fc, info = native.build_index(ref, offs, k=20, s=16, w_min=5, w_max=11, max_dist=80)
    print(f"index: {len(rs)} randstrobes, bits {info['bits']}, {time.time() - t:.1f} s", flush=True)
    idx = native.Index(rs, st, info["bits"], fc, 150, 20, 16, 1, 7, 255, 80, ref, offs,
                       [f"chr{i + 1}" for i in range(a.contigs)])
    ctx = native.GpuContext(idx)
    comp = bytes.maketrans(b"ACGT", b"TGCA")
    L = a.read_len

    def batch(seed):
        r = np.random.default_rng(seed)
        out = []
        starts = r.integers(0, n - L - 1, a.reads)
        for s in starts:
            b = bytearray(ref[s:s + L].tobytes())
            for j in r.integers(0, L, max(0, int(r.poisson(0.01 * L)))):
                b[j] = b"ACGT"[(b"ACGT".index(b[j]) + 1 + int(r.integers(0, 3))) % 4]
            b = bytes(b)
            out.append(b.translate(comp)[::-1] if r.integers(0, 2) else b)
        return out

    batches = [batch(100 + i) for i in range(4)]
    for bt in batches[:2]:                                        # warm-up
        ctx.seed(bt, sites=True, order=native.NAMS_BY_SCORE, hamming=(2, 8, 10))
    if a.ab:
        sets = [dict(kv.split("=", 1) for kv in x.split(",")) for x in a.ab.split("|")]
        acc = [dict() for _ in sets]
        for _ in range(a.rounds):
            for i, env in enumerate(sets):
                os.environ.update(env)
                ctx.reset_stats()
                for c in range(a.calls):
                    ctx.seed(batches[c % len(batches)], sites=True, order=native.NAMS_BY_SCORE, hamming=(2, 8, 10))
                for k, v in ctx.stats()["kernels"].items():
                    if v["launches"]:
                        x = acc[i].setdefault(k, [0.0, 0])
                        x[0] += v["ms"]; x[1] += v["launches"]
        for env, kv in zip(sets, acc):
            print(json.dumps({"env": env, "read_len": L, "us_per_launch":
                              {k: round(1e3 * ms / n, 1) for k, (ms, n) in kv.items()}}), flush=True)
        ctx.close()
        return
    ctx.reset_stats()
    t = time.time()
    for c in range(a.calls):
        ctx.seed(batches[c % len(batches)], sites=True, order=native.NAMS_BY_SCORE, hamming=(2, 8, 10))
    wall = time.time() - t
    s = ctx.stats()
    rows = {k: {"launches": v["launches"], "avg_us": round(1e3 * v["ms"] / max(1, v["launches"]), 2)}
            for k, v in s["kernels"].items() if v["launches"]}
    res = {"reads_per_call": a.reads, "calls": a.calls, "wall_ms_per_call": round(1e3 * wall / a.calls, 3),
           "kernels": rows, "nams": s.get("nams"), "reads": s.get("reads")}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
