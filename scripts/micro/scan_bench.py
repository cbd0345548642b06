#!/usr/bin/env python3
"""Isolated timing of the extension kernels on synthetic jobs shaped like the headline
workload (query 150 bp, window 257 bp, 1 % substitutions) -- measurement tool.

    python scripts/micro/scan_bench.py [n_jobs ...]

Prints per-launch k_ext_scan / band16 / band64 times (HIP events) and Gcells/s."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def make(rng, ref, n, L=150, W=257):
    starts = rng.integers(0, len(ref) - W, n)
    q = np.empty((n, L), np.uint8)
    for i, s in enumerate(starts):
        a = int(rng.integers(40, 60))
        q[i] = ref[s + a:s + a + L]
    sub = rng.random((n, L)) < 0.01
    q[sub] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(sub.sum()))]
    from jobgen import JOB_DTYPE
    jobs = np.zeros(n, JOB_DTYPE)
    jobs["query_offset"] = np.arange(n, dtype=np.uint64) * L
    jobs["query_len"] = L
    jobs["ref_id"] = 0
    jobs["ref_start"] = starts
    jobs["ref_len"] = W
    return q.tobytes(), jobs


def main():
    import torch  # noqa: F401
    from rabbitsalign_amd import native
    if os.environ.get("SCAN_BENCH_LIB"):          # A/B against another build of librsa_gpu.so
        native.load(os.environ["SCAN_BENCH_LIB"])
    sizes = [int(x) for x in sys.argv[1:]] or [16, 256, 1024, 4096, 7300, 16384, 65536]
    rng = np.random.default_rng(1)
    ref = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 4_000_000)].copy()
    ctx = native.GpuContext(native.empty_index(ref, np.array([0, len(ref)], np.uint64)))
    L = int(os.environ.get("SCAN_BENCH_L", "150"))      # query length; window = L + 107 (headline shape)
    W = int(os.environ.get("SCAN_BENCH_W", str(L + 107)))
    for n in sizes:
        q, jobs = make(rng, ref, n, L, W)
        ctx.extend(q, jobs)                       # warm-up (buffers, code)
        ctx.reset_stats()
        reps = max(1, min(20, 200_000 // n))
        t = time.perf_counter()
        for _ in range(reps):
            ctx.extend(q, jobs)
        wall = (time.perf_counter() - t) / reps
        st = ctx.stats()
        k = st["kernels"]
        us = {name: round(1e3 * k[name]["ms"] / max(1, k[name]["launches"]), 1)
              for name in ("ext_scan", "ext_band", "ext_band_wide")}
        cells = st["dp_cells"] / reps
        print(f"n={n:6d} scan {us['ext_scan']:8.1f} us  band16 {us['ext_band']:7.1f}  band64 {us['ext_band_wide']:7.1f}"
              f"  call {wall * 1e6:8.1f} us  scan {cells / (us['ext_scan'] * 1e-6) / 1e9:7.1f} Gcells/s", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
