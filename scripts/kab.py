#!/usr/bin/env python3
"""A/B of kernel variants on the headline workload, one host thread (so each
launch runs alone on the GPU and its HIP-event time is its isolated time).

    python scripts/kab.py VAR=a,VAR2=b  VAR=c ...   (one argument per variant)

Builds the 3 Gb synthetic mapper once, maps the same pairs under every
variant's environment and prints per-kernel mean launch times + the SAM hash
(identical across variants, or the variant is wrong)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="*")
    ap.add_argument("--ref-len", type=int, default=3_000_000_000)
    ap.add_argument("--contigs", type=int, default=24)
    ap.add_argument("--pairs", type=int, default=60_000)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--read-len", type=int, default=150)
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime first, see bench.py)
    from rabbitsalign_amd import mapper as M
    M.load()
    t = time.time()
    m = M.Mapper.synthetic(1, a.ref_len, a.contigs, a.read_len, device=0, threads=16)
    print(f"# index {time.time() - t:.1f}s", flush=True)
    mu, sd = (500.0, 50.0) if a.read_len == 250 else (300.0, 30.0)
    reads = m.synthetic_reads(7, 0, a.pairs, a.read_len, mu, sd, True)
    m.map(reads, threads=a.threads)   # warm-up
    out = {}
    for v in (a.variants or [""]):
        env = dict(kv.split("=", 1) for kv in v.split(",") if kv)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        m.reset_kernel_stats()
        st = m.map(reads, threads=a.threads)
        ks = m.kernel_stats()
        for k, x in old.items():
            if x is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = x
        row = {n: round(1e3 * k["ms"] / k["launches"], 1) for n, k in ks["kernels"].items() if k["launches"]}
        out[v or "default"] = {"Mreads_s": round(st.n_reads / st.map_seconds / 1e6, 4), "sam_hash": f"{st.sam_hash:016x}",
                               "avg_us": row}
        print(json.dumps({v or "default": out[v or "default"]}), flush=True)
    reads.close()
    m.close()


if __name__ == "__main__":
    main()
