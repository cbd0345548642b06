"""Where the streamed FASTQ -> SAM path spends host time (profiling tool).

Maps the same read set several ways and prints wall, user and system CPU per
step:  in-memory (rsam_map, SAM in memory), in-memory + SAM file, files ->
no SAM, files -> SAM file, each with the FASTQ/SAM in /dev/shm and in /tmp.
    python scripts/io_probe.py [--pairs N] [--ref-len BP] [--steps K]
"""
import argparse
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--ref-len", type=int, default=3_000_000_000)
    ap.add_argument("--contigs", type=int, default=24)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dirs", default="/dev/shm,/tmp")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime in the process, as in bench.py)
    from rabbitsalign_amd import mapper as M
    M.load()
    m = M.Mapper.synthetic(1, args.ref_len, args.contigs, 150, device=0, threads=args.threads)
    reads = m.synthetic_reads(7, 0, args.pairs, 150, 300.0, 30.0, True)

    def run(name, fn):
        if args.only and name not in args.only.split(","):
            return
        fn(0)                                   # warm-up
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        t0 = time.perf_counter()
        for i in range(args.steps):
            st = fn(i + 1)
        wall = (time.perf_counter() - t0) / args.steps
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        usr = (ru1.ru_utime - ru0.ru_utime) / args.steps
        sys_ = (ru1.ru_stime - ru0.ru_stime) / args.steps
        print(f"{name:28s} wall {wall:.3f} s  {st.n_reads / wall / 1e6:6.2f} Mreads/s  user {usr:.2f} s  "
              f"sys {sys_:.2f} s  minflt {(ru1.ru_minflt - ru0.ru_minflt) / args.steps:.0f}  "
              f"nvcsw {(ru1.ru_nvcsw - ru0.ru_nvcsw) / args.steps:.0f}  "
              f"nivcsw {(ru1.ru_nivcsw - ru0.ru_nivcsw) / args.steps:.0f}", flush=True)

    T = args.threads
    for _ in range(3):
        m.map(reads, threads=T)
    run("memory", lambda i: m.map(reads, threads=T))
    for d in args.dirs.split(","):
        f1, f2 = (os.path.join(d, f"probe_{os.getpid()}{x}") for x in ("_1.fq", "_2.fq"))
        sams = [os.path.join(d, f"probe_{os.getpid()}_{i}.sam") for i in range(args.steps + 1)]

        def clean():
            for f in sams:
                if os.path.exists(f):
                    os.remove(f)
        reads.write_fastq(f1, f2)
        try:
            run(f"memory+sam {d}", lambda i: m.map(reads, threads=T, sam_path=sams[i]))
            clean()
            run(f"files {d}", lambda i: m.map_files(f1, f2, threads=T))
            run(f"files+sam {d}", lambda i: m.map_files(f1, f2, threads=T, sam_path=sams[i]))
        finally:
            clean()
            for f in (f1, f2):
                if os.path.exists(f):
                    os.remove(f)
    reads.close()
    m.close()


if __name__ == "__main__":
    main()
