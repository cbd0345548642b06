#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X mapping path.

Metric (BASELINE.json): Mreads/s aligned, paired-end 2x150 bp against a 3 Gb
reference, SAM bit-exact with the CPU path.  One "step" maps one set of 10^6
synthetic pairs end to end as the CLI does: two FASTQ files -> reads streamed
by a reader thread per file while mapping -> seeding, NAMs, extension on the
GPU, pairing/rescue/SAM text on the host -> a SAM file, timed from the call to
the last SAM byte written: the reference's "consumer cost" (SURVEY.md §8d,
src/main.cpp:446,595).  Reference and index are built once before timing and
stay resident in HBM.  An in-memory leg (reads in RAM, SAM in memory) is
reported beside it.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload pe150_3g]

N>1: one process per GPU under torch.distributed.run; every rank holds the
replicated index, and all ranks map ONE shared FASTQ pair of N x --pairs pairs per
step in the product's rank/world mode (rsam_part_* / rsam_map_files_part, DESIGN.md
§7): each rank counts the newlines of its 1/N of each file, the counts are
all-gathered (the only exchange before mapping), and each rank maps its contiguous
chunks into its own SAM part; header + parts in rank order are the one-process SAM
(checked untimed, `parity.parts_equal_one_process`).  The wall time is the max over
ranks and the read count the sum ("weak": per-GPU work fixed).
rank 0 prints one JSON line.  `python3 bench.py --gpus N` without WORLD_SIZE
starts the N ranks itself (rabbitsalign_amd/launch.py; the launcher never
touches the GPU), then runs the product's one-process multi-device path
(rsam_add_devices, one SAM file) and adds it to the line as `multi_device`.  The cpu_baseline leg (rank 0, N=1) maps a
bounded sample of the same workload with oracle/_ref/librsalign_ref.so (the
reference's own seeding + SSW code inside the same host pipeline) and checks
that its SAM hash equals the GPU path's on that sample.
"""
from __future__ import annotations

import argparse
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    # name: reference bp, contigs, read length, insert mean/sd, paired
    "pe150_3g": dict(ref_len=3_000_000_000, n_contigs=24, read_len=150, mu=300.0, sigma=30.0, paired=True,
                     desc="PE 2x150 vs 3 Gb synthetic reference (24 x 125 Mb contigs), 1 GPU"),
    "pe250_3g": dict(ref_len=3_000_000_000, n_contigs=24, read_len=250, mu=500.0, sigma=50.0, paired=True,
                     desc="PE 2x250 vs 3 Gb synthetic reference (24 x 125 Mb contigs)"),
    "pe150_250m": dict(ref_len=250_000_000, n_contigs=1, read_len=150, mu=300.0, sigma=30.0, paired=True,
                       desc="PE 2x150 vs 250 Mb synthetic reference (chr1)"),
    "se100_5m": dict(ref_len=5_000_000, n_contigs=1, read_len=100, mu=300.0, sigma=30.0, paired=False,
                     desc="SE 1x100 vs 5 Mb synthetic reference"),
}

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md "Chip-level parameters")
# VALU ceilings of the DP scan (DESIGN.md §3 "Roofline reporting"), in cell updates/s.
# Measured issue cost on gfx950 (scripts/micro/valu_issue.hip, profiles/r04/valu_issue.txt,
# 4 waves per SIMD): a wave64 VOP3/VOP3P instruction (v_pk_maximum3_f16, v_pk_add_f16,
# v_max3_i32) 4.4 cycles, a VOP1/VOP2 one (v_add_u32, v_and_b32, v_add_f32) 2.35 cycles.
#  - peak: SSW's recurrence is 11.5 packed-f16 instructions per row of two cells (diag add,
#    three max3 for H/E/F, three gap decays, the gap-open term, the column max), i.e. 5.75
#    VOP3P per cell: 1024 SIMDs x 2.4 GHz / 4.4 cycles x 64 lanes / 5.75 = 6.2 T cells/s;
#  - spec model: 256 CUs x 128 lane-ops/clk x 2.4 GHz x 2 / 12 = 13.1 T
#    cells/s -- it assumes packed instructions issue at the VOP2 rate, which gfx950 does not
VOP3P_CYCLES, VOP2_CYCLES = 4.4, 2.35
VALU_SIMDS, VALU_CLOCK = 1024, 2.4e9
DP_PEAK_GCELLS = VALU_SIMDS * VALU_CLOCK / VOP3P_CYCLES * 64 / 5.75 / 1e9
DP_SPEC_GCELLS = 256 * 128 * 2.4 * 2 / 12
REF_CPU_LIB = os.path.join(ROOT, "oracle", "_ref", "librsalign_ref.so")


def log(rank, *a):
    print(f"[bench r{rank} {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def _cgroup_cpus():
    """CPUs granted by the cgroup v2 quota (cpu.max), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else max(1, int(int(quota) / int(period)))
    except (OSError, ValueError):
        return None


def pin_rank_cpus(local_rank: int, local_world: int):
    """N>1: give each rank of the node its own physical cores on the NUMA node its
    GPU number maps to (rabbitsalign_amd.shard.rank_cpu_groups); returns the CPU
    list, or None when nothing was pinned.  Threads started afterwards (the host
    pipeline's workers) inherit it."""
    if local_world <= 1 or os.environ.get("RSA_BENCH_NO_PIN"):
        return None
    from rabbitsalign_amd import shard
    allowed = sorted(os.sched_getaffinity(0))
    node_cpus, siblings = shard.host_topology(allowed)
    cpus = shard.rank_cpu_groups(node_cpus, siblings, local_world)[local_rank]
    if not cpus:
        return None
    os.sched_setaffinity(0, cpus)
    return cpus


def host_cores(pinned: bool = False) -> int:
    """Host threads for this rank: the CPUs this process may use (affinity, cgroup
    quota) shared among the ranks of the node, capped by OMP_NUM_THREADS / MAX_JOBS.
    torch.distributed.run exports OMP_NUM_THREADS=1 to every rank when the variable
    is unset; that default says nothing about the host pipeline and is ignored.
    `pinned`: the affinity is already this rank's share (pin_rank_cpus)."""
    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    n = len(os.sched_getaffinity(0))
    q = _cgroup_cpus()                       # the quota covers every rank of the node
    if pinned:
        n = min(n, max(1, q // local)) if q else n
    else:
        n = max(1, (min(n, q) if q else n) // local)
    for var in ("OMP_NUM_THREADS", "MAX_JOBS"):
        v = os.environ.get(var)
        if v and v.isdigit() and int(v) > 0:
            if var == "OMP_NUM_THREADS" and int(v) == 1 and local > 1:
                continue
            n = min(n, int(v))
    return max(1, n)


TRAFFIC_JSON = os.path.join(ROOT, "profiles", "latest_traffic.json")
LINE_PEAK_GLINES = 46.0      # random 128-B lines, 8 lanes a line, 32 GB table (scripts/micro/line_probe.hip)
EXT_PMC_JSON = os.path.join(ROOT, "profiles", "r06", "ext_pmc.json")


def scan_pmc(symbol: str):
    """(wave64 VALU instructions per DP cell, VOP3P share) of the scan kernel from the
    committed PMC pass (scripts/gpu_ext_pmc.sh: SQ_INSTS_VALU / cells of an isolated
    22000-job launch), or None."""
    try:
        with open(EXT_PMC_JSON) as f:
            d = json.load(f)[symbol]
        return float(d["wave_instr_per_cell"]), float(d.get("vop3p_share", 1.0))
    except (OSError, ValueError, KeyError):
        return None


def pmc_traffic(symbol: str):
    """HBM bytes per launch of `symbol` from the committed rocprofv3 PMC summary
    (scripts/prof_summary.py: 2 x FETCH_SIZE + WRITE_SIZE), or None."""
    try:
        with open(TRAFFIC_JSON) as f:
            t = json.load(f)
        per = t["traffic_per_launch"]
        # rocprof names carry the return type and template arguments ("void k_ext_scan<4, 2>")
        base = lambda n: n.split("(")[0].split("<")[0].split()[-1]
        v = per.get(symbol) or next((per[n] for n in per if base(n) == symbol), None)
        return (round(v["bytes"], 1) if v and v.get("bytes") is not None else None), t.get("source")
    except (OSError, ValueError, KeyError):
        return None, None


def kernel_roofline(name: str, k: dict, ks: dict) -> dict:
    """Roofline of one kernel of the path from its live HIP-event times.

    k_ext_scan (integer DP, no MFMA) is VALU-bound: achieved = forward DP cells
    per launch / average launch duration, against DP_PEAK_GCELLS.  The seeding,
    site and band kernels are memory kernels: achieved = algorithmic bytes per
    launch / average launch duration, against HBM peak.
    traffic = PMC HBM bytes per launch of the same kernel (committed profile).
    """
    from rabbitsalign_amd.native import KERNEL_SYMBOLS
    sym = KERNEL_SYMBOLS[name]
    avg_s = k["ms"] * 1e-3 / k["launches"]
    per_launch_bytes = k["alg_bytes"] / k["launches"]
    traffic, src = pmc_traffic(sym)
    out = {"kernel": sym, "launches": k["launches"], "avg_launch_us": round(avg_s * 1e6, 3),
           "alg_bytes_per_launch": round(per_launch_bytes, 1), "traffic": traffic, "traffic_source": src}
    if name == "ext_scan" and ks.get("dp_cells_timed"):
        cells = ks["dp_cells_timed"] / k["launches"]
        achieved = cells / avg_s / 1e9
        out.update({"bound": "valu", "achieved": round(achieved, 2), "peak": round(DP_PEAK_GCELLS, 1),
                    "unit": "Gcells/s", "frac": round(achieved / DP_PEAK_GCELLS, 5),
                    "peak_source": "measured VALU issue cost (4.4 cycles a wave64 VOP3P instruction, "
                                   "profiles/r04/valu_issue.txt) x 5.75 packed instructions a cell",
                    "spec_model": {"peak": round(DP_SPEC_GCELLS, 1),
                                   "frac": round(achieved / DP_SPEC_GCELLS, 5)},
                    "cells_per_launch": round(cells, 1),
                    "hbm_GBps": round(per_launch_bytes / avg_s / 1e9, 3)})
        pm = scan_pmc(sym)
        if pm:
            # what the kernel as written issues: its VALU instructions per cell (PMC) times the
            # live cell rate, against the issue ceiling of its VOP3P / VOP2 instruction mix
            ipc, share = pm
            cyc = share * VOP3P_CYCLES + (1 - share) * VOP2_CYCLES
            ceiling = VALU_SIMDS * VALU_CLOCK / cyc
            issued = achieved * 1e9 * ipc
            out["valu_issue"] = {"wave_instr_per_cell": ipc, "vop3p_share": share,
                                 "achieved": round(issued / 1e9, 2), "peak": round(ceiling / 1e9, 1),
                                 "unit": "G wave64 VALU instr/s", "frac": round(issued / ceiling, 4),
                                 "cells_ceiling_Gcells": round(ceiling / ipc / 1e9, 1),
                                 "source": "profiles/r06/ext_pmc.json"}
    else:
        achieved = per_launch_bytes / avg_s / 1e9
        out.update({"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 6)})
        if name in KERNEL_LIMITER:
            out["limiter"] = KERNEL_LIMITER[name]
        if name == "lookup" and ks.get("query_randstrobes") and ks.get("seed_calls"):
            # its real currency: one random 128-B bucket line per query randstrobe, against the
            # measured rate of random line fetches, 8 lanes a line, on a 32 GB table
            lines = ks["query_randstrobes"] / ks["seed_calls"]
            got = lines / avg_s / 1e9
            out["line_fetch"] = {"lines_per_launch": round(lines, 1), "achieved": round(got, 3),
                                 "peak": LINE_PEAK_GLINES, "unit": "G lines/s",
                                 "frac": round(got / LINE_PEAK_GLINES, 5),
                                 "peak_source": "profiles/r05/line_probe.txt (mode 1, 32 GB table)"}
    return out


# what actually limits the kernels reported against HBM: their HBM
# fraction is shown for the bytes they must move, not as their ceiling
KERNEL_LIMITER = {
    "ext_band": "dependent-issue latency: one 16-lane group walks a job's band row by row (F prefix scan "
                "over DPP row_shr), 4 jobs a wave, < 2 waves per SIMD at chunk size",
    "ext_band_wide": "latency of the few (~3 a call) 64-lane jobs, one wave each",
    "sites": "latency of random reference windows (one read per NAM)",
    "lookup": "k_seed_query (randstrobes + lookup fused, one wave per read): xxh64 and the syncmer window in "
              "LDS, then random HBM lines, 8 lanes a line: one 128-B bucket line per query randstrobe (bounds "
              "+ up to 7 entries); their issue stalls on address translation (0.87 UTCL1 misses a line, the "
              "stall grows with the 32 GB table: profiles/r05/seed_table_size.txt)",
    "find_nams": "one wave per read, the NAM merge wave-parallel (ballots); robin_hood map inserts per run "
                 "of equal keys on one lane per orientation",
    "randstrobes": "one lane per read (reads over 512 bp only)",
    "rescue": "latency, rescued reads only",
    "ext_redo": "latency: the jobs (about one a call) whose word result the band path could not certify, "
                "re-run through the two-layout scan (one wave a job) and the band kernels in the call's stream",
}


def roofline(ks: dict, elapsed: float) -> dict:
    """Roofline object: the kernel with the largest device time over all calls (the dominant
    kernel), the extension scan (k_ext_scan_v, the path's compute kernel) beside it, the three
    largest kernels and the whole path's HBM view."""
    kern = {n: k for n, k in ks["kernels"].items() if k["launches"] and k["ms"] > 0}
    if not kern:
        return {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None, "traffic": None}
    # kernel times and alg_bytes cover the timed calls (one in RSA_KTIMER_EVERY per lane), and
    # the timed share differs between seeding and (combined) extension calls: scale each
    # kernel's to all calls before ranking
    from rabbitsalign_amd.native import EXT_KERNELS
    def scale(n):
        calls, timed = (("ext_calls", "ext_calls_timed") if n in EXT_KERNELS else ("seed_calls", "seed_calls_timed"))
        return ks.get(calls, 0) / max(1, ks.get(timed, 0))
    top = sorted(kern, key=lambda n: -kern[n]["ms"] * scale(n))
    # the headline kernel is the one with the largest device time over all calls of the
    # timed steps (the dominant kernel); the extension scan -- the path's compute kernel --
    # is reported beside it (`ext_scan`), and top_kernels keeps the ranking
    head = top[0]
    out = kernel_roofline(head, kern[head], ks)
    out["device_ms_all_calls"] = round(kern[head]["ms"] * scale(head), 3)
    if head != "ext_scan" and "ext_scan" in kern:
        out["ext_scan"] = dict(kernel_roofline("ext_scan", kern["ext_scan"], ks),
                               device_ms_all_calls=round(kern["ext_scan"]["ms"] * scale("ext_scan"), 3))
    out["top_kernels"] = [dict(kernel_roofline(n, kern[n], ks), device_ms_all_calls=round(kern[n]["ms"] * scale(n), 3))
                          for n in top[:3]]
    # whole path: the algorithmic bytes of every kernel of the timed steps / wall time
    reads = max(1, ks.get("reads", 0))
    alg = sum(k["alg_bytes"] * scale(n) for n, k in kern.items())
    path = {"alg_bytes_per_read": round(alg / reads, 1), "achieved": round(alg / elapsed / 1e9, 3),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(alg / elapsed / 1e9 / HBM_PEAK_GBS, 6)}
    # SURVEY.md §8d's B_alg with this run's counters: 32 n_q + 24 n_hit + L n_site + n_sw (L + t + 16)
    if ks.get("reads") and ks.get("jobs"):
        L = ks["read_bases"] / ks["reads"]
        n_q = ks["query_randstrobes"] / ks["reads"]
        n_hit = ks["hits"] / ks["reads"]
        n_site = ks["nams"] / ks["reads"]
        n_sw = ks["jobs"] / ks["reads"]
        t_bar = ks["dp_cells"] / max(1, ks["jobs"]) / max(1.0, L)
        b = 32 * n_q + 24 * n_hit + L * n_site + n_sw * (L + t_bar + 16)
        path["survey_formula"] = {"bytes_per_read": round(b, 1), "n_q": round(n_q, 2), "n_hit": round(n_hit, 2),
                                  "n_site": round(n_site, 2), "n_sw": round(n_sw, 4), "t_bar": round(t_bar, 1),
                                  "frac": round(b * reads / elapsed / 1e9 / HBM_PEAK_GBS, 6)}
    out["path"] = path
    return out


def file_xxh64(path: str) -> str:
    import xxhash
    h = xxhash.xxh64()
    with open(path, "rb") as f:
        while True:
            b = f.read(1 << 24)
            if not b:
                break
            h.update(b)
    return h.hexdigest()


def pick_io_dir(requested: str, need_bytes: int) -> str:
    """The bench's FASTQ/SAM directory: the one asked for, else the system temp dir
    (a disk file system's page cache) when it has room for `need_bytes`, else
    /dev/shm.  Writing one SAM file into the page cache runs at the speed of one
    writer (the file's inode lock); on the box that is ~5.5 GB/s on the disk file
    system and ~3.7 GB/s on tmpfs (scripts/write_bw.py)."""
    import tempfile
    if requested:
        return requested
    # the node's ranks write their files side by side: room for all of them
    need_bytes *= max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    for d in (tempfile.gettempdir(), "/dev/shm"):
        try:
            st = os.statvfs(d)
            if os.access(d, os.W_OK) and st.f_bavail * st.f_frsize > 1.5 * need_bytes:
                return d
        except OSError:
            continue
    return tempfile.gettempdir()


def write_shared_fastq(reads, f1, f2, tag, io_dir, rank, world, barrier):
    """N>1: the ranks' slices of one read set as ONE FASTQ pair.  Each rank formats its slice
    into part files, the part sizes are all-gathered, rank 0 sizes the shared files, and
    every rank copies its part to its offset (copy_file_range)."""
    import torch.distributed as dist
    mine = [os.path.join(io_dir, f"{tag}_slice_1.fq"), os.path.join(io_dir, f"{tag}_slice_2.fq") if f2 else None]
    reads.write_fastq(mine[0], mine[1])
    sizes = [os.path.getsize(p) if p else 0 for p in mine]
    every = [None] * world
    dist.all_gather_object(every, sizes)
    targets = [f1, f2]
    if rank == 0:
        for i, t in enumerate(targets):
            if t:
                with open(t, "wb") as f:
                    f.truncate(sum(e[i] for e in every))
    barrier()
    for i, (src, dst) in enumerate(zip(mine, targets)):
        if not src:
            continue
        off = sum(e[i] for e in every[:rank])
        with open(src, "rb") as a, open(dst, "r+b") as b:
            left, o_in, o_out = sizes[i], 0, off
            while left:
                n = os.copy_file_range(a.fileno(), b.fileno(), left, o_in, o_out)
                if n <= 0:
                    raise OSError(f"copy_file_range into {dst} stopped")
                left, o_in, o_out = left - n, o_in + n, o_out + n
        os.remove(src)
    barrier()


def files_concat_equal(paths, one) -> bool:
    """The files in `paths` back to back == `one`, byte for byte (streamed)."""
    if sum(os.path.getsize(p) for p in paths) != os.path.getsize(one):
        return False
    with open(one, "rb") as f:
        for p in paths:
            with open(p, "rb") as g:
                while True:
                    b = g.read(1 << 24)
                    if not b:
                        break
                    if f.read(len(b)) != b:
                        return False
    return True


def host_cpu() -> dict:
    """CPU model and NUMA layout of the box (cpu_baseline context)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nodes = {}
    base = "/sys/devices/system/node"
    try:
        for d in sorted(os.listdir(base)):
            if d.startswith("node") and d[4:].isdigit():
                with open(os.path.join(base, d, "cpulist")) as f:
                    nodes[d] = f.read().strip()
    except OSError:
        pass
    return {"cpu_model": model, "numa_nodes": nodes, "affinity_cpus": len(os.sched_getaffinity(0)),
            "machine_cpus": os.cpu_count()}


def kernel_table(ks: dict) -> dict:
    out = {}
    for name, k in ks["kernels"].items():
        if k["launches"]:
            out[name] = {"ms": round(k["ms"], 3), "launches": k["launches"],
                         "avg_us": round(1e3 * k["ms"] / k["launches"], 3),
                         "GBps_alg": round(k["alg_bytes"] / (k["ms"] * 1e-3) / 1e9, 3) if k["ms"] > 0 else None}
    return out


def self_launch(args) -> int:
    """--gpus N > 1 without WORLD_SIZE: start N ranks (torch.distributed.run, one process
    per GPU), relay rank 0's line, then run the product's one-process multi-device leg
    and report it beside the per-rank weak-scaling value."""
    from rabbitsalign_amd import launch
    me = os.path.abspath(__file__)
    n_vis = launch.visible_gpus()
    # RSA_BENCH_REHEARSE=1: rehearse the N-rank path on fewer GPUs (every rank on GPU 0, a
    # gloo process group since RCCL refuses two ranks on one device); the line says so
    rehearse = os.environ.get("RSA_BENCH_REHEARSE") == "1"
    if rehearse and n_vis >= 1:
        log(0, f"rehearsal: {args.gpus} ranks share GPU 0 (gloo process group); not a scaling measurement")
        os.environ.setdefault("RSA_BENCH_DEVICES", ",".join("0" * args.gpus))
    elif n_vis < args.gpus:
        log(0, f"error: {args.gpus} GPUs requested, {n_vis} visible; nothing was run")
        return 2
    log(0, f"launching {args.gpus} ranks (torch.distributed.run, one process per GPU)")
    argv = sys.argv[1:]
    rc, line = launch.run_ranks(me, argv, args.gpus)
    if rc != 0 or line is None:
        log(0, f"error: the ranks exited with {rc}" + ("" if line else " and printed no result line"))
        return rc or 1
    if not args.no_multi_device:
        log(0, f"multi-device leg: one process, rsam_add_devices over {args.gpus} GPUs, one SAM file")
        # bounded: the rank leg's line is already in hand and must come out whatever this leg does
        md_timeout = float(os.environ.get("RSA_BENCH_MD_TIMEOUT", "600"))
        rc2, md = launch.run_child([sys.executable, me, "--multi-device-leg", *argv], timeout=md_timeout)
        line["multi_device"] = (md or {}).get("multi_device") if rc2 == 0 and md else \
            {"error": f"multi-device leg exited with {rc2}"}
    print(json.dumps(line), flush=True)
    return 0


def multi_device_leg(args) -> int:
    """The product's own multi-GPU path (rsalign --devices 0..N-1 / rsam_add_devices): one
    process, one chunk queue, one engine per GPU (index replica each), ONE ordered SAM
    file.  Each step maps N x --pairs pairs (the same per-GPU work as the rank leg) from
    FASTQ files to one SAM file.  Prints {"multi_device": {...}}."""
    wl = dict(WORKLOADS[args.workload])
    if args.ref_len:
        wl["ref_len"] = args.ref_len
    env_dev = os.environ.get("RSA_BENCH_DEVICES")           # e.g. "0,0": rehearse on one GPU
    devices = [int(x) for x in env_dev.split(",")] if env_dev else list(range(args.gpus))
    cores = host_cores(False)
    threads = args.threads or min(16 * len(devices), cores)
    import torch
    from rabbitsalign_amd import mapper as M
    M.load()
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (the product path has no CPU fallback)")
    t = time.time()
    m = M.Mapper.synthetic(args.ref_seed, wl["ref_len"], wl["n_contigs"], wl["read_len"], device=devices[0],
                           threads=threads)
    t_idx = time.time() - t
    t = time.time()
    m.add_devices(devices[1:])
    t_add = time.time() - t
    log(0, f"multi-device: index on device {devices[0]} in {t_idx:.1f} s, replicated to {devices[1:]} in "
           f"{t_add:.1f} s; engine {m.engine}; {threads} pipeline threads of {cores} cores")
    P = args.pairs * len(devices)
    reads = m.synthetic_reads(args.read_seed, 0, P, wl["read_len"], wl["mu"], wl["sigma"], wl["paired"])
    per_pair = (2 if wl["paired"] else 1)
    io_dir = pick_io_dir(args.io_dir, P * per_pair * (2 * wl["read_len"] + 80) * 2
                         + 2 * P * per_pair * (2 * wl["read_len"] + 120))
    tag = f"rsa_bench_md_{os.getpid()}"
    f1 = os.path.join(io_dir, f"{tag}_1.fq")
    f2 = os.path.join(io_dir, f"{tag}_2.fq") if wl["paired"] else None
    reads.write_fastq(f1, f2)
    reads.close()
    steps = max(1, args.md_steps)
    warm = os.path.join(io_dir, f"{tag}_warm.sam")
    sam = os.path.join(io_dir, f"{tag}_step.sam")
    out = {}
    try:
        w = m.map_files(f1, f2, threads=threads, chunk_size=args.chunk_size, sam_path=warm)
        log(0, f"multi-device warmup: {w.n_reads} reads in {w.map_seconds:.3f} s")
        warm_hash = file_xxh64(warm)
        m.set_sam_digest(False)
        m.reset_kernel_stats()
        walls, n_reads, identical = [], 0, True
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        for s in range(steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st = m.map_files(f1, f2, threads=threads, chunk_size=args.chunk_size, sam_path=sam)
            walls.append(time.perf_counter() - t0)
            n_reads += st.n_reads
            log(0, f"multi-device step {s}: {st.n_reads} reads in {walls[-1]:.3f} s "
                   f"({st.n_reads / walls[-1] / 1e6:.3f} Mreads/s)")
            identical = identical and file_xxh64(sam) == warm_hash      # untimed
            os.remove(sam)
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        ks = m.kernel_stats()
        elapsed = sum(walls)
        cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
        out = {"value": round(n_reads / elapsed / 1e6, 6), "unit": "Mreads/s", "devices": devices,
               "steps": steps, "ms_per_step": round(1e3 * elapsed / steps, 3), "pairs_per_step": P,
               "sam_file_bytes_per_step": w.sam_bytes,
               "sam_write_GBps": round(w.sam_bytes * steps / elapsed / 1e9, 3),
               "host_threads": threads, "host_cores": cores,
               "core_us_per_read": round(1e6 * cpu_s / max(1, n_reads), 4),
               "timed_files_identical_to_warmup": identical,
               "engine": m.engine, "index_replicate_seconds": round(t_add, 3),
               "calls": {"seed": ks.get("seed_calls"), "extend": ks.get("ext_calls")},
               "note": "product path: one process, rsam_add_devices (csrc/host/multi.cpp), one chunk queue, "
                       "one ordered SAM file; FASTQ files -> SAM file, timed per step from the call to the "
                       "last SAM byte (steps run back to back; each step's SAM file checked untimed)"}
    finally:
        for f in (f1, f2, warm, sam):
            if f and os.path.exists(f):
                os.remove(f)
        m.close()
    print(json.dumps({"multi_device": out}), flush=True)
    return 0


class _NoTorch:
    """the few torch calls of a 1-GPU run, without torch (RSA_BENCH_NO_TORCH=1)"""
    class cuda:
        @staticmethod
        def is_available():
            return True          # the mapper's open fails loudly without a GPU

        @staticmethod
        def set_device(d):
            pass                 # the device goes to the mapper explicitly

        @staticmethod
        def synchronize():
            pass                 # mapping calls return after their device work

    @staticmethod
    def device(*a):
        return None


def ab_run(args, m, map_step, sam_paths, n_sets, threads) -> int:
    """--ab: alternate environment settings of the host pipeline over the same read sets
    (streamed FASTQ -> SAM file, as the headline), --ab-steps steps per setting per round;
    per setting: every step's Mreads/s, the first chunk's extension bounds and the time the
    first SAM text reached the writer.  Settings are read per mapping call."""
    settings = [dict(kv.split("=", 1) for kv in grp.split(",") if kv) for grp in args.ab.split("|")]
    res = {i: {"env": st, "mreads_s": [], "first_ext_ms": [], "first_out_ms": [], "core_us_per_read": [],
               "kern": {}}
           for i, st in enumerate(settings)}
    kern_names = ("ext_scan", "ext_band", "lookup", "find_nams", "sites")
    base = {k: os.environ.get(k) for st in settings for k in st}
    s = args.warmup
    for r in range(args.ab_rounds):
        for i, st in enumerate(settings):
            for k, v in base.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            os.environ.update(st)
            m.reset_kernel_stats()
            for _ in range(args.ab_steps):
                idx = args.warmup + (s % max(1, args.steps))
                ru0 = resource.getrusage(resource.RUSAGE_SELF)
                x = map_step(idx)
                ru1 = resource.getrusage(resource.RUSAGE_SELF)
                cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
                res[i]["mreads_s"].append(round(x.n_reads / x.map_seconds / 1e6, 3))
                res[i]["first_ext_ms"].append([round(1e3 * x.t_first_ext_begin, 1), round(1e3 * x.t_first_ext_end, 1)])
                res[i]["first_out_ms"].append(round(1e3 * x.t_first_out, 1))
                res[i]["core_us_per_read"].append(round(1e6 * cpu / max(1, x.n_reads), 3))
                if os.path.exists(sam_paths[idx]):
                    os.remove(sam_paths[idx])
                s += 1
            ks = m.kernel_stats()
            for kn in kern_names:
                k = ks["kernels"].get(kn)
                if k:
                    acc = res[i]["kern"].setdefault(kn, {"ms": 0.0, "launches": 0})
                    acc["ms"] += k["ms"]
                    acc["launches"] += k["launches"]
            res[i]["kern"].setdefault("dp_cells", 0)
            res[i]["kern"]["dp_cells"] += ks.get("dp_cells_timed", 0)
    for v in res.values():
        kk = v["kern"]
        for kn in kern_names:
            if kn in kk:
                kk[kn]["us_per_launch"] = round(1e3 * kk[kn]["ms"] / max(1, kk[kn]["launches"]), 1)
        if "ext_scan" in kk and kk["ext_scan"]["ms"] > 0:
            kk["scan_gcells_s"] = round(kk["dp_cells"] / (kk["ext_scan"]["ms"] * 1e-3) / 1e9, 1)
        xs = sorted(v["mreads_s"])
        v["median"] = xs[len(xs) // 2]
        v["mean"] = round(sum(xs) / len(xs), 3)
    print(json.dumps({"ab": list(res.values()), "steps_each": args.ab_steps, "rounds": args.ab_rounds,
                      "threads": threads}), flush=True)
    m.close()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--workload", default="pe150_3g", choices=sorted(WORKLOADS))
    ap.add_argument("--pairs", type=int, default=1_000_000,
                    help="pairs (SE: reads) per step per GPU (SURVEY.md §8d: 10^6 pairs per config)")
    ap.add_argument("--threads", type=int, default=0,
                    help="host pipeline threads (0: one per host core, max 64; r9: 16 beat 24 on 16 cores)")
    ap.add_argument("--chunk-size", type=int, default=10000)
    ap.add_argument("--ref-seed", type=int, default=1)
    ap.add_argument("--read-seed", type=int, default=7)
    ap.add_argument("--cpu-pairs", type=int, default=2_000_000,
                    help="cpu_baseline sample (pairs; ~10 s of CPU work on 16 cores at 2x150)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--io-dir", default="",
                    help="where the FASTQ inputs and the SAM output go (default: the system temp dir when it "
                         "has room, else /dev/shm)")
    ap.add_argument("--read-sets", type=int, default=3,
                    help="distinct synthetic read sets (FASTQ file pairs) rotated over the steps")
    ap.add_argument("--ref-len", type=int, default=0, help="override reference length (testing only)")
    ap.add_argument("--stats-out", default="", help="write per-kernel stats JSON here")
    ap.add_argument("--no-multi-device", action="store_true",
                    help="N>1: skip the product's one-process multi-device leg (one SAM file over N GPUs)")
    ap.add_argument("--md-steps", type=int, default=3, help="timed steps of the multi-device leg")
    ap.add_argument("--multi-device-leg", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--ab", default="",
                    help="measurement mode (1 GPU): 'K=V,K2=V2|K=V3' -- environment settings of the host pipeline "
                         "run alternately after the warm-up, --ab-steps steps each, --ab-rounds times; prints one "
                         "{\"ab\": ...} line instead of the headline")
    ap.add_argument("--ab-rounds", type=int, default=3)
    ap.add_argument("--ab-steps", type=int, default=4)
    args = ap.parse_args()

    if os.environ.get("RSA_MAPS_OUT"):
        # diagnostics: the process's mappings as Python exits (before the C-level
        # destructors run), to attribute addresses in an exit-time native stack trace
        import atexit

        def _dump_maps(path=os.environ["RSA_MAPS_OUT"]):
            with open("/proc/self/maps") as src, open(path, "w") as dst:
                dst.write(src.read())
        atexit.register(_dump_maps)

    if args.multi_device_leg:
        return multi_device_leg(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python3 bench.py --gpus N` (the driver's form): this process is the launcher,
        # not a rank, and never initialises the GPU
        raise SystemExit(self_launch(args))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(rank, f"note: WORLD_SIZE={world} but --gpus {args.gpus}; using WORLD_SIZE")
    wl = dict(WORKLOADS[args.workload])
    if args.ref_len:
        wl["ref_len"] = args.ref_len
    local_world = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    pinned = pin_rank_cpus(local_rank, local_world)
    cores = host_cores(pinned is not None)
    threads = args.threads or min(64, cores)

    # torch first: its libamdhip64 (soname libamdhip64.so.7) is then the one
    # runtime of the process and librsa_gpu.so binds to it; loading ours first
    # would put two HIP runtimes in one process (torch needs "libamdhip64.so").
    # RSA_BENCH_NO_TORCH=1 (N=1, profiling runs): no torch at all, so the process has
    # the system ROCm's runtime only -- the one rocprofv3's tool library uses.  With
    # torch's bundled HSA runtime beside it, the tool's exit-time finalisation under
    # --memory-copy-trace touches GPU mappings the other runtime's teardown removed
    # (profiles/r06/exit_abort.txt).  A mapping call returns after its
    # device work, so torch.cuda.synchronize has nothing to wait for at N=1.
    if os.environ.get("RSA_BENCH_NO_TORCH") == "1" and world == 1:
        torch, dist = _NoTorch(), None
    else:
        import torch
        import torch.distributed as dist
    from rabbitsalign_amd import mapper as M
    from rabbitsalign_amd import shard
    M.load()

    has_gpu = torch.cuda.is_available()
    if not has_gpu:
        raise SystemExit("bench.py needs a GPU (the product path has no CPU fallback)")
    rehearse = os.environ.get("RSA_BENCH_REHEARSE") == "1"
    device = 0 if rehearse else local_rank
    torch.cuda.set_device(device)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    def barrier():
        if world > 1:
            dist.barrier()

    t = time.time()
    log(rank, f"building {wl['ref_len']/1e9:.3f} Gb reference ({wl['n_contigs']} contigs) + index; "
              f"host cores for this rank {cores}, pipeline threads {threads}")
    m = M.Mapper.synthetic(args.ref_seed, wl["ref_len"], wl["n_contigs"], wl["read_len"], device=device,
                           threads=threads)
    info = m.info()
    log(rank, f"index ready in {time.time()-t:.1f} s: {info['n_randstrobes']} randstrobes, bits {info['bits']}, "
              f"built on {'GPU' if info['index_on_device'] else 'host'} in {info['index_seconds']:.2f} s "
              f"(device phases ms {info['index_device_ms']}), upload {info['upload_seconds']:.2f} s, engine {m.engine}")

    P = args.pairs
    total_steps = args.warmup + args.steps
    # distinct read sets, rotated over the steps (each step maps one whole set)
    # at most one read set per warm-up step, so every set has a warm-up SAM digest the timed
    # steps and the in-memory leg are compared with
    n_sets = max(1, min(total_steps, args.read_sets, args.warmup))
    batches = []
    t = time.time()
    for s in range(n_sets):
        # set s holds pairs [s*world*P, (s+1)*world*P) of the synthetic stream; this rank generates
        # (and, at N>1, writes into the shared files) its slice, which its part maps
        first = shard.shared_set_first(s, rank, world, P)
        batches.append(m.synthetic_reads(args.read_seed, first, P, wl["read_len"], wl["mu"], wl["sigma"],
                                         wl["paired"]))
    log(rank, f"generated {n_sets} x {P} {'pairs' if wl['paired'] else 'reads'} in {time.time()-t:.1f} s")

    # the headline: FASTQ files -> SAM file, reads streamed while mapping, timed from the
    # call to the last SAM byte written (the reference's consumer cost, main.cpp:446,595).
    # The FASTQ files are written once before timing (page cache warm, as a re-run of a
    # mapper over the same files would find them); every step truncates and rewrites its SAM.
    io_dir = pick_io_dir(args.io_dir, n_sets * P * (2 if wl["paired"] else 1) * (2 * wl["read_len"] + 80)
                         + max(args.steps, args.warmup) * P * (2 if wl["paired"] else 1) * (2 * wl["read_len"] + 120))
    # one tag for the whole job (the ranks share the FASTQ files): rank 0's pid, broadcast
    job = [os.getpid()]
    if world > 1:
        dist.broadcast_object_list(job, src=0)
    tag = f"rsa_bench_{job[0]}"
    fqs = []
    t = time.time()
    for s, b in enumerate(batches):
        f1 = os.path.join(io_dir, f"{tag}_s{s}_1.fq")
        f2 = os.path.join(io_dir, f"{tag}_s{s}_2.fq") if wl["paired"] else None
        if world == 1:
            b.write_fastq(f1, f2)
        else:
            write_shared_fastq(b, f1, f2, f"{tag}_r{rank}", io_dir, rank, world, barrier)
        fqs.append((f1, f2))
    # every step writes a SAM file of its own (a new file, as a mapping run makes one; at N>1
    # the rank's part); the files are removed after the timed region
    sam_paths = [os.path.join(io_dir, f"{tag}_r{rank}_step{s}.sam") for s in range(total_steps)]
    fq_bytes = sum(os.path.getsize(f) for pair in fqs for f in pair if f)
    log(rank, f"{'wrote' if world == 1 else 'wrote shared'} {n_sets} FASTQ sets ({fq_bytes / 1e9:.2f} GB) to "
              f"{io_dir} in {time.time()-t:.1f} s")

    parts = {}
    def map_step(s):
        f1, f2 = fqs[s % n_sets]
        if world == 1:
            return m.map_files(f1, f2, threads=threads, chunk_size=args.chunk_size, sam_path=sam_paths[s])
        # rank/world mode: the plan (newline counts of this rank's 1/N of each file, all-gathered
        # over RCCL) is part of the step, then this rank's chunks -> its SAM part
        part = shard.plan_shared_input(f1, f2, args.chunk_size, threads, device="cpu" if rehearse else "cuda")
        parts[s % n_sets] = part.as_dict()
        return m.map_files_part(f1, f2, part, threads=threads, sam_path=sam_paths[s])

    def drop_sams(upto, keep=()):
        for f in sam_paths[:upto]:
            if f not in keep and os.path.exists(f):
                os.remove(f)

    try:
        # warm-up steps with the SAM digest (the in-memory leg and the CPU path are compared
        # with it); the timed steps without it, as a mapping run has no use for one -- their
        # SAM files are checked against the warm-up files of the same read set after timing
        set_hash, set_file = {}, {}
        for s in range(args.warmup):
            st = map_step(s)
            log(rank, f"warmup {s}: {st.n_reads} reads in {st.map_seconds:.3f} s")
            if s % n_sets not in set_hash:
                set_hash[s % n_sets] = st.sam_hash
                set_file[s % n_sets] = sam_paths[s]
        drop_sams(args.warmup, keep=set(set_file.values()))
        m.reset_kernel_stats()
        m.set_sam_digest(False)
        if args.ab and world == 1:
            return ab_run(args, m, map_step, sam_paths, n_sets, threads)

        barrier()
        torch.cuda.synchronize()
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        t0 = time.perf_counter()
        n_reads = 0
        totals = {f: 0 for f in shard.STAT_FIELDS}
        hashes = []
        sam_file_bytes = 0
        for s in range(args.warmup, total_steps):
            st = map_step(s)
            n_reads += st.n_reads
            for f in shard.STAT_FIELDS:
                totals[f] += getattr(st, f)
            sam_file_bytes = os.path.getsize(sam_paths[s])
            log(rank, f"step {s - args.warmup}: {st.n_reads} reads in {st.map_seconds:.3f} s "
                      f"({st.n_reads / st.map_seconds / 1e6:.4f} Mreads/s), SW {st.sw_calls}; thread-s: "
                      f"seed {st.t_seed:.2f} extend {st.t_extend:.2f} part {st.t_part:.2f} "
                      f"collect {st.t_collect:.2f} last {st.t_last:.2f}; sequential phase {st.t_sequential:.3f} s "
                      f"(chunk 0 seeded at {st.t_first_seeded:.3f} s), last chunk: finish {st.t_last_start:.3f} s, "
                      f"SAM out {st.t_last_put:.3f} s; workers done {st.t_workers_done:.3f} s; first chunk "
                      f"extension {st.t_first_ext_begin * 1e3:.1f}-{st.t_first_ext_end * 1e3:.1f} ms, first SAM "
                      f"text to the writer {st.t_first_out * 1e3:.1f} ms"
                      + (f", replayed chunks {st.replayed_chunks}" if st.replayed_chunks else ""))
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        ks = m.kernel_stats()
        m.set_sam_digest(True)
        # untimed: every timed step's SAM file == the warm-up file of its read set
        file_hash = {}
        def fhash(path):
            if path not in file_hash:
                file_hash[path] = file_xxh64(path)
            return file_hash[path]
        checked = [s for s in range(args.warmup, total_steps) if s % n_sets in set_file]
        timed_files_identical = all(fhash(sam_paths[s]) == fhash(set_file[s % n_sets])
                                    for s in checked) if checked else None
        hashes = [set_hash.get(s % n_sets, 0) for s in range(args.warmup, total_steps)]
        # N>1, untimed: header + every rank's part of read set 0 (its warm-up files) == one
        # process mapping the whole shared input (rank 0, rsam_map_files)
        parts_parity = None
        if world > 1 and 0 in set_file:
            paths = [None] * world
            dist.all_gather_object(paths, set_file[0])
            if rank == 0:
                one = os.path.join(io_dir, f"{tag}_one.sam")
                f1, f2 = fqs[0]
                o = m.map_files(f1, f2, threads=threads, chunk_size=args.chunk_size, sam_path=one)
                parts_parity = {"parts_equal_one_process": files_concat_equal(paths, one),
                                "one_process_reads": o.n_reads, "one_process_sam_bytes": os.path.getsize(one),
                                "read_set": 0, "plan": parts.get(0)}
                os.remove(one)
                log(rank, f"parts of set 0 concatenated == one-process SAM: {parts_parity['parts_equal_one_process']}")
            barrier()
    finally:
        barrier()
        if rank == 0:
            for pair in fqs:
                for f in pair:
                    if f and os.path.exists(f):
                        os.remove(f)
        drop_sams(total_steps)
    # host CPU time of this rank's timed steps (all threads, user + system): the
    # host-bound part of the path, steadier than wall-time throughput on a shared box
    host_cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)

    # the run's only collective: max wall time and summed statistics over ranks (RCCL)
    elapsed_max, totals_all = shard.reduce_run(elapsed, totals, device="cuda")
    reads_all = float(totals_all["n_reads"])

    # in-memory leg (every rank, after the headline): reads resident in host RAM, SAM
    # text kept in memory -- the mapping alone, without FASTQ parsing or the SAM file
    barrier()
    ru2 = resource.getrusage(resource.RUSAGE_SELF)
    t2 = time.perf_counter()
    mem_reads = 0
    mem_hashes = []
    for s in range(args.warmup, total_steps):
        st = m.map(batches[s % n_sets], threads=threads, chunk_size=args.chunk_size)
        mem_reads += st.n_reads
        mem_hashes.append(st.sam_hash)
    barrier()
    mem_elapsed = time.perf_counter() - t2
    ru3 = resource.getrusage(resource.RUSAGE_SELF)
    mem_elapsed_max, mem_tot = shard.reduce_run(mem_elapsed, {"n_reads": mem_reads}, device="cuda")
    mem_cpu_s = (ru3.ru_utime - ru2.ru_utime) + (ru3.ru_stime - ru2.ru_stime)
    in_memory = {"value": round(mem_tot["n_reads"] / mem_elapsed_max / 1e6, 6), "unit": "Mreads/s",
                 "ms_per_step": round(1e3 * mem_elapsed_max / args.steps, 3),
                 "core_us_per_read": round(1e6 * mem_cpu_s / max(1, mem_reads), 4),
                 # steps whose read set had a warm-up step (its digest is the headline's reference);
                 # None when no step could be compared
                 "sam_identical_to_headline": (all(mh == h for mh, h in zip(mem_hashes, hashes) if h)
                                               if any(hashes) else None),
                 "sam_compared_steps": sum(1 for h in hashes if h),
                 "note": "the same read sets held in host RAM (rsam_map), SAM text kept in memory"}
    log(rank, f"in-memory leg: {in_memory['value']} Mreads/s, {in_memory['core_us_per_read']} core-us a read")
    for b in batches:
        b.close()

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if os.path.exists(REF_CPU_LIB):
            # the same timeline as the headline (FASTQ files streamed -> SAM file) on a bounded
            # sample; the GPU path maps the same files and both SAM digests must agree
            n_cpu = args.cpu_pairs
            sample = m.synthetic_reads(args.read_seed, 0, n_cpu, wl["read_len"], wl["mu"], wl["sigma"], wl["paired"])
            cf1 = os.path.join(io_dir, f"{tag}_cpu_1.fq")
            cf2 = os.path.join(io_dir, f"{tag}_cpu_2.fq") if wl["paired"] else None
            csam = os.path.join(io_dir, f"{tag}_cpu.sam")
            try:
                sample.write_fastq(cf1, cf2)
                sample.close()
                g = m.map_files(cf1, cf2, threads=threads, chunk_size=args.chunk_size, sam_path=csam)
                log(rank, f"cpu_baseline: opening CPU path on the same index ({cores} cores)")
                cm = m.like(device=0, threads=cores, lib_path=REF_CPU_LIB)
                c = cm.map_files(cf1, cf2, threads=cores, chunk_size=args.chunk_size, sam_path=csam)
                cm.close()
            finally:
                for f in (cf1, cf2, csam):
                    if f and os.path.exists(f):
                        os.remove(f)
            per_core = c.n_reads / c.map_seconds / cores
            cpu = {"value": round(c.n_reads / c.map_seconds / 1e6, 6), "unit": "Mreads/s", "cores": cores,
                   "kind": "reference", "host": host_cpu(),
                   "reads_per_s_per_core": round(per_core, 1),
                   "vs_survey_probe_per_core": {
                       "probe": 21000, "ratio": round(per_core / 21000, 3), "within_25pct": abs(per_core / 21000 - 1) <= 0.25,
                       "note": "SURVEY.md §8d probe: the reference binary, 0.167 Mreads/s on 8 vCPU, 2x150 @ 250 Mb, "
                               "another CPU. This CPU path is the reference's own seeding/SSW objects inside the "
                               "restated host pipeline (pooled buffers, one reverse complement a read, SIMD "
                               "Hamming): per core it is faster than the reference's own pipeline, i.e. a "
                               "stronger baseline"},
                   "sample": f"{n_cpu} {'pairs' if wl['paired'] else 'reads'} of the same workload "
                             f"({c.n_reads} reads, {c.map_seconds:.2f} s wall), FASTQ files -> SAM file as the "
                             f"headline, -t {cores}, chunk {args.chunk_size}; reference randstrobes/nam/ssw.c "
                             "objects + restated host pipeline"}
            parity = {"sample_reads": c.n_reads, "sam_bytes": c.sam_bytes, "gpu_sam_hash": f"{g.sam_hash:016x}",
                      "cpu_sam_hash": f"{c.sam_hash:016x}", "sam_identical": g.sam_hash == c.sam_hash
                      and g.sam_bytes == c.sam_bytes}
            log(rank, f"cpu_baseline {cpu['value']} Mreads/s; SAM identical on sample: {parity['sam_identical']}")
        else:
            log(rank, f"cpu_baseline skipped: {REF_CPU_LIB} not built")

    if rank == 0:
        value = reads_all / elapsed_max / 1e6
        rl = roofline(ks, elapsed_max)
        line = {
            "metric": "Mreads/s aligned (PE 2x150 vs 3 Gb, SAM bit-exact vs CPU)" if args.workload == "pe150_3g"
            else f"Mreads/s aligned ({args.workload})",
            "value": round(value, 6), "unit": "Mreads/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed_max / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            # the DP's arithmetic: exact small integers in packed f16 (forward scan) and int32
            # (reverse pass, band traceback); hashing and lookups in 64-bit integers
            "dtype": "int: exact integers in packed f16x2 (SSW scan) and int32 (bands, seeding)",
            "data": "synthetic (seeded reference + reads, SURVEY.md Appendix D)",
            "config": {"workload": wl["desc"], "reference_bp": wl["ref_len"], "contigs": wl["n_contigs"],
                       "read_len": wl["read_len"], "paired": wl["paired"], "pairs_per_step_per_gpu": P,
                       "host_threads": threads, "host_cpus_pinned": len(pinned) if pinned else None,
                       "chunk_size": args.chunk_size, "index_bits": info["bits"],
                       "randstrobes": info["n_randstrobes"], "parallelism": f"dp{world} (replicated index)"},
            "index_build": {"on": "gpu" if info["index_on_device"] else "host",
                            "seconds": round(info["index_seconds"], 3), "device_ms": info["index_device_ms"],
                            "replayed_segments": info["index_replayed_segments"],
                            "position_ties": info["index_position_ties"],
                            "ms_tie_replay": round(info["index_ms_tie_replay"], 1),
                            "note": "StrobemerIndex::populate (index.cpp:141-309) via rsa_index_build_run; the "
                                    "index stays in HBM and the engine adopts it (rsa_open_built)"},
            "roofline": rl,
            **({"rehearsal": "RSA_BENCH_REHEARSE=1: every rank on GPU 0 with a gloo process group -- "
                             "exercises the N-rank path, not a scaling measurement"} if rehearse else {}),
            "cpu_baseline": cpu,
            "in_memory": in_memory,
            "io": {"dir": io_dir, "fastq_bytes_per_set": fq_bytes // n_sets, "read_sets": n_sets,
                   "sam_file_bytes_per_step": sam_file_bytes,
                   "note": "value = FASTQ files -> SAM file (rsam_map_files: reads streamed by a reader "
                           "thread per file while mapping); FASTQ in the page cache, SAM rewritten each step"},
            "parity": parity if world == 1 else parts_parity,
            **({"shared_input": {"pairs_per_step": P * world, "plan_rank0": parts.get(0),
                                 "note": "every rank maps its chunks of ONE FASTQ pair (rsam_map_files_part); the "
                                         "plan's newline counts are all-gathered over RCCL inside the timed step"}}
               if world > 1 else {}),
            "kernels": kernel_table(ks),
            "device_counters": {k: v for k, v in ks.items() if k != "kernels"},
            "host_cpu": {"cpu_s_per_step": round(host_cpu_s / args.steps, 4),
                         "core_us_per_read": round(1e6 * host_cpu_s / max(1, n_reads), 4),
                         "sys_fraction": round((ru1.ru_stime - ru0.ru_stime) / max(1e-9, host_cpu_s), 4),
                         "cores_per_rank": cores,
                         "note": "rank 0 process CPU time (getrusage) over the timed steps; cores_per_rank = "
                                 "the host CPUs each rank's pipeline may use (affinity / cgroup share)"},
            "mapping_stats_all_ranks": totals_all,
            "sam_hashes": [f"{h:016x}" for h in hashes],
            "sam_check": {"timed_files_identical_to_warmup": timed_files_identical,
                          "compared_steps": len(checked),
                          "note": "timed steps run without the SAM digest (rsam_set_sam_digest 0: a mapping run "
                                  "computes none); each timed step's SAM file is compared (xxh64 of the file, "
                                  "untimed) with the warm-up file of the same read set, whose digest is the one "
                                  "sam_hashes, in_memory and parity compare"},
        }
        if args.stats_out:
            with open(args.stats_out, "w") as f:
                json.dump({"kernel_stats": ks, "info": info, "line": line}, f, indent=1)
        print(json.dumps(line), flush=True)
    m.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
