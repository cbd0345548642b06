"""Read-chunk sharding across GPUs.

Every rank holds a full replica of the index and maps its own pairs, so the
data path has no collective.  The only exchanges are the end-of-run reductions
below -- the analogue of the reference summing its per-thread
AlignmentStatistics (src/main.cpp:597-600) -- over torch.distributed (RCCL on
GPUs, gloo in the CPU tests).
"""
from __future__ import annotations

STAT_FIELDS = ("n_reads", "sam_bytes", "sw_calls", "tried", "nam_rescue", "mate_rescue", "inconsistent")


def plan_shared_input(fq1, fq2, chunk_size: int, threads: int, device="cpu", lib_path=None):
    """This rank's part of ONE input pair mapped by every rank (rsam_part_*):
    each rank counts the newlines of its own 1/world of each file, the counts are
    all-gathered (world * 64 integers per file, the only exchange before mapping), and
    the plan follows.  Without a process group: the whole input as one part."""
    import torch
    import torch.distributed as dist
    from . import mapper
    kw = {"lib_path": lib_path} if lib_path else {}
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return mapper.part_plan(fq1, fq2, 0, 1, chunk_size, None, None, threads, **kw)
    rank, world = dist.get_rank(), dist.get_world_size()
    files = [f for f in (fq1, fq2) if f]
    mine = torch.tensor([c for f in files for c in mapper.part_count(f, rank, world, threads, **kw)],
                        dtype=torch.int64, device=device)
    got = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(got, mine)
    rows = [g.cpu().tolist() for g in got]
    B = mapper.PART_BLOCKS
    counts = [[c for r in rows for c in r[i * B:(i + 1) * B]] for i in range(len(files))]
    return mapper.part_plan(fq1, fq2, rank, world, chunk_size, counts[0], counts[1] if fq2 else None, threads, **kw)


def shared_set_first(read_set: int, rank: int, world: int, pairs_per_rank: int) -> int:
    """First synthetic pair of rank `rank`'s slice of read set `read_set`: set s is pairs
    [s*world*P, (s+1)*world*P), written as ONE FASTQ pair with the ranks' slices in rank
    order, so rank r's part (chunks [r*C/W, (r+1)*C/W) when P is a multiple of the chunk
    size) is exactly its slice."""
    return (read_set * world + rank) * pairs_per_rank


def first_pair(rank: int, step: int, total_steps: int, pairs_per_step: int) -> int:
    """Index of the first synthetic pair rank `rank` maps in step `step`.
    Ranges of different (rank, step) never overlap."""
    return (rank * total_steps + step) * pairs_per_step


def _reduce(values, op, device):
    import sys
    if "torch" not in sys.modules:       # no torch, no process group (a 1-GPU run without torch)
        return list(values)
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return list(values)
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=op)
    return [float(x) for x in t.tolist()]


def reduce_run(elapsed_s: float, stats: dict, device="cpu") -> tuple[float, dict]:
    """Max wall time over ranks and the sum of every counter in `stats`."""
    import sys
    if "torch" not in sys.modules:
        return elapsed_s, {k: int(round(float(v))) for k, v in stats.items()}
    import torch.distributed as dist
    (wall,) = _reduce([elapsed_s], dist.ReduceOp.MAX, device)
    keys = sorted(stats)
    summed = _reduce([float(stats[k]) for k in keys], dist.ReduceOp.SUM, device)
    return wall, {k: int(round(v)) for k, v in zip(keys, summed)}


def rank_cpu_groups(node_cpus, siblings, local_world):
    """Host CPUs of each of the `local_world` ranks of a node.

    node_cpus: per NUMA node, the CPUs this process may use; siblings: cpu ->
    tuple of its SMT siblings.  Ranks spread over the nodes in order (rank r on
    node r * n_nodes // local_world, matching the usual GPU numbering of a
    two-socket node), and each node's physical cores -- siblings kept together --
    are split into contiguous runs among its ranks, so no two ranks share a core
    and each rank's cores share its node's memory and last-level caches."""
    nodes = [sorted(c) for c in node_cpus if c]
    if not nodes or local_world < 1:
        return [[] for _ in range(max(local_world, 0))]
    n = len(nodes)
    on_node = [[r for r in range(local_world) if r * n // local_world == k] for k in range(n)]
    groups = [[] for _ in range(local_world)]
    for k, cpus in enumerate(nodes):
        ranks = on_node[k]
        if not ranks:
            continue
        allowed = set(cpus)
        cores, seen = [], set()
        for c in cpus:                               # physical cores in CPU order
            if c in seen:
                continue
            core = tuple(sorted(s for s in siblings.get(c, (c,)) if s in allowed)) or (c,)
            seen.update(core)
            cores.append(core)
        for j, r in enumerate(ranks):
            a = j * len(cores) // len(ranks)
            b = (j + 1) * len(cores) // len(ranks)
            groups[r] = sorted(c for core in cores[a:b] for c in core)
    # a node with more ranks than cores leaves some ranks empty: they share the node's CPUs
    for k, cpus in enumerate(nodes):
        for r in on_node[k]:
            if not groups[r]:
                groups[r] = sorted(cpus)
    return groups


def _parse_cpulist(s):
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def host_topology(allowed):
    """(node_cpus, siblings) of this machine from sysfs, restricted to `allowed`."""
    import glob
    allowed = set(allowed)
    node_cpus = []
    for path in sorted(glob.glob("/sys/devices/system/node/node[0-9]*/cpulist"),
                       key=lambda p: int(p.split("/node")[-1].split("/")[0])):
        with open(path) as f:
            node_cpus.append([c for c in _parse_cpulist(f.read()) if c in allowed])
    if not any(node_cpus):
        node_cpus = [sorted(allowed)]
    siblings = {}
    for c in allowed:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                siblings[c] = tuple(_parse_cpulist(f.read()))
        except OSError:
            siblings[c] = (c,)
    return node_cpus, siblings
