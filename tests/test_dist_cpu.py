"""CPU, world_size 2 over gloo: the multi-GPU sharding of bench.py.

Each rank maps its own shard of synthetic pairs (rabbitsalign_amd.shard) with
the CPU-path build of include/rsalign.h (the parity reference, test
infrastructure), then the ranks reduce wall time and statistics exactly as
bench.py does over RCCL.  Checks: shards are disjoint, the reduced read count
is the sum, and every rank's SAM equals a single-process mapping of the same
shard (placement does not change results)."""
import os
import socket

import pytest

from helpers import ROOT

REF_CPU_LIB = os.path.join(ROOT, "oracle", "_ref", "librsalign_ref.so")
CFG = dict(seed=3, ref_len=2_000_000, contigs=2, L=150, pairs=1500, steps=2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _map_shard(m, rank, step):
    from rabbitsalign_amd import shard
    first = shard.first_pair(rank, step, CFG["steps"], CFG["pairs"])
    reads = m.synthetic_reads(7, first, CFG["pairs"], CFG["L"], 300.0, 30.0, True)
    st = m.map(reads, threads=2, chunk_size=500)
    reads.close()
    return st


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from rabbitsalign_amd import mapper, shard
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = mapper.Mapper.synthetic(CFG["seed"], CFG["ref_len"], CFG["contigs"], CFG["L"], threads=2,
                                    lib_path=REF_CPU_LIB)
        totals = {f: 0 for f in shard.STAT_FIELDS}
        hashes = []
        for step in range(CFG["steps"]):
            st = _map_shard(m, rank, step)
            hashes.append(st.sam_hash)
            for f in shard.STAT_FIELDS:
                totals[f] += getattr(st, f)
        wall, tot = shard.reduce_run(1.0 + rank, totals, device="cpu")
        q.put((rank, hashes, totals, wall, tot))
        m.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(not os.path.exists(REF_CPU_LIB), reason="CPU-path library not built")
def test_two_rank_sharding_gloo():
    import torch.multiprocessing as mp
    from rabbitsalign_amd import mapper, shard
    ranges = {(r, s): shard.first_pair(r, s, CFG["steps"], CFG["pairs"]) for r in range(2) for s in range(CFG["steps"])}
    starts = sorted(ranges.values())
    assert all(b - a >= CFG["pairs"] for a, b in zip(starts, starts[1:]))

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, hashes, totals, wall, tot = q.get(timeout=600)
        res[rank] = (hashes, totals, wall, tot)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # reduced values identical on both ranks: max wall, summed counters
    for r in range(2):
        assert res[r][2] == 2.0
        assert res[r][3]["n_reads"] == 2 * CFG["steps"] * 2 * CFG["pairs"]
        assert res[r][3] == {k: res[0][1][k] + res[1][1][k] for k in shard.STAT_FIELDS}
    # a rank's SAM equals a single-process mapping of the same shard
    m = mapper.Mapper.synthetic(CFG["seed"], CFG["ref_len"], CFG["contigs"], CFG["L"], threads=2,
                                lib_path=REF_CPU_LIB)
    for r in range(2):
        assert _map_shard(m, r, 1).sam_hash == res[r][0][1]
    m.close()


# ---- one shared input over the ranks (rank/world mode, rsam_map_files_part) ------
PART = dict(pairs=2600, chunk=300)


def _part_worker(rank, world, port, fq1, fq2, out_dir, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from rabbitsalign_amd import mapper, shard
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = mapper.Mapper.synthetic(CFG["seed"], CFG["ref_len"], CFG["contigs"], CFG["L"], threads=2,
                                    lib_path=REF_CPU_LIB)
        part = shard.plan_shared_input(fq1, fq2, PART["chunk"], threads=2, lib_path=REF_CPU_LIB)
        sam = os.path.join(out_dir, f"part{rank}.sam")
        st = m.map_files_part(fq1, fq2, part, threads=2, sam_path=sam)
        wall, tot = shard.reduce_run(1.0, {f: getattr(st, f) for f in shard.STAT_FIELDS}, device="cpu")
        q.put((rank, part.as_dict(), tot))
        m.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(not os.path.exists(REF_CPU_LIB), reason="CPU-path library not built")
@pytest.mark.parametrize("world,gz", [(2, False), (4, False), (2, True)], ids=["w2", "w4", "w2_gzip"])
def test_shared_input_gloo(tmp_path, world, gz):
    """`world` ranks map ONE FASTQ pair: each counts its 1/world of each file, the counts
    are all-gathered over gloo, each maps its chunks into its own SAM part (every rank past
    the first replays the insert-size estimate from chunk 0).  Header + parts in rank order ==
    the single-process SAM of the same files, byte for byte; the summed statistics == the
    single process's.  gzip: the ranks map .fq.gz files (planned by records: each rank
    counts the records and skips to its part) and must still give the one-process SAM of
    the plain files."""
    import torch.multiprocessing as mp
    from rabbitsalign_amd import mapper, shard
    m = mapper.Mapper.synthetic(CFG["seed"], CFG["ref_len"], CFG["contigs"], CFG["L"], threads=2,
                                lib_path=REF_CPU_LIB)
    reads = m.synthetic_reads(7, 0, PART["pairs"], CFG["L"], 300.0, 30.0, True)
    fq1, fq2 = str(tmp_path / "r1.fq"), str(tmp_path / "r2.fq")
    reads.write_fastq(fq1, fq2)
    reads.close()
    one = str(tmp_path / "one.sam")
    st1 = m.map_files(fq1, fq2, threads=2, chunk_size=PART["chunk"], sam_path=one)
    m.close()
    if gz:
        import gzip
        import shutil
        for f in (fq1, fq2):
            with open(f, "rb") as a, gzip.open(f + ".gz", "wb", compresslevel=1) as b:
                shutil.copyfileobj(a, b)
        fq1, fq2 = fq1 + ".gz", fq2 + ".gz"

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_part_worker, args=(r, world, port, fq1, fq2, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, part, tot = q.get(timeout=600)
        res[rank] = (part, tot)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n_chunks = (PART["pairs"] + PART["chunk"] - 1) // PART["chunk"]
    assert res[0][0]["first_chunk"] == 0 and res[world - 1][0]["end_chunk"] == n_chunks
    assert all(res[r][0]["flags"] == (3 if gz else 0) for r in range(world))   # RSAM_PART_RECORDS1 | _RECORDS2
    for r in range(1, world):
        assert res[r][0]["first_chunk"] == res[r - 1][0]["end_chunk"] and res[r][0]["first_chunk"] > 0
    parts = b"".join(open(tmp_path / f"part{r}.sam", "rb").read() for r in range(world))
    assert parts == open(one, "rb").read()
    for r in range(world):
        assert res[r][1]["n_reads"] == st1.n_reads
        assert all(res[r][1][f] == getattr(st1, f) for f in shard.STAT_FIELDS)


@pytest.mark.skipif(not os.path.exists(REF_CPU_LIB), reason="CPU-path library not built")
def test_part_refuses_inconsistent_plan(tmp_path):
    """rsam_map_files_part re-checks the part it is handed: chunk bounds that do not follow
    from rank/world, a record range that does not match the chunks, or a byte offset that
    does not start a record are refused before anything is mapped."""
    from rabbitsalign_amd import mapper
    m = mapper.Mapper.synthetic(CFG["seed"], CFG["ref_len"], CFG["contigs"], CFG["L"], threads=2,
                                lib_path=REF_CPU_LIB)
    reads = m.synthetic_reads(7, 0, 900, CFG["L"], 300.0, 30.0, True)
    fq1, fq2 = str(tmp_path / "r1.fq"), str(tmp_path / "r2.fq")
    reads.write_fastq(fq1, fq2)
    reads.close()
    good = mapper.part_plan(fq1, fq2, 1, 2, 100, None, None, 2, lib_path=REF_CPU_LIB)
    assert good.first_chunk == 4 and good.first_pair == 400 and good.offset1 > 0
    st = m.map_files_part(fq1, fq2, good, threads=2, sam_path=str(tmp_path / "ok.sam"))
    assert st.n_reads == 2 * good.n_pairs
    for field, delta in (("offset1", 1), ("first_chunk", 1), ("first_pair", 100), ("n_pairs", -1), ("offset2", -3)):
        bad = mapper.Part.from_buffer_copy(good)
        setattr(bad, field, getattr(bad, field) + delta)
        with pytest.raises(RuntimeError, match="inconsistent part"):
            m.map_files_part(fq1, fq2, bad, threads=2, sam_path=str(tmp_path / "bad.sam"))
    m.close()
