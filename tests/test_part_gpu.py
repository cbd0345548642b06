"""rank/world mode on the GPU: ONE input pair mapped by several
processes, each writing the SAM of its own chunks.

- library: two ranks (spawned processes, both on GPU 0, a gloo group for the plan's
  count exchange) plan with rabbitsalign_amd.shard.plan_shared_input and map with
  rsam_map_files_part; header + part 0 + part 1 == one process's SAM, byte for byte,
  and the summed statistics are the one process's -- for plain and for gzip input;
- CLI: `rsalign --rank R --world 3` (each rank plans alone) -- the parts minus @PG
  concatenate to the one-process SAM, on a repetitive reference whose insert-size
  estimate stays open across chunks.
"""
import os
import socket

import pytest

from e2e import RSALIGN, make_dataset, map_reads, sam_body

CFG = dict(seed=5, ref_len=2_000_000, contigs=2, L=150, pairs=6000, chunk=700)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, fq1, fq2, out_dir, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    from rabbitsalign_amd import mapper, shard
    mapper.load()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = mapper.Mapper.synthetic(CFG["seed"], CFG["ref_len"], CFG["contigs"], CFG["L"], device=0, threads=4)
        part = shard.plan_shared_input(fq1, fq2, CFG["chunk"], threads=4)
        st = m.map_files_part(fq1, fq2, part, threads=4, sam_path=os.path.join(out_dir, f"part{rank}.sam"))
        _, tot = shard.reduce_run(1.0, {f: getattr(st, f) for f in shard.STAT_FIELDS}, device="cpu")
        q.put((rank, part.as_dict(), tot, m.engine))
        m.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("gz", [False, True], ids=["plain", "gzip"])
def test_two_ranks_on_gpu0_equal_one_process(tmp_path, gz):
    import torch.multiprocessing as mp
    from rabbitsalign_amd import mapper, shard
    m = mapper.Mapper.synthetic(CFG["seed"], CFG["ref_len"], CFG["contigs"], CFG["L"], device=0, threads=4)
    assert "gpu" in m.engine.lower() or "hip" in m.engine.lower()
    reads = m.synthetic_reads(11, 0, CFG["pairs"], CFG["L"], 300.0, 30.0, True)
    fq1, fq2 = str(tmp_path / "r1.fq"), str(tmp_path / "r2.fq")
    reads.write_fastq(fq1, fq2)
    reads.close()
    one = tmp_path / "one.sam"
    st1 = m.map_files(fq1, fq2, threads=4, chunk_size=CFG["chunk"], sam_path=str(one))
    m.close()
    if gz:                          # the ranks map .fq.gz (parts planned by records)
        import gzip
        import shutil
        for f in (fq1, fq2):
            with open(f, "rb") as a, gzip.open(f + ".gz", "wb", compresslevel=1) as b:
                shutil.copyfileobj(a, b)
        fq1, fq2 = fq1 + ".gz", fq2 + ".gz"

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, fq1, fq2, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(2):
            rank, part, tot, engine = q.get(timeout=300)
            res[rank] = (part, tot, engine)
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    assert res[0][0]["end_chunk"] == res[1][0]["first_chunk"] > 0
    assert res[1][0]["end_chunk"] == res[1][0]["n_chunks"]
    parts = b"".join((tmp_path / f"part{r}.sam").read_bytes() for r in range(2))
    assert parts == one.read_bytes()
    assert all(res[0][1][f] == getattr(st1, f) for f in shard.STAT_FIELDS)


@pytest.mark.gpu
def test_cli_rank_parts_equal_one_process(tmp_path):
    fa, reads = make_dataset(str(tmp_path), pairs=5000, repeat_frac=0.2, n_runs=50)
    opts = ["-t", "4", "--chunk-size", "90"]
    map_reads(RSALIGN, fa, reads, str(tmp_path / "one.sam"), *opts)
    parts = []
    for r in range(3):
        out = str(tmp_path / f"p{r}.sam")
        map_reads(RSALIGN, fa, reads, out, *opts, "--rank", str(r), "--world", "3")
        parts += sam_body(out)
    assert parts == sam_body(str(tmp_path / "one.sam"))
