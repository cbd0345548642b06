"""One rank of tests/test_launch_cpu.py: started by rabbitsalign_amd.launch.run_ranks
under torch.distributed.run exactly as bench.py's ranks are, but on gloo with the
CPU-path library (test infrastructure) in place of the GPU engine.  Each rank maps
its own shard (rabbitsalign_amd.shard.first_pair), the ranks reduce wall time and
counters with shard.reduce_run as bench.py does, and rank 0 prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch.distributed as dist
    from rabbitsalign_amd import mapper, shard
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    lib = os.path.join(ROOT, "oracle", "_ref", "librsalign_ref.so")
    m = mapper.Mapper.synthetic(3, 1_000_000, 2, 150, threads=2, lib_path=lib)
    pairs, steps = 400, 2
    totals = {f: 0 for f in shard.STAT_FIELDS}
    hashes = []
    t0 = time.perf_counter()
    for s in range(steps):
        r = m.synthetic_reads(7, shard.first_pair(rank, s, steps, pairs), pairs, 150, 300.0, 30.0, True)
        st = m.map(r, threads=2, chunk_size=100)
        r.close()
        hashes.append(f"{st.sam_hash:016x}")
        for f in shard.STAT_FIELDS:
            totals[f] += getattr(st, f)
    wall, tot = shard.reduce_run(time.perf_counter() - t0, totals, device="cpu")
    all_hashes = [None] * world
    dist.all_gather_object(all_hashes, hashes)
    m.close()
    if rank == 0:
        print(json.dumps({"n_ranks": world, "local_world": int(os.environ["LOCAL_WORLD_SIZE"]),
                          "reads": tot["n_reads"], "wall": wall, "hashes": all_hashes}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
