"""CPU: the bench's self-launch (`python3 bench.py --gpus N` without WORLD_SIZE).

- The launcher (rabbitsalign_amd.launch.run_ranks) starts N ranks under
  torch.distributed.run and relays rank 0's JSON line: run here with N = 2 on
  gloo, each rank mapping its own shard with the CPU-path library, reducing
  as bench.py does; every rank's SAM must equal a one-process mapping of its shard.
- bench.py with more GPUs requested than visible fails cleanly before any rank
  starts, and never prints a result line."""
import json
import os
import subprocess
import sys

import pytest

from helpers import ROOT

REF_CPU_LIB = os.path.join(ROOT, "oracle", "_ref", "librsalign_ref.so")


@pytest.mark.skipif(not os.path.exists(REF_CPU_LIB), reason="CPU-path library not built")
def test_self_launch_two_ranks_gloo():
    from rabbitsalign_amd import launch, mapper, shard
    env = dict(os.environ, OMP_NUM_THREADS="1")
    rc, line = launch.run_ranks(os.path.join(ROOT, "tests", "dist_rank_prog.py"), [], 2, env=env)
    assert rc == 0
    assert line is not None
    assert line["n_ranks"] == 2 and line["local_world"] == 2
    assert line["reads"] == 2 * 2 * 2 * 400               # ranks x steps x mates x pairs
    m = mapper.Mapper.synthetic(3, 1_000_000, 2, 150, threads=2, lib_path=REF_CPU_LIB)
    for rank in range(2):
        r = m.synthetic_reads(7, shard.first_pair(rank, 1, 2, 400), 400, 150, 300.0, 30.0, True)
        assert f"{m.map(r, threads=2, chunk_size=100).sam_hash:016x}" == line["hashes"][rank][1]
        r.close()
    m.close()


def test_bench_more_gpus_than_visible_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert p.returncode == 2, p.stderr[-2000:]
    assert "2 GPUs requested, 0 visible" in p.stderr
    assert not any(l.strip().startswith("{") for l in p.stdout.splitlines())


def test_run_child_timeout_kills_the_child():
    """The multi-device leg runs under a time limit (bench.py RSA_BENCH_MD_TIMEOUT): a child
    that outlives it is killed with its process group, and the caller gets 124 and no line
    instead of waiting, so the rank leg's result line still comes out."""
    import sys
    import time
    from rabbitsalign_amd import launch
    t = time.time()
    rc, line = launch.run_child([sys.executable, "-c", "import time; print('{\"x\": 1}', flush=True); time.sleep(60)"],
                                timeout=2)
    assert rc == 124 and line is None
    assert time.time() - t < 30
    rc, line = launch.run_child([sys.executable, "-c", "print('{\"x\": 2}')"], timeout=60)
    assert rc == 0 and line == {"x": 2}
