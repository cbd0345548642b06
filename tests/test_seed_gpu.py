"""GPU parity: rsa_randstrobes / rsa_seed (HIP) vs the oracle (pinned to the reference)."""
import os

import numpy as np
import pytest

import oracle_lib
from helpers import GOLDEN, build_sti


def _reads(name):
    with open(os.path.join(GOLDEN, f"{name}_reads.txt"), "rb") as f:
        return [l.rstrip(b"\n") for l in f]


@pytest.fixture(scope="module", params=["small", "rep"])
def setup(request, tmp_path_factory):
    from rabbitsalign_amd import native
    d = tmp_path_factory.mktemp(request.param)
    fa, sti = build_sti(d, request.param)
    idx = native.load_index(fa, sti)
    ctx = native.GpuContext(idx)
    yield request.param, idx, ctx, oracle_lib.OracleIndex(idx)
    ctx.close()


@pytest.mark.gpu
def test_randstrobes(setup):
    name, idx, ctx, ora = setup
    reads = _reads(name)
    got = ctx.randstrobes(reads)
    for r, g in zip(reads, got):
        w = ora.randstrobes(r)
        assert len(g) == len(w)
        assert np.array_equal(g["hash"], w["hash"]) and np.array_equal(g["start"], w["start"])
        assert np.array_equal(g["end"], w["end"]) and np.array_equal(g["is_reverse"], w["is_reverse"])


def _nam_equal(g, w):
    if len(g) != len(w):
        return False
    for f in ("nam_id", "query_start", "query_end", "query_prev_hit_startpos", "ref_start", "ref_end",
              "ref_prev_hit_startpos", "n_hits", "ref_id", "is_rc"):
        if not np.array_equal(g[f], w[f]):
            return False
    return np.array_equal(g["score"].view(np.uint32), w["score"].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("rescue_level", [2, 1])
def test_seed(setup, rescue_level):
    name, idx, ctx, ora = setup
    reads = _reads(name)
    nams, nonrep, resc = ctx.seed(reads, rescue_level=rescue_level)
    bad = []
    for i, r in enumerate(reads):
        w, wn, wr = ora.seed(r, rescue_level=rescue_level)
        if not _nam_equal(nams[i], w) or np.float32(nonrep[i]).view(np.uint32) != np.float32(wn).view(np.uint32) \
                or bool(resc[i]) != wr:
            bad.append(i)
    assert not bad, f"{len(bad)} reads differ, first {bad[:5]}"


@pytest.mark.gpu
def test_seed_batch_independent(setup):
    name, idx, ctx, ora = setup
    reads = _reads(name)
    a, _, _ = ctx.seed(reads)
    b, _, _ = ctx.seed(reads[::-1])
    for x, y in zip(a, b[::-1]):
        assert _nam_equal(x, y)
