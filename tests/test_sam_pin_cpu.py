"""CPU: the host pipeline's SAM pinned to a digest.

The GPU/CPU parity tests compare two engines through the same restated host code
(pairing, rescue, MAPQ, SAM), so a host change that altered the output would pass
them.  This pins the CPU path's SAM body on a seeded dataset (repeats, N runs,
pairs with several NAMs) to the digest the round-2 start of the host code (1958959) gives; the
round-2 host changes were also checked against it on 300 k reads: host
refactors must keep it."""
import hashlib
import os

import pytest

from e2e import CPU_REF, make_dataset, map_reads, sam_body

PINNED = {
    "N0": "6e7dccf9539120b59f314dbaa356bd89",
    "N3": "88a24e41688e9bba1a613b6b58f7142d",
}


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    d = tmp_path_factory.mktemp("sam_pin")
    return d, make_dataset(str(d), name="pin", pairs=6000, ref_len=400_000, contigs=3, seed=11, repeat_frac=0.08,
                           cpu_index=True)


def digest(path):
    return hashlib.sha256("".join(sam_body(path)).encode()).hexdigest()[:32]


@pytest.mark.skipif(not os.path.exists(CPU_REF), reason="reference build absent")
@pytest.mark.parametrize("key,opts", [("N0", ()), ("N3", ("-N", "3"))])
def test_sam_pinned(data, key, opts):
    d, (fa, reads) = data
    out = str(d / f"{key}.sam")
    map_reads(CPU_REF, fa, reads, out, "-t", "4", "--chunk-size", "1000", *opts)
    assert digest(out) == PINNED[key]
