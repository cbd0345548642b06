"""CPU: the product's SAM formatter (csrc/host/io.cpp Sam, reverse_complement) writes
the bytes the REFERENCE's own Sam class (src/sam.cpp, compiled unmodified into
oracle/_ref/refgen) wrote for the same 976 calls: add / add_pair / add_unmapped /
add_unmapped_pair / add_unmapped_mate over every constructor setting (=/X or M,
read group, -U, --details), with secondaries, proper/improper pairs, mates on other
contigs, unaligned mates, empty qualities, N/lowercase/U bases, /1 /2 name
suffixes, positions up to 2^31 (tests/golden/make_sam_golden.py).  SURVEY.md §8
rows a17 / f2."""
import gzip
import os
import subprocess

import pytest

from helpers import GOLDEN, ROOT

REPLAY = os.path.join(ROOT, "oracle", "_build", "sam_replay")
REFGEN = os.path.join(ROOT, "oracle", "_ref", "refgen")
FASTA = os.path.join(GOLDEN, "rep.fa")


@pytest.fixture(scope="module")
def calls(tmp_path_factory):
    d = tmp_path_factory.mktemp("sam")
    p = d / "calls.txt"
    with gzip.open(os.path.join(GOLDEN, "sam_calls.txt.gz"), "rb") as f:
        p.write_bytes(f.read())
    return d, p


def _diff(got: bytes, want: bytes):
    g, w = got.split(b"\n"), want.split(b"\n")
    for i, (x, y) in enumerate(zip(g, w)):
        if x != y:
            return f"line {i}:\n got  {x[:300]!r}\n want {y[:300]!r}"
    return f"{len(g)} vs {len(w)} lines"


def test_product_formatter_matches_reference_golden(calls):
    d, p = calls
    out = d / "product.sam"
    subprocess.run([REPLAY, FASTA, str(p), str(out)], check=True)
    with gzip.open(os.path.join(GOLDEN, "sam_calls.golden.sam.gz"), "rb") as f:
        want = f.read()
    got = out.read_bytes()
    assert got == want, _diff(got, want)


@pytest.mark.skipif(not os.path.exists(REFGEN), reason="reference build absent (golden file pins it)")
def test_golden_is_the_reference_live(calls):
    d, p = calls
    out = d / "ref.sam"
    subprocess.run([REFGEN, "sam", FASTA, str(p), str(out)], check=True)
    with gzip.open(os.path.join(GOLDEN, "sam_calls.golden.sam.gz"), "rb") as f:
        assert out.read_bytes() == f.read()
