"""CPU: the SAM digest rsam_map reports (rsam_stats.sam_hash, include/rsalign.h) is
the order-sensitive line digest of the SAM body it wrote -- folded line by line
while each record is written (Sam::digest_into) -- restated here in Python from
its definition (rsa_host.hpp SamDigest) and computed over the SAM file."""
import os

import pytest

from helpers import ROOT

REF_LIB = os.path.join(ROOT, "oracle", "_ref", "librsalign_ref.so")
M64 = (1 << 64) - 1


def _rot(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def _mix(a, w):
    a ^= (w * 0xC2B2AE3D27D4EB4F) & M64
    return (_rot(a, 31) * 0x9E3779B185EBCA87) & M64


def _line_hash(b: bytes) -> int:
    n = len(b)
    a, bb, c, d = 0x9E3779B97F4A7C15 ^ n, 0x165667B19E3779F9, 0x85EBCA77C2B2AE63, 0x27D4EB2F165667C5
    rd = lambda o: int.from_bytes(b[o:o + 8], "little")
    i = 0
    while i + 32 <= n:
        a, bb, c, d = _mix(a, rd(i)), _mix(bb, rd(i + 8)), _mix(c, rd(i + 16)), _mix(d, rd(i + 24))
        i += 32
    while i + 8 <= n:
        a = _mix(a, rd(i))
        i += 8
    t = int.from_bytes(b[i:n], "little")
    h = _mix(a, t) ^ _rot(bb, 17) ^ _rot(c, 29) ^ _rot(d, 43)
    h ^= h >> 33
    h = (h * 0xff51afd7ed558ccd) & M64
    h ^= h >> 33
    h = (h * 0xc4ceb9fe1a85ec53) & M64
    h ^= h >> 33
    return h


def digest(body: bytes) -> int:
    h = 0
    for line in body.split(b"\n")[:-1]:
        h = (h * 0x100000001b3 + _line_hash(line)) & M64
    return h


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="reference build absent")
@pytest.mark.parametrize("paired", [True, False])
def test_sam_hash_is_digest_of_written_sam(tmp_path, paired):
    from rabbitsalign_amd import mapper as M
    m = M.Mapper.synthetic(5, 1_000_000, 2, 150, device=0, threads=4, lib_path=REF_LIB)
    try:
        reads = m.synthetic_reads(3, 0, 3000, 150, 300.0, 30.0, paired)
        out = tmp_path / "o.sam"
        st = m.map(reads, threads=4, chunk_size=700, sam_path=out)
        body = b"".join(l for l in open(out, "rb") if not l.startswith(b"@"))
        assert st.sam_bytes == len(body)
        assert st.sam_hash == digest(body)
        reads.close()
    finally:
        m.close()
