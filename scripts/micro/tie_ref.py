#!/usr/bin/env python3
"""A 3 Gb synthetic FASTA (24 x 125 Mb uniform contigs) with a PAR-like region: chr1's
[1 Mb, 1 Mb + dup) copied onto chr2 at the same coordinates, so its randstrobes tie in
(hash, position) across the two contigs -- the index build's tie path at scale
(measurement tool, scripts/gpu_r06g.sh).

    python scripts/micro/tie_ref.py OUT.fa [dup_bp=10000000] [total=3000000000] [contigs=24]
"""
import sys

import numpy as np


def main():
    out = sys.argv[1]
    dup = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
    total = int(sys.argv[3]) if len(sys.argv) > 3 else 3_000_000_000
    nc = int(sys.argv[4]) if len(sys.argv) > 4 else 24
    rng = np.random.default_rng(12345)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    per = total // nc
    at = 1 << 20
    chr1 = None
    with open(out, "wb") as f:
        for c in range(nc):
            s = acgt[rng.integers(0, 4, per, dtype=np.uint8)]
            if c == 0:
                chr1 = s[at:at + dup].copy()
            elif c == 1:
                s[at:at + dup] = chr1
            f.write(b">chr%d\n" % (c + 1))
            f.write(s.tobytes())
            f.write(b"\n")


if __name__ == "__main__":
    main()
