#!/usr/bin/env python3
"""Golden SAM-formatting fixtures from the REFERENCE's own Sam class.

Writes tests/golden/sam_calls.txt.gz: a seeded list of Sam calls (add, add_pair,
add_unmapped, add_unmapped_pair, add_unmapped_mate; format in oracle/refgen.cpp
cmd_sam) over every constructor setting (=/X or M CIGARs, read group, -U,
--details), and tests/golden/sam_calls.golden.sam.gz: the bytes the reference's
src/sam.cpp (compiled unmodified into oracle/_ref/refgen) writes for them.
tests/test_sam_golden.py replays the calls through the product's formatter.
Run in the build container only:  python tests/golden/make_sam_golden.py
"""
import gzip
import os
import random
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REFGEN = os.path.join(ROOT, "oracle", "_ref", "refgen")
FASTA = os.path.join(HERE, "rep.fa")          # 140 contigs "ctgN extra words"
N_CONTIGS = 140


def seq(rnd, n, alphabet="ACGT"):
    return "".join(rnd.choice(alphabet) for _ in range(n))


def name(rnd, i, mate):
    style = rnd.random()
    if style < 0.6:
        return f"r{i}/{mate}"
    if style < 0.7:
        return f"r{i}"
    if style < 0.8:
        return f"r{i}/3"
    if style < 0.9:
        return f"read:{i}:x/{mate}/{mate}"
    return f"{i}/"


def record(rnd, i, mate, L):
    s = seq(rnd, L, "ACGT" if rnd.random() < 0.8 else "ACGTNacgtU")
    q = "*" if rnd.random() < 0.15 else "".join(chr(33 + rnd.randrange(42)) for _ in range(L))
    if L == 0:
        s = "*"
        q = "*"
    return [name(rnd, i, mate), s, q]


def cigar(rnd, L):
    """A CIGAR consistent with query length L: S? (=|X|I|D|M runs) S?"""
    ops = []
    left = L
    if rnd.random() < 0.3 and left > 2:
        k = rnd.randint(1, min(20, left - 1))
        ops.append((4, k)); left -= k
    clip_r = rnd.randint(1, min(20, left - 1)) if rnd.random() < 0.3 and left > 2 else 0
    left -= clip_r
    while left > 0:
        op = rnd.choice([7, 7, 7, 8, 1, 2, 0])
        k = rnd.randint(1, max(1, min(left, 60)))
        if op == 2:
            ops.append((2, rnd.randint(1, 12)))
            continue
        if ops and ops[-1][0] == op:          # Cigar::push merges equal neighbours
            ops[-1] = (op, ops[-1][1] + k)
        else:
            ops.append((op, k))
        left -= k
    if clip_r:
        ops.append((4, clip_r))
    return [str(l << 4 | o) for o, l in ops]


def aln(rnd, L, unaligned=False, ref_id=None, pos=None):
    cg = [] if unaligned and rnd.random() < 0.7 else cigar(rnd, L)
    rid = rnd.randrange(N_CONTIGS) if ref_id is None else ref_id
    p = rnd.choice([0, 1, rnd.randrange(2500), rnd.randrange(2 ** 31 - 1)]) if pos is None else pos
    return [str(rid), str(p), str(rnd.randint(0, L + 30)), str(rnd.randint(0, 40)),
            str(rnd.randint(-60, 2 * L + 20)), str(rnd.randint(0, 1)), "1" if unaligned else "0",
            str(len(cg))] + cg


def det(rnd):
    return [str(rnd.randint(0, 1)), str(rnd.randint(0, 50)), str(rnd.randint(0, 5)), str(rnd.randint(0, 3)),
            str(rnd.randint(0, 40)), str(rnd.randint(0, 20))]


def calls(seed=3):
    rnd = random.Random(seed)
    out = []
    i = 0
    for eqx in (0, 1):
        for rg in ("-", "grp1"):
            for unmapped in (1, 0):
                for details in (0, 1):
                    out.append(f"S {eqx} {rg} {unmapped} {details}")
                    for _ in range(60):
                        i += 1
                        L = rnd.choice([150, 150, 100, 250, 1, 37])
                        if rnd.random() < 0.01:
                            L = 0
                        u = rnd.random()
                        if u < 0.25:       # single-end alignment, primary or secondary
                            out.append(" ".join(["A"] + record(rnd, i, 1, L) + [str(rnd.choice([0, 1, 37, 60, 255])),
                                                 str(int(rnd.random() < 0.8))] + det(rnd) + aln(rnd, L)))
                        elif u < 0.75:     # pair: same / other contig, either mate unaligned, proper or not
                            L2 = rnd.choice([L, 150, 100])
                            r1, r2 = record(rnd, i, 1, L), record(rnd, i, 2, L2)
                            same = rnd.random() < 0.7
                            rid = rnd.randrange(N_CONTIGS)
                            p1 = rnd.randrange(10_000_000)
                            p2 = p1 + rnd.randint(-700, 700) if same else rnd.randrange(10_000_000)
                            un1, un2 = rnd.random() < 0.12, rnd.random() < 0.12
                            a1 = aln(rnd, L, un1, rid, p1)
                            a2 = aln(rnd, L2, un2, rid if same else rnd.randrange(N_CONTIGS), max(0, p2))
                            out.append(" ".join(["P"] + r1 + r2 + [str(rnd.choice([0, 3, 60, 255])),
                                                 str(rnd.choice([0, 8, 60])), str(int(rnd.random() < 0.6)),
                                                 str(int(rnd.random() < 0.85))] + det(rnd) + det(rnd) + a1 + a2))
                        elif u < 0.85:
                            flags = rnd.choice([4, 4 | 1 | 8 | 64, 4 | 1 | 8 | 128, 4 | 1 | 64, 4 | 1])
                            out.append(" ".join(["U"] + record(rnd, i, 1, L) + [str(flags)]))
                        elif u < 0.93:
                            out.append(" ".join(["UP"] + record(rnd, i, 1, L) + record(rnd, i, 2, L)))
                        else:
                            flags = rnd.choice([1 | 4 | 64, 1 | 4 | 128, 1 | 4 | 64 | 32, 1 | 4 | 128 | 32])
                            out.append(" ".join(["UM"] + record(rnd, i, 1, L) +
                                                [str(flags), f"ctg{rnd.randrange(N_CONTIGS)}",
                                                 str(rnd.randrange(2 ** 31))]))
    return out


def main():
    if not os.path.exists(REFGEN):
        sys.exit("oracle/_ref/refgen missing: make -C oracle ref (needs /root/reference)")
    lines = calls()
    with tempfile.TemporaryDirectory() as d:
        cf, sf = os.path.join(d, "calls.txt"), os.path.join(d, "out.sam")
        with open(cf, "w") as f:
            f.write("\n".join(lines) + "\n")
        subprocess.run([REFGEN, "sam", FASTA, cf, sf], check=True)
        with open(cf, "rb") as f, gzip.GzipFile(os.path.join(HERE, "sam_calls.txt.gz"), "wb", mtime=0) as g:
            g.write(f.read())
        with open(sf, "rb") as f, gzip.GzipFile(os.path.join(HERE, "sam_calls.golden.sam.gz"), "wb", mtime=0) as g:
            data = f.read()
            g.write(data)
    print(f"{len(lines)} calls, {len(data)} SAM bytes")


if __name__ == "__main__":
    main()
