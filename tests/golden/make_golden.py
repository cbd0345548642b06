#!/usr/bin/env python3
"""Regenerate the golden fixtures from the REFERENCE's own code.

Inputs (FASTA, reads, SW jobs) are synthetic and produced here with fixed
seeds.  Expected outputs come from oracle/_ref/refgen, i.e. the reference's
randstrobes.cpp / nam.cpp / index.cpp / ssw.c / sam.cpp compiled unmodified
from /root/reference by oracle/Makefile.  Run in the build container only:
    python tests/golden/make_golden.py
"""
import gzip
import hashlib
import os
import random
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REFGEN = os.path.join(ROOT, "oracle", "_ref", "refgen")
GEN = os.path.join(ROOT, "rabbitsalign_amd", "bin", "rsa_gen")


def run(*a):
    subprocess.run([str(x) for x in a], check=True, stdout=subprocess.DEVNULL)


def rep_fasta(path, seed=5, n=140, base_len=2000):
    rnd = random.Random(seed)
    B = "ACGT"
    base = "".join(rnd.choice(B) for _ in range(base_len))
    with open(path, "w") as f:
        for c in range(n):
            s = [ch if rnd.random() > 0.01 else rnd.choice(B) for ch in base]
            s = "".join(s) + "".join(rnd.choice(B) for _ in range(rnd.randint(0, 300)))
            f.write(">ctg%d extra words\n" % c)
            for i in range(0, len(s), 60):
                f.write(s[i:i + 60] + "\n")
    reads = []
    for i in range(40):
        p = rnd.randint(0, base_len - 150)
        r = "".join(ch if rnd.random() > 0.01 else rnd.choice(B) for ch in base[p:p + 150])
        if rnd.random() < 0.5:
            r = r[::-1].translate(str.maketrans("ACGT", "TGCA"))
        reads.append(r)
    return reads


def main():
    if not os.path.exists(REFGEN):
        sys.exit("oracle/_ref/refgen missing: make -C oracle (needs /root/reference)")
    os.chdir(HERE)
    # 1. small multi-contig reference with repeats and N runs + PE reads with N
    run(GEN, "ref", 11, 200000, 3, "small.fa", 0.05, 4)
    run(GEN, "reads", 12, "small.fa", 150, 150, 300, 30, "/tmp/g1.fq", "/tmp/g2.fq", 0.002)
    reads = []
    for fq in ("/tmp/g1.fq", "/tmp/g2.fq"):
        with open(fq) as f:
            reads += [l.strip() for i, l in enumerate(f) if i % 4 == 1]
    reads += ["ACGT", "N" * 60, "A" * 90, "ACGT" * 20, "acgtacgtnnACGTTGCA" * 8, "GATTACA" * 30]
    with open("small_reads.txt", "w") as f:
        f.write("\n".join(reads) + "\n")
    # 2. 140 near-identical contigs: many ref_ids per read (robin_hood rehash), rescue path
    with open("rep_reads.txt", "w") as f:
        f.write("\n".join(rep_fasta("rep.fa")) + "\n")
    shas = {}
    for name, r in (("small", 150), ("rep", 150)):
        sti = f"/tmp/{name}.fa.r{r}.sti"
        run(REFGEN, "index", f"{name}.fa", r, sti, 4)
        shas[name] = hashlib.sha256(open(sti, "rb").read()).hexdigest()
        out = f"/tmp/{name}_seeds.txt"
        run(REFGEN, "seeds", f"{name}.fa", sti, r, f"{name}_reads.txt", out, 2)
        with open(out, "rb") as f, gzip.GzipFile(f"{name}_seeds.golden.gz", "wb", mtime=0) as g:
            g.write(f.read())
    with open("sti.sha256", "w") as f:
        for k, v in shas.items():
            f.write(f"{v}  {k}.fa.r150.sti\n")
    # 3. SSW raw results for random extension/rescue-shaped jobs
    run(REFGEN, "sswrand", 99, 2500, "/tmp/ssw_golden.txt")
    with open("/tmp/ssw_golden.txt", "rb") as f, gzip.GzipFile("ssw.golden.gz", "wb", mtime=0) as g:
        g.write(f.read())
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
