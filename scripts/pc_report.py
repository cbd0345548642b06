#!/usr/bin/env python3
"""Attribute RSA_PC_SAMPLE output (capi.cpp PcSampler) to libraries and functions.

    python scripts/pc_report.py gpurun_out/pcsN/pcs.txt [top] [callee-substring]

Each "pc count" sample is mapped through the recorded /proc/self/maps lines to
(library, file offset) and symbolised with addr2line; libraries from the box
resolve here because the image is the same.  With a callee substring, the
samples whose function matches it are also broken down by the word at the
stack pointer ("#ra" lines), which is the caller for a leaf such as memmove."""
import collections
import os
import subprocess
import sys


def symbolise(maps, pcs):
    """{pc: "function [library]"} for a set of absolute addresses."""
    bylib = collections.defaultdict(list)
    for pc in pcs:
        for lo, hi, off, name in maps:
            if lo <= pc < hi:
                bylib[name].append((pc, pc - lo + off))
                break
        else:
            bylib["?"].append((pc, pc))
    sym = {}
    for name, v in bylib.items():
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        lib = name
        for part in ("/rabbitsalign_amd/", "/oracle/"):     # the box's copy of this tree -> here
            if part in name and not os.path.exists(name):
                lib = root + part + name.split(part, 1)[1]
        if not os.path.exists(lib):
            for pc, _ in v:
                sym[pc] = f"[{os.path.basename(name)}]"
            continue
        offs = sorted(set(o for _, o in v))
        # -i: the inline chain of each address; OUTER=1 reports its outermost
        # (really called) function instead of the innermost inlined one
        out = subprocess.run(["addr2line", "-a", "-i", "-f", "-C", "-e", lib] + [hex(o) for o in offs],
                             capture_output=True, text=True).stdout.split("\n")
        chains, cur = [], None
        for ln in out:
            if ln.startswith("0x"):
                cur = []
                chains.append(cur)
            elif cur is not None and ln and not (":" in ln and ln.split(":")[-1].split(" ")[0].isdigit()) \
                    and not ln.startswith("??:"):
                cur.append(ln)
        outer = os.environ.get("OUTER") == "1"
        by_off = {o: ((c[-1] if outer else c[0]) if c else "??") for o, c in zip(offs, chains)}
        for pc, o in v:
            sym[pc] = f"{by_off.get(o, '??')[:100]} [{os.path.basename(name)}]"
    return sym, bylib


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    callee = sys.argv[3] if len(sys.argv) > 3 else None
    maps, pcs, ras = [], collections.Counter(), collections.Counter()
    for line in open(path):
        if line.startswith("#map "):
            f = line[5:].split()
            lo, hi = (int(x, 16) for x in f[0].split("-"))
            maps.append((lo, hi, int(f[2], 16), f[5] if len(f) > 5 else "?"))
        elif line.startswith("#ra "):
            _, a, r, c = line.split()
            ras[(int(a, 16), int(r, 16))] += int(c)
        elif not line.startswith("#"):
            a, c = line.split()
            pcs[int(a, 16)] += int(c)
    tot = sum(pcs.values())
    sym, bylib = symbolise(maps, pcs)
    print(f"samples {tot}")
    for name, v in sorted(bylib.items(), key=lambda kv: -sum(pcs[pc] for pc, _ in kv[1])):
        print(f"{100 * sum(pcs[pc] for pc, _ in v) / tot:5.1f}%  {name}")
    fn = collections.Counter()
    for pc, c in pcs.items():
        fn[sym[pc]] += c
    for f, c in fn.most_common(top):
        print(f"{100 * c / tot:5.1f}%  {f}")
    if callee:
        hit = {(pc, ra): c for (pc, ra), c in ras.items() if callee in sym.get(pc, "")}
        rsym, _ = symbolise(maps, set(ra for _, ra in hit))
        callers = collections.Counter()
        for (pc, ra), c in hit.items():
            callers[rsym[ra]] += c
        print(f"\ncallers of samples in '{callee}' ({sum(hit.values())} samples):")
        for f, c in callers.most_common(top):
            print(f"{100 * c / tot:5.1f}%  {f}")


if __name__ == "__main__":
    main()
