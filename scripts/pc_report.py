#!/usr/bin/env python3
"""Attribute RSA_PC_SAMPLE output (capi.cpp PcSampler) to libraries and functions.

    python scripts/pc_report.py gpurun_out/pcsN/pcs.txt [top]

Each "pc count" sample is mapped through the recorded /proc/self/maps lines to
(library, file offset) and symbolised with addr2line; libraries from the box
resolve here because the image is the same."""
import collections
import os
import subprocess
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    maps, pcs = [], collections.Counter()
    for line in open(path):
        if line.startswith("#map "):
            f = line[5:].split()
            lo, hi = (int(x, 16) for x in f[0].split("-"))
            maps.append((lo, hi, int(f[2], 16), f[5] if len(f) > 5 else "?"))
        elif not line.startswith("#"):
            a, c = line.split()
            pcs[int(a, 16)] += int(c)
    tot = sum(pcs.values())
    bylib = collections.defaultdict(list)
    for pc, c in pcs.items():
        for lo, hi, off, name in maps:
            if lo <= pc < hi:
                bylib[name].append((pc - lo + off, c))
                break
        else:
            bylib["?"].append((pc, c))
    print(f"samples {tot}")
    for name, v in sorted(bylib.items(), key=lambda kv: -sum(c for _, c in kv[1])):
        print(f"{100 * sum(c for _, c in v) / tot:5.1f}%  {name}")
    fn = collections.Counter()
    for name, v in bylib.items():
        lib = name.replace("/tmp/code/RabbitBio__RabbitSAlign/repo", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        if not os.path.exists(lib):
            for off, c in v:
                fn[f"[{os.path.basename(name)}]"] += c
            continue
        offs = sorted(set(o for o, _ in v))
        out = subprocess.run(["addr2line", "-f", "-C", "-e", lib] + [hex(o) for o in offs], capture_output=True,
                             text=True).stdout.split("\n")
        sym = {o: out[2 * i] for i, o in enumerate(offs)}
        for off, c in v:
            s = sym.get(off, "??")
            fn[f"{s[:100]} [{os.path.basename(name)}]"] += c
    for f, c in fn.most_common(top):
        print(f"{100 * c / tot:5.1f}%  {f}")


if __name__ == "__main__":
    main()
