#!/usr/bin/env python3
"""Repeat the multi-device mapping (two contexts on one GPU, rsam_add_devices) and
diff its SAM against the one-context SAM -- measurement/debug tool for
test_multi_device_gpu.  python scripts/micro/multi_dev_diff.py [reps] [out_dir]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def body_lines(path):
    with open(path, "rb") as f:
        return [ln for ln in f if not ln.startswith(b"@")]


def main():
    import torch  # noqa: F401
    from rabbitsalign_amd import mapper as M
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    out = sys.argv[2] if len(sys.argv) > 2 else "/tmp/mdd"
    os.makedirs(out, exist_ok=True)
    m = M.Mapper.synthetic(3, 20_000_000, 4, 150, device=0, threads=8)
    reads = m.synthetic_reads(9, 0, 40_000, 150, 300.0, 30.0, True)
    a = m.map(reads, threads=8, sam_path=os.path.join(out, "one.sam"))
    ref = body_lines(os.path.join(out, "one.sam"))
    print("one", a.sam_hash, a.sam_bytes, flush=True)
    for i in range(2):
        b = m.map(reads, threads=8)
        print("one again", i, b.sam_hash == a.sam_hash, flush=True)
    if os.environ.get("MDD_LINES2") == "0":      # the added context without bucket lines (.sti table)
        os.environ["RSA_BUCKET_LINES"] = "0"
    m.add_devices([0])
    os.environ.pop("RSA_BUCKET_LINES", None)
    bad = 0
    for i in range(reps):
        p = os.path.join(out, f"multi_{i}.sam")
        b = m.map(reads, threads=8, sam_path=p)
        same = (b.sam_hash, b.sam_bytes) == (a.sam_hash, a.sam_bytes)
        print("multi", i, b.sam_hash, b.sam_bytes, "same" if same else "DIFF", flush=True)
        if not same:
            bad += 1
            cur = body_lines(p)
            nd = 0
            for k, (x, y) in enumerate(zip(ref, cur)):
                if x != y:
                    nd += 1
                    if nd <= 6:
                        print(" line", k, "\n  one:  ", x[:400].decode(errors="replace").rstrip(),
                              "\n  multi:", y[:400].decode(errors="replace").rstrip(), flush=True)
            print(" lines differing:", nd, "of", len(ref), len(cur), flush=True)
        else:
            os.remove(p)
    print("bad", bad, "of", reps)
    reads.close()
    m.close()


if __name__ == "__main__":
    main()
