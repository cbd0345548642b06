"""Page-cache write bandwidth of one SAM-sized file (profiling tool, no GPU).

For each directory: one thread writing 740 MB in 3.7 MB pwrites to a new file,
four threads writing disjoint quarters of one new file (the positional sink's
pattern), and four threads each writing its own file.
    python scripts/write_bw.py [dir ...]
"""
import os
import sys
import threading
import time

MB = 1 << 20
TOTAL, CHUNK = 740 * MB, 37 * MB // 10
buf = os.urandom(CHUNK)


def one_file(path, writers):
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    n = TOTAL // CHUNK

    def work(w):
        for i in range(w, n, writers):
            os.pwrite(fd, buf, i * CHUNK)
    t = time.perf_counter()
    ts = [threading.Thread(target=work, args=(w,)) for w in range(writers)]
    for x in ts:
        x.start()
    for x in ts:
        x.join()
    dt = time.perf_counter() - t
    os.close(fd)
    os.remove(path)
    return n * CHUNK / dt / 1e9


def own_files(d, writers):
    def work(w, out):
        out[w] = one_file(os.path.join(d, f"wbw_{os.getpid()}_{w}"), 1)
    out = [0.0] * writers
    t = time.perf_counter()
    ts = [threading.Thread(target=work, args=(w, out)) for w in range(writers)]
    for x in ts:
        x.start()
    for x in ts:
        x.join()
    return writers * TOTAL / (time.perf_counter() - t) / 1e9


for d in sys.argv[1:] or ["/tmp", "/dev/shm"]:
    p = os.path.join(d, f"wbw_{os.getpid()}")
    for rep in range(2):
        print(f"{d}: 1 writer {one_file(p, 1):.2f} GB/s, 4 writers one file {one_file(p, 4):.2f} GB/s, "
              f"4 writers own files {own_files(d, 4):.2f} GB/s", flush=True)
