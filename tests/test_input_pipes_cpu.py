"""CPU: reads from pipes, FIFOs and stdin.

The CLI estimates the read length from the first records (main.cpp:254-258,
readlen.cpp:16-29) when -r is not given.  The reference reads those records
through a RewindableFile and replays them to the mapper (fastq.cpp:1-65), so a
stream is read once and the estimate sees the real reads.  Here the estimate
comes from the streamed source's own queued records.  So:
- paired FIFOs without -r map every record, in step, with the profile of the
  real read length (100 bp here: an estimate of 150 would pick the r150 index
  parameters and fail against the r100 .sti);
- stdin ('-') single-end, and interleaved on stdin, likewise;
- each SAM equals the SAM of the same reads from regular files.
"""
import os
import subprocess
import threading

import pytest

from e2e import CPU_PORT, make_dataset, map_reads, sam_body
from test_input_cpu import _records, _write


@pytest.fixture(scope="module")
def data100(tmp_path_factory):
    d = tmp_path_factory.mktemp("pipes")
    fa, (f1, f2) = make_dataset(str(d), name="p100", pairs=1500, L=100, mu=250, sigma=25, ref_len=120_000,
                                cpu_index=True, n_rate=0.002)
    return d, fa, f1, f2


def _feed(path, fifo):
    with open(path, "rb") as src, open(fifo, "wb") as dst:
        while True:
            b = src.read(1 << 16)
            if not b:
                break
            dst.write(b)


def test_paired_fifos_without_r(data100):
    d, fa, f1, f2 = data100
    want = d / "files.sam"
    map_reads(CPU_PORT, fa, [f1, f2], str(want), "-t", "3", "--chunk-size", "128")
    p1, p2 = str(d / "in_1.fifo"), str(d / "in_2.fifo")
    for p in (p1, p2):
        if not os.path.exists(p):
            os.mkfifo(p)
    ts = [threading.Thread(target=_feed, args=(src, dst)) for src, dst in ((f1, p1), (f2, p2))]
    for t in ts:
        t.start()
    out = d / "fifo.sam"
    r = subprocess.run([CPU_PORT, "--use-index", "-t", "3", "--chunk-size", "128", "-o", str(out), fa, p1, p2],
                       capture_output=True, text=True, timeout=300)
    for t in ts:
        t.join(timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    assert sam_body(out) == sam_body(want)
    n_body = sum(1 for l in sam_body(out) if not l.startswith("@"))
    assert n_body >= 2 * 1500


@pytest.mark.parametrize("chunk", [128, 50])
def test_single_end_stdin_without_r(data100, chunk):
    """'-' is stdin; chunk 50 puts the 500-record estimate across ten blocks."""
    d, fa, f1, _ = data100
    want = d / f"se_file_{chunk}.sam"
    map_reads(CPU_PORT, fa, [f1], str(want), "-t", "2", "--chunk-size", str(chunk))
    out = d / f"se_stdin_{chunk}.sam"
    with open(f1, "rb") as fin:
        r = subprocess.run([CPU_PORT, "--use-index", "-t", "2", "--chunk-size", str(chunk), "-o", str(out), fa, "-"],
                           stdin=fin, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert sam_body(out) == sam_body(want)


def test_interleaved_stdin_without_r(data100):
    d, fa, f1, f2 = data100
    a, b = _records(f1), _records(f2)
    inter = d / "inter.fq"
    _write(inter, [x for pair in zip(a, b) for x in pair])
    want = d / "inter_file.sam"
    map_reads(CPU_PORT, fa, [str(inter)], str(want), "--interleaved", "-t", "2", "--chunk-size", "128")
    out = d / "inter_stdin.sam"
    with open(inter, "rb") as fin:
        r = subprocess.run([CPU_PORT, "--use-index", "--interleaved", "-t", "2", "--chunk-size", "128", "-o",
                            str(out), fa, "-"], stdin=fin, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert sam_body(out) == sam_body(want)
    # the interleaved pairs map as the two mate files do
    pe = d / "inter_pe.sam"
    map_reads(CPU_PORT, fa, [f1, f2], str(pe), "-t", "2", "--chunk-size", "128")
    assert [l for l in sam_body(out) if not l.startswith("@")] == [l for l in sam_body(pe) if not l.startswith("@")]


def test_error_with_stalled_pipe_exits(data100):
    """Mate files of different record counts, the second one a pipe whose writer
    stalls (keeps it open, writes no more) after some MB of records: the CLI reports
    the error and exits instead of waiting on the stalled producer (the workers'
    input waits are cancelled, and the blocked reader is given up after a bounded
    wait).  The reader fills 4 MB at a time, so the writer sends more than that."""
    d, fa, f1, f2 = data100
    a = _records(f1)
    short = d / "short_1.fq"
    _write(short, a[:40])
    recs = _records(f2)
    text = "".join("\n".join(x) + "\n" for x in recs).encode() * 20      # ~6 MB
    r_fd, w_fd = os.pipe()
    stop = threading.Event()

    def writer():
        try:
            os.write(w_fd, text)
        except OSError:
            pass
        stop.wait(300)                            # stalled: open, silent

    t = threading.Thread(target=writer, daemon=True)
    t.start()
    try:
        r = subprocess.run([CPU_PORT, "--use-index", "-r", "100", "-t", "2", "--chunk-size", "32", "-o",
                            str(d / "stall.sam"), fa, str(short), f"/dev/fd/{r_fd}"],
                           pass_fds=(r_fd,), capture_output=True, text=True, timeout=120)
    finally:
        os.close(r_fd)
        stop.set()
        t.join(timeout=10)
        os.close(w_fd)
    assert r.returncode == 1 and "different record counts" in r.stderr
