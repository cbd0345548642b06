"""CPU: streamed input (reference InputBuffer::read_records,
src/pc.cpp:74-107) and the SAM sinks.

- a file whose records leave the plain 4-line layout part-way (a wrapped record,
  a blank line, a FASTA record) switches from the mapped splitter to the kseq
  reader at that record and gives the SAM of the plain file;
- resident memory does not grow with the input: mapping twice the reads raises
  the peak RSS by far less than the extra FASTQ bytes (the old CLI loaded the
  whole file before mapping);
- SAM through `>> out.sam`, `> out.sam 2>&1`, `> out.sam` and a pipe is the
  same body as `-o` (one writer thread writes the chunks in order);
- rsam_map_files (files streamed) == rsam_map (records in memory) == CLI.
"""
import os
import subprocess

import pytest

from e2e import CPU_PORT, make_dataset, map_reads, run, sam_body
from test_input_cpu import _records, _write

REF_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                       "librsalign_ref.so")


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    d = tmp_path_factory.mktemp("stream")
    fa, (f1, f2) = make_dataset(str(d), pairs=3000, ref_len=150_000, cpu_index=True, n_rate=0.002)
    base = d / "base.sam"
    map_reads(CPU_PORT, fa, [f1, f2], str(base), "-t", "3", "--chunk-size", "256")
    return d, fa, f1, f2, sam_body(base)


def _write_mixed(path, recs, breaks):
    """The plain layout, except: record i in breaks gets its sequence and quality
    wrapped over two lines (kseq joins them), a blank line before it, or both."""
    out = []
    for i, (h, s, p, q) in enumerate(recs):
        kind = breaks.get(i)
        if kind == "blank":
            out.append("")
        if kind in ("wrap", "blank"):
            out += [h, s[:40], s[40:], p, q[:40], q[40:]]
        else:
            out += [h, s, p, q]
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")


@pytest.mark.parametrize("where", ["first", "chunk_edge", "middle", "last"])
def test_layout_switch_mid_file(data, where):
    d, fa, f1, f2, want = data
    a, b = _records(f1), _records(f2)
    n = len(a)
    at = dict(first=0, chunk_edge=256, middle=n // 2 + 3, last=n - 1)[where]
    paths = []
    for m, recs in ((1, a), (2, b)):
        p = d / f"mixed_{where}_{m}.fq"
        # only mate 1 leaves the layout at `at` (mate 2 a little later): the two
        # readers switch at different chunks
        _write_mixed(p, recs, {at: "wrap"} if m == 1 else {min(n - 1, at + 7): "blank", n - 1: "wrap"})
        paths.append(str(p))
    out = d / f"mixed_{where}.sam"
    map_reads(CPU_PORT, fa, paths, str(out), "-t", "3", "--chunk-size", "256")
    assert sam_body(out) == want


def test_fasta_after_fastq_records(data):
    """Records of both kinds in one file: the '>' record ends the mapped splitter."""
    d, fa, f1, f2, _ = data
    a, b = _records(f1)[:600], _records(f2)[:600]
    plain = []
    for m, recs in ((1, a), (2, b)):
        p = d / f"fqonly_{m}.fq"
        _write(p, recs)
        plain.append(str(p))
    ref = d / "fqonly.sam"
    map_reads(CPU_PORT, fa, plain, str(ref), "-t", "2", "--chunk-size", "100")
    mixed = []
    for m, recs in ((1, a), (2, b)):
        p = d / f"fqfa_{m}.fq"
        text = []
        for i, (h, s, pl, q) in enumerate(recs):
            text += ([">" + h[1:], s] if i == 300 else [h, s, pl, q])
        p.write_text("\n".join(text) + "\n")
        mixed.append(str(p))
    out = d / "fqfa.sam"
    map_reads(CPU_PORT, fa, mixed, str(out), "-t", "2", "--chunk-size", "100")
    got, want = sam_body(out), sam_body(ref)
    assert len(got) == len(want)
    diff = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    # only the FASTA records' own lines differ (pair r300: QUAL '*', the rest equal)
    assert diff and all(got[i].split("\t")[0] == "r300" for i in diff)
    for i in diff:
        g, w = got[i].rstrip("\n").split("\t"), want[i].rstrip("\n").split("\t")
        assert g[:10] == w[:10] and g[10] == "*" and g[11:] == w[11:]


def test_appended_and_shared_stderr_outputs(data):
    d, fa, f1, f2, want = data
    body = [l for l in want if not l.startswith("@")]
    app = d / "append.sam"
    app.write_text("previous content\n")
    with open(app, "a") as out:
        subprocess.run([CPU_PORT, "--use-index", "-t", "3", "--chunk-size", "256", fa, f1, f2], stdout=out,
                       stderr=subprocess.DEVNULL, check=True)
    lines = app.read_text().splitlines(keepends=True)
    assert lines[0] == "previous content\n"
    assert [l for l in lines[1:] if not l.startswith("@")] == body
    shared = d / "shared.sam"
    with open(shared, "w") as out:
        subprocess.run([CPU_PORT, "--use-index", "-v", "-t", "3", "--chunk-size", "256", fa, f1, f2], stdout=out,
                       stderr=subprocess.STDOUT, check=True)
    got = [l for l in shared.read_text().splitlines(keepends=True) if not l.startswith("@") and "\t" in l
           and l.split("\t")[0].startswith("r")]
    assert got == body


def _peak_rss_kb(cmd):
    """Peak resident set of a child process (wait4's rusage, KB)."""
    p = subprocess.Popen([str(c) for c in cmd], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    _, status, ru = os.wait4(p.pid, 0)
    p.returncode = os.waitstatus_to_exitcode(status)
    assert p.returncode == 0, cmd
    return ru.ru_maxrss


def test_resident_memory_flat_in_input_size(tmp_path):
    fa, (f1, f2) = make_dataset(str(tmp_path), name="small", pairs=40_000, ref_len=100_000, contigs=1,
                                cpu_index=True, n_rate=0.0)
    big1, big2 = tmp_path / "big_1.fq", tmp_path / "big_2.fq"
    for src, dst in ((f1, big1), (f2, big2)):
        text = open(src).read()
        dst.write_text(text * 3)
    extra = 2 * (os.path.getsize(f1) + os.path.getsize(f2))
    opts = ["--use-index", "-t", "4", "--chunk-size", "2000", "-o", os.devnull]
    small = _peak_rss_kb([CPU_PORT, *opts, fa, f1, f2])
    large = _peak_rss_kb([CPU_PORT, *opts, fa, big1, big2])
    assert extra > 40 << 20
    # 3x the reads: the peak grows by well under a tenth of the extra input
    assert (large - small) * 1024 < extra / 10, (small, large, extra)


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="CPU-path library not built")
def test_map_files_equals_map_in_memory(data):
    d, fa, f1, f2, want = data
    from rabbitsalign_amd import mapper
    sti = fa + ".r150.sti"
    m = mapper.Mapper.from_files(fa, sti, 150, device=0, threads=3, lib_path=REF_LIB)
    try:
        out = d / "lib_files.sam"
        s_files = m.map_files(f1, f2, threads=3, chunk_size=256, sam_path=out)
        reads = m.load_reads(f1, f2)
        s_mem = m.map(reads, threads=3, chunk_size=256)
        reads.close()
        assert (s_files.sam_hash, s_files.sam_bytes, s_files.n_reads) == (s_mem.sam_hash, s_mem.sam_bytes,
                                                                          s_mem.n_reads)
        body = [l for l in sam_body(out) if not l.startswith("@")]
        assert body == [l for l in want if not l.startswith("@")]
        # interleaved file streamed == the two mate files
        a, b = _records(f1), _records(f2)
        p = d / "lib_inter.fq"
        _write(p, [x for pair in zip(a, b) for x in pair])
        s_int = m.map_files(p, None, interleaved=True, threads=3, chunk_size=256)
        assert (s_int.sam_hash, s_int.n_reads) == (s_mem.sam_hash, s_mem.n_reads)
        # single-end streamed == single-end in memory
        s_se = m.map_files(f1, None, threads=2, chunk_size=300)
        r1 = m.load_reads(f1)
        s_se_mem = m.map(r1, threads=2, chunk_size=300)
        r1.close()
        assert (s_se.sam_hash, s_se.n_reads) == (s_se_mem.sam_hash, s_se_mem.n_reads)
        # without the digest (rsam_set_sam_digest 0): sam_hash 0, the same SAM file
        m.set_sam_digest(False)
        out2 = d / "lib_files_nodigest.sam"
        s_nd = m.map_files(f1, f2, threads=3, chunk_size=256, sam_path=out2)
        m.set_sam_digest(True)
        assert s_nd.sam_hash == 0 and s_nd.sam_bytes == s_files.sam_bytes
        assert open(out2, "rb").read() == open(out, "rb").read()
    finally:
        m.close()


def test_unequal_mate_files_fail(data):
    d, fa, f1, f2, _ = data
    a, b = _records(f1), _records(f2)
    p1, p2 = d / "uneq_1.fq", d / "uneq_2.fq"
    _write(p1, a)
    _write(p2, b[:-5])
    r = subprocess.run([CPU_PORT, "--use-index", "-t", "2", "-o", str(d / "uneq.sam"), fa, str(p1), str(p2)],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "different record counts" in r.stderr


@pytest.mark.parametrize("mode", ["stdout_file", "stdout_pipe"])
def test_sam_to_stdout(data, mode):
    """stdout redirected to a file or read through a pipe carries the -o bytes."""
    d, fa, f1, f2, want = data
    out = d / f"sink_{mode}.sam"
    args = [CPU_PORT, "--use-index", "-t", "4", "--chunk-size", "256", fa, f1, f2]
    if mode == "stdout_file":
        with open(out, "w") as fo:
            subprocess.run(args, stdout=fo, stderr=subprocess.DEVNULL, check=True)
    else:
        r = subprocess.run(args, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, check=True)
        out.write_bytes(r.stdout)
    assert sam_body(out) == want
