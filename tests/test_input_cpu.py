"""CPU: read input.

- FASTQ encodings the reader must parse into the same records (kseq++ semantics,
  src/fastq.cpp): gzip, CRLF line ends, sequences/qualities wrapped over several
  lines, no final newline -> the same SAM as the plain file; FASTA reads -> the
  same SAM with QUAL '*';
- --interleaved (src/pc.cpp:23-107, main.cpp:136-139): records paired per block of
  2 x chunk-size records by same_name; a perfectly interleaved file maps exactly
  like the two mate files; unpaired records and pairs split across blocks are
  not mapped (perform_task_async_pe ignores records3)."""
import gzip
import os
import subprocess

import pytest

from e2e import CPU_PORT, make_dataset, map_reads, run, sam_body


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    d = tmp_path_factory.mktemp("input")
    fa, (f1, f2) = make_dataset(str(d), pairs=1500, ref_len=150_000, cpu_index=True, n_rate=0.002)
    base = d / "base.sam"
    map_reads(CPU_PORT, fa, [f1, f2], str(base), "-t", "2", "--chunk-size", "300")
    return d, fa, f1, f2, sam_body(base)


def _records(path):
    with open(path) as f:
        lines = f.read().split("\n")
    return [lines[i:i + 4] for i in range(0, len(lines) - 3, 4)]


def _write(path, recs, nl="\n", wrap=0, final_nl=True, fasta=False):
    out = []
    for h, s, p, q in recs:
        if fasta:
            out.append(">" + h[1:])
        else:
            out.append(h)
        chunks = [s[i:i + wrap] for i in range(0, len(s), wrap)] if wrap else [s]
        out += chunks
        if not fasta:
            out.append(p)
            out += [q[i:i + wrap] for i in range(0, len(q), wrap)] if wrap else [q]
    text = nl.join(out) + (nl if final_nl else "")
    if str(path).endswith(".gz"):
        with gzip.open(path, "wt", newline="") as f:
            f.write(text)
    else:
        with open(path, "w", newline="") as f:
            f.write(text)


@pytest.mark.parametrize("variant", ["gzip", "crlf", "wrapped", "no_final_newline", "wrapped_crlf_gzip"])
def test_fastq_encodings_same_records(data, variant):
    d, fa, f1, f2, want = data
    opts = dict(gzip=dict(), crlf=dict(nl="\r\n"), wrapped=dict(wrap=60), no_final_newline=dict(final_nl=False),
                wrapped_crlf_gzip=dict(nl="\r\n", wrap=37))[variant]
    ext = ".fq.gz" if "gzip" in variant else ".fq"
    paths = []
    for m, f in ((1, f1), (2, f2)):
        p = d / f"{variant}_{m}{ext}"
        _write(p, _records(f), **opts)
        paths.append(str(p))
    out = d / f"{variant}.sam"
    map_reads(CPU_PORT, fa, paths, str(out), "-t", "2", "--chunk-size", "300")
    assert sam_body(out) == want


def test_fasta_reads(data):
    d, fa, f1, f2, want = data
    paths = []
    for m, f in ((1, f1), (2, f2)):
        p = d / f"fasta_{m}.fa"
        _write(p, _records(f), fasta=True, wrap=70)
        paths.append(str(p))
    out = d / "fasta.sam"
    map_reads(CPU_PORT, fa, paths, str(out), "-t", "2", "--chunk-size", "300")
    got = sam_body(out)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        if g.startswith("@"):
            assert g == w
            continue
        gf, wf = g.rstrip("\n").split("\t"), w.rstrip("\n").split("\t")
        assert gf[:10] == wf[:10] and gf[11:] == wf[11:] and gf[10] == "*"


def test_interleaved_equals_two_files(data):
    d, fa, f1, f2, want = data
    a, b = _records(f1), _records(f2)
    p = d / "inter.fq"
    _write(p, [x for pair in zip(a, b) for x in pair])
    out = d / "inter.sam"
    map_reads(CPU_PORT, fa, [str(p)], str(out), "--interleaved", "-t", "2", "--chunk-size", "300")
    assert sam_body(out) == want


def _same_name(n1, n2):                     # pc.cpp:23-35
    if len(n1) != len(n2):
        return False
    if len(n1) <= 2:
        return n1 == n2
    if n1[:-1] != n2[:-1]:
        return False
    if n1[-2] == "/" and n1[-1] == "1" and n2[-1] == "2":
        return True
    return n1[-1] == n2[-1]


def test_interleaved_singletons_not_mapped(data):
    d, fa, f1, f2, _ = data
    a, b = _records(f1), _records(f2)
    recs = []
    for i, (x, y) in enumerate(zip(a, b)):
        if i % 7 == 3:
            recs.append(x)                    # mate 2 missing: a singleton
        elif i % 11 == 5:
            recs += [y, x]                    # /2 before /1: two singletons
        else:
            recs += [x, y]
    chunk = 250
    expect = []                               # distribute_interleaved per block of 2 * chunk records
    names = [r[0][1:].split()[0] for r in recs]
    for s in range(0, len(recs), 2 * chunk):
        e = min(len(recs), s + 2 * chunk)
        i = s
        while i < e:
            if i + 1 < e and _same_name(names[i], names[i + 1]):
                expect.append(names[i].rsplit("/", 1)[0])
                i += 2
            else:
                i += 1
    p = d / "inter_single.fq"
    _write(p, recs)
    out = d / "inter_single.sam"
    map_reads(CPU_PORT, fa, [str(p)], str(out), "--interleaved", "-t", "3", "--chunk-size", str(chunk))
    got = [l.split("\t")[0] for l in sam_body(out) if not l.startswith("@")]
    assert got[0::2] == expect and got[1::2] == expect


def test_interleaved_with_two_files_is_an_error(data):
    d, fa, f1, f2, _ = data
    r = subprocess.run([CPU_PORT, "--use-index", "--interleaved", "-o", str(d / "x.sam"), fa, f1, f2],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "interleaved" in r.stderr


@pytest.fixture(scope="module")
def big(tmp_path_factory):
    d = tmp_path_factory.mktemp("input_big")
    fa, (f1, f2) = make_dataset(str(d), pairs=6000, ref_len=200_000, cpu_index=True, n_rate=0.002)
    return d, fa, f1, f2


def _tricky(recs, k):
    """Header comments, quality lines starting with '@' or '+', trailing blanks after sequences."""
    out = []
    for i, (h, s, p, q) in enumerate(recs):
        if i % 3 == k % 3:
            h = h + " BX:Z:cmt\tmore"
        if i % 5 == 1:
            q = "@" + q[1:]
        elif i % 5 == 2:
            q = "+" + q[1:]
        if i % 7 == 3:
            s = s + " \t"
        if i % 11 == 4:
            p = "+" + h[1:]
        out.append((h, s, p, q))
    return out


@pytest.mark.parametrize("variant", ["plain", "crlf_tricky", "wrapped"])
def test_parallel_fastq_parse_matches_sequential(big, variant):
    """Files over 1 MB in the plain 4-line layout are parsed by several threads
    (io.cpp parse_parallel); the gzip copy of the same text takes the sequential
    kseq reader.  Both must give the same SAM; a wrapped file falls back."""
    d, fa, f1, f2 = big
    opts = dict(plain=dict(), crlf_tricky=dict(nl="\r\n"), wrapped=dict(wrap=60))[variant]
    sams = []
    for ext in (".fq", ".fq.gz"):
        paths = []
        for m, f in ((1, f1), (2, f2)):
            recs = _records(f)
            if variant == "crlf_tricky":
                recs = _tricky(recs, m)
            p = d / f"{variant}_{m}{ext}"
            _write(p, recs, **opts)
            paths.append(str(p))
        assert os.path.getsize(paths[0]) > (1 << 20) or ext == ".fq.gz"
        out = d / f"{variant}{ext}.sam"
        map_reads(CPU_PORT, fa, paths, str(out), "-t", "4", "--chunk-size", "1000")
        sams.append(sam_body(out))
    assert len(sams[0]) > 12000 and sams[0] == sams[1]
