"""rank/world mode of the CLI (`rsalign --rank R --world W`) on the CPU
path build of the same host code (oracle/_ref/rsalign_ref: the reference's seeding and
SSW objects behind the product pipeline -- the engine does not matter for what is
tested here, which is the part plan, the insert-size replay and the ordered output).

The SAM parts of ranks 0..W-1 concatenated (minus @PG, which carries the command line)
must be byte for byte the one-process SAM, for: a reference whose repeats keep the
insert-size estimate open for dozens of chunks (the replay then runs through other
ranks' chunks, and past a part's end), tiny chunks and more ranks than chunks (empty
parts), single-end input, and --eqx -N; plus the plan's errors on files that are not
plain four-line FASTQ."""
import os
import subprocess

import pytest

from helpers import ROOT

REF_CLI = os.path.join(ROOT, "oracle", "_ref", "rsalign_ref")
GEN = os.path.join(ROOT, "rabbitsalign_amd", "bin", "rsa_gen")
pytestmark = pytest.mark.skipif(not (os.path.exists(REF_CLI) and os.path.exists(GEN)), reason="CPU CLI not built")


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    d = tmp_path_factory.mktemp("part")
    subprocess.run([GEN, "ref", "5", "3000000", "3", str(d / "ref.fa"), "0.2", "50"], check=True)
    subprocess.run([GEN, "reads", "9", str(d / "ref.fa"), "6001", "150", "300", "30", str(d / "r1.fq"),
                    str(d / "r2.fq"), "0.001"], check=True)
    return d


def _body(path):
    with open(path, "rb") as f:
        return b"".join(l for l in f.read().splitlines(keepends=True) if not l.startswith(b"@PG"))


def _run(d, out, *args):
    subprocess.run([REF_CLI, "-t", "3", "-o", str(out), *args], check=True, capture_output=True)


@pytest.mark.parametrize("chunk,world,extra,se", [
    (1000, 3, [], False),
    (50, 7, [], False),           # the estimate stays open past several parts' ends
    (7, 40, [], False),
    (5000, 5, [], False),         # 2 chunks, 5 ranks: empty parts
    (500, 4, [], True),           # single-end
    (300, 3, ["--eqx", "-N", "2"], False),
], ids=["c1000w3", "c50w7", "c7w40", "c5000w5", "se", "eqx_N2"])
def test_parts_concatenate_to_one_process_sam(data, chunk, world, extra, se):
    reads = [str(data / "r1.fq")] + ([] if se else [str(data / "r2.fq")])
    one = data / "one.sam"
    _run(data, one, "--chunk-size", str(chunk), *extra, str(data / "ref.fa"), *reads)
    parts = b""
    for r in range(world):
        p = data / f"p{r}.sam"
        _run(data, p, "--chunk-size", str(chunk), "--rank", str(r), "--world", str(world), *extra,
             str(data / "ref.fa"), *reads)
        body = _body(p)
        if r > 0:
            assert not body.startswith(b"@")                   # only rank 0 writes the header
        parts += body
    assert parts == _body(one)


def _write_gz(src, dst):
    import gzip
    import shutil
    with open(src, "rb") as a, gzip.open(dst, "wb", compresslevel=1) as b:
        shutil.copyfileobj(a, b)


@pytest.mark.parametrize("se", [False, True], ids=["pe", "se"])
def test_parts_of_gzip_input(data, tmp_path, se):
    """.fq.gz input (the reference's usual input): the parts are planned by records (each
    rank counts them with the kseq parser and skips to its part), and the concatenated parts
    are the one-process SAM of the same gzip files."""
    names = ["r1.fq"] + ([] if se else ["r2.fq"])
    reads = []
    for n in names:
        _write_gz(data / n, tmp_path / (n + ".gz"))
        reads.append(str(tmp_path / (n + ".gz")))
    one = tmp_path / "one.sam"
    _run(data, one, "--chunk-size", "400", str(data / "ref.fa"), *reads)
    parts = b""
    for r in range(3):
        p = tmp_path / f"p{r}.sam"
        _run(data, p, "--chunk-size", "400", "--rank", str(r), "--world", "3", str(data / "ref.fa"), *reads)
        parts += _body(p)
    assert parts == _body(one)


def _wrap(src, dst, n=None):
    """FASTQ with each sequence line wrapped after 70 bases (5 lines a record)"""
    with open(src) as f, open(dst, "w") as g:
        lines = f.read().splitlines()
        if n is not None:
            lines = lines[:4 * n]
        for i in range(0, len(lines), 4):
            g.write(lines[i] + "\n" + lines[i + 1][:70] + "\n" + lines[i + 1][70:] + "\n+\n" + lines[i + 3] + "\n")


def test_parts_of_wrapped_fastq(data, tmp_path):
    """A wrapped FASTQ whose line count is not four lines a record is planned by records,
    like gzip: the parts concatenate to the one-process SAM."""
    _wrap(data / "r1.fq", tmp_path / "w1.fq")          # 6001 records: 30005 lines
    one = tmp_path / "one.sam"
    _run(data, one, "--chunk-size", "700", str(data / "ref.fa"), str(tmp_path / "w1.fq"))
    parts = b""
    for r in range(2):
        p = tmp_path / f"p{r}.sam"
        _run(data, p, "--chunk-size", "700", "--rank", str(r), "--world", "2", str(data / "ref.fa"),
             str(tmp_path / "w1.fq"))
        parts += _body(p)
    assert parts == _body(one)


def test_part_rejects_wrapped_fastq_with_four_line_count(data, tmp_path):
    """A wrapped FASTQ whose line count happens to be a multiple of four cannot be told
    from the plain layout by its counts: the byte plan's layout check fails loudly, no
    wrong SAM."""
    _wrap(data / "r1.fq", tmp_path / "w1.fq", n=6000)   # 30000 lines
    r = subprocess.run([REF_CLI, "-t", "2", "--rank", "1", "--world", "2", "-o", str(tmp_path / "x.sam"),
                        str(data / "ref.fa"), str(tmp_path / "w1.fq")], capture_output=True, text=True)
    assert r.returncode != 0 and "four-line" in r.stderr


def test_parts_with_trailing_blank_line_and_empty_input(data, tmp_path):
    """Empty lines at the end of a plain FASTQ are not records (kseq skips them); an empty
    input gives rank 0 the header and every other rank an empty part."""
    for n in ("r1.fq", "r2.fq"):
        (tmp_path / n).write_bytes((data / n).read_bytes() + b"\n\n")
    reads = [str(tmp_path / "r1.fq"), str(tmp_path / "r2.fq")]
    one = tmp_path / "one.sam"
    _run(data, one, "--chunk-size", "1000", str(data / "ref.fa"), *reads)
    parts = b""
    for r in range(3):
        p = tmp_path / f"p{r}.sam"
        _run(data, p, "--chunk-size", "1000", "--rank", str(r), "--world", "3", str(data / "ref.fa"), *reads)
        parts += _body(p)
    assert parts == _body(one)
    (tmp_path / "e.fq").write_bytes(b"")
    _run(data, tmp_path / "e_one.sam", str(data / "ref.fa"), str(tmp_path / "e.fq"))
    for r in range(2):
        _run(data, tmp_path / f"e{r}.sam", "--rank", str(r), "--world", "2", str(data / "ref.fa"), str(tmp_path / "e.fq"))
    assert _body(tmp_path / "e0.sam") == _body(tmp_path / "e_one.sam")
    assert (tmp_path / "e1.sam").read_bytes() == b""


def test_pg_line_leaves_out_rank_and_world(data, tmp_path):
    """rank 0's @PG command line is the one-process command line (same other arguments)."""
    _run(data, tmp_path / "x.sam", "--chunk-size", "3000", "--rank", "0", "--world", "2", str(data / "ref.fa"),
         str(data / "r1.fq"))
    pg = [l for l in (tmp_path / "x.sam").read_text().splitlines() if l.startswith("@PG")]
    assert pg and "--rank" not in pg[0] and "--world" not in pg[0] and "--chunk-size 3000" in pg[0]
