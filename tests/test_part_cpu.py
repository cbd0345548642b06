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


def test_part_rejects_non_plain_fastq(data, tmp_path):
    """A wrapped (multi-line) FASTQ cannot be cut by line counts: an error, not a wrong SAM."""
    wrapped = tmp_path / "w1.fq"
    with open(data / "r1.fq") as f, open(wrapped, "w") as g:
        lines = f.read().splitlines()
        for i in range(0, len(lines), 4):
            g.write(lines[i] + "\n" + lines[i + 1][:70] + "\n" + lines[i + 1][70:] + "\n+\n" + lines[i + 3] + "\n")
    r = subprocess.run([REF_CLI, "-t", "2", "--rank", "1", "--world", "2", "-o", str(tmp_path / "x.sam"),
                        str(data / "ref.fa"), str(wrapped)], capture_output=True, text=True)
    assert r.returncode != 0 and "four-line" in r.stderr
