"""Shared test helpers: fixture paths, .sti construction."""
import gzip
import hashlib
import os
import subprocess

import pytest

import oracle_lib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = os.path.join(HERE, "golden")
INDEXER = os.path.join(ROOT, "rabbitsalign_amd", "bin", "rsalign")


def golden_sha(name):
    with open(os.path.join(GOLDEN, "sti.sha256")) as f:
        for line in f:
            sha, fn = line.split()
            if fn.startswith(name + "."):
                return sha
    raise KeyError(name)


def build_sti(tmpdir, name, read_len=150):
    """Build <name>.fa.r150.sti with the reference's own populate() (oracle/_ref/refgen)
    when available, else with our indexer; either way it must hash to the golden sha."""
    fa = os.path.join(GOLDEN, f"{name}.fa")
    sti = os.path.join(str(tmpdir), f"{name}.fa.r{read_len}.sti")
    if os.path.exists(oracle_lib.REFGEN):
        subprocess.run([oracle_lib.REFGEN, "index", fa, str(read_len), sti, "4"], check=True,
                       stdout=subprocess.DEVNULL)
    elif os.path.exists(INDEXER):
        subprocess.run([INDEXER, "index", "-r", str(read_len), "-o", sti, fa], check=True, stdout=subprocess.DEVNULL)
    else:
        pytest.skip("no index builder available")
    with open(sti, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == golden_sha(name)
    return fa, sti


def read_lines(path):
    if path.endswith(".gz"):
        with gzip.open(path, "rt") as f:
            return f.read()
    with open(path) as f:
        return f.read()
