"""CPU: the host pipeline's per-job arithmetic (extension / rescue windows and the
stored Alignment, src/pc.cpp:177-242, 291-368) on the hand-derived cases of
tests/host_cases.py, through the product's own functions (bin/rsa_host_cases)."""
import os
import subprocess

import pytest

from helpers import ROOT
from host_cases import EXTENSION_WINDOWS, RESCUE_WINDOWS, STORES

TOOL = os.path.join(ROOT, "rabbitsalign_amd", "bin", "rsa_host_cases")


def run_cases(lines):
    r = subprocess.run([TOOL], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True)
    return r.stdout.splitlines()


def nam_args(nam):
    return " ".join(str(x) for x in nam)


def info_args(info):
    rs, re, qs, qe, ed, sw, ops = info
    return f"{rs} {re} {qs} {qe} {ed} {sw} {len(ops)} " + " ".join(str(x) for x in ops)


def store_line(kind, nam, read_len, contig_len, mu, sigma, info):
    if kind == "ext":
        return f"ext_store {nam_args(nam)} {read_len} {info_args(info)}"
    return f"rescue_store {nam_args(nam)} {read_len} {contig_len} {mu} {sigma} {info_args(info)}"


def parse_aln(line):
    f = line.split()
    assert f[0] == "aln"
    v = [int(x) for x in f[1:]]
    return tuple(v[:8]) + (v[9:9 + v[8]],)


@pytest.mark.parametrize("case", EXTENSION_WINDOWS, ids=[c[0] for c in EXTENSION_WINDOWS])
def test_extension_window(case):
    name, nam, read_len, contig_len, want = case
    out = run_cases([f"ext_window {nam_args(nam)} {read_len} {contig_len}"])
    assert out == [f"window {want[0]} {want[1]}"]


@pytest.mark.parametrize("case", RESCUE_WINDOWS, ids=[c[0] for c in RESCUE_WINDOWS])
def test_rescue_window(case):
    name, nam, read_len, contig_len, mu, sigma, want = case
    out = run_cases([f"rescue_window {nam_args(nam)} {read_len} {contig_len} {mu} {sigma}"])
    assert out == [f"window {want[0]} {want[1]}"]


@pytest.mark.parametrize("case", STORES, ids=[c[0] for c in STORES])
def test_store(case):
    name, kind, nam, read_len, contig_len, mu, sigma, info, want = case
    out = run_cases([store_line(kind, nam, read_len, contig_len, mu, sigma, info)])
    assert parse_aln(out[0]) == want
