"""CPU: the drop-in libraries load into an FFI host whose static-TLS surplus is
already in use (torch imported first), both of them in one process, and map.

Round 3 built the host pipeline's scratch as initial-exec TLS; dlopen of
librsalign.so / librsalign_ref.so then failed with "cannot allocate memory in
static TLS block" once torch and one library were loaded.  The libraries must
carry no static-TLS requirement (no DF_STATIC_TLS flag) and load in any order."""
import os
import subprocess
import sys

import pytest

from helpers import ROOT

PRODUCT = os.path.join(ROOT, "rabbitsalign_amd", "lib", "librsalign.so")
GPU_LIB = os.path.join(ROOT, "rabbitsalign_amd", "lib", "librsa_gpu.so")
REF_CPU_LIB = os.path.join(ROOT, "oracle", "_ref", "librsalign_ref.so")


def _dynamic_flags(path):
    out = subprocess.run(["readelf", "-d", path], capture_output=True, text=True, check=True).stdout
    return [l for l in out.splitlines() if "FLAGS" in l]


@pytest.mark.parametrize("path", [PRODUCT, GPU_LIB, REF_CPU_LIB])
def test_no_static_tls_flag(path):
    if not os.path.exists(path):
        pytest.skip(f"{path} not built")
    flags = " ".join(_dynamic_flags(path))
    assert "STATIC_TLS" not in flags, f"{path}: {flags}"


SCRIPT = r"""
import sys
sys.path.insert(0, {root!r})
import torch, torch.distributed        # the FFI host: torch's own libraries first
from rabbitsalign_amd import mapper
mapper.load({product!r})               # the product library (GPU engine; loaded, no compute)
m = mapper.Mapper.synthetic(3, 400_000, 2, 150, threads=2, lib_path={ref!r})
r = m.synthetic_reads(7, 0, 400, 150, 300.0, 30.0, True)
st = m.map(r, threads=2, chunk_size=100)
assert st.n_reads == 800, st.n_reads
print("mapped", st.n_reads, hex(st.sam_hash))
"""


@pytest.mark.skipif(not (os.path.exists(PRODUCT) and os.path.exists(REF_CPU_LIB)), reason="libraries not built")
def test_torch_then_both_libraries_then_map():
    code = SCRIPT.format(root=ROOT, product=PRODUCT, ref=REF_CPU_LIB)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "mapped 800" in p.stdout
