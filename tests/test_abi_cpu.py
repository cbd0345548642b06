"""CPU: the C-ABI libraries load without a GPU and export every function their
headers declare (include/rsa_gpu.h -> librsa_gpu.so, include/rsalign.h ->
librsalign.so).  No compute call is made."""
import ctypes as C
import os
import re

import pytest

from helpers import ROOT

LIB = os.path.join(ROOT, "rabbitsalign_amd", "lib")
HEADERS = {
    "rsa_gpu.h": os.path.join(LIB, "librsa_gpu.so"),
    "rsalign.h": os.path.join(LIB, "librsalign.so"),
}
DECL = re.compile(r"^[A-Za-z_][\w\s\*]*?\b((?:rsa|rsam)_\w+)\s*\(", re.M)


def declared(header):
    with open(os.path.join(ROOT, "include", header)) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)      # drop comments
    text = re.sub(r"typedef[^;]*;", "", text, flags=re.S)   # and typedefs
    return sorted(set(DECL.findall(text)))


@pytest.mark.parametrize("header", sorted(HEADERS))
def test_header_symbols_exported(header):
    names = declared(header)
    assert len(names) >= 5, names
    lib = C.CDLL(HEADERS[header])
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"{HEADERS[header]} lacks {missing}"


def test_python_mirror_lists_every_symbol():
    from rabbitsalign_amd import native
    assert sorted(native.EXPORTED_SYMBOLS) == declared("rsa_gpu.h")


def test_gpu_library_fails_loudly_without_device():
    """rsa_open with no GPU visible returns NULL and an error, never a CPU path."""
    lib = C.CDLL(HEADERS["rsa_gpu.h"])
    lib.rsa_open.restype = C.c_void_p
    lib.rsa_open.argtypes = [C.c_int, C.c_void_p, C.c_char_p, C.c_size_t]
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from rabbitsalign_amd import native
    view = native.IndexView()
    offs = (C.c_uint64 * 2)(0, 0)
    view.contig_offsets = C.cast(offs, C.c_void_p)
    err = C.create_string_buffer(256)
    assert lib.rsa_open(0, C.byref(view), err, 256) is None
    assert b"device" in err.value, err.value
