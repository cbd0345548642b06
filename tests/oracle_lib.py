"""ctypes binding of the parity oracle (oracle/_build/librsa_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "_build", "librsa_oracle.so")
ORACLE_CLI = os.path.join(ORACLE_DIR, "_build", "oracle_cli")
REFGEN = os.path.join(ORACLE_DIR, "_ref", "refgen")


class AlnInfo(C.Structure):
    _fields_ = [("edit_distance", C.c_uint32), ("ref_start", C.c_uint32), ("ref_end", C.c_uint32),
                ("query_start", C.c_uint32), ("query_end", C.c_uint32), ("sw_score", C.c_int32),
                ("n_cigar", C.c_int32)]


class Params(C.Structure):
    _fields_ = [("k", C.c_int), ("s", C.c_int), ("t_syncmer", C.c_int), ("w_min", C.c_int), ("w_max", C.c_int),
                ("max_dist", C.c_int), ("q", C.c_uint64)]


class Qrs(C.Structure):
    _fields_ = [("hash", C.c_uint64), ("start", C.c_uint32), ("end", C.c_uint32), ("is_reverse", C.c_uint32)]


class Index(C.Structure):
    _fields_ = [("rs", C.c_void_p), ("n", C.c_uint64), ("starts", C.c_void_p), ("bits", C.c_int),
                ("filter_cutoff", C.c_uint), ("k", C.c_int)]


class Nam(C.Structure):
    _fields_ = [("nam_id", C.c_int32), ("query_start", C.c_int32), ("query_end", C.c_int32),
                ("query_prev_hit_startpos", C.c_int32), ("ref_start", C.c_int32), ("ref_end", C.c_int32),
                ("ref_prev_hit_startpos", C.c_int32), ("n_hits", C.c_int32), ("ref_id", C.c_int32),
                ("score", C.c_float), ("is_rc", C.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            raise RuntimeError("oracle not built: make -C oracle")
        L = C.CDLL(ORACLE_LIB)
        L.ora_aligner_align.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.c_int, C.c_int, C.POINTER(AlnInfo), C.c_void_p]
        L.ora_randstrobes_query.argtypes = [C.c_char_p, C.c_int, C.POINTER(Params), C.c_void_p, C.c_int]
        L.ora_find_nams.argtypes = [C.POINTER(Index), C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                    C.POINTER(C.c_float)]
        L.ora_find_nams_rescue.argtypes = [C.POINTER(Index), C.c_void_p, C.c_int, C.c_uint, C.c_void_p, C.c_int]
        L.ora_reverse_complement.argtypes = [C.c_char_p, C.c_int, C.c_char_p]
        L.ora_hamming_align.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                        C.POINTER(C.c_int), C.c_void_p]
        L.ora_nam_site.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_int, C.c_char_p, C.c_int64, C.c_int,
                                   C.c_void_p, C.POINTER(C.c_int)]
        _lib = L
    return _lib


def align(query: bytes, ref: bytes, match=2, mismatch=8, gap_open=12, gap_extend=1, end_bonus=10):
    """Aligner::align restated (src/aligner.cpp:114-210)."""
    info = AlnInfo()
    cig = np.zeros(2 * (len(query) + len(ref)) + 16, dtype=np.uint32)
    lib().ora_aligner_align(query, len(query), ref, len(ref), match, mismatch, gap_open, gap_extend, end_bonus,
                            C.byref(info), cig.ctypes.data)
    return dict(sw_score=info.sw_score, edit_distance=info.edit_distance, ref_start=info.ref_start,
                ref_end=info.ref_end, query_start=info.query_start, query_end=info.query_end,
                cigar=[int(x) for x in cig[:info.n_cigar]])


QRS_DTYPE = np.dtype([("hash", "<u8"), ("start", "<u4"), ("end", "<u4"), ("is_reverse", "<u4"), ("pad_", "<u4")])
NAM_DTYPE = np.dtype([("nam_id", "<i4"), ("query_start", "<i4"), ("query_end", "<i4"),
                      ("query_prev_hit_startpos", "<i4"), ("ref_start", "<i4"), ("ref_end", "<i4"),
                      ("ref_prev_hit_startpos", "<i4"), ("n_hits", "<i4"), ("ref_id", "<i4"),
                      ("score", "<f4"), ("is_rc", "<i4")])


class OracleIndex:
    def __init__(self, idx):
        """idx: rabbitsalign_amd.native.Index"""
        self.idx = idx
        self.rs = np.ascontiguousarray(idx.randstrobes)
        self.st = np.ascontiguousarray(idx.bucket_starts)
        self.c = Index(self.rs.ctypes.data if len(self.rs) else 0, len(self.rs), self.st.ctypes.data, idx.bits,
                       idx.filter_cutoff, idx.k)
        self.p = Params(idx.k, idx.s, idx.t_syncmer, idx.w_min, idx.w_max, idx.max_dist, idx.q)

    def randstrobes(self, seq: bytes):
        cap = 2 * len(seq) + 8
        out = np.zeros(cap, dtype=QRS_DTYPE)
        n = lib().ora_randstrobes_query(seq, len(seq), C.byref(self.p), out.ctypes.data, cap)
        assert n >= 0
        return out[:n]

    def find_nams(self, qrs):
        qrs = np.ascontiguousarray(qrs, dtype=QRS_DTYPE)
        cap = 1 << 16
        out = np.zeros(cap, dtype=NAM_DTYPE)
        nonrep = C.c_float()
        n = lib().ora_find_nams(C.byref(self.c), qrs.ctypes.data, len(qrs), out.ctypes.data, cap, C.byref(nonrep))
        assert n >= 0
        return out[:n], nonrep.value

    def find_nams_rescue(self, qrs, cutoff):
        qrs = np.ascontiguousarray(qrs, dtype=QRS_DTYPE)
        cap = 1 << 16
        out = np.zeros(cap, dtype=NAM_DTYPE)
        n = lib().ora_find_nams_rescue(C.byref(self.c), qrs.ctypes.data, len(qrs), cutoff, out.ctypes.data, cap)
        assert n >= 0
        return out[:n]

    def seed(self, seq: bytes, rescue_level=2, rescue_cutoff=None):
        """find_nams + rescue decision of align_*_read_part (src/aln.cpp:1946-1962)."""
        if rescue_cutoff is None:
            rescue_cutoff = rescue_level * self.idx.filter_cutoff if rescue_level < 100 else 1000
        q = self.randstrobes(seq)
        nams, nonrep = self.find_nams(q)
        rescued = False
        if rescue_level > 1 and (len(nams) == 0 or nonrep < 0.7):
            nams = self.find_nams_rescue(q, rescue_cutoff)
            rescued = True
        return nams, np.float32(nonrep), rescued


def reverse_complement(seq: bytes) -> bytes:
    """revcomp.hpp:11-38"""
    out = C.create_string_buffer(len(seq) + 1)
    lib().ora_reverse_complement(seq, len(seq), out)
    return out.raw[:len(seq)]


def nam_site(nam, read: bytes, contig: bytes, k: int):
    """reverse_nam_if_needed (aln.cpp:60-93) + extend_seed_part's Hamming test
    (aln.cpp:374-395): (flags, n_mm, mismatch positions) as rsa_nam_site reports them."""
    n = np.zeros(1, dtype=NAM_DTYPE)
    n[0] = nam
    pos = np.zeros(max(1, len(read)), dtype=np.uint16)
    n_mm = C.c_int()
    f = lib().ora_nam_site(n.ctypes.data, read, reverse_complement(read), len(read), contig, len(contig), k,
                           pos.ctypes.data, C.byref(n_mm))
    return int(f), int(n_mm.value), [int(x) for x in pos[:n_mm.value]] if f & 8 else []


def hamming_align(query: bytes, ref: bytes, match=2, mismatch=8, end_bonus=10):
    """hamming_align (aligner.cpp:219-302): (score, segment start, end, mismatches, CIGAR ops)."""
    n = len(query)
    cig = np.zeros(2 * n + 4, dtype=np.uint32)
    sc, st, en, mm = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    k = lib().ora_hamming_align(query, ref, n, match, mismatch, end_bonus, C.byref(sc), C.byref(st), C.byref(en),
                                C.byref(mm), cig.ctypes.data)
    return int(sc.value), int(st.value), int(en.value), int(mm.value), [int(x) for x in cig[:k]]
