"""ctypes binding of the C-ABI in include/rsa_gpu.h (librsa_gpu.so, gfx950).

This is the Python host mirror used by tests, bench.py and __graft_entry__.
It only marshals plain buffers; all compute runs in the HIP library.  There
is no fallback: if the library or a GPU is missing, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
BIN_DIR = os.path.join(_HERE, "bin")
GPU_LIB = os.path.join(LIB_DIR, "librsa_gpu.so")


class RefRandstrobe(C.Structure):
    _fields_ = [("hash", C.c_uint64), ("position", C.c_uint32), ("packed", C.c_uint32)]


class IndexView(C.Structure):
    _fields_ = [
        ("randstrobes", C.c_void_p), ("n_randstrobes", C.c_uint64), ("bucket_starts", C.c_void_p),
        ("bits", C.c_int32), ("filter_cutoff", C.c_int32),
        ("k", C.c_int32), ("s", C.c_int32), ("t_syncmer", C.c_int32),
        ("w_min", C.c_int32), ("w_max", C.c_int32), ("max_dist", C.c_int32), ("q", C.c_uint64),
        ("ref_seq", C.c_void_p), ("contig_offsets", C.c_void_p), ("n_contigs", C.c_int32),
    ]


class ReadBatch(C.Structure):
    _fields_ = [("seq", C.c_void_p), ("offsets", C.c_void_p), ("lengths", C.c_void_p), ("n_reads", C.c_uint32)]


class QueryRandstrobe(C.Structure):
    _fields_ = [("hash", C.c_uint64), ("start", C.c_uint32), ("end", C.c_uint32),
                ("is_reverse", C.c_uint32), ("pad_", C.c_uint32)]


class RandstrobeBatch(C.Structure):
    _fields_ = [("out", C.c_void_p), ("capacity", C.c_uint64), ("offsets", C.c_void_p), ("needed", C.c_uint64)]


NAM_DTYPE = np.dtype([("nam_id", "<i4"), ("query_start", "<i4"), ("query_end", "<i4"),
                      ("query_prev_hit_startpos", "<i4"), ("ref_start", "<i4"), ("ref_end", "<i4"),
                      ("ref_prev_hit_startpos", "<i4"), ("n_hits", "<i4"), ("ref_id", "<i4"),
                      ("score", "<f4"), ("is_rc", "<i4")])

QRS_DTYPE = np.dtype([("hash", "<u8"), ("start", "<u4"), ("end", "<u4"), ("is_reverse", "<u4"), ("pad_", "<u4")])

JOB_DTYPE = np.dtype([("query_offset", "<u8"), ("query_len", "<u4"), ("ref_id", "<i4"),
                      ("ref_start", "<u4"), ("ref_len", "<u4")])

ALN_DTYPE = np.dtype([("sw_score", "<i4"), ("edit_distance", "<u4"), ("ref_start", "<u4"), ("ref_end", "<u4"),
                      ("query_start", "<u4"), ("query_end", "<u4"), ("cigar_offset", "<u8"),
                      ("cigar_len", "<u4"), ("flags", "<u4")])


class NamBatch(C.Structure):
    _fields_ = [("nams", C.c_void_p), ("capacity", C.c_uint64), ("offsets", C.c_void_p),
                ("nonrepetitive_fraction", C.c_void_p), ("rescued", C.c_void_p), ("needed", C.c_uint64),
                ("sites", C.c_void_p), ("mm_pool", C.c_void_p), ("mm_capacity", C.c_uint64), ("mm_used", C.c_uint64),
                ("order", C.c_uint32), ("hamming_align", C.c_uint32), ("match", C.c_int32),
                ("mismatch", C.c_int32), ("end_bonus", C.c_int32), ("pad_", C.c_uint32)]


SITE_DTYPE = np.dtype([("flags", "u1"), ("orig_is_rc", "u1"), ("n_mm", "<u2"), ("mm_offset", "<u4"),
                       ("orig_query_start", "<i4"), ("orig_query_end", "<i4")])
NAMS_FOUND, NAMS_BY_SCORE = 0, 1


class JobBatch(C.Structure):
    _fields_ = [("queries", C.c_void_p), ("queries_len", C.c_uint64), ("jobs", C.c_void_p),
                ("n_jobs", C.c_uint32), ("match", C.c_int32), ("mismatch", C.c_int32),
                ("gap_open", C.c_int32), ("gap_extend", C.c_int32), ("end_bonus", C.c_int32)]


class AlnBatch(C.Structure):
    _fields_ = [("alns", C.c_void_p), ("cigar_pool", C.c_void_p), ("cigar_capacity", C.c_uint64),
                ("cigar_used", C.c_uint64)]


KERNELS = ["randstrobes", "lookup", "find_nams", "rescue", "compact", "ext_scan", "ext_band", "ext_band_wide",
           "ext_band_panel", "sites", "ext_redo"]
# the extension scan is k_ext_scan_v unless RSA_SCAN_V=0 selects the two-layout k_ext_scan_g (rsa_ctx.hip)
SCAN_SYMBOL = "k_ext_scan_g" if os.environ.get("RSA_SCAN_V", "1")[:1] == "0" else "k_ext_scan_v"
KERNEL_SYMBOLS = {"randstrobes": "k_randstrobes", "lookup": "k_seed_query", "find_nams": "k_find_nams_w2",
                  "rescue": "k_rescue_w", "compact": "k_compact", "ext_scan": SCAN_SYMBOL, "ext_band": "k_ext_band16",
                  "ext_band_wide": "k_ext_band64", "ext_band_panel": "k_ext_band_panel",
                  "sites": "k_sites", "ext_redo": "k_ext_scan"}
NK = len(KERNELS)
EXT_KERNELS = ("ext_scan", "ext_band", "ext_band_wide", "ext_band_panel", "ext_redo")   # launched by rsa_extend


class KernelStats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double * NK), ("launches", C.c_uint64 * NK), ("alg_bytes", C.c_double * NK),
                ("dp_cells_timed", C.c_uint64), ("seed_calls_timed", C.c_uint64),
                ("ext_calls_timed", C.c_uint64), ("seed_calls", C.c_uint64), ("ext_calls", C.c_uint64),
                ("reads", C.c_uint64), ("read_bases", C.c_uint64), ("query_randstrobes", C.c_uint64),
                ("lookups_found", C.c_uint64), ("filtered", C.c_uint64), ("hits", C.c_uint64),
                ("nams", C.c_uint64), ("rescued_reads", C.c_uint64),
                ("jobs", C.c_uint64), ("dp_cells", C.c_uint64),
                ("band_deferred", C.c_uint64), ("band_overflow", C.c_uint64),
                ("scan_certified", C.c_uint64), ("scan_redo", C.c_uint64),
                ("call_ms", C.c_double * 2), ("lane_wait_ms", C.c_double * 2), ("device_wait_ms", C.c_double * 2),
                ("query_written", C.c_uint64), ("query_fixed_reads", C.c_uint64),
                ("shared_checks", C.c_uint64), ("no_shared", C.c_uint64), ("seed_second_trips", C.c_uint64)]


def stats_dict(ks: "KernelStats") -> dict:
    """Flatten a KernelStats into {"kernels": {name: {ms, launches, alg_bytes}}, counters...}."""
    out = {"kernels": {k: {"ms": ks.kernel_ms[i], "launches": int(ks.launches[i]), "alg_bytes": ks.alg_bytes[i]}
                       for i, k in enumerate(KERNELS)}}
    for f, t in KernelStats._fields_[3:]:
        if t in (C.c_uint64,):
            out[f] = int(getattr(ks, f))
    # host-side view of the engine calls: {seed|extend: {call, lane_wait, device_wait} ms}
    out["calls_ms"] = {nm: {"call": round(ks.call_ms[i], 3), "lane_wait": round(ks.lane_wait_ms[i], 3),
                            "device_wait": round(ks.device_wait_ms[i], 3)} for i, nm in enumerate(("seed", "extend"))}
    return out


EXPORTED_SYMBOLS = ["rsa_open", "rsa_close", "rsa_last_error", "rsa_resident_bytes", "rsa_randstrobes",
                    "rsa_seed", "rsa_extend", "rsa_extend_cigar_bound", "rsa_host_alloc", "rsa_host_free",
                    "rsa_get_stats", "rsa_reset_stats", "rsa_index_build_run", "rsa_index_build_download",
                    "rsa_index_build_free", "rsa_open_built", "rsa_index_download", "rsa_extend_async",
                    "rsa_ready", "rsa_wait"]

_lib = None


def load(path: str = GPU_LIB):
    """Load librsa_gpu.so; raises if it is missing (no fallback path exists).
    RSA_GPU_LIB names another build of the same library (kernel A/B tooling)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("RSA_GPU_LIB", path)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not built: run __graft_entry__.build() (no CPU fallback exists)")
    lib = C.CDLL(path)
    lib.rsa_open.restype = C.c_void_p
    lib.rsa_open.argtypes = [C.c_int, C.POINTER(IndexView), C.c_char_p, C.c_size_t]
    lib.rsa_close.argtypes = [C.c_void_p]
    lib.rsa_last_error.restype = C.c_char_p
    lib.rsa_last_error.argtypes = [C.c_void_p]
    lib.rsa_resident_bytes.restype = C.c_uint64
    lib.rsa_resident_bytes.argtypes = [C.c_void_p]
    lib.rsa_randstrobes.argtypes = [C.c_void_p, C.POINTER(ReadBatch), C.POINTER(RandstrobeBatch)]
    lib.rsa_seed.argtypes = [C.c_void_p, C.POINTER(ReadBatch), C.c_int32, C.c_uint32, C.POINTER(NamBatch)]
    lib.rsa_extend.argtypes = [C.c_void_p, C.POINTER(JobBatch), C.POINTER(AlnBatch)]
    lib.rsa_extend_async.argtypes = [C.c_void_p, C.POINTER(JobBatch), C.POINTER(AlnBatch), C.POINTER(C.c_void_p)]
    lib.rsa_ready.argtypes = [C.c_void_p]
    lib.rsa_wait.argtypes = [C.c_void_p]
    lib.rsa_extend_cigar_bound.restype = C.c_uint64
    lib.rsa_extend_cigar_bound.argtypes = [C.POINTER(JobBatch)]
    lib.rsa_get_stats.argtypes = [C.c_void_p, C.POINTER(KernelStats)]
    lib.rsa_reset_stats.argtypes = [C.c_void_p]
    lib.rsa_index_build_run.restype = C.c_void_p
    lib.rsa_index_build_run.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(IndexBuildParams),
                                        C.POINTER(IndexBuildInfo), C.c_char_p, C.c_size_t]
    lib.rsa_index_build_download.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.rsa_index_build_free.argtypes = [C.c_void_p]
    lib.rsa_open_built.restype = C.c_void_p
    lib.rsa_open_built.argtypes = [C.c_void_p, C.POINTER(IndexView), C.c_char_p, C.c_size_t]
    _lib = lib
    return lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a is not None and a.size else 0


@dataclass
class Index:
    """A .sti index + reference held as numpy arrays (host side)."""
    randstrobes: np.ndarray      # structured (hash u8, position u4, packed u4)
    bucket_starts: np.ndarray    # uint64 [2^bits+1]
    bits: int
    filter_cutoff: int
    canonical_read_length: int
    k: int
    s: int
    l: int
    u: int
    q: int
    max_dist: int
    ref_seq: np.ndarray          # uint8 concatenated contigs
    contig_offsets: np.ndarray   # uint64 [n+1]
    names: list

    @property
    def t_syncmer(self):
        return (self.k - self.s) // 2 + 1

    @property
    def w_min(self):
        return max(0, self.k // (self.k - self.s + 1) + self.l)

    @property
    def w_max(self):
        return self.k // (self.k - self.s + 1) + self.u


RS_DTYPE = np.dtype([("hash", "<u8"), ("position", "<u4"), ("packed", "<u4")])


def read_fasta(path: str):
    """refs.cpp:20-58 semantics: name cut at the first ' ', bases uppercased (c & ~32)."""
    names, seqs = [], []
    cur = None
    with open(path, "rb") as f:
        for line in f:
            line = line.rstrip(b"\n")
            if line.startswith(b">"):
                if cur is not None and len(cur) > 0:
                    seqs.append(bytes(cur))
                    names.append(name)
                sp = line.find(b" ")
                name = (line[1:sp] if sp >= 0 else line[1:]).decode()
                cur = bytearray()
            else:
                cur += line
    if cur is not None and len(cur) > 0:
        seqs.append(bytes(cur))
        names.append(name)
    arrs = [np.frombuffer(s, dtype=np.uint8) & np.uint8(0xDF) for s in seqs]
    offs = np.zeros(len(arrs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(a) for a in arrs])
    ref = np.concatenate(arrs) if arrs else np.zeros(0, np.uint8)
    return names, ref, offs


def read_sti(path: str):
    """StrobemerIndex::read (src/index.cpp:91-132)."""
    with open(path, "rb") as f:
        buf = f.read()
    if buf[:4] != b"STI\x01":
        raise ValueError("bad .sti magic")
    ver = int.from_bytes(buf[4:8], "little")
    if ver != 2:
        raise ValueError("bad .sti version")
    res = int.from_bytes(buf[8:16], "little")
    o = 16 + res
    fc, bits = np.frombuffer(buf, dtype="<i4", count=2, offset=o)
    o += 8
    prm = np.frombuffer(buf, dtype="<i4", count=7, offset=o)
    o += 28
    n = int(np.frombuffer(buf, dtype="<u8", count=1, offset=o)[0])
    o += 8
    rs = np.frombuffer(buf, dtype=RS_DTYPE, count=n, offset=o)
    o += 16 * n
    ns = int(np.frombuffer(buf, dtype="<u8", count=1, offset=o)[0])
    o += 8
    st = np.frombuffer(buf, dtype="<u8", count=ns, offset=o)
    return dict(filter_cutoff=int(fc), bits=int(bits), r=int(prm[0]), k=int(prm[1]), s=int(prm[2]), l=int(prm[3]),
                u=int(prm[4]), q=int(prm[5]), max_dist=int(prm[6]), randstrobes=rs, bucket_starts=st)


def load_index(fasta: str, sti: str) -> Index:
    names, ref, offs = read_fasta(fasta)
    d = read_sti(sti)
    return Index(d["randstrobes"], d["bucket_starts"], d["bits"], d["filter_cutoff"], d["r"], d["k"], d["s"],
                 d["l"], d["u"], d["q"], d["max_dist"], ref, offs, names)


class IndexBuildParams(C.Structure):
    _fields_ = [("k", C.c_int32), ("s", C.c_int32), ("t_syncmer", C.c_int32), ("w_min", C.c_int32),
                ("w_max", C.c_int32), ("max_dist", C.c_int32), ("q", C.c_uint64), ("bits", C.c_int32),
                ("f", C.c_float), ("threads", C.c_int32)]


class IndexBuildInfo(C.Structure):
    _fields_ = [("n_randstrobes", C.c_uint64), ("n_syncmers", C.c_uint64), ("unique_hashes", C.c_uint64),
                ("bits", C.c_int32), ("filter_cutoff", C.c_int32), ("n_segments", C.c_uint64),
                ("replayed_segments", C.c_uint64), ("ms_upload", C.c_double), ("ms_syncmers", C.c_double),
                ("ms_randstrobes", C.c_double), ("ms_sort", C.c_double), ("ms_buckets", C.c_double),
                ("ms_total", C.c_double), ("position_ties", C.c_uint64), ("ms_tie_replay", C.c_double)]


def build_index(ref: np.ndarray, contig_offsets: np.ndarray, k=20, s=16, w_min=2, w_max=12, max_dist=80, q=255,
                bits=-1, f=0.0002, device=0, threads=0):
    """StrobemerIndex::populate on the GPU (rsa_index_build_run): returns
    (randstrobes [RS_DTYPE], bucket_starts [u64], filter_cutoff, info dict)."""
    lib = load()
    ref = np.ascontiguousarray(ref, dtype=np.uint8)
    offs = np.ascontiguousarray(contig_offsets, dtype=np.uint64)
    p = IndexBuildParams(k, s, (k - s) // 2 + 1, w_min, w_max, max_dist, q, bits, f, threads)
    info = IndexBuildInfo()
    err = C.create_string_buffer(512)
    h = lib.rsa_index_build_run(device, _ptr(ref), _ptr(offs), len(offs) - 1, C.byref(p), C.byref(info), err, 512)
    if not h:
        raise RuntimeError(err.value.decode())
    try:
        rs = np.zeros(info.n_randstrobes, dtype=RS_DTYPE)
        st = np.zeros((1 << info.bits) + 1, dtype=np.uint64)
        rc = lib.rsa_index_build_download(h, _ptr(rs), _ptr(st))
        if rc != 0:
            raise RuntimeError(f"rsa_index_build_download failed ({rc})")
    finally:
        lib.rsa_index_build_free(h)
    return rs, st, int(info.filter_cutoff), {f: getattr(info, f) for f, _ in IndexBuildInfo._fields_}


def empty_index(ref: np.ndarray, offs: np.ndarray, names=None) -> Index:
    """Index with no randstrobes (extension-only use)."""
    return Index(np.zeros(0, RS_DTYPE), np.zeros(257, np.uint64), 8, 30, 150, 20, 16, 1, 7, 255, 80,
                 ref, offs, names or [f"chr{i + 1}" for i in range(len(offs) - 1)])


class GpuContext:
    """One rsa_ctx (index + reference resident on one GPU)."""

    def __init__(self, index: Index, device: int = 0):
        self.lib = load()
        self.index = index
        v = IndexView()
        self._keep = [np.ascontiguousarray(index.randstrobes), np.ascontiguousarray(index.bucket_starts),
                      np.ascontiguousarray(index.ref_seq), np.ascontiguousarray(index.contig_offsets)]
        v.randstrobes = _ptr(self._keep[0])
        v.n_randstrobes = len(index.randstrobes)
        v.bucket_starts = _ptr(self._keep[1])
        v.bits = index.bits
        v.filter_cutoff = index.filter_cutoff
        v.k, v.s, v.t_syncmer = index.k, index.s, index.t_syncmer
        v.w_min, v.w_max, v.max_dist, v.q = index.w_min, index.w_max, index.max_dist, index.q
        v.ref_seq = _ptr(self._keep[2])
        v.contig_offsets = _ptr(self._keep[3])
        v.n_contigs = len(index.contig_offsets) - 1
        err = C.create_string_buffer(512)
        self.ctx = self.lib.rsa_open(device, C.byref(v), err, 512)
        if not self.ctx:
            raise RuntimeError(err.value.decode())

    def close(self):
        if self.ctx:
            self.lib.rsa_close(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed ({rc}): {self.lib.rsa_last_error(self.ctx).decode()}")

    @staticmethod
    def _reads(seqs):
        lens = np.array([len(s) for s in seqs], dtype=np.uint32)
        offs = np.zeros(len(seqs), dtype=np.uint64)
        if len(seqs):
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        blob = np.frombuffer(b"".join(seqs), dtype=np.uint8) if seqs else np.zeros(1, np.uint8)
        blob = np.ascontiguousarray(blob)
        rb = ReadBatch(_ptr(blob), _ptr(offs), _ptr(lens), len(seqs))
        return rb, (blob, offs, lens)

    def randstrobes(self, seqs):
        rb, keep = self._reads(seqs)
        cap = int(sum(2 * len(s) for s in seqs)) + 1
        out = np.zeros(cap, dtype=QRS_DTYPE)
        offs = np.zeros(len(seqs) + 1, dtype=np.uint64)
        b = RandstrobeBatch(_ptr(out), cap, _ptr(offs), 0)
        self._check(self.lib.rsa_randstrobes(self.ctx, C.byref(rb), C.byref(b)), "rsa_randstrobes")
        return [out[int(offs[i]):int(offs[i + 1])] for i in range(len(seqs))]

    def seed(self, seqs, rescue_level=2, rescue_cutoff=None, sites=False, mm_capacity=None, order=NAMS_FOUND,
             hamming=None):
        """NAM lists per read (+ nonrepetitive fraction, rescued flags); with sites=True
        also the per-NAM site checks (indexed by nam_id) and the mismatch-position pool
        (rsa_nam_site); order=NAMS_BY_SCORE returns lists of <= 16 NAMs sorted.
        hamming=(match, mismatch, end_bonus): accepted sites carry hamming_align's result
        in the pool instead of their positions (RSA_SITE_ALIGNED, decode_hamming)."""
        if rescue_cutoff is None:
            rescue_cutoff = rescue_level * self.index.filter_cutoff if rescue_level < 100 else 1000
        rb, keep = self._reads(seqs)
        cap = max(1024, 64 * len(seqs))
        while True:
            nams = np.zeros(cap, dtype=NAM_DTYPE)
            offs = np.zeros(len(seqs) + 1, dtype=np.uint64)
            nonrep = np.zeros(len(seqs), dtype=np.float32)
            resc = np.zeros(len(seqs), dtype=np.uint8)
            st = np.zeros(cap if sites else 0, dtype=SITE_DTYPE)
            mcap = (16 * cap if mm_capacity is None else mm_capacity) if sites else 0
            pool = np.zeros(max(1, mcap), dtype=np.uint16)
            hm = hamming or (0, 0, 0)
            b = NamBatch(_ptr(nams), cap, _ptr(offs), _ptr(nonrep), _ptr(resc), 0,
                         _ptr(st) if sites else 0, _ptr(pool) if sites else 0, mcap, 0, order,
                         1 if hamming else 0, hm[0], hm[1], hm[2], 0)
            rc = self.lib.rsa_seed(self.ctx, C.byref(rb), rescue_level, rescue_cutoff, C.byref(b))
            if rc == -3:
                cap = int(b.needed) + 1
                continue
            self._check(rc, "rsa_seed")
            lists = [nams[int(offs[i]):int(offs[i + 1])] for i in range(len(seqs))]
            if sites:
                return lists, nonrep, resc, [st[int(offs[i]):int(offs[i + 1])] for i in range(len(seqs))], \
                    pool[:int(b.mm_used)]
            return lists, nonrep, resc

    @staticmethod
    def decode_hamming(pool, offset):
        """hamming_align's result of an RSA_SITE_ALIGNED site: (score, start, end, mismatches, cigar ops)."""
        w = [int(x) for x in pool[offset:offset + 6]]
        score = w[0] | (w[1] << 16)
        if score >= 1 << 31:
            score -= 1 << 32
        ops = [int(pool[offset + 6 + 2 * i]) | (int(pool[offset + 7 + 2 * i]) << 16) for i in range(w[5])]
        return score, w[2], w[3], w[4], ops

    @staticmethod
    def _ext_batches(queries, jobs, match, mismatch, gap_open, gap_extend, end_bonus, lib):
        qb = np.frombuffer(queries, dtype=np.uint8) if len(queries) else np.zeros(1, np.uint8)
        jobs = np.ascontiguousarray(jobs, dtype=JOB_DTYPE)
        jb = JobBatch(_ptr(qb), len(queries), _ptr(jobs), len(jobs), match, mismatch, gap_open, gap_extend,
                      end_bonus)
        bound = int(lib.rsa_extend_cigar_bound(C.byref(jb)))
        alns = np.zeros(len(jobs), dtype=ALN_DTYPE)
        pool = np.zeros(bound + 1, dtype=np.uint32)
        ab = AlnBatch(_ptr(alns), _ptr(pool), bound + 1, 0)
        return jb, ab, alns, pool, (qb, jobs)

    def extend(self, queries, jobs, match=2, mismatch=8, gap_open=12, gap_extend=1, end_bonus=10):
        """queries: bytes blob; jobs: structured array JOB_DTYPE.  Returns (alns, cigar_pool)."""
        jb, ab, alns, pool, keep = self._ext_batches(queries, jobs, match, mismatch, gap_open, gap_extend,
                                                     end_bonus, self.lib)
        self._check(self.lib.rsa_extend(self.ctx, C.byref(jb), C.byref(ab)), "rsa_extend")
        return alns, pool

    def extend_async(self, queries, jobs, match=2, mismatch=8, gap_open=12, gap_extend=1, end_bonus=10):
        """rsa_extend_async: returns a PendingExtend; .ready() polls, .wait() -> (alns, cigar_pool)."""
        jb, ab, alns, pool, keep = self._ext_batches(queries, jobs, match, mismatch, gap_open, gap_extend,
                                                     end_bonus, self.lib)
        h = C.c_void_p()
        self._check(self.lib.rsa_extend_async(self.ctx, C.byref(jb), C.byref(ab), C.byref(h)), "rsa_extend_async")
        return PendingExtend(self, h, ab, alns, pool, keep)

    def stats(self) -> dict:
        s = KernelStats()
        self._check(self.lib.rsa_get_stats(self.ctx, C.byref(s)), "rsa_get_stats")
        return stats_dict(s)

    def reset_stats(self):
        self.lib.rsa_reset_stats(self.ctx)

    def resident_bytes(self) -> int:
        return int(self.lib.rsa_resident_bytes(self.ctx))


class PendingExtend:
    """An rsa_extend_async call: the batches it reads and writes live here until wait()."""

    def __init__(self, ctx, handle, ab, alns, pool, keep):
        self._ctx, self._h, self._ab, self.alns, self.pool, self._keep = ctx, handle, ab, alns, pool, keep

    def ready(self) -> bool:
        return bool(self._ctx.lib.rsa_ready(self._h))

    def wait(self):
        if self._h is None:
            raise RuntimeError("rsa_wait: already waited")
        h, self._h = self._h, None
        self._ctx._check(self._ctx.lib.rsa_wait(h), "rsa_wait")
        return self.alns, self.pool
