"""Python mirror of the reference's mapping entry (run_rabbitsalign,
src/main.cpp:240-617) over the C-ABI of include/rsalign.h (librsalign.so).

    m = Mapper.synthetic(seed=1, ref_len=3_000_000_000, n_contigs=24, read_len=150)
    reads = m.synthetic_reads(seed=7, first=0, n=1_000_000, read_len=150, mu=300, sigma=30)
    st = m.map(reads, threads=16)          # SAM kept in memory, FNV-1a hash in st.sam_hash

The product library drives the HIP engine (librsa_gpu.so); nothing here
computes.  ``lib_path`` may name another build of the same ABI (bench.py's
cpu_baseline leg points it at oracle/_ref/librsalign_ref.so).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

from .native import LIB_DIR, KernelStats, stats_dict

PRODUCT_LIB = os.path.join(LIB_DIR, "librsalign.so")


class _Stats(C.Structure):
    _fields_ = [("n_reads", C.c_uint64), ("sam_bytes", C.c_uint64), ("sam_hash", C.c_uint64),
                ("sw_calls", C.c_uint64), ("tried", C.c_uint64), ("nam_rescue", C.c_uint64),
                ("mate_rescue", C.c_uint64), ("inconsistent", C.c_uint64), ("map_seconds", C.c_double),
                ("t_seed", C.c_double), ("t_extend", C.c_double), ("t_part", C.c_double),
                ("t_collect", C.c_double), ("t_last", C.c_double), ("t_sequential", C.c_double),
                ("t_first_seeded", C.c_double), ("t_last_start", C.c_double), ("t_last_put", C.c_double),
                ("t_workers_done", C.c_double), ("t_first_out", C.c_double), ("t_first_ext_begin", C.c_double),
                ("t_first_ext_end", C.c_double), ("replayed_chunks", C.c_uint64)]


class _Info(C.Structure):
    _fields_ = [("ref_bases", C.c_uint64), ("n_randstrobes", C.c_uint64), ("n_contigs", C.c_int32),
                ("bits", C.c_int32), ("filter_cutoff", C.c_int32), ("k", C.c_int32),
                ("canonical_read_length", C.c_int32), ("index_seconds", C.c_double),
                ("upload_seconds", C.c_double), ("device_resident_bytes", C.c_uint64),
                ("index_on_device", C.c_int32), ("pad_", C.c_int32), ("index_device_ms", C.c_double * 6),
                ("index_replayed_segments", C.c_uint64), ("index_position_ties", C.c_uint64),
                ("index_ms_tie_replay", C.c_double)]


class Part(C.Structure):
    """rsam_part (include/rsalign.h): one rank's chunks of a shared input."""
    _fields_ = [("rank", C.c_int32), ("world", C.c_int32), ("chunk_size", C.c_uint64), ("total_pairs", C.c_uint64),
                ("n_chunks", C.c_uint64), ("first_chunk", C.c_uint64), ("end_chunk", C.c_uint64),
                ("first_pair", C.c_uint64), ("n_pairs", C.c_uint64), ("offset1", C.c_uint64), ("offset2", C.c_uint64),
                ("flags", C.c_uint32), ("reserved", C.c_uint32)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


PART_BLOCKS = 64     # RSAM_PART_BLOCKS


EXPORTED_SYMBOLS = [
    "rsam_open_files", "rsam_open_synthetic", "rsam_open_like", "rsam_close", "rsam_get_info",
    "rsam_reads_load", "rsam_reads_load_interleaved", "rsam_reads_synthetic", "rsam_reads_write_fastq", "rsam_reads_count", "rsam_reads_free", "rsam_map", "rsam_map_files",
    "rsam_set_sam_digest", "rsam_add_devices", "rsam_kernel_stats", "rsam_reset_kernel_stats", "rsam_engine_name", "rsam_last_error",
    "rsam_part_count", "rsam_part_plan", "rsam_map_files_part",
]

_LIBS: dict = {}


def load(path: str = PRODUCT_LIB) -> C.CDLL:
    if path in _LIBS:
        return _LIBS[path]
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is not built (run `make -C rabbitsalign_amd`); there is no fallback path")
    lib = C.CDLL(path)
    vp, sz, u64, i32, cp = C.c_void_p, C.c_size_t, C.c_uint64, C.c_int, C.c_char_p
    lib.rsam_open_files.restype = vp
    lib.rsam_open_files.argtypes = [cp, cp, i32, i32, i32, cp, sz]
    lib.rsam_open_synthetic.restype = vp
    lib.rsam_open_synthetic.argtypes = [u64, u64, i32, i32, i32, i32, cp, sz]
    lib.rsam_open_like.restype = vp
    lib.rsam_open_like.argtypes = [vp, i32, i32, cp, sz]
    lib.rsam_close.argtypes = [vp]
    lib.rsam_get_info.argtypes = [vp, C.POINTER(_Info)]
    lib.rsam_reads_load.restype = vp
    lib.rsam_reads_load.argtypes = [cp, cp]
    lib.rsam_add_devices.argtypes = [vp, C.POINTER(C.c_int), i32]
    lib.rsam_reads_write_fastq.argtypes = [vp, cp, cp]
    lib.rsam_reads_load_interleaved.restype = vp
    lib.rsam_reads_load_interleaved.argtypes = [cp]
    lib.rsam_reads_synthetic.restype = vp
    lib.rsam_reads_synthetic.argtypes = [vp, u64, u64, u64, i32, C.c_double, C.c_double, i32]
    lib.rsam_reads_count.restype = u64
    lib.rsam_reads_count.argtypes = [vp]
    lib.rsam_reads_free.argtypes = [vp]
    lib.rsam_map.argtypes = [vp, vp, i32, i32, cp, C.POINTER(_Stats)]
    lib.rsam_map_files.argtypes = [vp, cp, cp, i32, i32, i32, cp, C.POINTER(_Stats)]
    lib.rsam_set_sam_digest.argtypes = [vp, i32]
    lib.rsam_kernel_stats.argtypes = [vp, C.POINTER(KernelStats)]
    lib.rsam_reset_kernel_stats.argtypes = [vp]
    lib.rsam_engine_name.restype = cp
    lib.rsam_engine_name.argtypes = [vp]
    lib.rsam_last_error.restype = cp
    u64p = C.POINTER(C.c_uint64)
    lib.rsam_part_count.argtypes = [cp, i32, i32, i32, u64p]
    lib.rsam_part_plan.argtypes = [cp, cp, i32, i32, i32, u64p, u64p, i32, C.POINTER(Part)]
    lib.rsam_map_files_part.argtypes = [vp, cp, cp, C.POINTER(Part), i32, cp, C.POINTER(_Stats)]
    _LIBS[path] = lib
    return lib


def unload(path: str = PRODUCT_LIB) -> None:
    """dlclose a library load() opened (every mapper of it closed first: rsam_close of the
    last one joins the pipeline's threads and frees its pooled buffers)."""
    lib = _LIBS.pop(path, None)
    if lib is not None:
        import _ctypes
        _ctypes.dlclose(lib._handle)


def part_count(path, rank: int, world: int, threads: int = 8, lib_path: str = PRODUCT_LIB) -> list:
    """Newline counts of rank's PART_BLOCKS byte blocks of `path` (rsam_part_count)."""
    lib = load(lib_path)
    out = (C.c_uint64 * PART_BLOCKS)()
    if lib.rsam_part_count(str(path).encode(), rank, world, threads, out) != 0:
        raise RuntimeError(f"rsam_part_count: {lib.rsam_last_error().decode()}")
    return list(out)


def part_plan(fq1, fq2, rank: int, world: int, chunk_size: int = 10000, counts1=None, counts2=None,
              threads: int = 8, lib_path: str = PRODUCT_LIB) -> Part:
    """Rank's part of the input (rsam_part_plan); counts: all world * PART_BLOCKS block counts
    of each file (rank-major, e.g. all-gathered part_count results) or None to count here."""
    lib = load(lib_path)
    def arr(c):
        if c is None:
            return None
        if len(c) != world * PART_BLOCKS:
            raise ValueError("expected world * PART_BLOCKS counts")
        return (C.c_uint64 * len(c))(*[int(x) for x in c])
    part = Part()
    if lib.rsam_part_plan(str(fq1).encode(), str(fq2).encode() if fq2 else None, rank, world, chunk_size,
                          arr(counts1), arr(counts2), threads, C.byref(part)) != 0:
        raise RuntimeError(f"rsam_part_plan: {lib.rsam_last_error().decode()}")
    return part


@dataclass
class MapStats:
    n_reads: int
    sam_bytes: int
    sam_hash: int
    sw_calls: int
    tried: int
    nam_rescue: int
    mate_rescue: int
    inconsistent: int
    map_seconds: float
    t_seed: float = 0.0
    t_extend: float = 0.0
    t_part: float = 0.0
    t_collect: float = 0.0
    t_last: float = 0.0
    t_sequential: float = 0.0
    t_first_seeded: float = 0.0
    t_last_start: float = 0.0
    t_last_put: float = 0.0
    t_workers_done: float = 0.0
    t_first_out: float = 0.0
    t_first_ext_begin: float = 0.0
    t_first_ext_end: float = 0.0
    replayed_chunks: int = 0


class Reads:
    def __init__(self, lib, handle):
        self._lib, self._h = lib, handle

    def __len__(self):
        return int(self._lib.rsam_reads_count(self._h))

    def write_fastq(self, fq1, fq2=None):
        if self._lib.rsam_reads_write_fastq(self._h, str(fq1).encode(), str(fq2).encode() if fq2 else None) != 0:
            raise RuntimeError(f"rsam_reads_write_fastq: {self._lib.rsam_last_error().decode()}")

    def close(self):
        if self._h:
            self._lib.rsam_reads_free(self._h)
            self._h = None

    def __del__(self):
        self.close()


class Mapper:
    """Reference + .sti index resident on one device, plus the host pipeline."""

    def __init__(self, lib, handle):
        self._lib, self._h = lib, handle

    @classmethod
    def _open(cls, lib, fn, *args):
        err = C.create_string_buffer(1024)
        h = fn(*args, err, len(err))
        if not h:
            raise RuntimeError(f"rsalign open failed: {err.value.decode(errors='replace')}")
        return cls(lib, h)

    @classmethod
    def from_files(cls, ref_fa, sti=None, read_len=150, device=0, threads=8, lib_path=PRODUCT_LIB):
        lib = load(lib_path)
        return cls._open(lib, lib.rsam_open_files, str(ref_fa).encode(), (str(sti).encode() if sti else None),
                         read_len, device, threads)

    @classmethod
    def synthetic(cls, seed, ref_len, n_contigs, read_len=150, device=0, threads=8, lib_path=PRODUCT_LIB):
        lib = load(lib_path)
        return cls._open(lib, lib.rsam_open_synthetic, seed, ref_len, n_contigs, read_len, device, threads)

    def like(self, device=0, threads=8, lib_path=PRODUCT_LIB):
        """Same reference + index (host copy), another engine build or device."""
        lib = load(lib_path)
        return Mapper._open(lib, lib.rsam_open_like, self._h, device, threads)

    @property
    def engine(self) -> str:
        return self._lib.rsam_engine_name(self._h).decode()

    def info(self) -> dict:
        i = _Info()
        self._lib.rsam_get_info(self._h, C.byref(i))
        out = {f: getattr(i, f) for f, _ in _Info._fields_ if f != "pad_"}
        out["index_device_ms"] = dict(zip(("upload", "syncmers", "randstrobes", "sort", "buckets", "total"),
                                          [round(x, 3) for x in i.index_device_ms]))
        return out

    def synthetic_reads(self, seed, first, n, read_len=150, mu=300.0, sigma=30.0, paired=True) -> Reads:
        return Reads(self._lib, self._lib.rsam_reads_synthetic(self._h, seed, first, n, read_len, mu, sigma,
                                                               1 if paired else 0))

    def load_reads(self, fq1, fq2=None, interleaved=False) -> Reads:
        if interleaved:
            h = self._lib.rsam_reads_load_interleaved(str(fq1).encode())
        else:
            h = self._lib.rsam_reads_load(str(fq1).encode(), str(fq2).encode() if fq2 else None)
        if not h:
            raise RuntimeError(self._lib.rsam_last_error().decode())
        return Reads(self._lib, h)

    def map(self, reads: Reads, threads=8, chunk_size=10000, sam_path=None) -> MapStats:
        st = _Stats()
        rc = self._lib.rsam_map(self._h, reads._h, threads, chunk_size,
                                str(sam_path).encode() if sam_path else None, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"rsam_map: {self._lib.rsam_last_error().decode()}")
        return MapStats(**{f: getattr(st, f) for f, _ in _Stats._fields_})

    def map_files(self, fq1, fq2=None, interleaved=False, threads=8, chunk_size=10000, sam_path=None) -> MapStats:
        """FASTQ files -> SAM, the reads streamed while mapping (the CLI's path);
        map_seconds = call -> last SAM byte written."""
        st = _Stats()
        rc = self._lib.rsam_map_files(self._h, str(fq1).encode(), str(fq2).encode() if fq2 else None,
                                      1 if interleaved else 0, threads, chunk_size,
                                      str(sam_path).encode() if sam_path else None, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"rsam_map_files: {self._lib.rsam_last_error().decode()}")
        return MapStats(**{f: getattr(st, f) for f, _ in _Stats._fields_})

    def map_files_part(self, fq1, fq2, part: Part, threads=8, sam_path=None) -> MapStats:
        """A rank's part of one input (rsam_map_files_part): its chunks' SAM records to
        sam_path (rank 0: header first); the parts in rank order are the one-process SAM."""
        st = _Stats()
        rc = self._lib.rsam_map_files_part(self._h, str(fq1).encode(), str(fq2).encode() if fq2 else None,
                                           C.byref(part), threads, str(sam_path).encode() if sam_path else None,
                                           C.byref(st))
        if rc != 0:
            raise RuntimeError(f"rsam_map_files_part: {self._lib.rsam_last_error().decode()}")
        return MapStats(**{f: getattr(st, f) for f, _ in _Stats._fields_})

    def set_sam_digest(self, on: bool):
        """MapStats.sam_hash computed while mapping (default) or not (sam_hash 0, less host CPU)."""
        self._lib.rsam_set_sam_digest(self._h, 1 if on else 0)

    def add_devices(self, devices):
        """Replicate the index on more devices and spread the mapping calls over them."""
        arr = (C.c_int * len(devices))(*devices)
        if self._lib.rsam_add_devices(self._h, arr, len(devices)) != 0:
            raise RuntimeError(f"rsam_add_devices: {self._lib.rsam_last_error().decode()}")

    def kernel_stats(self) -> dict:
        ks = KernelStats()
        self._lib.rsam_kernel_stats(self._h, C.byref(ks))
        return stats_dict(ks)

    def reset_kernel_stats(self):
        self._lib.rsam_reset_kernel_stats(self._h)

    def close(self):
        if self._h:
            self._lib.rsam_close(self._h)
            self._h = None

    def __del__(self):
        self.close()
