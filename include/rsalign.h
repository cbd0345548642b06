/*
 * rsalign.h -- C-ABI of the whole mapping path (host pipeline + GPU engine),
 * librsalign.so.  It is the library form of the reference's CLI entry
 * (run_rabbitsalign, src/main.cpp:240-617: read references, load/build the
 * .sti index, spawn workers over read chunks, write SAM) so that a binding can
 * drive mapping without a subprocess.  bench.py and the Python mirror
 * (rabbitsalign_amd/mapper.py) use it through ctypes.
 */
#ifndef RSALIGN_H
#define RSALIGN_H

#include <stddef.h>
#include <stdint.h>

#include "rsa_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rsam rsam;              /* reference + index (+ engine) */
typedef struct rsam_reads rsam_reads;  /* a read set held in host memory */

typedef struct rsam_stats {
    uint64_t n_reads;         /* reads mapped (each mate counts, pc.cpp:1596) */
    uint64_t sam_bytes;       /* SAM body bytes produced */
    uint64_t sam_hash;        /* sum_k line_hash(line_k) * 0x100000001b3^(N-1-k) mod 2^64 over SAM body lines
                                 (line_hash: rsa_host.hpp SamDigest) */
    uint64_t sw_calls, tried, nam_rescue, mate_rescue, inconsistent;
    double map_seconds;       /* first chunk read -> last SAM byte (consumer cost, main.cpp:446,595) */
    /* host pipeline phases, seconds summed over worker threads (PE path) */
    double t_seed, t_extend, t_part, t_collect, t_last, t_sequential;
    /* s from the call: chunk 0 seeded; the last chunk's extension + store began; the last
     * chunk's SAM text went to the sink; all workers done (map_seconds: the sink closed) */
    double t_first_seeded, t_last_start, t_last_put, t_workers_done;
    /* s from the call: the first SAM text reached the writer; the first chunk's extension
     * call began and returned; chunks parted only for the insert-size estimate (rank mode) */
    double t_first_out, t_first_ext_begin, t_first_ext_end;
    uint64_t replayed_chunks;
} rsam_stats;

/* Open from files: FASTA + optional .sti (NULL: build the index in memory). */
rsam* rsam_open_files(const char* ref_fa, const char* sti, int read_len, int device, int threads, char* err,
                      size_t err_len);
/* Open on a synthetic reference (seeded): n_contigs equal contigs.
 * RSA_SYNTH_DUP=<bp> (measurement): chr1[1 Mb, 1 Mb + bp) is copied onto chr2 at the same
 * coordinates, a PAR-like region whose randstrobes tie in (hash, position). */
rsam* rsam_open_synthetic(uint64_t seed, uint64_t ref_len, int n_contigs, int read_len, int device, int threads,
                          char* err, size_t err_len);
/* Open on the host-side reference + index of another mapper (no rebuild). */
rsam* rsam_open_like(const rsam* other, int device, int threads, char* err, size_t err_len);
void rsam_close(rsam* m);

/* index/reference shape of a mapper */
typedef struct rsam_info {
    uint64_t ref_bases, n_randstrobes;
    int32_t n_contigs, bits, filter_cutoff, k, canonical_read_length;
    double index_seconds, upload_seconds;
    uint64_t device_resident_bytes;
    int32_t index_on_device;           /* 1: built on the GPU (rsa_index_build_run), 0: host build or .sti */
    int32_t pad_;
    double index_device_ms[6];         /* GPU build phases: upload, syncmers, randstrobes, sort, buckets, total */
    uint64_t index_replayed_segments;  /* GPU build: segments replayed past their warm-up (tandem repeats) */
    uint64_t index_position_ties;      /* entries equal in (hash, position) to their predecessor (other contigs) */
    double index_ms_tie_replay;        /* GPU build: host replay of pdqsort's order of those ties, incl. transfers */
} rsam_info;
int rsam_get_info(const rsam* m, rsam_info* out);

rsam_reads* rsam_reads_load(const char* fq1, const char* fq2 /* NULL: single-end */);
/* --interleaved input (one file, mates as consecutive records): rsam_map pairs the
 * records per chunk of 2 x chunk_size records as the reference's InputBuffer does
 * (src/pc.cpp:23-107) and maps the pairs; unpaired records are not mapped, as in
 * the reference's paired-end task (perform_task_async_pe). */
rsam_reads* rsam_reads_load_interleaved(const char* fq);
/* pairs p in [first, first + n) of the synthetic stream `seed` (paired or SE with mate 1 only) */
rsam_reads* rsam_reads_synthetic(const rsam* m, uint64_t seed, uint64_t first, uint64_t n, int read_len,
                                 double mu, double sigma, int paired);
/* FASTQ of a read set (mate 2 to fq2 when paired): test data and the I/O-inclusive bench leg */
int rsam_reads_write_fastq(const rsam_reads* r, const char* fq1, const char* fq2);
uint64_t rsam_reads_count(const rsam_reads* r);
void rsam_reads_free(rsam_reads* r);

/* Map every read; SAM to `sam_path` (header + body) or kept in memory only when NULL. */
int rsam_map(rsam* m, const rsam_reads* reads, int threads, int chunk_size, const char* sam_path,
             rsam_stats* out);
/* Map FASTQ/FASTA files as the CLI does: the reads are streamed (a reader thread per
 * file parses chunks of chunk_size pairs while the workers map, InputBuffer::read_records,
 * src/pc.cpp:74-107), so memory does not grow with the input.  fq2 NULL or "": single-end,
 * or interleaved pairs when `interleaved` != 0.  map_seconds runs from the call to the last
 * SAM byte written (the reference's consumer cost, src/main.cpp:446,595). */
int rsam_map_files(rsam* m, const char* fq1, const char* fq2, int interleaved, int threads, int chunk_size,
                   const char* sam_path, rsam_stats* out);
/* Note for long-lived hosts: a run that fails while a reader thread is blocked in
 * read() of a stalled pipe or terminal (not a regular file) returns after 2 s and
 * leaves that thread detached, holding its descriptor, until the read returns. */

/* ---- a rank's part of one input (rank/world mode) -----------
 * `world` processes (one per GPU, each with its own rsam) map ONE pair of FASTQ
 * files (plain or gzip).  The records are cut into the chunks of chunk_size pairs a
 * single process maps (each keeps its chunk_index, the minstd_rand seed of
 * src/pc.cpp:1583); rank r maps chunks [r*C/W, (r+1)*C/W) of the C chunks, after
 * replaying chunk 0.. until the insert-size estimate freezes (src/aln.cpp, 400
 * samples; output discarded) so every rank works with the same estimate.  Its SAM
 * part holds exactly its chunks' records, rank 0's after the header: the parts
 * concatenated in rank order are byte for byte the one-process SAM.  Statistics are
 * per part; the caller sums them over ranks (src/main.cpp:597-600).
 *
 * Planning needs each part's first record.  Each plain file is cut into world * 64 equal
 * byte blocks; rsam_part_count counts the newlines of rank's 64 blocks, the caller
 * all-gathers them (world * 64 integers per file, rank-major), and rsam_part_plan
 * turns them into the part.  NULL counts: the rank counts every block itself. */
#define RSAM_PART_BLOCKS 64
typedef struct rsam_part {
    int32_t rank, world;
    uint64_t chunk_size;
    uint64_t total_pairs, n_chunks;    /* of the whole input */
    uint64_t first_chunk, end_chunk;   /* this rank's chunks */
    uint64_t first_pair, n_pairs;      /* this rank's records (pairs; single-end: reads) */
    uint64_t offset1, offset2;         /* byte offset of first_pair in each file (record index when planned by records) */
    uint32_t flags;                    /* RSAM_PART_RECORDS1 / _RECORDS2: that file is planned by records */
    uint32_t reserved;
} rsam_part;
/* A file that is not plain four-line FASTQ -- gzip (the reference's usual input,
 * src/fastq.cpp:1-65), wrapped lines, FASTA -- is planned by records: every rank counts
 * its records with the kseq parser and streams it from the start, dropping the records
 * before its part.  rsam_part_count returns zeros for a gzip file (no byte blocks). */
#define RSAM_PART_RECORDS1 1u
#define RSAM_PART_RECORDS2 2u
/* newline counts of rank's RSAM_PART_BLOCKS blocks of `path` (threads: readers) */
int rsam_part_count(const char* path, int rank, int world, int threads, uint64_t* counts);
/* the part of `rank` (fq2 NULL or "": single-end); counts1/counts2: world * 64 each or NULL */
int rsam_part_plan(const char* fq1, const char* fq2, int rank, int world, int chunk_size, const uint64_t* counts1,
                   const uint64_t* counts2, int threads, rsam_part* out);
/* map a planned part: SAM body of its chunks to sam_path (rank 0: header first); a part
 * whose chunk or record bounds do not follow from (rank, world, chunk_size, total_pairs),
 * or whose byte offsets do not start a record, is refused (-1) */
int rsam_map_files_part(rsam* m, const char* fq1, const char* fq2, const rsam_part* part, int threads,
                        const char* sam_path, rsam_stats* out);

/* SAM digest (rsam_stats.sam_hash): an order-sensitive hash of the SAM body, folded in
 * by the workers as they format the records; on by default.  Off, sam_hash is 0 and the
 * hashing (about 5 % of the host pipeline's CPU time) is skipped. */
int rsam_set_sam_digest(rsam* m, int on);

/* Map on more devices of this node: each listed device gets its own engine with a
 * full replica of the index; rsam_map then sends every seeding / extension call to
 * the least busy device.  The SAM is the same for any number of devices (one chunk
 * queue, global chunk_index seeding, one insert-size freeze, one ordered writer). */
int rsam_add_devices(rsam* m, const int* devices, int n);

/* GPU kernel statistics of the engine (summed over devices; zeros for a CPU engine). */
int rsam_kernel_stats(rsam* m, rsa_kernel_stats* out);
void rsam_reset_kernel_stats(rsam* m);
const char* rsam_engine_name(const rsam* m);
const char* rsam_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
