/*
 * rsa_gpu.h -- C-ABI boundary of the MI355X seed-and-extend path.
 *
 * This library (rabbitsalign_amd/lib/librsa_gpu.so, HIP/gfx950) replaces the
 * reference's hot path behind plain C entry points (no torch types, plain
 * pointers and sizes, int status returns, no exceptions across the boundary):
 *
 *   rsa_open / rsa_close  <- per-thread GASAL2 state set up lazily inside
 *                            solve_ssw_on_gpu (src/gasal2_ssw.cpp:29-102) and
 *                            the host-resident StrobemerIndex (src/index.hpp:37-183)
 *   rsa_randstrobes       <- randstrobes_query        (src/randstrobes.hpp:62, .cpp:207-253)
 *   rsa_seed              <- randstrobes_query + find_nams + find_nams_rescue as called by
 *                            align_{PE,SE}_read_part  (src/nam.hpp:40-49, src/aln.cpp:1946-1962)
 *   rsa_extend            <- solve_ssw_on_gpu         (src/gasal2_ssw.h:46-47) followed by the
 *                            gasal_fail / Aligner::align fallback (src/pc.cpp:1779-1788); the
 *                            result is exactly Aligner::align's AlignmentInfo
 *                            (src/aligner.cpp:114-210, src/aligner.hpp:20-30)
 *   rsa_index_build_*     <- StrobemerIndex::populate (src/index.cpp:141-309)
 *
 * Threading: every entry point is thread-safe on one context; concurrent calls
 * run on distinct HIP streams of the context (one stream "lane" per call).
 * Ownership: the caller owns every input and output buffer.  Results are
 * deterministic and independent of batch composition and job order.
 * Errors: a negative return value; rsa_last_error() describes it.  A missing
 * GPU or a failed HIP call is an error -- there is no CPU fallback.
 */
#ifndef RSA_GPU_H
#define RSA_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSA_OK 0
#define RSA_ERR_HIP (-1)
#define RSA_ERR_ARG (-2)
#define RSA_ERR_CAPACITY (-3)   /* an output buffer is too small; *_needed fields say how much */
#define RSA_ERR_NOMEM (-4)
#define RSA_ERR_BUSY (-5)       /* rsa_extend_async: RSA_MAX_PENDING calls not yet waited for */
#define RSA_ERR_INTERNAL (-6)   /* a device-side consistency check failed (a defect, not an input error) */

/* RefRandstrobe exactly as stored in a .sti file (src/randstrobes.hpp:20-49) */
typedef struct rsa_ref_randstrobe {
    uint64_t hash;
    uint32_t position;
    uint32_t packed;          /* ref_index << 8 | (strobe2 - strobe1) */
} rsa_ref_randstrobe;

/* Index + reference as loaded from <ref>.r<N>.sti and the FASTA
 * (src/index.cpp:91-132, IndexParameters src/indexparameters.hpp:73-104). */
typedef struct rsa_index_view {
    const rsa_ref_randstrobe* randstrobes;
    uint64_t n_randstrobes;
    const uint64_t* bucket_starts;     /* [2^bits + 1] */
    int32_t bits;
    int32_t filter_cutoff;
    int32_t k, s, t_syncmer;           /* SyncmerParameters */
    int32_t w_min, w_max, max_dist;    /* RandstrobeParameters */
    uint64_t q;
    const char* ref_seq;               /* contigs concatenated, uppercase (refs.cpp:8-16) */
    const uint64_t* contig_offsets;    /* [n_contigs + 1] */
    int32_t n_contigs;
} rsa_index_view;

typedef struct rsa_ctx rsa_ctx;

/* Upload index + reference to `device` (replicated per GPU). NULL on error. */
rsa_ctx* rsa_open(int device, const rsa_index_view* view, char* err, size_t err_len);
void rsa_close(rsa_ctx* ctx);
/* message of the CALLING THREAD's last failed call (valid until that thread's next
 * failing call); concurrent calls on one context never see each other's messages */
const char* rsa_last_error(rsa_ctx* ctx);
/* bytes of HBM the context holds resident (index + reference) */
uint64_t rsa_resident_bytes(const rsa_ctx* ctx);

/* ---- seeding ------------------------------------------------------------ */

typedef struct rsa_read_batch {
    const char* seq;          /* read bases, concatenated */
    const uint64_t* offsets;  /* [n_reads] start of read i in seq */
    const uint32_t* lengths;  /* [n_reads] */
    uint32_t n_reads;
} rsa_read_batch;

/* QueryRandstrobe (src/randstrobes.hpp:51-56) */
typedef struct rsa_query_randstrobe {
    uint64_t hash;
    uint32_t start;
    uint32_t end;
    uint32_t is_reverse;
    uint32_t pad_;
} rsa_query_randstrobe;

typedef struct rsa_randstrobe_batch {
    rsa_query_randstrobe* out;   /* caller-owned */
    uint64_t capacity;
    uint64_t* offsets;           /* [n_reads + 1] */
    uint64_t needed;             /* out: total count */
} rsa_randstrobe_batch;

int rsa_randstrobes(rsa_ctx* ctx, const rsa_read_batch* reads, rsa_randstrobe_batch* out);

/* Nam (src/nam.hpp:11-38), field order preserved, bool widened to int32 */
typedef struct rsa_nam {
    int32_t nam_id;
    int32_t query_start, query_end, query_prev_hit_startpos;
    int32_t ref_start, ref_end, ref_prev_hit_startpos;
    int32_t n_hits;
    int32_t ref_id;
    float score;
    int32_t is_rc;
} rsa_nam;

/* Per-NAM site checks, what align_*_read_part computes next
 * for a NAM against the reference window: reverse_nam_if_needed
 * (src/aln.cpp:60-93) and the Hamming test + mismatch positions of
 * extend_seed_part (src/aln.cpp:374-431, aligner.cpp:219-302). */
enum {
    RSA_SITE_ORIENT_MASK = 3,    /* 0 consistent as is, 1 consistent once reversed, 2 inconsistent */
    RSA_SITE_HAMMING = 4,        /* (reversed if 1) projection is read-length and consistent: n_mm = Hamming distance */
    RSA_SITE_POSITIONS = 8,      /* n_mm / read length < 0.05 and mm_pool[mm_offset .. + n_mm) holds the positions */
    RSA_SITE_POOL_FULL = 16,     /* as 8, but the pool was too small: the positions were not stored */
    RSA_SITE_ALIGNED = 32        /* with 8 (rsa_nam_batch.hamming_align set): mm_pool[mm_offset ..] holds
                                  * hamming_align's result (aligner.cpp:219-302) instead of the positions:
                                  * u16 words [score lo, score hi, segment start, segment end, mismatches in
                                  * the segment, n_ops], then n_ops CIGAR ops (len<<4|op) as (lo, hi) pairs;
                                  * 12 + 4 n_mm words at most */
};
/* One per NAM, at the NAM's nam_id within its read's list (sites + offsets[i] +
 * nam_id: the index the NAM had in find_nams' / find_nams_rescue's list, whatever
 * order the NAMs are returned in).  orig_*: the NAM as found, before any reversal
 * (reverse_nam_if_needed reverses from these, aln.cpp:78-90). */
typedef struct rsa_nam_site {
    uint8_t flags;
    uint8_t orig_is_rc;
    uint16_t n_mm;               /* mismatches of the read-length window (RSA_SITE_HAMMING), capped at 65535 */
    uint32_t mm_offset;          /* into mm_pool (RSA_SITE_POSITIONS) */
    int32_t orig_query_start, orig_query_end;
} rsa_nam_site;

/* rsa_nam_batch.order */
enum {
    RSA_NAMS_FOUND = 0,          /* each read's NAMs in the order find_nams / find_nams_rescue made them */
    RSA_NAMS_BY_SCORE = 1        /* lists of at most 16 NAMs in std::sort(by_score) order (aln.cpp:1962-1964:
                                  * libstdc++ sorts such lists by insertion, i.e. stable by descending score);
                                  * longer lists as found (the caller sorts them) */
};

typedef struct rsa_nam_batch {
    rsa_nam* nams;               /* caller-owned, NAMs of read i at [offsets[i], offsets[i+1]) */
    uint64_t capacity;
    uint64_t* offsets;           /* [n_reads + 1] */
    float* nonrepetitive_fraction; /* [n_reads], bit-equal to find_nams' .first */
    uint8_t* rescued;            /* [n_reads], 1 if find_nams_rescue produced the list */
    uint64_t needed;             /* out: total NAM count */
    /* optional (NULL: not computed): one site per NAM, mismatch positions (query
     * coordinates of the oriented read) in mm_pool[mm_capacity] */
    rsa_nam_site* sites;
    uint16_t* mm_pool;
    uint64_t mm_capacity;
    uint64_t mm_used;            /* out */
    uint32_t order;              /* RSA_NAMS_FOUND (0) or RSA_NAMS_BY_SCORE */
    uint32_t hamming_align;      /* 1: sites accepted by the Hamming test get hamming_align's result
                                  * (RSA_SITE_ALIGNED) with the scores below, not their positions */
    int32_t match, mismatch, end_bonus;   /* -A -B -L, for hamming_align */
    uint32_t pad_;
} rsa_nam_batch;

/* For every read: NAMs = find_nams(randstrobes_query(read)); if rescue_level > 1
 * and (NAMs empty or nonrepetitive_fraction < 0.7) then NAMs =
 * find_nams_rescue(..., rescue_cutoff)  (src/aln.cpp:1946-1962).  With
 * order = RSA_NAMS_FOUND the NAMs come in the reference's exact pre-sort order
 * (robin_hood slot order per orientation); RSA_NAMS_BY_SCORE hands lists of up
 * to 16 over already sorted, as the caller's std::sort would leave them. */
int rsa_seed(rsa_ctx* ctx, const rsa_read_batch* reads, int32_t rescue_level, uint32_t rescue_cutoff,
             rsa_nam_batch* out);

/* ---- extension ---------------------------------------------------------- */

/* One Smith-Waterman job: query bytes (caller buffer) vs a window of the
 * device-resident reference (contig ref_id, [ref_start, ref_start+ref_len)).
 * query_len holds the length in its low 24 bits.  A mate-rescue job may ask for
 * rescue_mate_part's pre-check as well (has_shared_substring, src/aln.cpp:1000-1013,
 * called at 1058): RSA_JOB_SHARED_CHECK | RSA_JOB_K(k) in query_len's high bits, for a
 * query of up to 1024 bp and a window of up to 4096.  The result then carries
 * RSA_ALN_NO_SHARED in rsa_aln.flags when no (2k/3)-mer of the query taken every k/3
 * bases occurs in the window: the caller's rescue is unaligned, and the SW result
 * (still computed) is not used. */
#define RSA_JOB_LEN_MASK 0x00FFFFFFu
#define RSA_JOB_SHARED_CHECK 0x80000000u
#define RSA_JOB_K(k) ((((uint32_t)(k)) & 0x7Fu) << 24)
#define RSA_SHARED_QMAX 1024
#define RSA_SHARED_WMAX 4096
typedef struct rsa_job {
    uint64_t query_offset;
    uint32_t query_len;
    int32_t ref_id;
    uint32_t ref_start;
    uint32_t ref_len;
} rsa_job;

typedef struct rsa_job_batch {
    const char* queries;       /* host buffer holding all query bytes */
    uint64_t queries_len;
    const rsa_job* jobs;
    uint32_t n_jobs;
    int32_t match, mismatch, gap_open, gap_extend, end_bonus;   /* -A -B -O -E -L */
} rsa_job_batch;

/* AlignmentInfo (src/aligner.hpp:20-30); CIGAR ops len<<4|op (src/cigar.hpp:11-21) */
typedef struct rsa_aln {
    int32_t sw_score;
    uint32_t edit_distance;
    uint32_t ref_start, ref_end;       /* half-open, relative to the job window */
    uint32_t query_start, query_end;   /* half-open */
    uint64_t cigar_offset;             /* into cigar_pool */
    uint32_t cigar_len;
    uint32_t flags;                    /* RSA_ALN_NO_SHARED (jobs with RSA_JOB_SHARED_CHECK) */
} rsa_aln;
#define RSA_ALN_NO_SHARED 1u
#define RSA_ALN_WORD_CERT 2u       /* informational: the scan's word-layout result stood on its band-path
                                      certificate (no byte-layout pass ran) */

typedef struct rsa_aln_batch {
    rsa_aln* alns;             /* [n_jobs] */
    uint32_t* cigar_pool;
    uint64_t cigar_capacity;
    uint64_t cigar_used;       /* out */
} rsa_aln_batch;

/* Aligner::align for every job.  ref_len > 2000 gives the reference's
 * sentinel (sw_score -1000000), a failed SSW the -100000 sentinel. */
int rsa_extend(rsa_ctx* ctx, const rsa_job_batch* jobs, rsa_aln_batch* out);

/* The same call split at the device boundary, so one host thread can overlap
 * its CPU work with the GPU, as the reference's worker does with gasal_aln_async
 * + gasal_is_aln_async_done (src/gasal2_ssw.cpp:114-249; pc.cpp:1699-1770 runs
 * part(N+1) while batch N extends).  rsa_extend_async validates the jobs, stages
 * them and enqueues every kernel and copy on a stream of its own, and returns;
 * `jobs` may be released then, but the query bytes and `out` must stay valid
 * until rsa_wait.  rsa_ready says whether the device part has finished (never
 * blocks); rsa_wait finishes the call (the rare one-lane band pass and the CIGAR
 * tail copy need the host), frees the handle and returns the call's status.
 * Results equal rsa_extend's.  At most RSA_MAX_PENDING calls per context may be
 * pending; the next one returns RSA_ERR_BUSY. */
#define RSA_MAX_PENDING 12
typedef struct rsa_pending rsa_pending;
int rsa_extend_async(rsa_ctx* ctx, const rsa_job_batch* jobs, rsa_aln_batch* out, rsa_pending** pending);
int rsa_ready(const rsa_pending* pending);
int rsa_wait(rsa_pending* pending);

/* upper bound of cigar_pool entries needed for a batch (the pool comes back
 * packed: cigar_used <= bound entries, alns[i].cigar_offset indexes it) */
uint64_t rsa_extend_cigar_bound(const rsa_job_batch* jobs);

/* Page-locked host memory for batch buffers (DMA-speed H2D/D2H); any caller
 * buffer works, these are only faster.  Portable: usable with every device's
 * context.  NULL on failure. */
void* rsa_host_alloc(size_t bytes);
void rsa_host_free(void* p);

/* ---- index construction -------------------------------- */

/* StrobemerIndex::populate (src/index.cpp:141-239) on the GPU: syncmers and
 * randstrobes of every contig (count_all_randstrobes / assign_all_randstrobes,
 * index.cpp:28-69, 244-309), the sort by (hash, position) (index.cpp:168),
 * the bucket table with the reference's exact fill rule (index.cpp:174-212)
 * and the filter cutoff (index.cpp:214-238).  The result is byte-identical to
 * the host build and to the .sti the reference writes: entries equal in (hash,
 * position) (duplicated sequence in two contigs) compare equal under
 * RefRandstrobe::operator< (randstrobes.hpp:32-35), and their order is the one
 * pdqsort_branchless's element moves produce; when the device sort finds any
 * (info.position_ties), the entries in generation order go to the host, where
 * that sort is replayed (sti_order.hpp), and come back. */
typedef struct rsa_index_build_params {
    int32_t k, s, t_syncmer;           /* SyncmerParameters */
    int32_t w_min, w_max, max_dist;    /* RandstrobeParameters */
    uint64_t q;
    int32_t bits;                      /* < 0: pick_bits (index.cpp:135-139) */
    float f;                           /* top fraction of repetitive hashes (-f, default 0.0002) */
    int32_t threads;                   /* host threads for the tie-order replay (<= 0: the machine's, max 64) */
} rsa_index_build_params;

typedef struct rsa_index_build_info {
    uint64_t n_randstrobes, n_syncmers, unique_hashes;
    int32_t bits, filter_cutoff;
    uint64_t n_segments;               /* reference segments processed in parallel */
    uint64_t replayed_segments;        /* segments whose warm-up did not converge (replayed from further back) */
    /* HIP-event times (ms): reference upload, syncmers (all passes), randstrobes,
     * sort (both radix passes + gathers), bucket table + counts; wall of the call */
    double ms_upload, ms_syncmers, ms_randstrobes, ms_sort, ms_buckets, ms_total;
    uint64_t position_ties;            /* entries equal in (hash, position) to their predecessor */
    double ms_tie_replay;              /* host replay of pdqsort's order (0 without ties), incl. transfers */
} rsa_index_build_info;

typedef struct rsa_index_build rsa_index_build;

/* Build the index of `ref_seq` (contigs back to back, contig i at
 * [contig_offsets[i], contig_offsets[i+1])) on `device`; the result stays in
 * HBM until freed.  NULL on error (message in err). */
rsa_index_build* rsa_index_build_run(int device, const char* ref_seq, const uint64_t* contig_offsets, int32_t n_contigs,
                                     const rsa_index_build_params* params, rsa_index_build_info* info, char* err,
                                     size_t err_len);
/* Copy the result into caller buffers: randstrobes[info.n_randstrobes],
 * bucket_starts[2^info.bits + 1]. */
int rsa_index_build_download(rsa_index_build* b, rsa_ref_randstrobe* randstrobes, uint64_t* bucket_starts);
void rsa_index_build_free(rsa_index_build* b);

/* Open a context on a GPU-built index without a copy: the context adopts the
 * build's device buffers (reference, entries, bucket table) and `b` is freed;
 * on error `b` stays valid.  `view` supplies the parameters, bits, filter cutoff
 * and contig offsets; its randstrobes, bucket_starts and ref_seq are not read. */
rsa_ctx* rsa_open_built(rsa_index_build* b, const rsa_index_view* view, char* err, size_t err_len);
/* Copy a context's resident index into caller buffers: randstrobes[n_randstrobes],
 * bucket_starts[2^bits + 1] (the host copy a GPU-built index does not keep). */
int rsa_index_download(rsa_ctx* ctx, rsa_ref_randstrobe* randstrobes, uint64_t* bucket_starts);

/* ---- instrumentation ------------------------------------------------------ */

/* kernels of the path, in stats arrays */
enum {
    RSA_K_RANDSTROBES = 0, /* syncmers + randstrobes per read (randstrobes.cpp:57-254) */
    RSA_K_LOOKUP = 1,      /* randstrobes + bucket lookup, filter probe, min_diff count, fused (k_seed_query;
                            * randstrobes.cpp:57-254, nam.cpp:68-85,920-943); RANDSTROBES then times only
                            * the lane kernel of reads over 512 bp */
    RSA_K_FIND_NAMS = 2,   /* hits_per_ref + merge_hits_into_nams (nam.cpp:87-245) */
    RSA_K_RESCUE = 3,      /* find_nams_rescue (nam.cpp:946-1010) */
    RSA_K_COMPACT = 4,     /* NAM output compaction */
    RSA_K_EXT_SCAN = 5,    /* SSW forward/reverse score scans (ssw.c:121-620) */
    RSA_K_EXT_BAND = 6,    /* banded_sw + traceback + Aligner::align, 16 lanes/job (ssw.c:622-790, aligner.cpp:114-210) */
    RSA_K_EXT_BAND_WIDE = 7, /* the same, 64 lanes/job, for the jobs the 16-lane kernel queues */
    RSA_K_EXT_BAND_PANEL = 8, /* the same, one wave per job sweeping 64-cell panels (bands > 64 cells) */
    RSA_K_SITES = 9,       /* per-NAM orientation + Hamming site checks (aln.cpp:60-93, 374-431) */
    RSA_K_EXT_REDO = 10,   /* the re-run of uncertified scan results: two-layout scan + band kernels */
    RSA_K_COUNT = 11
};

typedef struct rsa_kernel_stats {
    /* kernel_ms / launches / alg_bytes / dp_cells_timed: over the timed calls only
     * (one call in RSA_KTIMER_EVERY per lane, default 4) */
    double kernel_ms[RSA_K_COUNT];   /* sum of per-launch HIP-event durations (launch stream) */
    uint64_t launches[RSA_K_COUNT];
    double alg_bytes[RSA_K_COUNT];   /* algorithmic HBM bytes (DESIGN.md "Kernels") */
    uint64_t dp_cells_timed;         /* dp_cells of the timed rsa_extend calls */
    uint64_t seed_calls_timed, ext_calls_timed;
    uint64_t seed_calls, ext_calls;
    uint64_t reads, read_bases, query_randstrobes, lookups_found, filtered, hits, nams, rescued_reads;
    uint64_t jobs, dp_cells;         /* dp_cells: sum query_len * ref_len of the forward scan */
    uint64_t band_deferred, band_overflow;   /* jobs handed to the 64-lane / panel band kernels */
    uint64_t scan_certified, scan_redo;      /* word results taken without the byte pass (certified by the
                                              * band path), and those re-run through the two-layout scan */
    /* wall time of the calls ([0] rsa_seed, [1] rsa_extend), ms summed over calls: whole call,
     * waiting for a free stream lane, blocked on the device (event waits); the rest is host work */
    double call_ms[2], lane_wait_ms[2], device_wait_ms[2];
    /* query randstrobes the seeding call wrote out (the reads k_seed_query predicted the
     * global-map / rescue passes need), and reads whose randstrobes those passes had to make */
    uint64_t query_written, query_fixed_reads;
    /* extension jobs that carried RSA_JOB_SHARED_CHECK, and those that came back RSA_ALN_NO_SHARED */
    uint64_t shared_checks, no_shared;
    /* seeding calls whose first download was short and took a second round trip */
    uint64_t seed_second_trips;
} rsa_kernel_stats;

int rsa_get_stats(rsa_ctx* ctx, rsa_kernel_stats* out);
void rsa_reset_stats(rsa_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
