/*
 * rsa_oracle.h -- CPU restatement of the RabbitSAlign seed-and-extend hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: only tests/, the
 * __graft_entry__.smoke() check and bench.py's cpu_baseline leg may link or
 * call it.  The product (rabbitsalign_amd/) never links it and has no CPU
 * fallback.
 *
 * Every function restates the reference's behaviour (file:line cited at the
 * definition in rsa_oracle.c).  Parity of this restatement is PINNED against
 * golden vectors produced by the reference's own sources compiled from
 * /root/reference (oracle/Makefile -> oracle/_ref/refgen), see
 * tests/golden/README.md.
 */
#ifndef RSA_ORACLE_H
#define RSA_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- seeding ---------------------------------------------------------- */

typedef struct ora_params {
    int k, s, t_syncmer;        /* SyncmerParameters (indexparameters.hpp:11-37) */
    int w_min, w_max, max_dist; /* RandstrobeParameters (indexparameters.hpp:39-70) */
    uint64_t q;
} ora_params;

typedef struct ora_qrs {        /* QueryRandstrobe (randstrobes.hpp:51-56) */
    uint64_t hash;
    uint32_t start;
    uint32_t end;
    uint32_t is_reverse;
} ora_qrs;

uint64_t ora_xxh64(uint64_t x);

/* returns number of query randstrobes written (<= cap), or -1 if cap too small */
int ora_randstrobes_query(const char* seq, int len, const ora_params* p, ora_qrs* out, int cap);

/* ---- index ------------------------------------------------------------ */

typedef struct ora_refrs {      /* RefRandstrobe (randstrobes.hpp:20-49), 16-byte AoS as in .sti */
    uint64_t hash;
    uint32_t position;
    uint32_t packed;            /* ref_index << 8 | strobe2 offset */
} ora_refrs;

typedef struct ora_index {
    const ora_refrs* rs;
    uint64_t n;
    const uint64_t* starts;     /* [2^bits + 1] */
    int bits;
    unsigned filter_cutoff;
    int k;
} ora_index;

typedef struct ora_nam {        /* Nam (nam.hpp:11-38) */
    int32_t nam_id, query_start, query_end, query_prev_hit_startpos;
    int32_t ref_start, ref_end, ref_prev_hit_startpos, n_hits, ref_id;
    float score;
    int32_t is_rc;
} ora_nam;

/* find_nams (nam.cpp:771-926): returns #NAMs (pre-sort order), -1 if cap too small */
int ora_find_nams(const ora_index* idx, const ora_qrs* q, int nq, ora_nam* out, int cap, float* nonrep);
/* find_nams_rescue (nam.cpp:955-1012, pre_sort branch) */
int ora_find_nams_rescue(const ora_index* idx, const ora_qrs* q, int nq, unsigned rescue_cutoff,
                         ora_nam* out, int cap);

/* reverse_complement (revcomp.hpp:11-38) */
void ora_reverse_complement(const char* s, int len, char* out);
/* reverse_nam_if_needed (aln.cpp:60-93) + extend_seed_part's Hamming test
 * (aln.cpp:374-395) for one NAM; returns rsa_nam_site flags (rsa_gpu.h),
 * mismatch positions into mm_pos[L] when accepted (flag 8) */
int ora_nam_site(const ora_nam* nam, const char* read, const char* read_rc, int L, const char* contig, int64_t clen,
                 int k, uint16_t* mm_pos, int* n_mm);

/* ---- extension -------------------------------------------------------- */

typedef struct ora_ssw_res {    /* s_align (ssw.h) fields used by the C++ wrapper */
    int score1;
    int ref_begin1, ref_end1;
    int read_begin1, read_end1;
    int flag;
    int n_cigar;                /* ops written to cigar buffer (SSW encoding len<<4|op) */
} ora_ssw_res;

/* ssw_align(flag=0x0f, filters=0, filterd=32767) on translated (0..4) sequences
 * (ssw.c:818-922).  cigar must hold >= 2*(qlen+rlen)+8 ops. */
void ora_ssw_align(const int8_t* q, int qlen, const int8_t* r, int rlen, int match, int mismatch,
                   int gap_open, int gap_extend, ora_ssw_res* res, uint32_t* cigar);

/* the scan kernel's word-result certificate on one job (rsa_oracle.c): 0 not a
 * candidate, 1 path with an I next to a D, 2 certified and the byte layout saturates,
 * -1 certified but it does not (a counterexample) */
int ora_scan_certificate(const int8_t* q, int qlen, const int8_t* r, int rlen, int match, int mismatch,
                         int gap_open, int gap_extend);

typedef struct ora_aln_info {   /* AlignmentInfo (aligner.hpp:20-30) */
    uint32_t edit_distance, ref_start, ref_end, query_start, query_end;
    int32_t sw_score;
    int32_t n_cigar;            /* Cigar ops len<<4|op (cigar.hpp:11-21) */
} ora_aln_info;

/* Aligner::align (aligner.cpp:114-210) incl. SSW wrapper (ssw_cpp.cpp:54-210,432-471).
 * cigar must hold >= 2*(qlen+rlen)+8 ops. */
void ora_aligner_align(const char* query, int qlen, const char* ref, int rlen, int match, int mismatch,
                       int gap_open, int gap_extend, int end_bonus, ora_aln_info* out, uint32_t* cigar);

/* hamming_align (aligner.cpp:219-302) on equal-length query/ref: CIGAR ops in cigar
 * (>= 2n + 3 entries), their count returned */
int ora_hamming_align(const char* query, const char* ref, int n, int match, int mismatch, int end_bonus,
                      int* score, int* start, int* end, int* mismatches, uint32_t* cigar);

#ifdef __cplusplus
}
#endif
#endif
