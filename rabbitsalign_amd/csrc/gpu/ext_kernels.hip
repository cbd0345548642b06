// ext_kernels.hip -- SSW-exact batched extension for gfx950.
//
// Replaces GASAL2's one-thread-per-alignment local kernel + get_tb
// (GASAL2/src/kernels/local_kernel_template.h:71-519, get_tb.h:4-149) and the
// CPU re-run through Aligner::align (src/aligner.cpp:114-210).  Results are
// bit-identical to the reference CPU path (ext/ssw/ssw.c + ssw_cpp.cpp):
//
//  k_ext_scan  one 64-lane wavefront per job.  The query is split over the
//              lanes (R consecutive rows per lane) and the reference streams
//              through them as an anti-diagonal systolic array: at step s lane l
//              owns column s-l; the row-above values (F, within-stripe F, H)
//              move one lane per step with a DPP wave_shr:1.  Both SSW passes
//              run here: forward (score1, ref_end1, read_end1) and the reverse
//              pass that stops at the first column reaching score1.  The SSW
//              striping artefact (cross-stripe F never feeds E, ssw.c:275-289)
//              is reproduced with the byte (16 stripes) / word (8 stripes)
//              layout of the reference.  Query/reference codes sit in LDS.
//  k_ext_band16 / k_ext_band64 / k_ext_band_panel  banded_sw (ssw.c:590-774)
//              with 16 or 64 lanes per job, one band cell per lane, or 64-lane
//              panels swept along each band row for the widest bands; then the
//              traceback, =/X CIGAR (ssw_cpp.cpp:126-210) and the end-bonus
//              extension (aligner.cpp:147-207).
//
// Integer DP, no MFMA.  Roofline: VALU-bound (cells/s), see DESIGN.md.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>

#include "rsa_dev.h"
#include "rsa_ext.h"

#define SCAN_WAVES 4
#define MAXQ_LDS 1024
#define MAXR_LDS 2048

__device__ __forceinline__ int subst(int a, int b, int match, int mismatch) {
    return (a == b && a < 4) ? match : -mismatch;
}

struct PassOut {
    int best, col, row;      // forward: max, first col, min row; reverse: see below
    int tcol, trow;          // reverse: first column reaching terminate
};

// One SSW pass over `ncol` reference columns with `nrow` query rows.
// fwd: row p -> qc[p], column c -> rc[c]
// rev: row p -> qc[qend - p], column c -> rc[rend - c]
// Per cell: E, Fw and F are kept >= 0 (result-neutral, as in SSW), so
// H' = max(0, diag + s, E, Fw) is a single max3.  The best-cell bookkeeping is
// per column: a lane takes its column maximum over its valid rows and only
// looks for the row when that maximum improves (same first-column /
// smallest-row tie rules as the per-cell strict '>').
template <int R, bool REV>
__device__ PassOut sw_pass(const uint8_t* __restrict__ qc, int nrow, const uint8_t* __restrict__ rc, int ncol,
                           int qend, int rend, int match, int mismatch, int gO, int gE, int seg,
                           int terminate, int lane) {
    const int lanes_used = (nrow + R - 1) / R;
    int E[R], Hc[R], qv[R];
    bool ss[R], valid[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        E[r] = 0;
        Hc[r] = 0;
        const int p = lane * R + r;
        ss[r] = (p % seg) == 0;
        valid[r] = p < nrow;
        const int code = valid[r] ? (int)qc[REV ? (qend - p) : p] : 7;
        qv[r] = code < 4 ? code : 7;          // N (and padding) never scores a match, not even vs N
    }
    int F_out = 0, Fw_out = 0, H_last = 0, diag_top = 0;
    int best = 0, bcol = INT_MAX, brow = INT_MAX;
    int tcol = INT_MAX, trow = INT_MAX;
    const int steps = ncol + lanes_used - 1;
    for (int s = 0; s < steps; ++s) {
        const int F_in = wave_shr1(F_out);
        const int Fw_in = wave_shr1(Fw_out);
        const int Hl_in = wave_shr1(H_last);
        const int c = s - lane;
        if (lane < lanes_used && c >= 0 && c < ncol) {
            const int rcode = rc[REV ? (rend - c) : c];
            int dg = diag_top, F = F_in, Fw = Fw_in, cm = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (ss[r]) Fw = 0;
                const int diag = dg + (qv[r] == rcode ? match : -mismatch);
                const int hm = max(max(diag, E[r]), Fw);
                const int h = max(hm, F);
                dg = Hc[r];
                Hc[r] = h;
                const int t = hm - gO;
                E[r] = max(max(E[r] - gE, t), 0);
                Fw = max(max(Fw - gE, t), 0);
                F = max(max(F - gE, h - gO), 0);
                cm = max(cm, valid[r] ? h : 0);
            }
            F_out = F;
            Fw_out = Fw;
            H_last = Hc[R - 1];
            if (!REV) {
                if (cm > best) {
                    best = cm;
                    bcol = c;
                    int row = INT_MAX;
#pragma unroll
                    for (int r = R - 1; r >= 0; --r)
                        if (valid[r] && Hc[r] == cm) row = lane * R + r;
                    brow = row;
                }
            } else {
                if (cm > best) best = cm;
                if (cm == terminate && tcol == INT_MAX) {
                    tcol = c;
                    int row = INT_MAX;
#pragma unroll
                    for (int r = R - 1; r >= 0; --r)
                        if (valid[r] && Hc[r] == terminate) row = lane * R + r;
                    trow = row;
                }
            }
        }
        diag_top = Hl_in;
        if (REV && (s & 7) == 7) {
            const int m = wave_min_i32(tcol);
            if (m != INT_MAX && s >= m + lanes_used - 1) break;
        }
        // forward byte pass: once the running max reaches the overflow bound
        // the word pass recomputes everything, so the rest is moot (ssw.c:846-849)
        if (!REV && terminate > 0 && (s & 7) == 7 && wave_max_i32(best) >= terminate) break;
    }
    PassOut o;
    o.best = best; o.col = bcol; o.row = brow; o.tcol = tcol; o.trow = trow;
    return o;
}

// Fused forward pass: the byte-mode (16 stripes) and word-mode (8 stripes)
// recurrences of SSW differ only in where the within-stripe F restarts, so
// both run in one sweep as the two 16-bit halves of packed registers
// (v_pk_*_i16): low half = byte layout, high half = word layout.  The caller
// keeps the byte result unless its max reaches the overflow bound, exactly
// like ssw_align (ssw.c:838-850) -- without the second pass.  Needs every
// score to fit int16 (host-checked: match * qlen < 30000).
typedef short pk16 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ pk16 pk_from(uint32_t x) { return __builtin_bit_cast(pk16, x); }
__device__ __forceinline__ uint32_t pk_bits(pk16 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ pk16 pk_max(pk16 a, pk16 b) { return __builtin_elementwise_max(a, b); }

struct FusedOut {
    int best[2], col[2], row[2];     // [0] byte layout, [1] word layout
};

template <int R>
__device__ FusedOut sw_fwd_fused(const uint8_t* __restrict__ qc, int nrow, const uint8_t* __restrict__ rc, int ncol,
                                 int match, int mismatch, int gO, int gE, int lane) {
    const int lanes_used = (nrow + R - 1) / R;
    const int seg_b = (nrow + 15) / 16, seg_w = (nrow + 7) / 8;
    pk16 E[R], Hc[R];
    int qv[R];
    uint32_t ssm[R], vm[R];
    const pk16 zero = {0, 0};
    const pk16 GO2 = {(short)gO, (short)gO}, GE2 = {(short)gE, (short)gE};
    const uint32_t M2 = pk_bits((pk16){(short)match, (short)match});
    const uint32_t X2 = pk_bits((pk16){(short)-mismatch, (short)-mismatch});
#pragma unroll
    for (int r = 0; r < R; ++r) {
        E[r] = zero;
        Hc[r] = zero;
        const int p = lane * R + r;
        ssm[r] = ((p % seg_b) == 0 ? 0u : 0x0000FFFFu) | ((p % seg_w) == 0 ? 0u : 0xFFFF0000u);
        vm[r] = p < nrow ? 0xFFFFFFFFu : 0u;
        const int code = p < nrow ? (int)qc[p] : 7;
        qv[r] = code < 4 ? code : 7;
    }
    uint32_t F_out = 0, Fw_out = 0, H_last = 0, diag_top = 0;
    FusedOut o;
    o.best[0] = o.best[1] = 0;
    o.col[0] = o.col[1] = INT_MAX;
    o.row[0] = o.row[1] = INT_MAX;
    const int steps = ncol + lanes_used - 1;
    for (int s = 0; s < steps; ++s) {
        const uint32_t F_in = (uint32_t)wave_shr1((int)F_out);
        const uint32_t Fw_in = (uint32_t)wave_shr1((int)Fw_out);
        const uint32_t Hl_in = (uint32_t)wave_shr1((int)H_last);
        const int c = s - lane;
        if (lane < lanes_used && c >= 0 && c < ncol) {
            const int rcode = rc[c];
            pk16 dg = pk_from(diag_top), F = pk_from(F_in), Fw = pk_from(Fw_in), cm = zero;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                Fw = pk_from(pk_bits(Fw) & ssm[r]);
                const pk16 diag = dg + pk_from(qv[r] == rcode ? M2 : X2);
                const pk16 hm = pk_max(pk_max(diag, E[r]), Fw);
                const pk16 h = pk_max(hm, F);
                dg = Hc[r];
                Hc[r] = h;
                const pk16 t = hm - GO2;
                E[r] = pk_max(pk_max(E[r] - GE2, t), zero);
                Fw = pk_max(pk_max(Fw - GE2, t), zero);
                F = pk_max(pk_max(F - GE2, h - GO2), zero);
                cm = pk_max(cm, pk_from(pk_bits(h) & vm[r]));
            }
            F_out = pk_bits(F);
            Fw_out = pk_bits(Fw);
            H_last = pk_bits(Hc[R - 1]);
            const uint32_t cmb = pk_bits(cm);
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int v = (int)((cmb >> (16 * hf)) & 0xFFFFu);
                if (v > o.best[hf]) {
                    o.best[hf] = v;
                    o.col[hf] = c;
                    int row = INT_MAX;
#pragma unroll
                    for (int r = R - 1; r >= 0; --r)
                        if (vm[r] && (int)((pk_bits(Hc[r]) >> (16 * hf)) & 0xFFFFu) == v) row = lane * R + r;
                    o.row[hf] = row;
                }
            }
        }
        diag_top = Hl_in;
    }
    return o;
}

template <int RMAX>
__device__ FusedOut sw_fwd_fused_dispatch(const uint8_t* qc, int nrow, const uint8_t* rc, int ncol, int match,
                                          int mismatch, int gO, int gE, int lane) {
    const int R = (nrow + 63) / 64;
#define RSA_FUSED(N) if constexpr (N <= RMAX) return sw_fwd_fused<N>(qc, nrow, rc, ncol, match, mismatch, gO, gE, lane);
    if (R <= 1) { RSA_FUSED(1) }
    if (R == 2) { RSA_FUSED(2) }
    if (R == 3) { RSA_FUSED(3) }
    if (R == 4) { RSA_FUSED(4) }
    if (R <= 6) { RSA_FUSED(6) }
    if (R <= 8) { RSA_FUSED(8) }
    if (R <= 12) { RSA_FUSED(12) }
    RSA_FUSED(16)
#undef RSA_FUSED
    FusedOut o{};
    return o;
}

// R = rows per lane; the kernel is instantiated per RMAX so its register
// allocation (and occupancy) is that of the largest R it can take, not 16.
template <bool REV, int RMAX>
__device__ PassOut sw_pass_dispatch(const uint8_t* qc, int nrow, const uint8_t* rc, int ncol, int qend, int rend,
                                    int match, int mismatch, int gO, int gE, int seg, int terminate, int lane) {
    const int R = (nrow + 63) / 64;
#define RSA_PASS(N)                                                                                              \
    if constexpr (N <= RMAX) return sw_pass<N, REV>(qc, nrow, rc, ncol, qend, rend, match, mismatch, gO, gE, seg, \
                                                    terminate, lane);
    if (R <= 1) { RSA_PASS(1) }
    if (R == 2) { RSA_PASS(2) }
    if (R == 3) { RSA_PASS(3) }
    if (R == 4) { RSA_PASS(4) }
    if (R <= 6) { RSA_PASS(6) }
    if (R <= 8) { RSA_PASS(8) }
    if (R <= 12) { RSA_PASS(12) }
    RSA_PASS(16)
#undef RSA_PASS
    PassOut o{};
    return o;   // unreachable: the host picks RMAX >= R of every job
}

template <int RMAX>
__global__ void __launch_bounds__(64 * SCAN_WAVES)
k_ext_scan(const ExtJobDev* __restrict__ jobs, int n_jobs, const int* __restrict__ idx, const char* __restrict__ qbuf,
           const char* __restrict__ ref, ScanRes* __restrict__ out, int match, int mismatch, int gO, int gE,
           const int* __restrict__ n_dev) {
    // n_dev: the list's length as the device counted it (the in-stream redo pass); the
    // grid covers n_jobs at most
    if (n_dev) n_jobs = min(n_jobs, *n_dev);
    __shared__ uint8_t s_q[SCAN_WAVES][MAXQ_LDS];
    // every packed 16-bit score stays far inside int16
    const bool fused_ok = match >= 0 && match <= 28 && mismatch >= 0 && mismatch < 4000 && gO >= 0 && gO < 4000 &&
                          gE >= 0 && gE < 4000;
    __shared__ uint8_t s_r[SCAN_WAVES][MAXR_LDS];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int k = blockIdx.x * SCAN_WAVES + wave;
    // every wave reaches the barrier; invalid / sentinel jobs skip the work after it
    const bool in_range = k < n_jobs;
    const int j = in_range ? (idx ? idx[k] : k) : 0;
    ExtJobDev jb;
    jb.q_off = 0; jb.r_off = 0; jb.qlen = 0; jb.rlen = 0; jb.cig_off = 0;
    if (in_range) jb = jobs[j];
    const bool sentinel = in_range && (jb.rlen > 2000 || jb.qlen == 0 || jb.qlen > MAXQ_LDS);
    const bool work = in_range && !sentinel;
    ScanRes res;
    res.score1 = 0; res.ref_end1 = -1; res.read_end1 = 0; res.ref_begin1 = -1; res.read_begin1 = 0;
    res.flag = 0; res.word = 0; res.status = 0;
    const int qlen = (int)jb.qlen, rlen = (int)jb.rlen;
    uint8_t* qc = s_q[wave];
    uint8_t* rc = s_r[wave];
    if (work) {
        for (int i = lane; i < qlen; i += 64) qc[i] = (uint8_t)ssw_code((unsigned char)qbuf[jb.q_off + i]);
        for (int i = lane; i < rlen; i += 64) rc[i] = (uint8_t)ssw_code((unsigned char)ref[jb.r_off + i]);
    }
    __syncthreads();
    if (!work) {
        if (sentinel && lane == 0) { res.status = jb.qlen > MAXQ_LDS ? 2 : 1; out[j] = res; }
        return;
    }

    // forward pass, byte layout first (sw_sse2_byte), word layout on overflow (ssw.c:838-850)
    int word = 0;
    PassOut f;
    int score1;
    if (fused_ok) {
        const FusedOut fo = sw_fwd_fused_dispatch<RMAX>(qc, qlen, rc, rlen, match, mismatch, gO, gE, lane);
        const int sb = wave_max_i32(fo.best[0]);
        word = sb + mismatch >= 255 ? 1 : 0;
        f.best = fo.best[word]; f.col = fo.col[word]; f.row = fo.row[word];
        score1 = word ? wave_max_i32(fo.best[1]) : sb;
    } else {
        f = sw_pass_dispatch<false, RMAX>(qc, qlen, rc, rlen, 0, 0, match, mismatch, gO, gE, (qlen + 15) / 16,
                                             255 - mismatch, lane);
        score1 = wave_max_i32(f.best);
        if (score1 + mismatch >= 255) {
            word = 1;
            f = sw_pass_dispatch<false, RMAX>(qc, qlen, rc, rlen, 0, 0, match, mismatch, gO, gE, (qlen + 7) / 8, 0,
                                                 lane);
            score1 = wave_max_i32(f.best);
        }
    }
    int ref_end1, read_end1;
    if (score1 == 0) {
        ref_end1 = word ? 0 : -1;
        read_end1 = 0;
    } else {
        ref_end1 = wave_min_i32(f.best == score1 ? f.col : INT_MAX);
        read_end1 = wave_min_i32((f.best == score1 && f.col == ref_end1) ? f.row : INT_MAX);
    }
    res.score1 = score1; res.ref_end1 = ref_end1; res.read_end1 = read_end1; res.word = word;

    if (score1 > 0) {
        // reverse pass (ssw.c:877-893)
        const int nrow = read_end1 + 1, ncol = ref_end1 + 1;
        const int seg = word ? (nrow + 7) / 8 : (nrow + 15) / 16;
        PassOut b = sw_pass_dispatch<true, RMAX>(qc, nrow, rc, ncol, read_end1, ref_end1, match, mismatch,
                                                             gO, gE, seg, score1, lane);
        const int tcol = wave_min_i32(b.tcol);
        if (tcol == INT_MAX) {
            res.flag = 2;   // reverse max < score1: "may miss a small part"
            res.ref_begin1 = 0;
            res.read_begin1 = 0;
        } else {
            const int trow = wave_min_i32(b.tcol == tcol ? b.trow : INT_MAX);
            res.ref_begin1 = ref_end1 - tcol;
            res.read_begin1 = read_end1 - trow;
        }
    } else {
        res.ref_begin1 = word ? 0 : -1;
        res.read_begin1 = 0;
    }
    if (lane == 0) out[j] = res;
}

__device__ __forceinline__ uint32_t cig(uint32_t len, uint32_t op) { return (len << 4) | op; }

// Cigar::push merge rule (src/cigar.hpp:52-59)
__device__ __forceinline__ void cpush(uint32_t* c, int& n, uint32_t op, uint32_t len) {
    if (n == 0 || (c[n - 1] & 0xf) != op) c[n++] = (len << 4) | op;
    else c[n - 1] += len << 4;
}

// ConvertAlignment + CalculateNumberMismatch + the end-bonus step of
// Aligner::align, given the raw banded_sw ops of a job (shared by both band kernels).
// qcs/rcs (optional): SSW codes of the aligned segment, read_begin1.. and
// ref_begin1.. (the band kernels hold them in LDS); without them the =/X split
// translates the bytes from global memory.
//
__device__ void ext_finish(const ExtJobDev& jb, const ScanRes& sr, const char* __restrict__ q,
                          const char* __restrict__ r, const uint32_t* __restrict__ raw, int nraw,
                          uint32_t* __restrict__ c, rsa_aln& a, int match, int mismatch, int bonus, int gO, int gE,
                          const uint8_t* qcs = nullptr, const uint8_t* rcs = nullptr) {
    const int qlen = (int)jb.qlen, rlen = (int)jb.rlen;
    // ConvertAlignment + CalculateNumberMismatch (ssw_cpp.cpp:54-90, 126-210).
    // Core ops are built after a gap of qs+2 entries (room for the left end-bonus ops).
    const int qs0 = sr.read_begin1;
    int base = qs0 + 2;
    int n = 0;
    uint32_t* core = c + base;
    int mism = 0;
    if (qs0 > 0) core[n++] = cig((uint32_t)qs0, 4);
    int rp = sr.ref_begin1, qp = qs0;
    int in_m = 0, in_x = 0;
    uint32_t len_m = 0, len_x = 0;
    for (int k = 0; k < nraw; ++k) {
        const uint32_t opk = raw[k] & 0xf, lenk = raw[k] >> 4;
        if (opk == 0) {
            // the =/X split 32 bases at a time: a branch-free pass builds the chunk's mismatch
            // mask (its LDS loads issue back to back), then its runs are emitted from the mask
            // -- the same ops as comparing base by base
            for (uint32_t z = 0; z < lenk; z += 32) {
                const uint32_t cnt = lenk - z < 32 ? lenk - z : 32;
                const int qo = qp - qs0, ro = rp - sr.ref_begin1;
                uint32_t mm = 0;
                if (qcs && qo >= 0 && qo + (int)cnt - 1 <= sr.read_end1 - qs0 && ro >= 0 &&
                    ro + (int)cnt - 1 <= sr.ref_end1 - sr.ref_begin1) {
#pragma unroll 8
                    for (uint32_t b = 0; b < cnt; ++b) mm |= (uint32_t)(rcs[ro + b] != qcs[qo + b]) << b;
                } else {
                    for (uint32_t b = 0; b < cnt; ++b) {
                        const int rr = rp + (int)b;
                        const int rcode = (rr >= 0 && rr < rlen) ? ssw_code((unsigned char)r[rr]) : 4;
                        const int qcode = ssw_code((unsigned char)q[qp + (int)b]);
                        mm |= (uint32_t)(rcode != qcode) << b;
                    }
                }
                uint64_t m = mm;                            // 64-bit: a shift by 32 stays defined
                uint32_t rem = cnt;
                while (rem) {
                    if (m & 1) {                            // a run of mismatches
                        uint32_t run = (uint32_t)__builtin_ctzll(~m);
                        run = run < rem ? run : rem;
                        if (in_m) core[n++] = cig(len_m, 7);
                        mism += (int)run;
                        len_m = 0; len_x += run; in_m = 0; in_x = 1;
                        m >>= run; rem -= run;
                    } else {                                // a run of matches
                        uint32_t run = m ? (uint32_t)__builtin_ctzll(m) : rem;
                        run = run < rem ? run : rem;
                        if (in_x) core[n++] = cig(len_x, 8);
                        len_m += run; len_x = 0; in_m = 1; in_x = 0;
                        m >>= run; rem -= run;
                    }
                }
                rp += (int)cnt; qp += (int)cnt;
            }
        } else if (opk == 1 || opk == 2) {
            const uint32_t rawk = raw[k];
            if (opk == 1) qp += (int)lenk; else rp += (int)lenk;
            mism += (int)lenk;
            if (in_m) core[n++] = cig(len_m, 7);
            else if (in_x) core[n++] = cig(len_x, 8);
            in_m = in_x = 0; len_m = len_x = 0;
            core[n++] = rawk;
        }
    }
    if (in_m) core[n++] = cig(len_m, 7);
    else if (in_x) core[n++] = cig(len_x, 8);
    const int tail = qlen - sr.read_end1 - 1;
    if (tail > 0) core[n++] = cig((uint32_t)tail, 4);

    // Aligner::align end bonus (aligner.cpp:138-207).  The scans over the clipped ends are
    // sums (no early exit), so they run branch-free with their loads issued ahead, and the
    // =/X ops of a taken end are pushed run by run from 32-base match masks.
    auto end_scan = [&](const char* qa, const char* rb, uint32_t len, int& score, uint32_t& edits) {
#pragma unroll 8
        for (uint32_t i = 0; i < len; ++i) {
            const bool eq = qa[i] == rb[i];
            score += eq ? match : -mismatch;
            edits += eq ? 0u : 1u;
        }
    };
    auto push_eq_runs = [&](int& fn, const char* qa, const char* rb, uint32_t len) {
        for (uint32_t z = 0; z < len; z += 32) {
            const uint32_t cnt = len - z < 32 ? len - z : 32;
            uint32_t eqm = 0;
#pragma unroll 8
            for (uint32_t b = 0; b < cnt; ++b) eqm |= (uint32_t)(qa[z + b] == rb[z + b]) << b;
            uint64_t m = eqm;
            uint32_t rem = cnt;
            while (rem) {
                const bool eq = m & 1;
                uint32_t run = eq ? (uint32_t)__builtin_ctzll(~m) : (m ? (uint32_t)__builtin_ctzll(m) : rem);
                run = run < rem ? run : rem;
                cpush(c, fn, eq ? 7u : 8u, run);
                m >>= run;
                rem -= run;
            }
        }
    };
    uint32_t ed = (uint32_t)mism;
    int sw = sr.score1;
    uint32_t rs = (uint32_t)sr.ref_begin1, re = (uint32_t)sr.ref_end1 + 1;
    uint32_t qs = (uint32_t)qs0, qe = (uint32_t)sr.read_end1 + 1;
    int final_n;
    {
        const uint32_t steps = qs < rs ? qs : rs;      // while (q0 > 0 && r0 > 0)
        const uint32_t q0 = qs - steps, r0 = rs - steps;
        int score = sw;
        uint32_t edits = ed;
        end_scan(q + q0, r + r0, steps, score, edits);
        if (q0 == 0 && score + bonus > sw) {
            if (qs > 0) {
                // front ops in left-to-right order, then core without its leading S
                int fn = 0;
                push_eq_runs(fn, q, r + (rs - qs), qs);
                for (int k = 1; k < n; ++k) cpush(c, fn, core[k] & 0xf, core[k] >> 4);
                final_n = fn;
            } else {
                for (int k = 0; k < n; ++k) c[k] = core[k];
                final_n = n;
            }
            qs = 0; rs = r0; sw = score + bonus; ed = edits;
        } else {
            for (int k = 0; k < n; ++k) c[k] = core[k];
            final_n = n;
        }
    }
    {
        const uint32_t qrem = (uint32_t)qlen - qe, rrem = (uint32_t)rlen - re;
        const uint32_t steps = qrem < rrem ? qrem : rrem;   // while (q1 < qlen && r1 < rlen)
        const uint32_t q1 = qe + steps, r1 = re + steps;
        int score = sw;
        uint32_t edits = ed;
        end_scan(q + qe, r + re, steps, score, edits);
        if (q1 == (uint32_t)qlen && score + bonus > sw) {
            if (qe < (uint32_t)qlen) {
                final_n--;   // drop trailing soft clip
                push_eq_runs(final_n, q + qe, r + re, (uint32_t)qlen - qe);
            }
            qe = (uint32_t)qlen; re = r1; sw = score + bonus; ed = edits;
        }
    }
    a.sw_score = sw; a.edit_distance = ed; a.ref_start = rs; a.ref_end = re; a.query_start = qs; a.query_end = qe;
    a.cigar_len = (uint32_t)final_n;
}

// ---------------------------------------------------------------------------
// Group-parallel banded_sw: G lanes per job (G = 16: 4 jobs per wave; G = 64:
// one job per wave).
//
// Same result as banded_sw_dev, computed row by row with one band cell per
// lane.  The band arrays (h_b, e_b) and the direction matrix keep the
// reference's exact index layout (SET_U / SET_D), in LDS, so the traceback --
// including its out-of-band reads -- sees the same bytes.  Within a row the
// only serial term is F (horizontal gap); with gap_open >= gap_extend
//     F_j = max(H'_{j-1} - gO, F_{j-1} - gE),  H' = max(E+, diag)
// equals the reference's recurrence on the full H (the F-arm of H never wins
// the next F), so it is a max-plus prefix scan over the lanes of the group
// (DPP row_shr 1,2,4,8 for G = 16; shuffles for the 64-lane group).
//
//  k_ext_band16  every job; jobs whose band is wider than 16 cells, whose
//                direction matrix exceeds 4 KB or whose segments are long are
//                appended to a device queue (no host round trip).
//  k_ext_band64  drains that queue, one wave per job, 32 KB direction matrix
//                in LDS.  Whatever still does not fit is flagged in `overflow`
//                for the panel kernel with global scratch (k_ext_band_panel).
// ---------------------------------------------------------------------------
#define BG_NEG (-0x20000000)

template <int G, int S>
__device__ __forceinline__ int gshr(int v) {
    // lane z of the group receives lane z-S; z < S receives BG_NEG
    if constexpr (G == 16) {
        return __builtin_amdgcn_update_dpp(BG_NEG, v, 0x110 + S, 0xf, 0xf, false);
    } else if constexpr (S == 1) {
        return __builtin_amdgcn_update_dpp(BG_NEG, v, 0x138, 0xf, 0xf, false);   // DPP wave_shr:1
    } else {
        const int x = __shfl_up(v, S, 64);
        return (int)(threadIdx.x & 63) < S ? BG_NEG : x;
    }
}

// lane z of the group receives lane z+1 (band index z+2 is held by lane z+1); the last lane receives 0
// (16 lanes: DPP bound_ctrl writes the 0 itself, so no register is preset with it)
template <int G>
__device__ __forceinline__ int gshl1z(int v) {
    if constexpr (G == 16) return __builtin_amdgcn_mov_dpp(v, 0x101, 0xf, 0xf, true);
    else return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xf, 0xf, false);
}

// lane z receives lane z-1; lane 0 receives 0
template <int G>
__device__ __forceinline__ int gshr1z(int v) {
    if constexpr (G == 16) return __builtin_amdgcn_mov_dpp(v, 0x111, 0xf, 0xf, true);
    else return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false);
}

// 16 lanes: lane z receives lane z-S, lanes z < S receive 0 (bound_ctrl)
template <int S>
__device__ __forceinline__ int rshr0(int v) { return __builtin_amdgcn_mov_dpp(v, 0x110 + S, 0xf, 0xf, true); }

// max-plus prefix scan offset so that the 0 a DPP shift brings in at the group's
// start is below every real value: X + GSCAN_OFF stays positive for |X| < 2^20
#define GSCAN_OFF (1 << 24)

template <int G>
__device__ __forceinline__ int gmax(int v) {
    for (int o = G / 2; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, G));
    return v;
}

// X_z = max over m <= z of (A_m - (z - m) gE): a max-plus prefix scan.  16 lanes:
// DPP row_shr 1, 2, 4, 8.  64 lanes: the same within each 16-lane row, then the
// rows joined with the GFX9 DPP broadcasts (row_bcast:15 hands lane 15 of rows
// 0 and 2 to rows 1 and 3, row_bcast:31 lane 31 to rows 2 and 3), each lane
// charging the gap extension over its distance to the broadcasting lane -- no
// LDS round trip (ds_bpermute) in the row loop.
template <int G>
__device__ __forceinline__ int gscan_f(int A, int gE) {
    if constexpr (G == 16) {
        // values offset by GSCAN_OFF, so the 0 shifted in below lane S loses every max
        // (A >= -gO - 64 gE here): bound_ctrl shifts, no preset registers
        int X = A + GSCAN_OFF;
        X = max(X, rshr0<1>(X) - gE);
        X = max(X, rshr0<2>(X) - 2 * gE);
        X = max(X, rshr0<4>(X) - 4 * gE);
        X = max(X, rshr0<8>(X) - 8 * gE);
        return X - GSCAN_OFF;
    } else {
        const int z = (int)(threadIdx.x & 63), zr = z & 15;
        int X = A;
        X = max(X, __builtin_amdgcn_update_dpp(BG_NEG, X, 0x111, 0xf, 0xf, false) - gE);
        X = max(X, __builtin_amdgcn_update_dpp(BG_NEG, X, 0x112, 0xf, 0xf, false) - 2 * gE);
        X = max(X, __builtin_amdgcn_update_dpp(BG_NEG, X, 0x114, 0xf, 0xf, false) - 4 * gE);
        X = max(X, __builtin_amdgcn_update_dpp(BG_NEG, X, 0x118, 0xf, 0xf, false) - 8 * gE);
        const int b15 = __builtin_amdgcn_update_dpp(BG_NEG, X, 0x142, 0xa, 0xf, false);   // row_bcast:15
        X = max(X, b15 - (zr + 1) * gE);
        const int b31 = __builtin_amdgcn_update_dpp(BG_NEG, X, 0x143, 0xc, 0xf, false);   // row_bcast:31
        X = max(X, b31 - (z - 31) * gE);
        return X;
    }
}

#define WSYNC() do { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); } while (0)

__device__ __forceinline__ void aln_sentinel(rsa_aln* out, int j, const ExtJobDev& jb, int score) {
    rsa_aln a;
    a.sw_score = score; a.edit_distance = 100000; a.ref_start = a.ref_end = a.query_start = a.query_end = 0;
    a.cigar_offset = jb.cig_off; a.cigar_len = 0; a.flags = 0;
    out[j] = a;
}

// The direction matrix keeps the reference's byte layout for addressing (cell c of
// band row i at byte 3 (width_d i + c), bytes [de, df, dh], SET_D in ssw.c), but LDS holds
// one code per cell: the band fill always writes a cell's three bytes together, so a
// packed cell decodes to exactly the bytes the reference layout would hold there (an
// unwritten cell, 0, to three zeros; a cell a wider band pass left behind to what that
// pass wrote).  Code: bit 0 de - 2, bit 1 df - 4, bits 2-3 dh as 1 (1), de (2), df (3) --
// never 0 for a written cell, and 4 bits wide.  NIB = false: one byte a cell (a third
// of the reference's bytes); NIB = true: a nibble a cell, two cells a byte in the
// reference's cell order (cell c in byte c / 2, low nibble for even c), a sixth.  The
// nibbles cost a lane-pair merge per row; k_ext_band16 takes them where LDS sets its
// occupancy (the 8192 / 16384 classes: 5 instead of 2-3 waves a SIMD at 250 bp).
__device__ __forceinline__ int dir_pack(int de, int df, int dh) {
    const int dhc = dh == 1 ? 1 : (dh == de ? 2 : 3);
    return (de - 2) | ((df - 4) << 1) | (dhc << 2);
}
// byte `sub` (0..2) of cell `cell`, i.e. reference byte 3 cell + sub
template <bool NIB>
__device__ __forceinline__ int dir_byte(const int8_t* dirp, int cell, int sub) {
    const int v = NIB ? ((int)(uint8_t)dirp[cell >> 1] >> ((cell & 1) * 4)) & 15 : (int)(uint8_t)dirp[cell];
    if (v == 0) return 0;
    const int de = 2 + (v & 1), df = 4 + ((v >> 1) & 1), dhc = (v >> 2) & 3;
    return sub == 0 ? de : (sub == 1 ? df : (dhc == 1 ? 1 : (dhc == 2 ? de : df)));
}
// Certificate of a word-layout result taken without the byte pass (k_ext_scan_v,
// ScanRes.word bit 1): the job's banded path must have no insertion next to a
// deletion, or the job is listed for the exact two-layout scan (rsa_ctx.hip).
// raw: the path's ops in order (0 M, 1 I, 2 D); ok = false lists the job as is.
// Returns true when the job's word result stands on the certificate (its rsa_aln gets
// RSA_ALN_WORD_CERT, which the context counts as scan_certified).
__device__ __forceinline__ bool cert_check(const ScanRes& sr, int j, const uint32_t* raw, int nraw, bool ok,
                                           int* redo, int* redo_count) {
    if (!(sr.word & 2) || !redo) return false;
    bool bad = !ok;
    for (int k = 1; k < nraw && !bad; ++k) {
        const uint32_t a = raw[k - 1] & 0xf, b = raw[k] & 0xf;
        bad = (a == 1 && b == 2) || (a == 2 && b == 1);
    }
    if (bad) redo[atomicAdd(redo_count, 1)] = j;
    return !bad;
}

template <int DIRCAP, bool NIB> struct DirCells {
    static constexpr int CELLS = (DIRCAP + 2) / 3;
    static constexpr int BYTES = ((NIB ? (CELLS + 1) / 2 : CELLS) + 15) & ~15;
};

// banded_sw + traceback + ext_finish of job j by a group of G lanes (z = lane in
// group).  LDS: dir[DIRCAP], qc[QCAP], rc[RCAP].  Returns false when the job does
// not fit the group (nothing written).  Lane z keeps the reference's h_b[z+1] and
// e_b[z+1] in registers; its reads of h_b[e], e_b[e] and h_b[e-1] are DPP shifts
// (index 0 and indices past the group are always 0), so the row loop has no LDS
// round trip and no barrier.  NIB: the direction cells' packing (dir_byte).
template <int G, int DIRCAP, int QCAP, int RCAP, bool NIB>
__device__ bool band_group(int j, int z, const ExtJobDev& jb, const ScanRes& sr, const char* __restrict__ qbuf,
                           const char* __restrict__ ref, uint32_t* __restrict__ cig_pool,
                           uint32_t* __restrict__ raw_pool, rsa_aln* __restrict__ out, int match, int mismatch,
                           int gO, int gE, int bonus, int8_t* dir, uint8_t* qc, uint8_t* rc, int* redo,
                           int* redo_count) {
    const char* q = qbuf + jb.q_off;
    const char* r = ref + jb.r_off;
    const int rlen = (int)jb.rlen;
    const int ref_begin = sr.ref_begin1;
    const int ref_l = sr.ref_end1 - sr.ref_begin1 + 1;
    const int read_l = sr.read_end1 - sr.read_begin1 + 1;
    int bw = abs(ref_l - read_l) + 1;
    if (read_l > QCAP || ref_l > RCAP || read_l <= 0 || ref_l <= 0 || gO < gE || 2 * bw + 1 > G) return false;
    {   // the direction matrix of the first band must fit, too
        int s2 = 1024;
        while ((2 * bw + 1) * read_l * 3 >= s2) s2 *= 2;
        if (s2 > DIRCAP) return false;
    }
    for (int x = z; x < read_l; x += G) qc[x] = (uint8_t)ssw_code((unsigned char)q[sr.read_begin1 + x]);
    for (int x = z; x < ref_l; x += G) {
        const int gj = ref_begin + x;
        rc[x] = (uint8_t)((gj >= 0 && gj < rlen) ? ssw_code((unsigned char)r[gj]) : 4);
    }
    for (int x = z * 16; x < DirCells<DIRCAP, NIB>::BYTES; x += G * 16) *(int4*)(dir + x) = make_int4(0, 0, 0, 0);
    WSYNC();

    const int len = ref_l > read_l ? ref_l : read_l;
    int s2 = 1024, max_v = 0, width_d = 0;
    bool deferred = false;
    int HB = 0, EB = 0;                              // h_b[z+1], e_b[z+1]
    do {
        const int width = bw * 2 + 3;
        width_d = bw * 2 + 1;
        if (width_d > G) { deferred = true; break; }
        while (width_d * read_l * 3 >= s2) s2 *= 2;
        if (s2 > DIRCAP) { deferred = true; break; }
        if (z + 1 >= 1 && z + 1 <= width - 2) HB = 0;
        int lmax = 0;
        for (int i = 0; i < read_l; ++i) {
            const int beg = max(0, i - bw), end = min(ref_l - 1, i + bw);
            const int edge = end + 1 < width - 1 ? end + 1 : width - 1;
            const int jj = beg + z;
            const bool on = jj <= end;
            // Row i's cells are one run of nibbles from cell width_d i; lane pairs (even
            // cell, odd cell) of the row write whole bytes.  The row's first byte when its
            // cell is odd, and its last when its cell is even, hold a nibble of another row
            // or of a cell this pass leaves alone: those two lanes merge into the byte in
            // LDS, read here, well before the store, so the wait is hidden by the row's work.
            const int cell = width_d * i + z;
            const bool odd = NIB && (cell & 1);
            const bool merge = NIB && on && (odd ? z == 0 : jj == end);
            int held = 0;
            if (merge) held = (int)(uint8_t)dir[cell >> 1];
            const int sh = i - bw >= 1 ? 1 : 0;
            const bool clr = z == edge - 1;
            HB = clr ? 0 : HB;
            EB = clr ? 0 : EB;
            const int HBl = gshl1z<G>(HB), EBl = gshl1z<G>(EB), HBr = gshr1z<G>(HB);
            const int hb_e = sh ? HBl : HB;
            const int eb_e = sh ? EBl : EB;
            const int hb_d = sh ? HB : HBr;
            const int qv = qc[i];
            const int rv = on ? rc[min(jj, RCAP - 1)] : 4;   // in-bounds read, no branch
            const int t1 = i == 0 ? -gO : hb_e - gO;
            const int t2 = i == 0 ? -gE : eb_e - gE;
            const int E = t1 > t2 ? t1 : t2;
            const int de = t1 > t2 ? 3 : 2;
            const int diag = hb_d + ((rv == qv && rv < 4) ? match : -mismatch);
            const int e1 = E > 0 ? E : 0;
            const int hp = e1 > diag ? e1 : diag;
            // lane 0's shifted-in value is never used (A, f_prev take their boundary values)
            const int prev_hp = G == 16 ? rshr0<1>(hp) : gshr<G, 1>(hp);
            const int A = z == 0 ? -gO : prev_hp - gO;
            const int F = max(gscan_f<G>(A, gE), -(z + 1) * gE);
            const int f_prev = G == 16 ? rshr0<1>(F) : (z == 0 ? 0 : gshr<G, 1>(F));
            const int df = A > f_prev - gE ? 5 : 4;
            const int f1 = F > 0 ? F : 0;
            const int m = e1 > f1 ? e1 : f1;
            const int H = m > diag ? m : diag;
            const int dh = m <= diag ? 1 : (e1 > f1 ? de : df);
            const int code = on ? dir_pack(de, df, dh) : 0;
            if constexpr (NIB) {
                const int code_up = gshl1z<G>(code);    // the odd cell after an even one
                if (on && (!odd || z == 0)) {
                    const int b = odd ? ((held & 0x0f) | (code << 4))
                                      : (merge ? ((held & 0xf0) | code) : (code | (code_up << 4)));
                    dir[cell >> 1] = (int8_t)b;
                }
            } else if (on) {
                dir[cell] = (int8_t)code;
            }
            lmax = (on && H > lmax) ? H : lmax;
            EB = on ? E : EB;                            // h_b[1..u] = h_c[1..u]
            HB = on ? H : HB;
        }
        lmax = gmax<G>(lmax);
        if (lmax > max_v) max_v = lmax;
        bw *= 2;
    } while (max_v < sr.score1 && bw <= len);
    WSYNC();                                         // direction bytes visible to the traceback lane
    if (deferred) return false;
    if (z != 0) return true;
    bw /= 2;

    // traceback (ssw.c:748-776), leader lane
    rsa_aln a;
    a.sw_score = 0; a.edit_distance = 0; a.ref_start = a.ref_end = a.query_start = a.query_end = 0;
    a.cigar_offset = jb.cig_off; a.cigar_len = 0; a.flags = 0;
    uint32_t* raw = raw_pool + jb.cig_off;
    int i = read_l - 1, jx = ref_l - 1, ecount = 0, l = 0, temp2 = 2;
    int line = width_d * 3 * (read_l - 1);
    int lineC = width_d * (read_l - 1);           // line / 3: the row's first cell
    uint32_t op = 0, prev_op = 0;
    bool fail = false;
    const int W3 = width_d * 3;
    // one traceback step from the direction byte dv at the current cell; false = failure
    auto step = [&](int dv) -> bool {
        if (dv == 1) { --i; --jx; temp2 = 2; line -= W3; lineC -= width_d; op = 0; }
        else if (dv == 2) { --i; temp2 = 0; line -= W3; lineC -= width_d; op = 1; }
        else if (dv == 3) { --i; temp2 = 2; line -= W3; lineC -= width_d; op = 1; }
        else if (dv == 4) { --jx; temp2 = 1; op = 2; }
        else if (dv == 5) { --jx; temp2 = 2; op = 2; }
        else return false;
        if (op == prev_op) ++ecount;
        else { ++l; raw[l - 1] = cig((uint32_t)ecount, prev_op); prev_op = op; ecount = 1; }
        return true;
    };
    // Each step's byte address depends on the byte before it, so the walk is a chain of LDS
    // latencies.  From a cell entered with temp2 = 2, the next 8 cells along the diagonal
    // are loaded together (the addresses a run of diagonal moves would visit) and consumed
    // while the moves are diagonal; the first other move is taken from its byte as usual.
    // The same cells and bytes as the one-step walk (ssw.c:748-776).
    constexpr int TB_AHEAD = 8;
    while (i >= 0 && jx > 0) {
        if (temp2 == 2) {
            int dvs[TB_AHEAD];
#pragma unroll
            for (int k = 0; k < TB_AHEAD; ++k) {
                const int ik = i - k, jk = jx - k;
                const int ck = lineC - k * width_d + (jk - max(ik - bw, 0));
                const int atk = 3 * ck + 2;
                dvs[k] = (ik >= 0 && jk > 0 && atk >= 0 && atk < s2) ? dir_byte<NIB>(dir, ck, 2) : 0;
            }
            bool more = true;
#pragma unroll
            for (int k = 0; k < TB_AHEAD; ++k) {
                if (!more || !(i >= 0 && jx > 0)) { more = false; continue; }
                const int at = line + (jx - max(i - bw, 0)) * 3 + 2;
                if (at < 0 || at >= s2) { fail = true; more = false; continue; }
                if (!step(dvs[k])) { fail = true; more = false; continue; }
                if (dvs[k] != 1) more = false;             // left the diagonal: back to single steps
            }
            if (fail) break;
            continue;
        }
        const int cell = lineC + (jx - max(i - bw, 0));
        const int at = 3 * cell + temp2;                   // = line + (jx - max(i - bw, 0)) * 3 + temp2
        if (at < 0 || at >= s2) { fail = true; break; }
        if (!step(dir_byte<NIB>(dir, cell, temp2))) { fail = true; break; }
    }
    if (fail) {                                     // banded_sw failed -> flag 1 sentinel
        aln_sentinel(out, j, jb, -100000);
        cert_check(sr, j, raw, 0, false, redo, redo_count);
        return true;
    }
    if (op == 0) { ++l; raw[l - 1] = cig((uint32_t)ecount + 1, op); }
    else { l += 2; raw[l - 2] = cig((uint32_t)ecount, op); raw[l - 1] = cig(1, 0); }
    for (int s = 0, t = l - 1; s < t; ++s, --t) { const uint32_t x = raw[s]; raw[s] = raw[t]; raw[t] = x; }
    const bool certified = cert_check(sr, j, raw, l, true, redo, redo_count);
    ext_finish(jb, sr, q, r, raw, l, cig_pool + jb.cig_off, a, match, mismatch, bonus, gO, gE, qc, rc);
    if (certified) a.flags |= RSA_ALN_WORD_CERT;
    out[j] = a;
    return true;
}

#define B16_GROUPS 4
#define B16_SEGCAP 320

// DIRCAP: direction bytes of one job in the reference's 3-a-cell count.  4096 holds the
// bands of 150-bp reads up to 9 cells wide (deferral 0.04 % on the headline) in a byte a
// cell (8 KB of LDS a wave, 5 waves a SIMD); for 250-bp reads only 5 cells, which sent
// 15 % of the PE 2x250 jobs to the one-wave kernel.  8192 (chosen for batches with
// queries over 200 bp) holds 9 cells at 250 bp; with a byte a cell it took 13.5 KB a wave
// (2-3 waves a SIMD), with a nibble a cell 7.9 KB (5 waves).  16384 holds every band a
// 16-lane group can (15 cells at 250 bp) in 13.2 KB.
#define B16_NIB (DIRCAP > 4096)
template <int DIRCAP>
__global__ void __launch_bounds__(64)
k_ext_band16(const ExtJobDev* __restrict__ jobs, const ScanRes* __restrict__ scan, int n_jobs,
             const int* __restrict__ idx, const char* __restrict__ qbuf, const char* __restrict__ ref,
             uint32_t* __restrict__ cig_pool, uint32_t* __restrict__ raw_pool, rsa_aln* __restrict__ out, int match,
             int mismatch, int gO, int gE, int bonus, int* __restrict__ queue, int* __restrict__ qcount,
             int* __restrict__ overflow, int* __restrict__ redo, int* __restrict__ redo_count, int prio,
             const int* __restrict__ n_dev) {
    // the extension finishes chunks the SAM writer waits for: its waves may claim the
    // SIMDs they share with the seeding kernels first (s_setprio, RSA_EXT_SETPRIO)
    if (prio) __builtin_amdgcn_s_setprio(2);
    if (n_dev) n_jobs = min(n_jobs, *n_dev);      // the in-stream redo pass: the device's count
    __shared__ __attribute__((aligned(16))) int8_t s_dir[B16_GROUPS][DirCells<DIRCAP, B16_NIB>::BYTES];
    __shared__ uint8_t s_qc[B16_GROUPS][B16_SEGCAP];
    __shared__ uint8_t s_rc[B16_GROUPS][B16_SEGCAP];
    const int lane = threadIdx.x & 63, g = lane >> 4, z = lane & 15;
    const int t = blockIdx.x * B16_GROUPS + g;
    if (t >= n_jobs) return;                       // whole group leaves together
    const int j = idx ? idx[t] : t;
    const ExtJobDev jb = jobs[j];
    const ScanRes sr = scan[j];
    if (z == 0) overflow[j] = 0;                   // k_ext_band64 sets the jobs it cannot hold
    if (sr.status != 0) {                          // ref > 2000 (aligner.cpp:119-125)
        if (z == 0) aln_sentinel(out, j, jb, -1000000);
        return;
    }
    if (sr.flag != 0) {                            // aligner.cpp:131-136
        if (z == 0) {
            aln_sentinel(out, j, jb, -100000);
            cert_check(sr, j, nullptr, 0, false, redo, redo_count);
        }
        return;
    }
    const bool done = band_group<16, DIRCAP, B16_SEGCAP, B16_SEGCAP, B16_NIB>(
        j, z, jb, sr, qbuf, ref, cig_pool, raw_pool, out, match, mismatch, gO, gE, bonus, s_dir[g], s_qc[g], s_rc[g],
        redo, redo_count);
    if (!done && z == 0) {
        // an empty result until a wider kernel writes it: the CIGAR compaction reads
        // every job, including one the 64-lane kernel leaves to the one-lane pass
        rsa_aln a;
        a.sw_score = 0; a.edit_distance = 0; a.ref_start = a.ref_end = a.query_start = a.query_end = 0;
        a.cigar_offset = jb.cig_off; a.cigar_len = 0; a.flags = 0;
        out[j] = a;
        queue[atomicAdd(qcount, 1)] = j;
    }
}

#define B64_DIRCAP 32768
#define B64_QCAP 1024
#define B64_RCAP 2048

__global__ void __launch_bounds__(64)
k_ext_band64(const ExtJobDev* __restrict__ jobs, const ScanRes* __restrict__ scan, const char* __restrict__ qbuf,
             const char* __restrict__ ref, uint32_t* __restrict__ cig_pool, uint32_t* __restrict__ raw_pool,
             rsa_aln* __restrict__ out, int match, int mismatch, int gO, int gE, int bonus,
             const int* __restrict__ queue, const int* __restrict__ qcount, int* __restrict__ overflow,
             int* __restrict__ ocount, int* __restrict__ redo, int* __restrict__ redo_count) {
    __shared__ __attribute__((aligned(16))) int8_t s_dir[DirCells<B64_DIRCAP, false>::BYTES];
    __shared__ uint8_t s_qc[B64_QCAP];
    __shared__ uint8_t s_rc[B64_RCAP];
    const int z = threadIdx.x & 63;
    const int nq = *qcount;
    for (int t = blockIdx.x; t < nq; t += gridDim.x) {
        const int j = queue[t];
        const ExtJobDev jb = jobs[j];
        const ScanRes sr = scan[j];
        const bool done = band_group<64, B64_DIRCAP, B64_QCAP, B64_RCAP, false>(
            j, z, jb, sr, qbuf, ref, cig_pool, raw_pool, out, match, mismatch, gO, gE, bonus, s_dir, s_qc, s_rc,
            redo, redo_count);
        if (!done && z == 0) { overflow[j] = 1; atomicAdd(ocount, 1); }
        WSYNC();
    }
}

// ---------------------------------------------------------------------------
// k_ext_band_panel: bands too wide for one wave (band rows longer than 64 cells,
// up to the 2 x 2000 + 1 cells a 2 kb window can need) or direction matrices
// larger than LDS.  One wave per job.  Each band row is swept in panels of 64
// cells: lane z computes cell 64p + z + 1 of panel p, E and the diagonal from
// the previous row's h_b / e_b, and F as the same max-plus prefix scan as the
// 16/64-lane kernels, entered with the F and H' of the panel before it (a
// scalar carry read from lane 63).  h_b / e_b live in LDS with the reference's
// index layout (SET_U, ssw.c:600-601), so every out-of-band read and the
// values a band doubling leaves behind are the reference's; the current row's
// H reaches h_b one panel late (after the next panel has read the previous
// row), which is the reference's end-of-row copy h_b[1..u] = h_c[1..u].  The
// direction matrix (SET_D layout, zero-filled as it grows) is in global
// scratch; lane 0 walks the traceback over it once the band passes are done.
// ---------------------------------------------------------------------------
#define BP_KW 4104        // h_b / e_b entries: width = 2 * bw + 3 <= 2 * 2000 + 3
#define BP_QCAP 1024      // query segment (rsa_extend refuses longer queries)
#define BP_RCAP 2048      // reference segment (windows > 2000 are sentinels)

__global__ void __launch_bounds__(64)
k_ext_band_panel(const ExtJobDev* __restrict__ jobs, const ScanRes* __restrict__ scan, int n_jobs,
                 const int* __restrict__ idx_list, const char* __restrict__ qbuf, const char* __restrict__ ref,
                 uint32_t* __restrict__ cig_pool, rsa_aln* __restrict__ out, uint8_t* __restrict__ scratch,
                 int64_t scr_stride, int64_t dir_cap, int match, int mismatch, int gO, int gE, int bonus,
                 int* __restrict__ overflow, int over_code, int* __restrict__ redo, int* __restrict__ redo_count) {
    __shared__ int s_hb[BP_KW];
    __shared__ int s_eb[BP_KW];
    __shared__ uint8_t s_qc[BP_QCAP];
    __shared__ uint8_t s_rc[BP_RCAP];
    const int z = threadIdx.x & 63;
    const int t = blockIdx.x;
    if (t >= n_jobs) return;
    const int j = idx_list[t];
    const ExtJobDev jb = jobs[j];
    const ScanRes sr = scan[j];
    if (sr.status != 0) {                            // ref > 2000 (aligner.cpp:119-125)
        if (z == 0) aln_sentinel(out, j, jb, -1000000);
        return;
    }
    if (sr.flag != 0) {                              // aligner.cpp:131-136
        if (z == 0) aln_sentinel(out, j, jb, -100000);
        return;
    }
    const char* q = qbuf + jb.q_off;
    const char* r = ref + jb.r_off;
    const int rlen = (int)jb.rlen;
    const int ref_begin = sr.ref_begin1;
    const int ref_l = sr.ref_end1 - sr.ref_begin1 + 1;
    const int read_l = sr.read_end1 - sr.read_begin1 + 1;
    const int len = ref_l > read_l ? ref_l : read_l;
    if (read_l <= 0 || ref_l <= 0 || read_l > BP_QCAP || ref_l > BP_RCAP || gO < gE || 2 * len + 3 > BP_KW) {
        if (z == 0) overflow[j] = over_code;
        return;
    }
    int8_t* dir = (int8_t*)(scratch + (int64_t)t * scr_stride);
    uint32_t* raw = (uint32_t*)(scratch + (int64_t)t * scr_stride + dir_cap);
    for (int x = z; x < read_l; x += 64) s_qc[x] = (uint8_t)ssw_code((unsigned char)q[sr.read_begin1 + x]);
    for (int x = z; x < ref_l; x += 64) {
        const int gj = ref_begin + x;
        s_rc[x] = (uint8_t)((gj >= 0 && gj < rlen) ? ssw_code((unsigned char)r[gj]) : 4);
    }
    for (int x = z; x < BP_KW; x += 64) { s_hb[x] = 0; s_eb[x] = 0; }
    int64_t s2 = 0;                                  // direction bytes zeroed so far
    int64_t s2_ref = 1024;                           // the reference's direction size (traceback bound)
    int bw = abs(ref_l - read_l) + 1, max_v = 0, width_d = 0;
    WSYNC();
    do {
        const int width = bw * 2 + 3;
        width_d = bw * 2 + 1;
        while ((int64_t)width_d * read_l * 3 >= s2_ref) s2_ref *= 2;
        if (s2_ref > dir_cap) {
            if (z == 0) overflow[j] = over_code;
            return;
        }
        // the direction matrix grows zero-filled (only its first s2_ref bytes are ever read)
        for (int64_t x = s2 + 4 * z; x < s2_ref; x += 256) *(int*)(dir + x) = 0;
        s2 = s2_ref;
        for (int x = 1 + z; x <= width - 2; x += 64) s_hb[x] = 0;
        __threadfence();                             // zeroes before the band's own stores, from any lane
        WSYNC();
        int lmax = 0;
        for (int i = 0; i < read_l; ++i) {
            const int beg = max(0, i - bw), end = min(ref_l - 1, i + bw);
            const int edge = end + 1 < width - 1 ? end + 1 : width - 1;
            const int ncell = end - beg + 1;         // u = 1 .. ncell
            const int sh = i - bw >= 1 ? 1 : 0;       // SET_U(i-1, j) - SET_U(i, j)
            if (z == 0) { s_hb[0] = 0; s_eb[0] = 0; s_hb[edge] = 0; s_eb[edge] = 0; }
            WSYNC();
            const int qv = s_qc[i];
            int8_t* dline = dir + (int64_t)width_d * 3 * i;
            int Fc = 0, HPc = 0;                     // f and h_c[u-1]'s H' entering the panel
            int H_prev = 0, u_prev = 0;
            bool on_prev = false;
            for (int base = 0; base < ncell; base += 64) {
                const int u = base + z + 1;
                const bool on = u <= ncell;
                const int ue = min(u + sh, BP_KW - 1), ud = u - 1 + sh;
                const int hb_e = s_hb[ue], eb_e = s_eb[ue], hb_d = s_hb[ud];
                WSYNC();                             // the previous row's values are read: update them
                if (on_prev) s_hb[u_prev] = H_prev;
                const int t1 = i == 0 ? -gO : hb_e - gO;
                const int t2 = i == 0 ? -gE : eb_e - gE;
                const int E = t1 > t2 ? t1 : t2;
                const int de = t1 > t2 ? 3 : 2;
                if (on) s_eb[u] = E;
                const int rv = on ? s_rc[beg + u - 1] : 4;
                const int diag = hb_d + ((rv == qv && rv < 4) ? match : -mismatch);
                const int e1 = E > 0 ? E : 0;
                const int hp = e1 > diag ? e1 : diag;
                const int left_hp = __builtin_amdgcn_update_dpp(0, hp, 0x138, 0xf, 0xf, false);   // lane z-1
                const int A = (z == 0 ? HPc : left_hp) - gO;
                const int F = max(gscan_f<64>(A, gE), Fc - (z + 1) * gE);
                const int left_f = __builtin_amdgcn_update_dpp(0, F, 0x138, 0xf, 0xf, false);
                const int f_prev = z == 0 ? Fc : left_f;
                const int df = A > f_prev - gE ? 5 : 4;
                const int f1 = F > 0 ? F : 0;
                const int m = e1 > f1 ? e1 : f1;
                const int H = m > diag ? m : diag;
                const int dh = m <= diag ? 1 : (e1 > f1 ? de : df);
                if (on) {
                    int8_t* dl = dline + 3 * (u - 1);
                    dl[0] = (int8_t)de; dl[1] = (int8_t)df; dl[2] = (int8_t)dh;
                    lmax = H > lmax ? H : lmax;
                }
                Fc = __builtin_amdgcn_readlane(F, 63);
                HPc = __builtin_amdgcn_readlane(hp, 63);
                H_prev = H;
                u_prev = u;
                on_prev = on;
            }
            if (on_prev) s_hb[u_prev] = H_prev;      // the row's last panel: h_b[1..u] = h_c[1..u]
            WSYNC();
        }
        lmax = gmax<64>(lmax);
        if (lmax > max_v) max_v = lmax;
        bw *= 2;
    } while (max_v < sr.score1 && bw <= len);
    __threadfence();                                 // direction bytes of every lane visible to lane 0
    WSYNC();
    if (z != 0) return;
    bw /= 2;

    // traceback (ssw.c:748-776)
    rsa_aln a;
    a.sw_score = 0; a.edit_distance = 0; a.ref_start = a.ref_end = a.query_start = a.query_end = 0;
    a.cigar_offset = jb.cig_off; a.cigar_len = 0; a.flags = 0;
    int i = read_l - 1, jx = ref_l - 1, ecount = 0, l = 0, temp2 = 2;
    int64_t line = (int64_t)width_d * 3 * (read_l - 1);
    uint32_t op = 0, prev_op = 0;
    while (i >= 0 && jx > 0) {
        const int64_t at = line + (int64_t)(jx - max(i - bw, 0)) * 3 + temp2;
        if (at < 0 || at >= s2_ref) {
            aln_sentinel(out, j, jb, -100000);
            cert_check(sr, j, raw, 0, false, redo, redo_count);
            return;
        }
        const int dv = dir[at];
        if (dv == 1) { --i; --jx; temp2 = 2; line -= width_d * 3; op = 0; }
        else if (dv == 2) { --i; temp2 = 0; line -= width_d * 3; op = 1; }
        else if (dv == 3) { --i; temp2 = 2; line -= width_d * 3; op = 1; }
        else if (dv == 4) { --jx; temp2 = 1; op = 2; }
        else if (dv == 5) { --jx; temp2 = 2; op = 2; }
        else {                                               // banded_sw failed -> flag 1
            aln_sentinel(out, j, jb, -100000);
            cert_check(sr, j, raw, 0, false, redo, redo_count);
            return;
        }
        if (op == prev_op) ++ecount;
        else { ++l; raw[l - 1] = cig((uint32_t)ecount, prev_op); prev_op = op; ecount = 1; }
    }
    if (op == 0) { ++l; raw[l - 1] = cig((uint32_t)ecount + 1, op); }
    else { l += 2; raw[l - 2] = cig((uint32_t)ecount, op); raw[l - 1] = cig(1, 0); }
    for (int s = 0, e = l - 1; s < e; ++s, --e) { const uint32_t x = raw[s]; raw[s] = raw[e]; raw[e] = x; }
    const bool certified = cert_check(sr, j, raw, l, true, redo, redo_count);
    ext_finish(jb, sr, q, r, raw, l, cig_pool + jb.cig_off, a, match, mismatch, bonus, gO, gE, s_qc, s_rc);
    if (certified) a.flags |= RSA_ALN_WORD_CERT;
    out[j] = a;
}

// ---------------------------------------------------------------------------
// CIGAR compaction: every job's CIGAR is written into its qlen+rlen+8 slot; these
// kernels pack them back to back and rewrite cigar_offset, so the host copies only
// the ops that exist.  Per-block totals, a scan of the block totals, then every
// block lays its jobs' ops out with a flat, coalesced copy.
// ---------------------------------------------------------------------------
#define CCP_THREADS 256
__device__ __forceinline__ uint64_t block_incl_scan(uint64_t v, uint64_t* s) {
    const int t = threadIdx.x;
    s[t] = v;
    __syncthreads();
    for (int o = 1; o < CCP_THREADS; o <<= 1) {
        const uint64_t x = t >= o ? s[t - o] : 0;
        __syncthreads();
        s[t] += x;
        __syncthreads();
    }
    return s[t];
}

__global__ void __launch_bounds__(CCP_THREADS)
k_cig_bsum(const rsa_aln* __restrict__ alns, int n_jobs, uint64_t* __restrict__ bsum) {
    __shared__ uint64_t s[CCP_THREADS];
    const int i = blockIdx.x * CCP_THREADS + threadIdx.x;
    const uint64_t v = i < n_jobs ? alns[i].cigar_len : 0;
    const uint64_t incl = block_incl_scan(v, s);
    if (threadIdx.x == CCP_THREADS - 1) bsum[blockIdx.x] = incl;
}

// exclusive scan of nb block totals in place (one workgroup); *total = their sum
__global__ void __launch_bounds__(1024) k_cig_bscan(uint64_t* __restrict__ bsum, int nb, uint64_t* __restrict__ total) {
    __shared__ uint64_t s[1024];
    const int t = threadIdx.x;
    const int per = (nb + 1023) / 1024;
    const int a = min(nb, t * per), b = min(nb, a + per);
    uint64_t mine = 0;
    for (int i = a; i < b; ++i) mine += bsum[i];
    s[t] = mine;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint64_t x = t >= o ? s[t - o] : 0;
        __syncthreads();
        s[t] += x;
        __syncthreads();
    }
    uint64_t off = s[t] - mine;
    for (int i = a; i < b; ++i) {
        const uint64_t v = bsum[i];
        bsum[i] = off;
        off += v;
    }
    if (t == 1023) *total = s[t];
}

__global__ void __launch_bounds__(CCP_THREADS)
k_cig_copy(const rsa_aln* __restrict__ alns, rsa_aln* __restrict__ alns_out, int n_jobs,
           const uint64_t* __restrict__ bbase, const uint32_t* __restrict__ slots, uint32_t* __restrict__ dense) {
    __shared__ uint64_t s[CCP_THREADS];
    __shared__ uint64_t s_src[CCP_THREADS];
    const int t = threadIdx.x;
    const int i = blockIdx.x * CCP_THREADS + t;
    const uint32_t len = i < n_jobs ? alns[i].cigar_len : 0;
    const uint64_t src = i < n_jobs ? alns[i].cigar_offset : 0;
    const uint64_t incl = block_incl_scan(len, s);     // s[] now holds inclusive offsets
    s_src[t] = src;
    __syncthreads();
    const uint64_t base = bbase[blockIdx.x];
    const uint64_t tot = s[CCP_THREADS - 1];
    for (uint64_t f = t; f < tot; f += CCP_THREADS) {
        int lo = 0, hi = CCP_THREADS - 1;                // first job whose inclusive end exceeds f
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s[mid] > f) hi = mid; else lo = mid + 1;
        }
        const uint64_t start = lo ? s[lo - 1] : 0;
        dense[base + f] = slots[s_src[lo] + (f - start)];
    }
    if (i < n_jobs) {                                // the results with packed offsets; alns keeps the slots
        rsa_aln a = alns[i];
        a.cigar_offset = base + incl - len;
        alns_out[i] = a;
    }
}

void launch_cigar_compact(hipStream_t st, const rsa_aln* alns, rsa_aln* alns_out, int n_jobs, const uint32_t* slots,
                          uint32_t* dense, uint64_t* bsum, uint64_t* total) {
    const int nb = (n_jobs + CCP_THREADS - 1) / CCP_THREADS;
    hipLaunchKernelGGL(k_cig_bsum, dim3(nb), dim3(CCP_THREADS), 0, st, alns, n_jobs, bsum);
    hipLaunchKernelGGL(k_cig_bscan, dim3(1), dim3(1024), 0, st, bsum, nb, total);
    hipLaunchKernelGGL(k_cig_copy, dim3(nb), dim3(CCP_THREADS), 0, st, alns, alns_out, n_jobs, bsum, slots, dense);
}

// ---------------------------------------------------------------------------
// k_shared_check: rescue_mate_part's pre-check has_shared_substring (aln.cpp:1000-1013)
// for the jobs that ask for it (RSA_JOB_SHARED_CHECK): is any substring of sub = 2k/3
// query bytes starting at i = 0, step, 2 step, ... (i + sub < qlen, step = k/3) found
// in the window (std::string::find: exact bytes, whole match inside the window)?  One
// wave a job, the window staged in LDS; lane x tries window positions x, x + 64, ...
// for one substring at a time (8-byte words composed from aligned LDS loads, the last
// one masked), and the wave stops at the first substring found anywhere.
// list[2f] = job index, list[2f + 1] = k; res[f] = 1 when nothing is shared.
// ---------------------------------------------------------------------------
#define SH_WAVES 4
__device__ __forceinline__ uint64_t sh_word(const uint8_t* w, int p) {   // bytes w[p .. p+8), first lowest
    const int a = p & ~7, o = (p & 7) * 8;
    const uint64_t lo = *(const uint64_t*)(w + a), hi = *(const uint64_t*)(w + a + 8);
    return o ? (lo >> o) | (hi << (64 - o)) : lo;
}
__device__ __forceinline__ uint64_t sh_qword(const char* q, int p, int n) {   // n <= 8 bytes of q at p
    uint64_t x = 0;
    for (int b = 0; b < n; ++b) x |= (uint64_t)(uint8_t)q[p + b] << (8 * b);
    return x;
}

__global__ void __launch_bounds__(64 * SH_WAVES)
k_shared_check(const ExtJobDev* __restrict__ jobs, const uint32_t* __restrict__ list, int nl,
               const char* __restrict__ qbuf, const char* __restrict__ ref, uint8_t* __restrict__ res) {
    __shared__ __attribute__((aligned(8))) uint8_t s_w[SH_WAVES][RSA_SHARED_WMAX + 32];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int f = blockIdx.x * SH_WAVES + w;
    if (f >= nl) return;                             // the whole wave
    const ExtJobDev jb = jobs[list[2 * f]];
    const int k = (int)list[2 * f + 1];
    const int qlen = (int)jb.qlen, rlen = (int)jb.rlen;
    const int sub = 2 * k / 3, step = k / 3;
    uint8_t* win = s_w[w];
    const char* r = ref + jb.r_off;
    for (int x = lane; x < rlen + 32; x += 64) win[x] = x < rlen ? (uint8_t)r[x] : 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const char* q = qbuf + jb.q_off;
    const int nw = (sub + 7) / 8;                    // words a substring spans (sub <= 2 * 127 / 3)
    bool found = false;
    if (sub > 0 && step > 0 && sub <= 24) {
        for (int i = 0; i + sub < qlen; i += step) {
            uint64_t qw[3], mk[3];
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const int n = t < nw ? min(8, sub - 8 * t) : 0;
                qw[t] = n ? sh_qword(q, i + 8 * t, n) : 0;
                mk[t] = n == 8 ? ~0ull : ((1ull << (8 * n)) - 1);
            }
            bool hit = false;
            for (int p = lane; p + sub <= rlen; p += 64) {
                bool eq = true;
#pragma unroll
                for (int t = 0; t < 3; ++t)
                    if (t < nw) eq = eq && ((sh_word(win, p + 8 * t) & mk[t]) == qw[t]);
                hit = hit || eq;
            }
            if (__builtin_amdgcn_ballot_w64(hit)) { found = true; break; }
        }
    } else if (sub > 24) {
        found = true;                                // outside the kernel's shapes: the host never asks
    }
    if (lane == 0) res[f] = found ? 0 : 1;
}

void launch_shared_check(int nl, hipStream_t st, const ExtJobDev* jobs, const uint32_t* list, const char* q,
                         const char* ref, uint8_t* res) {
    if (nl <= 0) return;
    hipLaunchKernelGGL(k_shared_check, dim3((nl + SH_WAVES - 1) / SH_WAVES), dim3(64 * SH_WAVES), 0, st, jobs, list,
                       nl, q, ref, res);
}

// host-side launcher: RMAX from the longest query of the batch
void launch_ext_scan(int rmax, dim3 grid, dim3 block, hipStream_t st, const ExtJobDev* jobs, int n, const int* idx,
                     const char* q, const char* ref, ScanRes* out, int match, int mismatch, int gO, int gE,
                     const int* n_dev) {
#define RSA_L(RM) hipLaunchKernelGGL((k_ext_scan<RM>), grid, block, 0, st, jobs, n, idx, q, ref, out, match, mismatch, gO, gE, n_dev)
    if (rmax <= 2) RSA_L(2); else if (rmax <= 4) RSA_L(4); else if (rmax <= 8) RSA_L(8); else RSA_L(16);
#undef RSA_L
}

void launch_ext_band16(int dircap, dim3 grid, hipStream_t st, const ExtJobDev* jobs, const ScanRes* scan, int n,
                       const int* idx, const char* q, const char* ref, uint32_t* cig, uint32_t* raw, rsa_aln* out,
                       int match, int mismatch, int gO, int gE, int bonus, int* queue, int* qcount, int* overflow,
                       int* redo, int* redo_count, int prio, const int* n_dev) {
#define RSA_B16(DC)                                                                                                \
    hipLaunchKernelGGL(k_ext_band16<DC>, grid, dim3(64), 0, st, jobs, scan, n, idx, q, ref, cig, raw, out, match, \
                       mismatch, gO, gE, bonus, queue, qcount, overflow, redo, redo_count, prio, n_dev)
    if (dircap >= 16384) RSA_B16(16384);
    else if (dircap >= 8192) RSA_B16(8192);
    else RSA_B16(4096);
#undef RSA_B16
}

void launch_ext_band64(dim3 grid, hipStream_t st, const ExtJobDev* jobs, const ScanRes* scan, const char* q,
                       const char* ref, uint32_t* cig, uint32_t* raw, rsa_aln* out, int match, int mismatch, int gO,
                       int gE, int bonus, const int* queue, const int* qcount, int* overflow, int* ocount, int* redo,
                       int* redo_count) {
    hipLaunchKernelGGL(k_ext_band64, grid, dim3(64), 0, st, jobs, scan, q, ref, cig, raw, out, match, mismatch, gO, gE,
                       bonus, queue, qcount, overflow, ocount, redo, redo_count);
}
