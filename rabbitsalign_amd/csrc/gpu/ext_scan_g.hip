// ext_scan_g.hip -- grouped SSW scan for gfx950: 16 lanes per job, 4 jobs per
// wavefront.
//
// Same results as k_ext_scan (ext_kernels.hip) -- the SSW forward pass with the
// byte (16-stripe) and word (8-stripe) layouts fused in the two int16 halves of
// packed registers, then the reverse pass that stops at the first column
// reaching score1 (ssw.c:197-588, 838-893) -- with a different mapping:
//
//   * a job occupies one 16-lane DPP row; the query rows are striped R per lane
//     (R = 10 for 150 bp reads), the reference streams through the row as an
//     anti-diagonal systolic array, and the row-above values move one lane per
//     step with DPP row_shr:1 (the row's first lane reads the zero boundary);
//   * four jobs share a wavefront in lockstep, so the per-step overhead (three
//     DPP moves, one LDS read of the reference code, the column-max bookkeeping)
//     is paid once per R rows instead of once per 3, and the systolic ramp is
//     15 steps instead of 50.  The host hands the jobs over sorted by window
//     length, so the four jobs of a wave run nearly the same number of steps.
//
// Cell recurrence (SSW's, ssw.c:197-588): E, Fw (within-stripe F) and F are
// kept >= 0 as SSW saturates them, so H = max(diag, E, Fw, F, 0) is
// max3(diag, E, Fw) then a max with F; E and Fw take hm - gap_open, where hm
// leaves out the cross-stripe F (the striping artefact: that F never feeds E).
// F' = max(F - gE, H - gO) = max(F - gE, hm - gO) because F - gO <= F - gE
// (the host routes gap_open < gap_extend elsewhere): F's dependency chain
// through the rows is two instructions.
//
// Arithmetic: the forward pass runs in packed half precision (v_pk_*_f16 and
// gfx950's three-input v_pk_maximum3_f16): every value is an integer of
// magnitude < 2048 (host-checked: match * 256 <= 2048 and penalties <= 1024),
// which f16 holds exactly, so every H is SSW's.  Scores are >= +0, whose f16
// bit patterns order like the values: the column maximum is tracked on bits.
// The reverse pass is int32 with v_max3_i32.
//
// Column maxima of the forward pass include the padding rows of the last lane
// (rows >= nrow) without a mask: with non-negative mismatch/gap penalties
// every move into a padding row loses or keeps score (never a match there) and
// its only entries are this lane's last valid row, so a padding cell never
// exceeds the best valid cell of the same lane so far; whenever the column max
// improves the lane's best it is a valid cell's value, and the row search only
// looks at valid rows.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>

#include "rsa_dev.h"
#include "rsa_ext.h"

#define GS_WAVES 4
#define GS_G 16                  // lanes per job: a DPP row (32, half a wave, measured slower at chunk size)
#define GS_JOBS (GS_WAVES * (64 / GS_G))   // jobs per workgroup
#define GS_MAXR 1024             // reference window bytes staged in LDS per job
#define GS_RPAD 32               // code-4 bytes staged on both sides of a window: the scans read
                                 // a column's code ahead of time without a range check

namespace {

typedef _Float16 hh2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ hh2 h2_from(uint32_t x) { return __builtin_bit_cast(hh2, x); }
__device__ __forceinline__ uint32_t h2_bits(hh2 x) { return __builtin_bit_cast(uint32_t, x); }
// IEEE maximum: one v_pk_maximum3_f16, no canonicalisation (values are never NaN)
__device__ __forceinline__ hh2 hmax(hh2 a, hh2 b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ hh2 hmax3(hh2 a, hh2 b, hh2 c) { return hmax(hmax(a, b), c); }
__device__ __forceinline__ uint32_t h2_pair(int v) {
    const _Float16 h = (_Float16)v;
    const uint32_t b = (uint32_t)__builtin_bit_cast(uint16_t, h);
    return b | (b << 16);
}
__device__ __forceinline__ int h_bits_to_int(uint32_t bits16) {
    return (int)(float)__builtin_bit_cast(_Float16, (uint16_t)bits16);
}

// lane l of a job's lane group receives lane l-1; the group's first lane receives 0
// (16 lanes: DPP row_shr:1; 32 lanes: DPP wave_shr:1 with the group's first lane cleared)
__device__ __forceinline__ uint32_t row_shr1(uint32_t v) {
    if constexpr (GS_G == 16) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
    } else {
        const uint32_t x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
        return (threadIdx.x & (GS_G - 1)) ? x : 0u;
    }
}
__device__ __forceinline__ int grp_max(int v) {
    for (int o = GS_G / 2; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, GS_G));
    return v;
}
__device__ __forceinline__ int grp_min(int v) {
    for (int o = GS_G / 2; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, GS_G));
    return v;
}

// ssw_code as selects (no divergent branch tree)
__device__ __forceinline__ int ssw_code_sel(uint32_t c) {
    const uint32_t u = c | 0x20;              // 'A'..'Z' -> 'a'..'z'; other bytes map outside a/c/g/t/u
    int r = 4;
    r = u == 't' ? 3 : r;
    r = u == 'g' ? 2 : r;
    r = u == 'c' ? 1 : r;
    r = (u == 'a' || u == 'u') ? 0 : r;
    return r;
}

struct FwdG {
    int best[2], col[2], row[2];     // [0] byte layout, [1] word layout; best as f16 bits
};

// query profile of one job in LDS: [code 0..4][lane][GS_RP] f16 scores (match or
// -mismatch) of the lane's rows, so a step reads its column's R scores with
// ds_read_b64s instead of a compare + select per row
template <int R> struct ProfDim {
    static constexpr int RP = (R + 3) & ~3;                  // rows padded to 8 bytes
    static constexpr int CODE_STRIDE = GS_G * RP;            // u16 entries per reference code
    static constexpr int JOB = 5 * CODE_STRIDE;              // u16 entries per job
};

template <int R>
__device__ __forceinline__ void prof_load(const uint16_t* __restrict__ lane_prof, int code, uint32_t (&w)[ProfDim<R>::RP / 2]) {
    const uint2* src = reinterpret_cast<const uint2*>(lane_prof + code * ProfDim<R>::CODE_STRIDE);
#pragma unroll
    for (int k = 0; k < ProfDim<R>::RP / 4; ++k) {
        const uint2 v = src[k];
        w[2 * k] = v.x;
        w[2 * k + 1] = v.y;
    }
}

// forward pass, both layouts at once (low half: byte layout, 16 stripes; high
// half: word layout, 8 stripes); row p of this lane is gl * R + r.  lane_prof is
// this lane's profile slice; code(x) of column x is rc[x] for 0 <= x < ncol.
template <int R>
__device__ __forceinline__ FwdG fwd_g(const uint16_t* __restrict__ lane_prof, int nrow,
                                      const uint8_t* __restrict__ rc, int ncol, int S, bool on, int gO, int gE,
                                      int gl) {
    constexpr int RP = ProfDim<R>::RP;
    const int seg_b = (nrow + 15) / 16, seg_w = (nrow + 7) / 8;
    // H of the previous and of the current column in two arrays that trade roles
    // every step (the loop runs two steps an iteration), so no register copies
    // rotate the column; both start at zero, and an inactive step (column outside
    // the window) only ever precedes the first active one or follows the last
    hh2 E[R], HA[R], HB[R];
    uint32_t ssm[R], B0[R], B1[R];
    const hh2 zero = h2_from(0u);
    const hh2 GO2 = h2_from(h2_pair(gO)), GE2 = h2_from(h2_pair(gE));
#pragma unroll
    for (int r = 0; r < R; ++r) {
        E[r] = zero;
        HA[r] = zero;
        HB[r] = zero;
        B0[r] = 0;
        B1[r] = 0;
        const int p = gl * R + r;
        ssm[r] = ((p % seg_b) == 0 ? 0u : 0x0000FFFFu) | ((p % seg_w) == 0 ? 0u : 0xFFFF0000u);
    }
    uint32_t F_out = 0, Fw_out = 0, H_last = 0, diag_top = 0;
    FwdG o;
    o.best[0] = o.best[1] = 0;
    o.col[0] = o.col[1] = INT_MAX;
    o.row[0] = o.row[1] = INT_MAX;
    // software pipeline over columns: at step s this lane works on column c = s - gl
    // with the profile words P of code(c); code(c + 1) is known, and the step loads
    // the profile of code(c + 1) and the code of c + 2 (LDS latency hidden by a step)
    // columns outside [0, ncol) read the padding (or bytes of no active column)
    auto code_at = [&](int x) -> int { return (int)rc[x]; };
    uint32_t P[RP / 2], Pn[RP / 2];
    prof_load<R>(lane_prof, code_at(-gl), P);
    int code1 = code_at(1 - gl);
    // one step; the loop below runs two per iteration with the profile buffers
    // swapped, so no register copies carry P between steps
    auto step = [&](int s, const uint32_t (&P)[RP / 2], uint32_t (&Pn)[RP / 2], const hh2 (&Hin)[R], hh2 (&Hout)[R]) {
        const uint32_t F_in = row_shr1(F_out);
        const uint32_t Fw_in = row_shr1(Fw_out);
        const uint32_t Hl_in = row_shr1(H_last);
        const int c = s - gl;
        prof_load<R>(lane_prof, code1, Pn);
        const int code2 = code_at(c + 2);
        if (on && c >= 0 && c < ncol) {
            hh2 dg = h2_from(diag_top), F = h2_from(F_in), Fw = h2_from(Fw_in), cm = zero;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                Fw = h2_from(h2_bits(Fw) & ssm[r]);
                const hh2 pw = h2_from(P[r >> 1]);
                const hh2 sc = (r & 1) ? __builtin_shufflevector(pw, pw, 1, 1) : __builtin_shufflevector(pw, pw, 0, 0);
                const hh2 diag = dg + sc;
                const hh2 hm = hmax3(diag, E[r], Fw);
                const hh2 h = hmax(hm, F);
                dg = Hin[r];
                Hout[r] = h;
                const hh2 t = hm - GO2;
                E[r] = hmax3(E[r] - GE2, t, zero);
                Fw = hmax3(Fw - GE2, t, zero);
                F = hmax3(F - GE2, t, zero);
                cm = hmax(cm, h);
            }
            F_out = h2_bits(F);
            Fw_out = h2_bits(Fw);
            H_last = h2_bits(Hout[R - 1]);
            const uint32_t cmb = h2_bits(cm);
            // a new best of a layout: remember the column and this column's rows; the
            // row itself is searched once after the pass
            const int v0 = (int)(cmb & 0xFFFFu), v1 = (int)(cmb >> 16);
            if (v0 > o.best[0]) {
                o.best[0] = v0;
                o.col[0] = c;
#pragma unroll
                for (int r = 0; r < R; ++r) B0[r] = h2_bits(Hout[r]);
            }
            if (v1 > o.best[1]) {
                o.best[1] = v1;
                o.col[1] = c;
#pragma unroll
                for (int r = 0; r < R; ++r) B1[r] = h2_bits(Hout[r]);
            }
        }
        diag_top = Hl_in;
        code1 = code2;
    };
    int s = 0;
    for (; s + 1 < S; s += 2) {
        step(s, P, Pn, HA, HB);
        step(s + 1, Pn, P, HB, HA);
    }
    if (s < S) step(s, P, Pn, HA, HB);
    // the smallest valid row of the best column reaching the best (per layout)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        if (o.col[hf] == INT_MAX) continue;
        int row = INT_MAX;
#pragma unroll
        for (int r = R - 1; r >= 0; --r) {
            const uint32_t b = hf ? B1[r] : B0[r];
            if (gl * R + r < nrow && (int)((b >> (16 * hf)) & 0xFFFFu) == o.best[hf]) row = gl * R + r;
        }
        o.row[hf] = row;
    }
    return o;
}

__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }

// reverse pass (one layout, int32): row p -> query qend - p, column c -> ref rend - c.
// lane_prof holds this lane's rows of the reversed query's profile (int16 scores).
// Returns the first column whose valid-row maximum equals `terminate` (and its
// smallest such row) through tcol/trow, INT_MAX if none.
template <int R>
__device__ __forceinline__ void rev_g(const uint16_t* __restrict__ lane_prof, int nrow, const uint8_t* __restrict__ rc,
                                      int ncol, int rend, int seg, int terminate, int S, bool on, int gO, int gE,
                                      int gl, int& tcol, int& trow) {
    constexpr int RP = ProfDim<R>::RP;
    const int lanes_used = (nrow + R - 1) / R;
    int E[R], HA[R], HB[R], ssm[R];                    // HA / HB: previous / current column, trading roles
    bool valid[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        E[r] = 0;
        HA[r] = 0;
        HB[r] = 0;
        const int p = gl * R + r;
        ssm[r] = (p % seg) == 0 ? 0 : -1;
        valid[r] = p < nrow;
    }
    int F_out = 0, Fw_out = 0, H_last = 0, diag_top = 0;
    tcol = INT_MAX;
    trow = INT_MAX;
    bool done = !on;
    auto code_at = [&](int x) -> int { return (int)rc[rend - x]; };   // padded window: no range check
    uint32_t P[RP / 2], Pn[RP / 2];
    prof_load<R>(lane_prof, code_at(-gl), P);
    int code1 = code_at(1 - gl);
    // one step (two per loop iteration, profile buffers swapped); true once every
    // job of the wave is finished
    auto step = [&](int s, const uint32_t (&P)[RP / 2], uint32_t (&Pn)[RP / 2], const int (&Hin)[R],
                    int (&Hout)[R]) -> bool {
        const int F_in = (int)row_shr1((uint32_t)F_out);
        const int Fw_in = (int)row_shr1((uint32_t)Fw_out);
        const int Hl_in = (int)row_shr1((uint32_t)H_last);
        const int c = s - gl;
        prof_load<R>(lane_prof, code1, Pn);
        const int code2 = code_at(c + 2);
        if (on && c >= 0 && c < ncol) {
            int dg = diag_top, F = F_in, Fw = Fw_in, cm = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                Fw &= ssm[r];
                const uint32_t w = P[r >> 1];
                const int sc = (r & 1) ? ((int)w >> 16) : ((int)(w << 16) >> 16);
                const int diag = dg + sc;
                const int hm = max3i(diag, E[r], Fw);          // E, Fw >= 0: the 0 of max(diag, 0)
                const int h = max(hm, F);
                dg = Hin[r];
                Hout[r] = h;
                const int t = hm - gO;
                E[r] = max3i(E[r] - gE, t, 0);
                Fw = max3i(Fw - gE, t, 0);
                F = max3i(F - gE, t, 0);
                cm = max(cm, h);                   // padding rows included: cm >= the valid rows' maximum
            }
            F_out = F;
            Fw_out = Fw;
            H_last = Hout[R - 1];
            // a column whose maximum over every row reaches terminate may hold a valid row
            // that equals it: only such columns (at most a few a job) look at the valid rows
            const bool cand = cm >= terminate && tcol == INT_MAX;
            if (__builtin_amdgcn_ballot_w64(cand)) {
                if (cand) {
                    int row = INT_MAX;
#pragma unroll
                    for (int r = R - 1; r >= 0; --r)
                        if (valid[r] && Hout[r] == terminate) row = gl * R + r;
                    int cmv = 0;
#pragma unroll
                    for (int r = 0; r < R; ++r) cmv = max(cmv, valid[r] ? Hout[r] : 0);
                    if (cmv == terminate) {
                        tcol = c;
                        trow = row;
                    }
                }
            }
        }
        diag_top = Hl_in;
        code1 = code2;
        if ((s & 7) == 7) {
            // a job is finished once its first terminating column has crossed every lane
            const int m = grp_min(tcol);
            if (m != INT_MAX && s >= m + lanes_used - 1) done = true;
            if (wave_min_i32(done ? 1 : 0)) return true;
        }
        return false;
    };
    int s = 0;
    for (; s + 1 < S; s += 2) {
        if (step(s, P, Pn, HA, HB)) return;
        if (step(s + 1, Pn, P, HB, HA)) return;
    }
    if (s < S) (void)step(s, P, Pn, HA, HB);
}

// this lane's rows of a query profile: the f16 (fwd) or int16 (rev) score of row
// p (query code q[r], 7 = never matches) against reference code 0..4
template <int R>
__device__ __forceinline__ void prof_build(uint16_t* __restrict__ lane_prof, const int (&q)[ProfDim<R>::RP], uint32_t m16,
                                           uint32_t x16) {
    constexpr int RP = ProfDim<R>::RP;
#pragma unroll
    for (int code = 0; code < 5; ++code) {
        uint2* dst = reinterpret_cast<uint2*>(lane_prof + code * ProfDim<R>::CODE_STRIDE);
#pragma unroll
        for (int k = 0; k < RP / 4; ++k) {
            uint32_t w[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t lo = q[4 * k + 2 * h] == code ? m16 : x16;
                const uint32_t hi = q[4 * k + 2 * h + 1] == code ? m16 : x16;
                w[h] = lo | (hi << 16);
            }
            dst[k] = make_uint2(w[0], w[1]);
        }
    }
}

// stages one job into its LDS slot: the reference window as SSW codes with GS_RPAD
// code-4 bytes on both sides (rc points past the leading pad), and this lane's
// rows of the forward query profile (score of row p against reference code 0..4;
// N and padding rows never score a match, not even vs N)
template <int R>
__device__ __forceinline__ void stage_job(uint8_t* __restrict__ rc, uint16_t* __restrict__ lane_prof,
                                          const ExtJobDev& jb, int gl, const char* __restrict__ qbuf,
                                          const char* __restrict__ ref, int match, int mismatch) {
    const int qlen = (int)jb.qlen, rlen = (int)jb.rlen;
    for (int i = gl; i < GS_RPAD; i += GS_G) {
        rc[i - GS_RPAD] = 4;
        rc[rlen + i] = 4;
    }
    {
        // aligned dwords covering the window (the device reference carries 64 bytes of tail padding)
        const int pre = (int)(jb.r_off & 3);
        const uint32_t* w = (const uint32_t*)(ref + (jb.r_off - (uint64_t)pre));
        const int nw = (pre + rlen + 3) >> 2;
        for (int i = gl; i < nw; i += GS_G) {
            const uint32_t x = w[i];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int pos = 4 * i + b - pre;
                if (pos >= 0 && pos < rlen) rc[pos] = (uint8_t)ssw_code_sel((x >> (8 * b)) & 0xFF);
            }
        }
    }
    int qv[ProfDim<R>::RP];
#pragma unroll
    for (int r = 0; r < ProfDim<R>::RP; ++r) {
        const int p = gl * R + r;
        const int code = (r < R && p < qlen) ? ssw_code_sel((unsigned char)qbuf[jb.q_off + p]) : 7;
        qv[r] = code < 4 ? code : 7;
    }
    prof_build<R>(lane_prof, qv, h2_pair(match) & 0xFFFFu, h2_pair(-mismatch) & 0xFFFFu);
}

// the reversed query's profile (int16 scores) of rows 0..nrow-1 = query
// read_end1 .. 0 replaces the forward one in the job's LDS slot (only the job's
// own lanes, one wavefront, read and write it: LDS operations of a wave complete
// in order, and the fence orders the writes before the reads)
template <int R>
__device__ __forceinline__ void stage_rev_prof(uint16_t* __restrict__ lane_prof, const ExtJobDev& jb, int gl,
                                               const char* __restrict__ qbuf, int nrow, int read_end1, int match,
                                               int mismatch) {
    int qr[ProfDim<R>::RP];
#pragma unroll
    for (int r = 0; r < ProfDim<R>::RP; ++r) {
        const int p = gl * R + r;
        int code = 7;
        if (r < R && p < nrow) {
            code = ssw_code_sel((unsigned char)qbuf[jb.q_off + (read_end1 - p)]);
            code = code < 4 ? code : 7;
        }
        qr[r] = code;
    }
    prof_build<R>(lane_prof, qr, (uint32_t)match & 0xFFFFu, (uint32_t)(-mismatch) & 0xFFFFu);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// SSW's choice between the layouts (ssw.c:838-850) from the two-layout forward
// pass: byte unless it saturates; score, ref end (first best column) and read
// end (smallest row of that column reaching the score).  Group-collective.
__device__ __forceinline__ void pick_g(const FwdG& fo, int mismatch, int& word, int& score1, int& ref_end1,
                                       int& read_end1) {
    // maxima as f16 bit patterns (order-preserving for values >= +0)
    const int bb = grp_max(fo.best[0]);
    const int sb = h_bits_to_int((uint32_t)bb);
    word = sb + mismatch >= 255 ? 1 : 0;
    const int bw = word ? grp_max(fo.best[1]) : bb;
    score1 = word ? h_bits_to_int((uint32_t)bw) : sb;
    if (score1 == 0) {
        ref_end1 = word ? 0 : -1;
        read_end1 = 0;
    } else {
        const int e = grp_min(fo.best[word] == bw ? fo.col[word] : INT_MAX);
        read_end1 = grp_min((fo.best[word] == bw && fo.col[word] == e) ? fo.row[word] : INT_MAX);
        ref_end1 = e;
    }
}

// reverse pass (ssw.c:877-893) on read[0..read_end1] x ref[0..ref_end1],
// reversed, and the job's ScanRes (lane 0 of the group writes it).
// Wave-collective: every lane calls it.
template <int R>
__device__ __forceinline__ void rev_write(uint16_t* __restrict__ lane_prof, const ExtJobDev& jb, int j, bool on,
                                          int gl, const char* __restrict__ qbuf, const uint8_t* __restrict__ rc,
                                          int word, int score1, int ref_end1, int read_end1,
                                          int match, int mismatch, int gO, int gE, ScanRes* __restrict__ out) {
    const bool ron = on && score1 > 0;
    const int nrow = ron ? read_end1 + 1 : 0, ncol = ron ? ref_end1 + 1 : 0;
    const int rl_used = (nrow + R - 1) / R;
    stage_rev_prof<R>(lane_prof, jb, gl, qbuf, nrow, read_end1, match, mismatch);
    const int seg = word ? (nrow + 7) / 8 : (nrow + 15) / 16;
    const int S2 = wave_max_i32(ron ? ncol + rl_used - 1 : 0);
    int tc = INT_MAX, tr = INT_MAX;
    if (S2 > 0)
        rev_g<R>(lane_prof, nrow, rc, ncol, ref_end1, seg > 0 ? seg : 1, score1, S2, ron && gl < rl_used, gO, gE, gl,
                 tc, tr);
    const int tcol = grp_min(tc);
    const int trow = grp_min(tc == tcol ? tr : INT_MAX);
    if (!on || gl != 0) return;
    ScanRes res;
    res.score1 = score1; res.ref_end1 = ref_end1; res.read_end1 = read_end1; res.word = word;
    res.flag = 0; res.status = 0;
    if (score1 > 0) {
        if (tcol == INT_MAX) {
            res.flag = 2;   // reverse max < score1: "may miss a small part"
            res.ref_begin1 = 0;
            res.read_begin1 = 0;
        } else {
            res.ref_begin1 = ref_end1 - tcol;
            res.read_begin1 = read_end1 - trow;
        }
    } else {
        res.ref_begin1 = word ? 0 : -1;
        res.read_begin1 = 0;
    }
    out[j] = res;
}

}  // namespace

// jobs[order[k]] for k < n; results land at out[order[k]].  Every job handed
// here has 0 < qlen <= GS_G * R and rlen <= GS_MAXR (the host routes the rest to
// k_ext_scan).
template <int R>
__global__ void __launch_bounds__(64 * GS_WAVES)
k_ext_scan_g(const ExtJobDev* __restrict__ jobs, const int* __restrict__ order, int n,
             const char* __restrict__ qbuf, const char* __restrict__ ref, ScanRes* __restrict__ out,
             int match, int mismatch, int gO, int gE) {
    __shared__ uint8_t s_r[GS_JOBS][GS_RPAD + GS_MAXR + GS_RPAD];
    __shared__ __attribute__((aligned(16))) uint16_t s_prof[GS_JOBS][ProfDim<R>::JOB];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int slot = wave * (64 / GS_G) + lane / GS_G, gl = lane & (GS_G - 1);
    const int k = blockIdx.x * GS_JOBS + slot;
    const bool on = k < n;
    const int j = on ? order[k] : 0;
    ExtJobDev jb;
    jb.q_off = 0; jb.r_off = 0; jb.qlen = 0; jb.rlen = 0; jb.cig_off = 0;
    if (on) jb = jobs[j];
    const int qlen = (int)jb.qlen, rlen = (int)jb.rlen;
    uint8_t* rc = s_r[slot] + GS_RPAD;
    uint16_t* lane_prof = s_prof[slot] + gl * ProfDim<R>::RP;
    stage_job<R>(rc, lane_prof, jb, gl, qbuf, ref, match, mismatch);
    __syncthreads();

    // forward pass: every job of the wave runs until the longest one is done
    const int lanes_used = (qlen + R - 1) / R;
    const int S = wave_max_i32(on ? rlen + lanes_used - 1 : 0);
    const FwdG fo = fwd_g<R>(lane_prof, qlen, rc, rlen, S, on && gl < lanes_used, gO, gE, gl);
    int word, score1, ref_end1, read_end1;
    pick_g(fo, mismatch, word, score1, ref_end1, read_end1);
    rev_write<R>(lane_prof, jb, j, on, gl, qbuf, rc, word, score1, ref_end1, read_end1, match, mismatch, gO, gE, out);
}

// rows per lane of the grouped scan for a query length (0: not handled here)
int scan_g_rows(uint32_t qlen) {
    if (qlen == 0) return 0;
    if constexpr (GS_G == 16) {
        if (qlen <= 64) return 4;
        if (qlen <= 112) return 7;
        if (qlen <= 160) return 10;
        if (qlen <= 208) return 13;
        if (qlen <= 256) return 16;
    } else {
        if (qlen <= 64) return 2;
        if (qlen <= 128) return 4;
        if (qlen <= 160) return 5;
        if (qlen <= 224) return 7;
        if (qlen <= 256) return 8;
    }
    return 0;
}

int scan_g_max_ref() { return GS_MAXR; }

// the five rows-per-lane classes, ascending
void scan_g_classes(int* rows5) {
    static const int r16[5] = {4, 7, 10, 13, 16}, r32[5] = {2, 4, 5, 7, 8};
    for (int i = 0; i < 5; ++i) rows5[i] = GS_G == 16 ? r16[i] : r32[i];
}

void launch_ext_scan_g(int rows, int n, hipStream_t st, const ExtJobDev* jobs, const int* order, const char* q,
                       const char* ref, ScanRes* out, int match, int mismatch, int gO, int gE) {
    if (n <= 0) return;
    const dim3 grid((n + GS_JOBS - 1) / GS_JOBS), block(64 * GS_WAVES);
#define RSA_G(RR)                                                                                               \
    if (rows == RR) {                                                                                           \
        hipLaunchKernelGGL((k_ext_scan_g<RR>), grid, block, 0, st, jobs, order, n, q, ref, out, match, mismatch, \
                           gO, gE);                                                                             \
        return;                                                                                                 \
    }
    if constexpr (GS_G == 16) { RSA_G(4) RSA_G(7) RSA_G(10) RSA_G(13) RSA_G(16) }
    else { RSA_G(2) RSA_G(4) RSA_G(5) RSA_G(7) RSA_G(8) }
#undef RSA_G
}

bool scan_g_params_ok(int match, int mismatch, int gO, int gE);

// parameters the grouped scan computes exactly: half-precision integers stay
// below 2048 in magnitude (scores up to match * 256, penalties), and F's
// shortened recurrence needs gap_open >= gap_extend
bool scan_g_params_ok(int match, int mismatch, int gO, int gE) {
    return match >= 0 && match * 256 <= 2048 && mismatch >= 0 && mismatch <= 1024 && gO >= 0 && gO <= 1024 &&
           gE >= 0 && gE <= gO;
}
