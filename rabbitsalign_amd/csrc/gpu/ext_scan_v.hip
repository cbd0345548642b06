// ext_scan_v.hip -- the SSW scan with 32 virtual lanes per job: 16 lanes, each
// lane's packed-f16 registers holding two row blocks of the same job.
//
// Same results as k_ext_scan_g / k_ext_scan (SSW's forward pass, byte layout
// unless it saturates, then the reverse pass that stops at the first column
// reaching score1; ssw.c:197-588, 838-893), computed differently:
//
//   * one layout per pass.  The grouped scan (ext_scan_g.hip) runs the byte
//     (16-stripe) and word (8-stripe) layouts of one cell in the two halves of
//     a packed register, although the byte layout only decides whether SSW
//     switches to words, and on the headline workload nearly every job does.
//     Here the two halves hold two *rows* of the same job and the same layout:
//     virtual lane v = gl (low halves) and v = 16 + gl (high halves) of a
//     16-lane group own query rows v * RV .. v * RV + RV - 1, and the reference
//     streams through the 32 virtual lanes as an anti-diagonal systolic array
//     (virtual lane v works on column s - v at step s).  Every packed
//     instruction does two cells' work of the layout that is needed;
//   * the row-above values move one virtual lane per step with one DPP
//     row_ror:1 and one shift: lane gl receives lane gl-1's register, lane 0
//     lane 15's shifted up a half (its low half reads the zero boundary above
//     row 0, its high half -- virtual lane 16 -- virtual lane 15's low half);
//   * a query too short to reach the byte bound (match * qlen + bias < 255)
//     runs the byte layout alone.  Otherwise the word pass runs first.  SSW
//     takes the word result exactly when the byte pass saturates (byte score +
//     bias >= 255).  A job whose word score
//     is below that bound runs the byte pass too (inline, same kernel) and
//     takes SSW's decision from both.  A job whose word score reaches it takes
//     the word result, *certified later*: the byte layout differs from the
//     word layout only where a vertical gap (F) that crossed a byte stripe
//     boundary would have opened a horizontal gap (E), i.e. an insertion
//     directly followed by a deletion.  An alignment path with no insertion
//     next to a deletion is therefore scored by the byte layout at least as
//     high as its own score; the banded traceback (ext_kernels.hip) produces
//     such a path for the job, of score >= the word score, so the byte pass
//     provably saturates.  The band kernels list every job whose path has an
//     I next to a D (or whose band pass fails) and rsa_extend re-runs those
//     through the two-layout scan (k_ext_scan) and the band kernels -- results
//     are SSW's in every case (ScanRes.word bit 1 marks a certified job);
//   * per row the score comes from a query profile in LDS laid out
//     [code][row][virtual lane], read as two 16-bit loads (the low half's
//     column code, the high half's) per row;
//   * columns outside a job's window read code-4 padding (a score of
//     -mismatch everywhere): before the window every value stays 0, after it
//     no value can exceed an earlier one, so no step needs an activity mask.
//
// Arithmetic: packed f16 holding exact integers, as in ext_scan_g.hip (host
// check: match * 256 <= 2048, penalties <= 1024, gap_open >= gap_extend).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>

#include "rsa_dev.h"
#include "rsa_ext.h"

#define VS_WAVES 2
#define VS_G 16                              // lanes per job
#define VS_JOBS (VS_WAVES * (64 / VS_G))     // jobs per workgroup
#define VS_PAD 40                            // code-4 bytes before a staged window, and after the slot's capacity

namespace {

typedef _Float16 hh2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ hh2 h2_from(uint32_t x) { return __builtin_bit_cast(hh2, x); }
__device__ __forceinline__ uint32_t h2_bits(hh2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ hh2 hmax(hh2 a, hh2 b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ hh2 hmax3(hh2 a, hh2 b, hh2 c) { return hmax(hmax(a, b), c); }
__device__ __forceinline__ uint32_t h_bits16(int v) {
    const _Float16 h = (_Float16)v;
    return (uint32_t)__builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ int h_bits_to_int(uint32_t bits16) {
    return (int)(float)__builtin_bit_cast(_Float16, (uint16_t)bits16);
}

// one virtual lane down (see the file comment); sh0 = 16 on lane 0, else 0
__device__ __forceinline__ uint32_t vshr1(uint32_t v, uint32_t sh0) {
    const uint32_t x = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x121, 0xf, 0xf, true);   // row_ror:1
    return x << sh0;
}

__device__ __forceinline__ int grp_max(int v) {
    for (int o = VS_G / 2; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, VS_G));
    return v;
}
__device__ __forceinline__ int grp_min(int v) {
    for (int o = VS_G / 2; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, VS_G));
    return v;
}

// query profile of one job: [code 0..3][row r of a virtual lane][virtual lane 0..31], f16 bits.
// Reference code 4 (N, and the padding around a window) scores -mismatch against every
// query row, so its row is one block-wide constant row after the jobs' profiles: a job in
// slot j stages code 4 as the row offset 4 * (VS_JOBS - j), which lands there.  One row a
// job fewer in LDS (4 codes, not 5): 6 workgroups a CU instead of 5 at 8 rows a virtual
// lane (2 x 250 bp), the same address arithmetic a step.
template <int RV> struct VProf {
    static constexpr int CODE = RV * 32;            // u16 entries per reference code
    static constexpr int JOB = 4 * CODE;
};
// the staged code of reference code 4 for the job in `slot`
__device__ __forceinline__ uint32_t pad_code(int slot) { return 4u * (uint32_t)(VS_JOBS - slot); }

// The packed scores of a step's rows: low halves against code clo (virtual lane
// gl), high halves against code chi (virtual lane 16 + gl).  Two 16-bit LDS
// loads a row; the high one is merged with one SDWA move (dst_sel:WORD_1,
// UNUSED_PRESERVE: the low half stays), a single 32-bit-encoded VALU op.  (A
// d16_hi load straight into the register would merge against the register's
// value at issue, i.e. before the low half's own load returned.)
__device__ __forceinline__ uint32_t put_hi16(uint32_t lo, uint32_t hi) {
    asm("v_mov_b32_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0" : "+v"(lo) : "v"(hi));
    return lo;
}
template <int RV>
__device__ __forceinline__ void prof_pair(const uint16_t* __restrict__ prof, int clo, int chi, int gl,
                                          uint32_t (&P)[RV]) {
    const uint16_t* a = prof + clo * VProf<RV>::CODE + gl;
    const uint16_t* b = prof + chi * VProf<RV>::CODE + 16 + gl;
#pragma unroll
    for (int r = 0; r < RV; ++r) P[r] = put_hi16((uint32_t)a[r * 32], (uint32_t)b[r * 32]);
}

// this lane's two virtual lanes' rows of a profile: row p of virtual lane v is
// query code qcode(p) (7 = padding / N: never a match, not even vs N)
template <int RV, typename QF>
__device__ __forceinline__ void prof_build(uint16_t* __restrict__ prof, int gl, QF qcode, uint32_t m16, uint32_t x16) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        const int v = hf * 16 + gl;
#pragma unroll
        for (int r = 0; r < RV; ++r) {
            const int q = qcode(v * RV + r);
#pragma unroll
            for (int code = 0; code < 4; ++code)
                prof[code * VProf<RV>::CODE + r * 32 + v] = (uint16_t)(q == code ? m16 : x16);
        }
    }
}

struct FwdV {
    int best[2], col[2], row[2];    // [0] low half (virtual lane gl), [1] high half (16 + gl); best as f16 bits
};

// forward pass of one layout (stripe length seg) over ncol columns; rc[-40..-1]
// and rc[ncol..] (to the slot's end) are code-4 padding.  S steps (the wave's
// longest job).
template <int RV>
__device__ __forceinline__ FwdV fwd_v(const uint16_t* __restrict__ prof, int nrow, const uint8_t* __restrict__ rc,
                                      int S, int seg, int gO, int gE, int gl) {
    hh2 E[RV], HA[RV], HB[RV];
    uint32_t ssm[RV], B0[RV], B1[RV];
    const hh2 zero = h2_from(0u);
    const uint32_t go = h_bits16(gO), ge = h_bits16(gE);
    const hh2 GO2 = h2_from(go | (go << 16)), GE2 = h2_from(ge | (ge << 16));
#pragma unroll
    for (int r = 0; r < RV; ++r) {
        E[r] = zero;
        HA[r] = zero;
        HB[r] = zero;
        B0[r] = 0;
        B1[r] = 0;
        const int p0 = gl * RV + r, p1 = (16 + gl) * RV + r;
        ssm[r] = ((p0 % seg) == 0 ? 0u : 0x0000FFFFu) | ((p1 % seg) == 0 ? 0u : 0xFFFF0000u);
    }
    const uint32_t sh0 = gl == 0 ? 16u : 0u;
    uint32_t F_out = 0, Fw_out = 0, H_last = 0, diag_top = 0;
    FwdV o;
    o.best[0] = o.best[1] = 0;
    o.col[0] = o.col[1] = INT_MAX;
    o.row[0] = o.row[1] = INT_MAX;
    // the high half's column is the low half's - 16: rcq[x + 16] / rcq[x] are the codes of
    // column x - gl for the low / high half
    const uint8_t* rcq = rc - 16 - gl;
    uint32_t P[RV], Pn[RV];
    prof_pair<RV>(prof, rcq[16], rcq[0], gl, P);
    int c1lo = rcq[17], c1hi = rcq[1];
    auto step = [&](int s, const uint32_t (&P)[RV], uint32_t (&Pn)[RV], const hh2 (&Hin)[RV], hh2 (&Hout)[RV]) {
        prof_pair<RV>(prof, c1lo, c1hi, gl, Pn);
        const uint32_t F_in = vshr1(F_out, sh0);
        const uint32_t Fw_in = vshr1(Fw_out, sh0);
        const uint32_t Hl_in = vshr1(H_last, sh0);
        const int c = s - gl;                        // the low half's column; the high half's is c - 16
        const int c2lo = rcq[s + 18], c2hi = rcq[s + 2];
        hh2 dg = h2_from(diag_top), F = h2_from(F_in), Fw = h2_from(Fw_in), cm = zero;
#pragma unroll
        for (int r = 0; r < RV; ++r) {
            Fw = h2_from(h2_bits(Fw) & ssm[r]);
            const hh2 diag = dg + h2_from(P[r]);
            const hh2 hm = hmax3(diag, E[r], Fw);
            const hh2 h = hmax(hm, F);
            dg = Hin[r];
            Hout[r] = h;
            const hh2 t = hm - GO2;
            E[r] = hmax3(E[r] - GE2, t, zero);
            Fw = hmax3(Fw - GE2, t, zero);
            F = hmax3(F - GE2, t, zero);
        }
        // the column maximum over row pairs: one three-input max per two rows
#pragma unroll
        for (int r = 0; r < RV; r += 2) cm = r + 1 < RV ? hmax3(cm, Hout[r], Hout[r + 1]) : hmax(cm, Hout[r]);
        F_out = h2_bits(F);
        Fw_out = h2_bits(Fw);
        H_last = h2_bits(Hout[RV - 1]);
        const uint32_t cmb = h2_bits(cm);
        const int v0 = (int)(cmb & 0xFFFFu), v1 = (int)(cmb >> 16);
        if (v0 > o.best[0]) {
            o.best[0] = v0;
            o.col[0] = c;
#pragma unroll
            for (int r = 0; r < RV; ++r) B0[r] = h2_bits(Hout[r]);
        }
        if (v1 > o.best[1]) {
            o.best[1] = v1;
            o.col[1] = c - 16;
#pragma unroll
            for (int r = 0; r < RV; ++r) B1[r] = h2_bits(Hout[r]);
        }
        diag_top = Hl_in;
        c1lo = c2lo;
        c1hi = c2hi;
    };
    int s = 0;
    for (; s + 1 < S; s += 2) {
        step(s, P, Pn, HA, HB);
        step(s + 1, Pn, P, HB, HA);
    }
    if (s < S) step(s, P, Pn, HA, HB);
    // the smallest valid row of each half's best column reaching its best
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        if (o.col[hf] == INT_MAX) continue;
        int row = INT_MAX;
#pragma unroll
        for (int r = RV - 1; r >= 0; --r) {
            const uint32_t b = hf ? B1[r] : B0[r];
            const int p = (hf * 16 + gl) * RV + r;
            if (p < nrow && (int)((b >> (16 * hf)) & 0xFFFFu) == o.best[hf]) row = p;
        }
        o.row[hf] = row;
    }
    return o;
}

// score1, ref end (first best column) and read end (smallest row of that column
// reaching the score) of one layout; byte-layout convention for a zero score
// (ssw.c:838-850).  Group-collective.
__device__ __forceinline__ void pick_v(const FwdV& fo, bool word, int& score1, int& ref_end1, int& read_end1) {
    const int b = grp_max(max(fo.best[0], fo.best[1]));      // f16 bits: order-preserving for values >= +0
    score1 = h_bits_to_int((uint32_t)b);
    if (score1 == 0) {
        ref_end1 = word ? 0 : -1;
        read_end1 = 0;
        return;
    }
    const int e = grp_min(min(fo.best[0] == b ? fo.col[0] : INT_MAX, fo.best[1] == b ? fo.col[1] : INT_MAX));
    read_end1 = grp_min(min((fo.best[0] == b && fo.col[0] == e) ? fo.row[0] : INT_MAX,
                            (fo.best[1] == b && fo.col[1] == e) ? fo.row[1] : INT_MAX));
    ref_end1 = e;
}

// reverse pass (one layout): row p -> query read_end1 - p, column c -> ref
// rend - c.  rc[rend + 1 .. rend + 40] and rc[-40 .. -1] are code-4 padding
// (columns before the first read the former, columns past the last are clamped
// to rc[-1]).  The first column whose valid-row maximum equals `terminate` and
// its smallest such row, per half, through tcol/trow (INT_MAX if none).
template <int RV>
__device__ __forceinline__ void rev_v(const uint16_t* __restrict__ prof, int nrow, const uint8_t* __restrict__ rc,
                                      int rend, int seg, int terminate, int S, bool active, int gO, int gE, int gl,
                                      int (&tcol)[2], int (&trow)[2]) {
    const int vl_used = (nrow + RV - 1) / RV;
    hh2 E[RV], HA[RV], HB[RV];
    uint32_t ssm[RV], vmask[RV];
    const hh2 zero = h2_from(0u);
    const uint32_t go = h_bits16(gO), ge = h_bits16(gE);
    const hh2 GO2 = h2_from(go | (go << 16)), GE2 = h2_from(ge | (ge << 16));
    const uint32_t tb = h_bits16(terminate);
#pragma unroll
    for (int r = 0; r < RV; ++r) {
        E[r] = zero;
        HA[r] = zero;
        HB[r] = zero;
        const int p0 = gl * RV + r, p1 = (16 + gl) * RV + r;
        ssm[r] = ((p0 % seg) == 0 ? 0u : 0x0000FFFFu) | ((p1 % seg) == 0 ? 0u : 0xFFFF0000u);
        vmask[r] = (p0 < nrow ? 0x0000FFFFu : 0u) | (p1 < nrow ? 0xFFFF0000u : 0u);
    }
    const uint32_t sh0 = gl == 0 ? 16u : 0u;
    uint32_t F_out = 0, Fw_out = 0, H_last = 0, diag_top = 0;
    tcol[0] = tcol[1] = INT_MAX;
    trow[0] = trow[1] = INT_MAX;
    bool done = !active;
    // code of column x (of the reversed window) for the low half; the high half's is x - 16
    const int base = rend + gl;
    auto code_at = [&](int x) -> int { return (int)rc[max(base - x, -1)]; };
    uint32_t P[RV], Pn[RV];
    prof_pair<RV>(prof, code_at(0), code_at(-16), gl, P);
    int c1lo = code_at(1), c1hi = code_at(1 - 16);
    // one step; true once every job of the wave is finished
    auto step = [&](int s, const uint32_t (&P)[RV], uint32_t (&Pn)[RV], const hh2 (&Hin)[RV],
                    hh2 (&Hout)[RV]) -> bool {
        prof_pair<RV>(prof, c1lo, c1hi, gl, Pn);
        const uint32_t F_in = vshr1(F_out, sh0);
        const uint32_t Fw_in = vshr1(Fw_out, sh0);
        const uint32_t Hl_in = vshr1(H_last, sh0);
        const int c = s - gl;
        const int c2lo = code_at(s + 2), c2hi = code_at(s + 2 - 16);
        hh2 dg = h2_from(diag_top), F = h2_from(F_in), Fw = h2_from(Fw_in), cm = zero;
#pragma unroll
        for (int r = 0; r < RV; ++r) {
            Fw = h2_from(h2_bits(Fw) & ssm[r]);
            const hh2 diag = dg + h2_from(P[r]);
            const hh2 hm = hmax3(diag, E[r], Fw);
            const hh2 h = hmax(hm, F);
            dg = Hin[r];
            Hout[r] = h;
            const hh2 t = hm - GO2;
            E[r] = hmax3(E[r] - GE2, t, zero);
            Fw = hmax3(Fw - GE2, t, zero);
            F = hmax3(F - GE2, t, zero);
        }
        // padding rows included: cm >= the valid rows' maximum
#pragma unroll
        for (int r = 0; r < RV; r += 2) cm = r + 1 < RV ? hmax3(cm, Hout[r], Hout[r + 1]) : hmax(cm, Hout[r]);
        F_out = h2_bits(F);
        Fw_out = h2_bits(Fw);
        H_last = h2_bits(Hout[RV - 1]);
        // a column whose maximum over every row reaches terminate may hold a valid row that
        // equals it: only such columns (a few a job) look at the valid rows
        const uint32_t cmb = h2_bits(cm);
        const bool cand0 = (cmb & 0xFFFFu) >= tb && tcol[0] == INT_MAX;
        const bool cand1 = (cmb >> 16) >= tb && tcol[1] == INT_MAX;
        if (__builtin_amdgcn_ballot_w64(cand0 || cand1)) {
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                if (!(hf ? cand1 : cand0)) continue;
                int row = INT_MAX;
                uint32_t cmv = 0;
#pragma unroll
                for (int r = RV - 1; r >= 0; --r) {
                    const uint32_t hv = ((h2_bits(Hout[r]) & vmask[r]) >> (16 * hf)) & 0xFFFFu;
                    if (hv == tb) row = (hf * 16 + gl) * RV + r;
                    cmv = hv > cmv ? hv : cmv;
                }
                if (cmv == tb) {
                    tcol[hf] = c - 16 * hf;
                    trow[hf] = row;
                }
            }
        }
        diag_top = Hl_in;
        c1lo = c2lo;
        c1hi = c2hi;
        if ((s & 7) == 7) {
            // a job is finished once its first terminating column has crossed every virtual lane
            const int m = grp_min(min(tcol[0], tcol[1]));
            if (m != INT_MAX && s >= m + vl_used - 1) done = true;
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

// SSW base translation as selects (rsa_dev.h ssw_code); 7 for codes that never match
__device__ __forceinline__ int qcode7(unsigned char b) {
    const int c = ssw_code(b);
    return c < 4 ? c : 7;
}

// 4 bytes as 4 codes, packed: byte b (at position pos0 + b) -> code(byte) when the
// position is in [0, len), else `pad`
template <class CF>
__device__ __forceinline__ uint32_t codes4(uint32_t x, int pos0, int len, CF code, uint32_t pad) {
    uint32_t r = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int pos = pos0 + b;
        const uint32_t c = (pos >= 0 && pos < len) ? (uint32_t)code((x >> (8 * b)) & 0xFF) : pad;
        r |= c << (8 * b);
    }
    return r;
}

}  // namespace

// Job k < n is sjobs[k] (the descriptors in scan order, staged so by the host) and
// its result lands at out[order[k]].  Every job handed
// here has 0 < qlen <= 32 * RV and rlen <= WCAP (the host routes the rest to
// k_ext_scan).
// waves per SIMD the register allocation is held to (VS_MINW_SHORT for RV <= 5, VS_MINW_LONG
// above; 0 = the compiler's choice)
#ifndef VS_MINW_SHORT
#define VS_MINW_SHORT 0
#endif
#ifndef VS_MINW_LONG
#define VS_MINW_LONG 0
#endif
template <int RV> struct VsMinW { static constexpr int value = RV <= 5 ? VS_MINW_SHORT : VS_MINW_LONG; };

template <int RV, int WCAP>
__global__ void __launch_bounds__(64 * VS_WAVES, VsMinW<RV>::value)
k_ext_scan_v(const ExtJobDev* __restrict__ sjobs, const int* __restrict__ order, int n,
             const char* __restrict__ qbuf, const char* __restrict__ ref, ScanRes* __restrict__ out,
             int match, int mismatch, int gO, int gE, int* __restrict__ err, int prio) {
    // the extension finishes chunks the SAM writer waits for: its waves may claim the
    // SIMDs they share with the seeding kernels first (s_setprio, RSA_EXT_SETPRIO)
    if (prio) __builtin_amdgcn_s_setprio(2);
    // a slot: VS_PAD bytes of padding, the window from the dword-aligned base (its first
    // byte at base + (r_off & 3)), WCAP + VS_PAD bytes after the base in all
    constexpr int SLOT = WCAP + 2 * VS_PAD + 4;
    constexpr int QSLOT = 32 * RV + 4;
    __shared__ __attribute__((aligned(4))) uint8_t s_r[VS_JOBS][SLOT];
    __shared__ __attribute__((aligned(16))) uint16_t s_prof[VS_JOBS + 1][VProf<RV>::JOB];   // + the code-4 row
    __shared__ __attribute__((aligned(4))) uint8_t s_q[VS_JOBS][QSLOT];   // query codes (qcode7), 7 past the query
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int slot = wave * (64 / VS_G) + lane / VS_G, gl = lane & (VS_G - 1);
    const int k = blockIdx.x * VS_JOBS + slot;
    const bool on = k < n;
    // the descriptor and the result index in one round trip (both indexed by k)
    const int j = on ? order[k] : 0;
    ExtJobDev jb;
    jb.q_off = 0; jb.r_off = 0; jb.qlen = 0; jb.rlen = 0; jb.cig_off = 0;
    if (on) jb = sjobs[k];
    const int qlen = (int)jb.qlen, rlen = (int)jb.rlen;
    const int pre = (int)(jb.r_off & 3), preq = (int)(jb.q_off & 3);
    uint8_t* rcb = s_r[slot] + VS_PAD;
    uint8_t* rc = rcb + pre;
    uint16_t* prof = s_prof[slot];
    const uint32_t pc = pad_code(slot), pc4 = pc * 0x01010101u;
    uint8_t* qc = s_q[slot] + preq;

    // stage the window and the query as SSW codes, a dword (4 codes) at a time.  Every
    // load of a lane is issued before any is used (indices clamped into the job's own
    // dwords; the device reference carries 64 bytes of tail padding and the query
    // buffer a dword past its end), then the codes are written: code-4 padding before
    // the window and from its end to the end of the slot (the wave's steps read up to
    // 32 columns past its longest window), query code 7 past the query.
    {
        constexpr int WD = ((WCAP + 6) / 4 + VS_G - 1) / VS_G;      // window dwords a lane loads at most
        constexpr int QD = (32 * RV + 3 + 4 * VS_G - 1) / (4 * VS_G);   // query dwords a lane loads at most
        const uint32_t* w = (const uint32_t*)(ref + (jb.r_off - (uint64_t)pre));
        const uint32_t* qw = (const uint32_t*)(qbuf + (jb.q_off - (uint64_t)preq));
        const int nw = (pre + rlen + 3) >> 2, nq = (preq + qlen + 3) >> 2;
        const int wl = max(nw - 1, 0), ql = max(nq - 1, 0);
        uint32_t x[WD], y[QD];
#pragma unroll
        for (int t = 0; t < WD; ++t) x[t] = w[min(gl + t * VS_G, wl)];
#pragma unroll
        for (int t = 0; t < QD; ++t) y[t] = qw[min(gl + t * VS_G, ql)];
        uint32_t* rcw = (uint32_t*)rcb;
        for (int i = gl; i < VS_PAD / 4; i += VS_G) rcw[i - VS_PAD / 4] = pc4;
#pragma unroll
        for (int t = 0; t < WD; ++t) {
            const int i = gl + t * VS_G;
            if (i < nw)
                rcw[i] = codes4(x[t], 4 * i - pre, rlen, [&](uint32_t b) {
                    const uint32_t c = (uint32_t)ssw_code((unsigned char)b);
                    return c < 4 ? c : pc;
                }, pc);
        }
        for (int i = nw + gl; i < (WCAP + VS_PAD + 4) / 4; i += VS_G) rcw[i] = pc4;
        // the block's code-4 row (every wave writes the same values; the barrier after the
        // profiles orders them before any read)
        for (int i = threadIdx.x; i < VProf<RV>::CODE; i += 64 * VS_WAVES) s_prof[VS_JOBS][i] = (uint16_t)h_bits16(-mismatch);
        uint32_t* qcw = (uint32_t*)s_q[slot];
#pragma unroll
        for (int t = 0; t < QD; ++t) {
            const int i = gl + t * VS_G;
            if (i < QSLOT / 4) qcw[i] = codes4(y[t], 4 * i - preq, qlen, [](uint32_t b) { return qcode7((unsigned char)b); }, 7u);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t m16 = h_bits16(match), x16 = h_bits16(-mismatch);
    prof_build<RV>(prof, gl, [&](int p) { return (int)qc[p]; }, m16, x16);
    __syncthreads();

    const int vl_used = (qlen + RV - 1) / RV;
    const int S = wave_max_i32(on ? rlen + vl_used - 1 : 0);
    const int seg_w = (qlen + 7) / 8, seg_b = (qlen + 15) / 16;
    // A query whose every-base-matches score stays below the byte bound can only take the
    // byte layout: one pass.  Otherwise the word layout first: its score decides whether
    // the byte layout could still be SSW's choice.
    const bool byte_only = match * qlen + mismatch < 255;
    int score1, ref_end1, read_end1;
    {
        const int seg = byte_only ? seg_b : seg_w;
        const FwdV fw = fwd_v<RV>(prof, qlen, rc, S, seg > 0 ? seg : 1, gO, gE, gl);
        pick_v(fw, !byte_only, score1, ref_end1, read_end1);
    }
    int word = byte_only ? 0 : 1;
    bool cert = on && !byte_only;     // word taken on the word score alone: certified by the band traceback
    const bool need_b = on && !byte_only && score1 + mismatch < 255;
    if (__builtin_amdgcn_ballot_w64(need_b)) {
        const FwdV fb = fwd_v<RV>(prof, qlen, rc, S, seg_b > 0 ? seg_b : 1, gO, gE, gl);
        int sb, eb, rb;
        pick_v(fb, false, sb, eb, rb);
        if (need_b) {
            cert = false;             // both layouts computed: SSW's decision exactly (ssw.c:838-850)
            if (sb + mismatch < 255) {
                word = 0;
                score1 = sb;
                ref_end1 = eb;
                read_end1 = rb;
            }
        }
    }

    // an end outside the job is a defect of this kernel: no reverse pass reads past the
    // query for it, the job gets status 3 (a sentinel for the band kernels) and the call fails
    const bool bad = on && score1 > 0 && (read_end1 < 0 || read_end1 >= qlen || ref_end1 < 0 || ref_end1 >= rlen);
    // reverse pass (ssw.c:877-893) on read[0..read_end1] x ref[0..ref_end1], reversed
    const bool ron = on && score1 > 0 && !bad;
    const int nrow = ron ? read_end1 + 1 : 0, ncol = ron ? ref_end1 + 1 : 0;
    const int rl_used = (nrow + RV - 1) / RV;
    const int S2 = wave_max_i32(ron ? ncol + rl_used - 1 : 0);
    int tc[2] = {INT_MAX, INT_MAX}, tr[2] = {INT_MAX, INT_MAX};
    if (S2 > 0) {
        // the reversed query's profile replaces the forward one, and the window byte after
        // ref_end1 becomes padding (only this job's lanes, one wavefront, touch the slot: LDS
        // operations of a wave complete in order, and the fence orders writes before reads)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (ron)
            for (int i = gl; i < VS_PAD; i += VS_G) rc[ref_end1 + 1 + i] = (uint8_t)pc;
        prof_build<RV>(prof, gl, [&](int p) { return p < nrow ? (int)qc[read_end1 - p] : 7; }, m16, x16);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const int seg = word ? (nrow + 7) / 8 : (nrow + 15) / 16;
        rev_v<RV>(prof, nrow, rc, ron ? ref_end1 : 0, seg > 0 ? seg : 1, ron ? score1 : INT_MAX, S2, ron, gO, gE, gl,
                  tc, tr);
    }
    const int tcol = grp_min(min(tc[0], tc[1]));
    const int trow = grp_min(min(tc[0] == tcol ? tr[0] : INT_MAX, tc[1] == tcol ? tr[1] : INT_MAX));
    if (!on || gl != 0) return;
    ScanRes res;
    res.score1 = score1; res.ref_end1 = ref_end1; res.read_end1 = read_end1;
    res.word = word | (cert ? 2 : 0);
    res.flag = 0; res.status = 0;
    if (bad) {
        res.status = 3;
        res.ref_begin1 = res.read_begin1 = 0;
        atomicOr(err, 1);
    } else if (score1 > 0) {
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

// rows per virtual lane for a query length (0: not handled here)
int scan_v_rows(uint32_t qlen) {
    if (qlen == 0 || qlen > 256) return 0;
    const int rv = (int)((qlen + 31) / 32);
    return rv < 2 ? 2 : rv;
}

// window capacity class for a window length (0: not handled here)
int scan_v_wcap(uint32_t rlen) {
    if (rlen <= 512) return 512;
    if (rlen <= 1024) return 1024;
    return 0;
}

// sjobs: the class's descriptors in scan order; order: their indices (results go to out[order[k]])
void launch_ext_scan_v(int rv, int wcap, int n, hipStream_t st, const ExtJobDev* sjobs, const int* order, const char* q,
                       const char* ref, ScanRes* out, int match, int mismatch, int gO, int gE, int* err, int prio) {
    if (n <= 0) return;
    const dim3 grid((n + VS_JOBS - 1) / VS_JOBS), block(64 * VS_WAVES);
#define RSA_V(RR, WW)                                                                                             \
    if (rv == RR && wcap == WW) {                                                                                 \
        hipLaunchKernelGGL((k_ext_scan_v<RR, WW>), grid, block, 0, st, sjobs, order, n, q, ref, out, match,       \
                           mismatch, gO, gE, err, prio);                                                          \
        return;                                                                                                   \
    }
    RSA_V(2, 512) RSA_V(3, 512) RSA_V(4, 512) RSA_V(5, 512) RSA_V(6, 512) RSA_V(7, 512) RSA_V(8, 512)
    RSA_V(2, 1024) RSA_V(3, 1024) RSA_V(4, 1024) RSA_V(5, 1024) RSA_V(6, 1024) RSA_V(7, 1024) RSA_V(8, 1024)
#undef RSA_V
}
