// seed_kernels.hip -- randstrobe seeding + find_nams / find_nams_rescue on gfx950.
//
// Replaces the per-read CPU loop of align_{PE,SE}_read_part
// (src/aln.cpp:1946-1962): randstrobes_query (src/randstrobes.cpp:207-253),
// find_nams (src/nam.cpp:771-926), find_nams_rescue (src/nam.cpp:955-1012).
// Output is the reference's exact pre-sort NAM vector (robin_hood iteration
// order emulated, ext/robin_hood.h v3.11.1).
//
//  k_randstrobes  one lane per read: canonical syncmers (stateful window-min
//                 with the reference's tie rules) and fwd/rc randstrobes.
//  k_lookup       one wavefront per read, one lane per query randstrobe:
//                 bucket bounds + binary search in the 16-B RefRandstrobe AoS,
//                 the filter probe, the occurrence count and the min_diff hit
//                 count.  These random 16-B reads are the HBM-bound part.
//  k_find_nams    one lane per read: hits into per-read robin_hood emulations,
//                 merge_hits_into_nams (sort=true) fwd then rc.
//  k_rescue       one lane per flagged read: find_nams_rescue (pre_sort
//                 branch) with merge_hits_into_nams_fast.
//  k_compact      gathers the final per-read NAM lists.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "rsa_dev.h"
#include "rsa_seed.h"
#include "rsa_timer.h"

#define END64 0xFFFFFFFFFFFFFFFFULL
#define WSYNC_SEED() do { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); } while (0)

struct QrsInfo {            // per query randstrobe, filled by k_lookup
    uint64_t pos;           // first index with equal hash, END64 if absent
    uint32_t count;         // occurrences of the hash
    uint32_t hits;          // entries passing the min_diff filter (count <= 1000), else 0
    uint32_t flags;         // bit0 found, bit1 filtered
    uint32_t pad;
};

struct ReadStat {
    uint32_t found, good, hits_find, hits_all;
    uint32_t scan_find, scan_all;   // index entries read by the min_diff pass (instrumentation)
    uint32_t qw;                    // the read's query randstrobes and QrsInfo are in qrs / qi
    uint32_t pad;
};

struct HitD {
    int32_t qs, qe, rs, re;
    int32_t list;           // map value (list id) ; orientation in bit 30
    int32_t pad;
};

// Device-side state of one rsa_seed call.  The host uploads it zeroed with the
// read offsets and downloads it with the results, once: every count that used to
// come back between the kernels (hits per read, big-map reads, rescued reads, the
// final NAM offsets) is a device counter, scan or list now.
#define SEED_E_POOL 1u      // the call's pool ran out: the host grows it and runs again
#define SEED_E_FIND 2u      // robin_hood emulation overflow in the global-map pass
#define SEED_E_RESCUE 4u    // the same in the rescue pass
#define SEED_E_SITE 8u      // k_sites met a NAM whose nam_id is outside its read's list (a broken permutation)
// RSA_SEED_PROF builds (never the product): per-phase shader cycles of the fused
// query kernel and k_find_nams_w2, summed over waves, printed by seed_run
#ifdef RSA_SEED_PROF
#define SPROF_READS 32768
__device__ unsigned int g_seed_prof[SPROF_READS][20];    // per read (r < SPROF_READS), plain stores
__device__ unsigned int g_sites_prof[4096 * 4][8];       // k_sites: per (block, wave), summed over its NAM rounds
#define SPROF_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define SPROF_ADD(i, d) do { if (lane == 0 && r < SPROF_READS) g_seed_prof[r][i] = (unsigned int)(d); } while (0)
#else
#define SPROF_T(v)
#define SPROF_ADD(i, d)
#endif
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// one 16-byte part of a bucket line (non-temporal loads measured no better: 146 / 157 µs
// against 143 / 146, profiles/r05/seed_ab_nt.txt)
__device__ __forceinline__ uint4 line_part(const BucketLine* L, int part) { return ((const uint4*)L)[part]; }
struct SeedHdr {
    unsigned long long pool_used;   // pool entries handed out
    unsigned long long total;       // final NAMs of the batch
    unsigned long long mm_used;     // mismatch positions of the site checks
    uint32_t big_count;             // reads listed for k_find_nams_big
    uint32_t rcount;                // reads listed for find_nams_rescue
    uint32_t rbig_count;            // rescued reads listed for k_rescue_big
    uint32_t errors;                // SEED_E_*
    // statistics (DESIGN.md "Kernels": algorithmic bytes and per-read counts)
    unsigned long long qrs, found, good, hits_find, hits_all, scan_find, scan_all, n1, n2, resc_reads, resc_q,
        resc_scan, resc_hits, qw_q;   // qw_q: query randstrobes written out (reads with ReadStat::qw)
    unsigned long long qfix;        // reads query_lane made the randstrobes of (k_seed_query's prediction missed)
};

// The call's pool: per entry one hit, one open NAM, one NAM, one group hit and
// one added flag (the global-map and rescue passes take one run of entries per
// read, as many as the read has hits).  The NAMs sit at arena_base + entry in
// the NAM arena, after the n x FN2_HCAP fixed slots of k_find_nams_w2.
struct SeedPool {
    HitD* hits;
    rsa_nam* open;
    rsa_nam* nams;
    HitD* grp;
    uint8_t* added;
    uint64_t n;             // entries
    uint64_t arena_base;    // index of nams[0] in the NAM arena
};

// ---------------------------------------------------------------------------
// k_randstrobes
// ---------------------------------------------------------------------------
struct SyncD { uint64_t hash; uint32_t pos; uint32_t pad; };
struct RescueD { uint64_t pos; uint32_t count, qs, qe, pad; };
// query_lane's syncmer scratch for read r inside the rescue buffer: RescueD room for
// 2 len entries at qbase[r] holds len SyncD (the rescue pass overwrites it afterwards)
struct RescueScratch {
    RescueD* rbuf;
    __device__ __forceinline__ SyncD* sync(uint64_t qb) const { return (SyncD*)(rbuf + qb); }
};

__device__ void rs_get(const SyncD* sm, int n, int i, const SeedIndexParams& p, uint64_t& h, uint32_t& a,
                       uint32_t& b) {
    const int w_end = i + p.w_max < n - 1 ? i + p.w_max : n - 1;
    const uint64_t max_position = (uint64_t)sm[i].pos + (unsigned)p.max_dist;
    uint64_t min_val = END64;
    int best = i;
    const uint64_t hi = sm[i].hash;
    for (int j = i + p.w_min; j <= w_end && sm[j].pos <= max_position; ++j) {
        const uint64_t res = (uint64_t)__popcll((hi ^ sm[j].hash) & p.q);
        if (res < min_val) { min_val = res; best = j; }
    }
    h = hi + sm[best].hash;
    a = sm[i].pos;
    b = sm[best].pos;
}

// Syncmer window of the last W s-mer hashes, oldest first.  WC > 0: W == WC
// held in registers as a shift register (all indices static); WC == 0: any W
// in a ring buffer (private memory).
template <int WC>
struct SmWindow {
    uint64_t q[WC > 0 ? WC : 32];
    int qn = 0, qhead = 0, W;
    __device__ explicit SmWindow(int w) : W(WC > 0 ? WC : w) {}
    __device__ __forceinline__ uint64_t at(int j) const {
        if constexpr (WC > 0) {
            uint64_t v = q[0];
#pragma unroll
            for (int x = 1; x < WC; ++x) if (j == x) v = q[x];
            return v;
        } else {
            return q[(qhead + j) & 31];
        }
    }
    // push h; returns true when the window was already full (front popped)
    __device__ __forceinline__ bool push(uint64_t h) {
        if constexpr (WC > 0) {
            if (qn < WC) {
#pragma unroll
                for (int x = 0; x < WC; ++x) if (x == qn) q[x] = h;
                qn++;
                return false;
            }
#pragma unroll
            for (int x = 0; x + 1 < WC; ++x) q[x] = q[x + 1];
            q[WC - 1] = h;
            return true;
        } else {
            q[(qhead + qn) & 31] = h;
            if (qn < W) { qn++; return false; }
            qhead = (qhead + 1) & 31;
            return true;
        }
    }
    __device__ __forceinline__ void reset() { qn = 0; qhead = 0; }
};

// SyncmerIterator::next (randstrobes.cpp:57-118) over the whole read; returns
// the number of syncmers written to sm.
template <int WC>
__device__ int syncmers_lane(const char* __restrict__ s, int len, const SeedIndexParams& p, SyncD* __restrict__ sm) {
    const int k = p.k, sl = p.s, t = p.t;
    const uint64_t kmask = (k == 32) ? ~0ULL : ((1ULL << (2 * k)) - 1);
    const uint64_t smask = (1ULL << (2 * sl)) - 1;
    const int kshift = (k - 1) * 2, sshift = (sl - 1) * 2;
    SmWindow<WC> win(k - sl + 1);
    const int W = win.W;
    uint64_t min_val = END64;
    long long min_pos = -1;
    int l = 0, n = 0;
    uint64_t xk0 = 0, xk1 = 0, xs0 = 0, xs1 = 0;
    for (int i = 0; i < len; ++i) {
        const int c = nt4_code((unsigned char)s[i]);
        if (c < 4) {
            xk0 = ((xk0 << 2) | (uint64_t)c) & kmask;
            xk1 = (xk1 >> 2) | ((uint64_t)(3 - c) << kshift);
            xs0 = ((xs0 << 2) | (uint64_t)c) & smask;
            xs1 = (xs1 >> 2) | ((uint64_t)(3 - c) << sshift);
            if (++l < sl) continue;
            const uint64_t hs = xxh64_u64(xs0 < xs1 ? xs0 : xs1);
            const bool popped = win.push(hs);
            if (!popped) {
                if (win.qn < W) continue;
                for (int j = 0; j < W; ++j) {          // first fill: leftmost minimum
                    const uint64_t v = win.at(j);
                    if (v < min_val) { min_val = v; min_pos = (long long)i - k + j + 1; }
                }
            } else if (min_pos == (long long)i - k) {   // the minimum left: rescan, rightmost wins
                min_val = END64;
                min_pos = (long long)i - sl + 1;
                for (int j = W - 1; j >= 0; --j) {
                    const uint64_t v = win.at(j);
                    if (v < min_val) { min_val = v; min_pos = (long long)i - k + j + 1; }
                }
            } else if (hs < min_val) {
                min_val = hs;
                min_pos = (long long)i - sl + 1;
            }
            if (min_pos == (long long)i - k + t) {
                sm[n].hash = xxh64_u64(xk0 < xk1 ? xk0 : xk1);
                sm[n].pos = (uint32_t)(i - k + 1);
                n++;
            }
        } else {
            min_val = END64; min_pos = -1;
            l = 0; xs0 = xs1 = xk0 = xk1 = 0;
            win.reset();
        }
    }
    return n;
}

// one lane per read: reads longer than RW_MAXLEN and seeding parameters the
// wave kernel below does not take (list: the reads, NULL = all of them)
template <int WC>
__global__ void __launch_bounds__(64)
k_randstrobes(const char* __restrict__ seq, const uint64_t* __restrict__ roff, const uint32_t* __restrict__ rlen,
              const uint64_t* __restrict__ qbase, int n_reads, const int* __restrict__ list, SeedIndexParams p,
              SyncD* __restrict__ sync, rsa_query_randstrobe* __restrict__ qrs, uint32_t* __restrict__ qcnt) {
    const int t = blockIdx.x * 64 + (threadIdx.x & 63);
    if (t >= n_reads) return;
    const int r = list ? list[t] : t;
    const int len = (int)rlen[r];
    const char* s = seq + roff[r];
    SyncD* sm = sync + qbase[r] / 2;
    rsa_query_randstrobe* out = qrs + qbase[r];
    if (len < p.w_max) { qcnt[r] = 0; return; }     // randstrobes.cpp:209
    const int k = p.k;
    const int n = syncmers_lane<WC>(s, len, p, sm);
    int cnt = 0;
    if (n > 0) {
        for (int i = 0; i + p.w_min < n; ++i) {
            uint64_t h; uint32_t a, b;
            rs_get(sm, n, i, p, h, a, b);
            out[cnt].hash = h; out[cnt].start = a; out[cnt].end = b + (uint32_t)k; out[cnt].is_reverse = 0;
            out[cnt].pad_ = 0;
            cnt++;
        }
        for (int i = 0, j = n - 1; i < j; ++i, --j) { const SyncD x = sm[i]; sm[i] = sm[j]; sm[j] = x; }
        for (int i = 0; i < n; ++i) sm[i].pos = (uint32_t)(len - (int)sm[i].pos - k);
        for (int i = 0; i + p.w_min < n; ++i) {
            uint64_t h; uint32_t a, b;
            rs_get(sm, n, i, p, h, a, b);
            out[cnt].hash = h; out[cnt].start = a; out[cnt].end = b + (uint32_t)k; out[cnt].is_reverse = 1;
            out[cnt].pad_ = 0;
            cnt++;
        }
    }
    qcnt[r] = (uint32_t)cnt;
}

// ---------------------------------------------------------------------------
// k_rs_wave: one wavefront per read (reads of up to RW_MAXLEN bases), every
// step lane-parallel and LDS-resident -- no global scratch:
//   1. the read is loaded coalesced (one base a lane) into two LDS bit arrays:
//      2-bit base codes (ds_or) and an N mask (wave ballot);
//   2. every s-mer ending at i: canonical value = min(fwd, rc) of the rolling
//      registers of SyncmerIterator::next (randstrobes.cpp:57-118), extracted
//      from the code array (rc = complemented codes, first base lowest; fwd = the
//      2-bit groups reversed), xxh64 -> LDS;
//   3. every k-mer ending at p without an N: the window of its k-s+1 s-mer
//      hashes.  The iterator's tracked minimum always holds the window's
//      minimum value, so when that value occurs once the syncmer test is
//      stateless (argmin at offset t-1).  Only equal minima depend on history
//      (first fill keeps the leftmost, a rescan the rightmost, an equal
//      newcomer does not replace): a read with such a tie anywhere runs the
//      reference's walk exactly, on lane 0, over the same LDS hashes.  Random
//      reads never tie (equal 64-bit hashes need a repeated s-mer within k-s+1
//      bases); low-complexity reads do.  Syncmer positions are compacted in
//      order with a ballot prefix;
//   4. lanes: canonical k-mer hash of every syncmer, then one randstrobe per
//      lane (RandstrobeIterator::get, 148-171), forward then reverse complement
//      (207-253), stored coalesced.
// ---------------------------------------------------------------------------
#define RW_WAVES 4
#define RW_MAXLEN 512
#define RW_WMAX 16            // window k - s + 1 the wave kernel takes

// base codes [a, a + n) (first base in the low bits), n <= 32
__device__ __forceinline__ uint64_t rw_bases(const uint32_t* w, int a, int n) {
    const int wi = a >> 4, off = 2 * (a & 15);
    uint64_t x = ((uint64_t)w[wi] | ((uint64_t)w[wi + 1] << 32)) >> off;
    if (off) x |= (uint64_t)w[wi + 2] << (64 - off);
    return n >= 32 ? x : (x & ((1ULL << (2 * n)) - 1));
}
// an N among bases [a, a + n), n <= 32
__device__ __forceinline__ bool rw_has_n(const uint32_t* nm, int a, int n) {
    const int wi = a >> 5, off = a & 31;
    const uint64_t x = ((uint64_t)nm[wi] | ((uint64_t)nm[wi + 1] << 32)) >> off;
    return (x & ((1ULL << n) - 1)) != 0;
}
// min(xk[0], xk[1]) of the n-mer whose codes X holds: xk[1] (complement, first
// base lowest) is X ^ mask; xk[0] (first base highest) is X with its 2-bit groups reversed
__device__ __forceinline__ uint64_t rw_canon(uint64_t X, int n) {
    const uint64_t mask = n >= 32 ? ~0ULL : ((1ULL << (2 * n)) - 1);
    const uint64_t rc = X ^ mask;
    uint64_t r = __builtin_bitreverse64(X);
    r = ((r >> 1) & 0x5555555555555555ULL) | ((r & 0x5555555555555555ULL) << 1);
    const uint64_t fwd = r >> (64 - 2 * n);
    return fwd < rc ? fwd : rc;
}

__device__ __forceinline__ void rs_pick(const uint64_t* __restrict__ sh, const uint16_t* __restrict__ sp, int n, int i,
                                        bool rc, int len, const SeedIndexParams& p, uint64_t& h, uint32_t& a,
                                        uint32_t& b) {
    // syncmer x of the (possibly reversed) list: index n-1-x, position len - pos - k when reversed
    auto pos = [&](int x) -> uint32_t { return rc ? (uint32_t)(len - (int)sp[n - 1 - x] - p.k) : sp[x]; };
    auto hsh = [&](int x) -> uint64_t { return rc ? sh[n - 1 - x] : sh[x]; };
    const int w_end = i + p.w_max < n - 1 ? i + p.w_max : n - 1;
    const uint32_t pi = pos(i);
    const uint64_t max_position = (uint64_t)pi + (unsigned)p.max_dist;
    uint64_t min_val = END64;
    int best = i;
    const uint64_t hi = hsh(i);
    for (int j = i + p.w_min; j <= w_end && pos(j) <= max_position; ++j) {
        const uint64_t res = (uint64_t)__popcll((hi ^ hsh(j)) & p.q);
        if (res < min_val) { min_val = res; best = j; }
    }
    h = hi + hsh(best);
    a = pi;
    b = pos(best);
}

// Steps 1-4a for one read on one wave (len <= RW_MAXLEN, len >= p.w_max): returns the
// syncmer count n, with their canonical k-mer hashes in hs[0, n) and positions in sp[0, n).
// s_nw is a wave-private LDS int (the tie walk's count).
__device__ __forceinline__ int rw_syncmers(const char* __restrict__ sq, int len, const SeedIndexParams& p, int lane,
                                           uint32_t* cw, uint32_t* nm, uint64_t* hs, uint16_t* sp, int* s_nw) {
    const int k = p.k, sl = p.s, W = k - sl + 1;
    // 1. codes and N mask
    for (int i = lane; i < RW_MAXLEN / 16 + 4; i += 64) cw[i] = 0;
    WSYNC_SEED();
    for (int base = 0; base < len; base += 64) {
        const int i = base + lane;
        const int c = i < len ? nt4_code((unsigned char)sq[i]) : 4;
        const uint64_t nb = __ballot(c >= 4);
        if (c < 4) atomicOr(&cw[i >> 4], (uint32_t)c << (2 * (i & 15)));
        if (lane == 0) { nm[base >> 5] = (uint32_t)nb; nm[(base >> 5) + 1] = (uint32_t)(nb >> 32); }
    }
    WSYNC_SEED();
    // 2. s-mer hashes (only s-mers without an N are ever read)
    for (int i = sl - 1 + lane; i < len; i += 64) {
        const int a = i - sl + 1;
        hs[i] = rw_has_n(nm, a, sl) ? 0 : xxh64_u64(rw_canon(rw_bases(cw, a, sl), sl));
    }
    WSYNC_SEED();
    // 3. syncmer test per k-mer end p
    int n = 0;
    bool tie = false;
    for (int base = 0; base < len; base += 64) {
        const int pe = base + lane;
        bool sync = false;
        if (pe >= k - 1 && pe < len && !rw_has_n(nm, pe - k + 1, k)) {
            const uint64_t* hw = hs + (pe - k + sl);      // window s-mers, by start offset 0..W-1
            uint64_t mv = hw[0];
            int mo = 0, cnt = 1;
            for (int o = 1; o < W; ++o) {
                const uint64_t v = hw[o];
                if (v < mv) { mv = v; mo = o; cnt = 1; }
                else if (v == mv) cnt++;
            }
            tie |= cnt > 1;
            sync = mo == p.t - 1;
        }
        const uint64_t b = __ballot(sync);
        if (sync) sp[n + __popcll(b & ((1ULL << lane) - 1))] = (uint16_t)(pe - k + 1);
        n += __popcll(b);
    }
    if (__ballot(tie)) {                                // wave-uniform
        WSYNC_SEED();
        if (lane == 0) {
            // SyncmerIterator::next exactly (randstrobes.cpp:57-118); the window of the
            // k-mer ending at i is hs[i-W+1 .. i], all valid once l >= k
            int l = 0, nn = 0;
            uint64_t min_val = END64;
            int min_pos = -1;
            for (int i = 0; i < len; ++i) {
                if ((nm[i >> 5] >> (i & 31)) & 1u) { l = 0; min_val = END64; min_pos = -1; continue; }
                if (++l < sl) continue;
                const int qn = l - sl + 1;
                if (qn < W) continue;
                const uint64_t* hw = hs + (i - W + 1);
                if (qn == W) {                            // first fill: leftmost minimum
                    for (int j = 0; j < W; ++j)
                        if (hw[j] < min_val) { min_val = hw[j]; min_pos = i - k + j + 1; }
                } else if (min_pos == i - k) {            // the minimum left: rescan, rightmost wins
                    min_val = END64;
                    min_pos = i - sl + 1;
                    for (int j = W - 1; j >= 0; --j)
                        if (hw[j] < min_val) { min_val = hw[j]; min_pos = i - k + j + 1; }
                } else if (hw[W - 1] < min_val) {
                    min_val = hw[W - 1];
                    min_pos = i - sl + 1;
                }
                if (min_pos == i - k + p.t) sp[nn++] = (uint16_t)(i - k + 1);
            }
            *s_nw = nn;
        }
        WSYNC_SEED();
        n = *s_nw;
    }
    WSYNC_SEED();                                       // every read of the s-mer hashes is done
    // 4a. syncmer k-mer hashes (into the s-mer hash array)
    for (int x = lane; x < n; x += 64) hs[x] = xxh64_u64(rw_canon(rw_bases(cw, (int)sp[x], k), k));
    WSYNC_SEED();
    return n;
}

// the wave kernel's LDS, per wave
#define RW_LDS_DECL                                                                          \
    __shared__ uint32_t s_code[RW_WAVES][RW_MAXLEN / 16 + 4];                                \
    __shared__ uint32_t s_nm[RW_WAVES][RW_MAXLEN / 32 + 4];                                  \
    __shared__ uint64_t s_h[RW_WAVES][RW_MAXLEN];   /* s-mer hash by end, then k-mer hashes */ \
    __shared__ uint16_t s_sp[RW_WAVES][RW_MAXLEN];  /* syncmer positions (< RW_MAXLEN) */    \
    __shared__ int s_n[RW_WAVES]

// rsa_randstrobes (the randstrobe API): every query randstrobe written out
__global__ void __launch_bounds__(64 * RW_WAVES)
k_rs_wave(const char* __restrict__ seq, const uint64_t* __restrict__ roff, const uint32_t* __restrict__ rlen,
          const uint64_t* __restrict__ qbase, int n_reads, SeedIndexParams p, rsa_query_randstrobe* __restrict__ qrs,
          uint32_t* __restrict__ qcnt) {
    RW_LDS_DECL;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = blockIdx.x * RW_WAVES + w;
    if (r >= n_reads) return;                           // the whole wave leaves together
    const int len = (int)rlen[r];
    if (len > RW_MAXLEN) return;                        // k_randstrobes takes it
    if (len < p.w_max) { if (lane == 0) qcnt[r] = 0; return; }   // randstrobes.cpp:209
    uint64_t* hs = s_h[w];
    uint16_t* sp = s_sp[w];
    const int n = rw_syncmers(seq + roff[r], len, p, lane, s_code[w], s_nm[w], hs, sp, &s_n[w]);
    // 4b. randstrobes, forward then reverse complement
    const int m = n > p.w_min ? n - p.w_min : 0;
    rsa_query_randstrobe* out = qrs + qbase[r];
    for (int x = lane; x < 2 * m; x += 64) {
        const bool rcx = x >= m;
        uint64_t h; uint32_t a, b;
        rs_pick(hs, sp, n, rcx ? x - m : x, rcx, len, p, h, a, b);
        rsa_query_randstrobe o;
        o.hash = h; o.start = a; o.end = b + (uint32_t)p.k; o.is_reverse = rcx ? 1 : 0; o.pad_ = 0;
        out[x] = o;
    }
    if (lane == 0) qcnt[r] = (uint32_t)(2 * m);
}

// ---------------------------------------------------------------------------
// k_lookup: one wavefront per read
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t lower_bound_hash(const rsa_ref_randstrobe* rs, uint64_t lo, uint64_t hi,
                                                     uint64_t key) {
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (rs[mid].hash < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint64_t upper_bound_hash(const rsa_ref_randstrobe* rs, uint64_t lo, uint64_t hi,
                                                     uint64_t key) {
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (rs[mid].hash <= key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// hits (add_to_hits_per_ref order) of reads with at most LK_HCAP of them are
// also written to a fixed per-read slot, so k_find_nams_w2 starts from them
// instead of re-reading the index
#define LK_HCAP 128

__device__ __forceinline__ int wave_excl_scan_lk(int v, int lane, int& total) {
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    total = __shfl(x, 63, 64);
    return x - v;
}

__device__ __forceinline__ QrsInfo lookup_hit(const rsa_query_randstrobe& q, const SeedIndexParams& p, bool hit,
                                              uint64_t a, uint64_t lo, uint64_t ub, const rsa_ref_randstrobe* eb,
                                              bool one = false);

// One query randstrobe against the index (index.hpp:57-93, nam.cpp:68-85): its
// QrsInfo, and the run of equal hashes as eb[lo, ub)
__device__ __forceinline__ QrsInfo lookup_one(const rsa_query_randstrobe& q, const SeedIndexParams& p, uint64_t& lo,
                                              uint64_t& ub, const rsa_ref_randstrobe*& eb) {
    QrsInfo o;
    o.pos = END64; o.count = 0; o.hits = 0; o.flags = 0; o.pad = 0;
    // the bucket's entries are eb[0, b - a) (in its line or in p.rs); lo/ub index eb
    lo = 0; ub = 0;
    eb = p.rs;
    const uint64_t top = q.hash >> (64 - p.bits);
    uint64_t a, b;
    bool hit = false;
    if (p.lines) {
        // the whole line in one go (eight independent 16-byte loads, one
        // miss): bounds and up to BL_CAP entries, searched in registers
        const BucketLine* L = p.lines + top;
        const uint4* lv = (const uint4*)L;
        uint4 w[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) w[t] = lv[t];
        a = (uint64_t)w[0].x | (uint64_t)w[0].y << 32;
        b = (uint64_t)w[0].z | (uint64_t)w[0].w << 32;
        if (b - a <= BL_CAP) {
            eb = L->e;
            const uint64_t c = b - a;
            lo = c; ub = c;            // first entry >= / > the key (entries sorted)
#pragma unroll
            for (int t = BL_CAP - 1; t >= 0; --t) {
                const uint64_t h = (uint64_t)w[1 + t].x | (uint64_t)w[1 + t].y << 32;
                if ((uint64_t)t < c) {
                    if (h >= q.hash) lo = t;
                    if (h > q.hash) ub = t;
                }
            }
            hit = ub > lo;
        } else {
            eb = p.rs + a;
            lo = lower_bound_hash(eb, 0, b - a, q.hash);
            hit = lo < b - a && eb[lo].hash == q.hash;
            if (hit) ub = upper_bound_hash(eb, lo, b - a, q.hash);
        }
    } else {
        a = p.starts[top]; b = p.starts[top + 1];
        eb = p.rs + a;
        if (a != b) {
            lo = lower_bound_hash(eb, 0, b - a, q.hash);
            hit = lo < b - a && eb[lo].hash == q.hash;
            if (hit) ub = upper_bound_hash(eb, lo, b - a, q.hash);
        }
    }
    return lookup_hit(q, p, hit, a, lo, ub, eb);
}

// The QrsInfo of a query randstrobe whose run of equal hashes is eb[lo, ub) (hit)
// in the bucket starting at index entry a
// (one: the run is a single entry, whose span the caller holds: one hit)
__device__ __forceinline__ QrsInfo lookup_hit(const rsa_query_randstrobe& q, const SeedIndexParams& p, bool hit,
                                              uint64_t a, uint64_t lo, uint64_t ub, const rsa_ref_randstrobe* eb,
                                              bool one) {
    QrsInfo o;
    o.pos = END64; o.count = 0; o.hits = 0; o.flags = 0; o.pad = 0;
    if (hit) {
        o.pos = a + lo;
        o.flags = 1;
        // is_filtered (index.hpp:91-93) probes rs[lo + filter_cutoff].hash == hash;
        // equal hashes are contiguous from lo to ub (one bucket), so that is
        // ub - lo > filter_cutoff, and the probe's random line is not fetched
        if (ub - lo > (uint64_t)p.filter_cutoff) o.flags |= 2;
        o.count = (uint32_t)min<uint64_t>(ub - lo, 0xFFFFFFFFull);
        if (one) {
            o.hits = 1;                                 // the first entry always passes the min_diff filter
        } else if (o.count <= 1000) {
            // add_to_hits_per_ref min_diff filter (nam.cpp:68-85)
            int min_diff = INT_MAX;
            uint32_t h = 0;
            const int qspan = (int)q.end - (int)q.start;
            for (uint64_t e = lo; e < ub; ++e) {
                const rsa_ref_randstrobe x = eb[e];
                const int rspan = (int)(x.packed & 0xFF) + p.k;
                int d = qspan - rspan;
                d = d < 0 ? -d : d;
                if (d <= min_diff) { h++; min_diff = d; }
            }
            o.hits = h;
        }
    }
    return o;
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return (uint64_t)hi << 32 | lo;
}

// lookup_one for a whole wave over the BucketLine table (p.lines set; called by
// every lane, `valid` marks the lanes with a query randstrobe).  The lines are
// fetched cooperatively: in instruction j the 8 lanes of group g = lane / 8 load
// the 16-byte parts of the line of lane 8j + g, so each load instruction touches
// 8 lines, whole, instead of 64 (a lane walking its own line issues 8 loads to
// it: 8x the address translations and requests).  Lines and keys go to the
// groups through the wave's LDS (s_top, s_key: 64 entries), each group compares
// its line's entries with the owner's key (two ballots), and the bounds come
// back to the owners through s_ab; buckets over BL_CAP are searched in p.rs by
// the owner as before.
__device__ __forceinline__ QrsInfo lookup_coop(const rsa_query_randstrobe& q, bool valid, const SeedIndexParams& p,
                                               int lane, uint64_t& lo, uint64_t& ub, const rsa_ref_randstrobe*& eb,
                                               uint64_t* s_top, uint64_t* s_key, uint4* s_ab, uint2* s_ent,
                                               bool& one, uint2& ent, unsigned long long* prof) {
    // a lane without a randstrobe fetches line 0 (its results are dropped): the
    // loads stay unconditional, so all eight are in flight at once
    const uint64_t top = valid ? q.hash >> (64 - p.bits) : 0;
    const int g = lane >> 3, part = lane & 7;
#ifdef RSA_SEED_PROF
    const unsigned long long cs = __builtin_amdgcn_s_memtime();
#endif
    s_top[lane] = top;
    s_key[lane] = q.hash;
    WSYNC_SEED();
    uint4 w[8];
#ifdef RSA_SEED_PROF
    uint64_t tj[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) tj[j] = s_top[8 * j + g];
    __builtin_amdgcn_s_waitcnt(0xC07F & ~0x0F00);           // lgkmcnt(0): the line indices are in
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long ca = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = line_part(p.lines + tj[j], part);
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long cm = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 4; j < 8; ++j) w[j] = line_part(p.lines + tj[j], part);
    __builtin_amdgcn_sched_barrier(0);
    prof[4] += ca - cs; prof[5] += cm - ca;
#else
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = line_part(p.lines + s_top[8 * j + g], part);
#endif
#ifdef RSA_SEED_PROF
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    prof[6] += c0 - cm;
    __builtin_amdgcn_s_waitcnt(0x0F70);                   // vmcnt(0): the lines are in
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    prof[0] += c1 - c0;
#endif
    uint32_t own_lt = 0, own_le = 0;                      // the owner's group: entries < / <= its key
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint64_t kj = s_key[8 * j + g];
        const uint64_t x0 = (uint64_t)w[j].x | (uint64_t)w[j].y << 32;    // part 0: start; else: entry hash
        const uint64_t mlt = __ballot(part >= 1 && x0 < kj), mle = __ballot(part >= 1 && x0 <= kj);
        if (part == 0) s_ab[8 * j + g] = w[j];            // the bounds of line 8j + g
        if (part >= 1 && x0 == kj) s_ent[8 * j + g] = make_uint2(w[j].z, w[j].w);   // an equal entry's position, packed
        if ((lane >> 3) == j) {
            own_lt = (uint32_t)(mlt >> (8 * (lane & 7))) & 0xFFu;
            own_le = (uint32_t)(mle >> (8 * (lane & 7))) & 0xFFu;
        }
    }
    WSYNC_SEED();
    const uint4 ab = s_ab[lane];
    ent = s_ent[lane];
    one = false;
    const uint64_t a = (uint64_t)ab.x | (uint64_t)ab.y << 32, b = (uint64_t)ab.z | (uint64_t)ab.w << 32;
#ifdef RSA_SEED_PROF
    const unsigned long long c2 = __builtin_amdgcn_s_memtime();
    prof[1] += c2 - c1;
#endif
    bool hit = false;
    lo = 0; ub = 0;
    eb = p.rs;
    if (valid) {
        if (b - a <= BL_CAP) {
            eb = p.lines[top].e;
            const uint32_t in = ((1u << (uint32_t)(b - a)) - 1u) << 1;   // parts 1 .. c hold the entries
            lo = (uint32_t)__popc(own_lt & in); ub = (uint32_t)__popc(own_le & in);
            hit = ub > lo;
            // a run of one entry, and the only equal part of the line (so s_ent holds it)
            one = ub == lo + 1 && __popc(own_le ^ own_lt) == 1;
        } else {
            eb = p.rs + a;
            lo = lower_bound_hash(eb, 0, b - a, q.hash);
            hit = lo < b - a && eb[lo].hash == q.hash;
            if (hit) ub = upper_bound_hash(eb, lo, b - a, q.hash);
        }
    }
#ifdef RSA_SEED_PROF
    const unsigned long long c3 = __builtin_amdgcn_s_memtime();
    prof[2] += c3 - c2;
    const QrsInfo o = lookup_hit(q, p, hit, a, lo, ub, eb, one);
    const unsigned long long c4 = __builtin_amdgcn_s_memtime();
    prof[3] += c4 - c3;
    return o;
#else
    return lookup_hit(q, p, hit, a, lo, ub, eb, one);
#endif
}

// a read's lookup statistics (ReadStat fields)
struct LkStat {
    uint32_t found = 0, good = 0, hfind = 0, hall = 0, sfind = 0, sall = 0;
    __device__ __forceinline__ void add(const QrsInfo& o) {
        if (!(o.flags & 1)) return;
        found++;
        const uint32_t scanned = o.count <= 1000 ? o.count : 0;
        if (!(o.flags & 2)) { good++; hfind += o.hits; sfind += scanned; }
        if (o.count <= 1000) hall += o.hits;
        sall += scanned;
    }
    __device__ __forceinline__ void wave_sum() {
        for (int off = 32; off > 0; off >>= 1) {
            found += __shfl_xor(found, off, 64);
            good += __shfl_xor(good, off, 64);
            hfind += __shfl_xor(hfind, off, 64);
            hall += __shfl_xor(hall, off, 64);
            sfind += __shfl_xor(sfind, off, 64);
            sall += __shfl_xor(sall, off, 64);
        }
    }
    __device__ __forceinline__ ReadStat to_stat(uint32_t qw) const {
        ReadStat s;
        s.found = found; s.good = good; s.hits_find = hfind; s.hits_all = hall; s.scan_find = sfind; s.scan_all = sall;
        s.qw = qw; s.pad = 0;
        return s;
    }
};

// the hits of one non-filtered randstrobe (add_to_hits_per_ref order) into slot[at, ...)
// (one: the run is the single entry {position, packed} = ent)
__device__ __forceinline__ void lk_emit(const rsa_query_randstrobe& q, uint64_t lo, uint64_t ub,
                                        const rsa_ref_randstrobe* eb, const SeedIndexParams& p, HitD* slot, int at,
                                        bool one = false, uint2 ent = make_uint2(0u, 0u)) {
    const int qs = (int)q.start, qe = (int)q.end;
    if (one) {
        HitD hd;
        hd.qs = qs; hd.qe = qe; hd.rs = (int)ent.x; hd.re = (int)ent.x + (int)(ent.y & 0xFF) + p.k;
        hd.list = (int32_t)(ent.y >> 8);
        hd.pad = q.is_reverse ? 1 : 0;
        slot[at] = hd;
        return;
    }
    int min_diff = INT_MAX, h = at;
    for (uint64_t e = lo; e < ub; ++e) {
        const rsa_ref_randstrobe x = eb[e];
        const int rs0 = (int)x.position;
        const int re0 = rs0 + (int)(x.packed & 0xFF) + p.k;
        int d = (qe - qs) - (re0 - rs0);
        d = d < 0 ? -d : d;
        if (d <= min_diff) {
            HitD hd;
            hd.qs = qs; hd.qe = qe; hd.rs = rs0; hd.re = re0;
            hd.list = (int32_t)(x.packed >> 8);
            hd.pad = q.is_reverse ? 1 : 0;
            slot[h++] = hd;
            min_diff = d;
        }
    }
}

// k_lookup: the reads k_randstrobes took (list; NULL = every read), one wave a read
__global__ void __launch_bounds__(256)
k_lookup(const rsa_query_randstrobe* __restrict__ qrs, const uint32_t* __restrict__ qcnt,
         const uint64_t* __restrict__ qbase, int n_list, const int* __restrict__ list, SeedIndexParams p,
         QrsInfo* __restrict__ qi, ReadStat* __restrict__ st, HitD* __restrict__ hit_slots) {
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (wave >= n_list) return;
    const int r = list ? list[wave] : wave;
    const int nq = (int)qcnt[r];
    const uint64_t base = qbase[r];
    HitD* slot = hit_slots + (size_t)r * LK_HCAP;
    LkStat ls;
    int hoff = 0;                                      // hits of the read written so far
    for (int i0 = 0; i0 < nq; i0 += 64) {
        const int i = i0 + lane;
        QrsInfo o;
        o.flags = 0; o.hits = 0;
        rsa_query_randstrobe q;
        uint64_t lo = 0, ub = 0;
        const rsa_ref_randstrobe* eb = p.rs;
        if (i < nq) {
            q = qrs[base + i];
            o = lookup_one(q, p, lo, ub, eb);
            ls.add(o);
            qi[base + i] = o;
        }
        // the non-filtered randstrobes' hits, in randstrobe order, into the read's slot
        const bool emit = (o.flags & 1) && !(o.flags & 2) && o.hits > 0;
        int tot;
        const int at = hoff + wave_excl_scan_lk(emit ? (int)o.hits : 0, lane, tot);
        if (emit && at + (int)o.hits <= LK_HCAP) lk_emit(q, lo, ub, eb, p, slot, at);
        hoff += tot;
    }
    ls.wave_sum();
    if (lane == 0) st[r] = ls.to_stat(1);
}

// Reads the fused kernel predicts to need their query randstrobes and QrsInfo
// written out: the global-map pass (k_find_nams_w2 lists reads with more than
// FN2_HCAP hits, or whose LDS maps would rehash at ~102 lists an orientation)
// and find_nams_rescue (the rescue decision of k_rescue_select: no NAMs, which
// is no hits, since every hit opens or extends a NAM, or nonrepetitive fraction
// < 0.7).  A read the prediction misses is recomputed by query_lane.
#define SQ_BIG_HITS 96

// RSA_SEED_QW (qw_mode) overrides the prediction in the tests: 0 = never, 2 = always.
// k_seed_query: k_rs_wave + k_lookup fused, one wave a read (len <= RW_MAXLEN).
// Randstrobe x of the read is made on lane x % 64 (rs_pick from the LDS syncmers)
// and looked up straight from registers; only its hits leave the kernel (the
// read's fixed slot), and the per-read statistics.  The randstrobes and their
// QrsInfo are written only for the reads predicted above (a second, rare pass
// that repeats the picks and lookups: their lines are in L2 by then).
__global__ void __launch_bounds__(64 * RW_WAVES)
k_seed_query(const char* __restrict__ seq, const uint64_t* __restrict__ roff, const uint32_t* __restrict__ rlen,
             const uint64_t* __restrict__ qbase, int n_reads, SeedIndexParams p, int32_t rescue_level, int qw_mode,
             rsa_query_randstrobe* __restrict__ qrs, uint32_t* __restrict__ qcnt, QrsInfo* __restrict__ qi,
             ReadStat* __restrict__ st, HitD* __restrict__ hit_slots) {
    RW_LDS_DECL;
    __shared__ uint64_t s_top[RW_WAVES][64], s_key[RW_WAVES][64];   // lookup_coop's exchange
    __shared__ uint4 s_ab[RW_WAVES][64];
    __shared__ uint2 s_ent[RW_WAVES][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = blockIdx.x * RW_WAVES + w;
    if (r >= n_reads) return;                           // the whole wave leaves together
    const int len = (int)rlen[r];
    if (len > RW_MAXLEN) return;                        // k_randstrobes + k_lookup take it
    if (len < p.w_max) {                                // randstrobes.cpp:209: no randstrobes
        if (lane == 0) { qcnt[r] = 0; st[r] = LkStat().to_stat(1); }
        return;
    }
    uint64_t* hs = s_h[w];
    uint16_t* sp = s_sp[w];
    SPROF_T(q0);
    const int n = rw_syncmers(seq + roff[r], len, p, lane, s_code[w], s_nm[w], hs, sp, &s_n[w]);
    SPROF_T(q1);
    const int m = n > p.w_min ? n - p.w_min : 0;
    const int nq = 2 * m;
    HitD* slot = hit_slots + (size_t)r * LK_HCAP;
    LkStat ls;
    int hoff = 0;
    unsigned long long acc_wait[7] = {0, 0, 0, 0, 0, 0, 0};   // RSA_SEED_PROF: lookup_coop's phases
#ifdef RSA_SEED_PROF
    unsigned long long acc_pick = 0, acc_coop = 0, acc_emit = 0;
#endif
    for (int i0 = 0; i0 < nq; i0 += 64) {
        SPROF_T(l0);
        const int x = i0 + lane;
        QrsInfo o;
        o.flags = 0; o.hits = 0;
        rsa_query_randstrobe q;
        uint64_t lo = 0, ub = 0;
        bool one = false;                               // lookup_coop: a single-entry run, held in ent
        uint2 ent = make_uint2(0u, 0u);
        const rsa_ref_randstrobe* eb = p.rs;
        q.hash = 0; q.start = 0; q.end = 0; q.is_reverse = 0; q.pad_ = 0;
        if (x < nq) {
            const bool rcx = x >= m;
            uint64_t h; uint32_t a, b;
            rs_pick(hs, sp, n, rcx ? x - m : x, rcx, len, p, h, a, b);
            q.hash = h; q.start = a; q.end = b + (uint32_t)p.k; q.is_reverse = rcx ? 1 : 0; q.pad_ = 0;
        }
        SPROF_T(l1);
        if (p.lines) {                                  // kernel-uniform: the whole wave
            const QrsInfo oc = lookup_coop(q, x < nq, p, lane, lo, ub, eb, s_top[w], s_key[w], s_ab[w], s_ent[w], one,
                                           ent, acc_wait);
            if (x < nq) o = oc;
        } else if (x < nq) {
            o = lookup_one(q, p, lo, ub, eb);
        }
        if (x < nq) ls.add(o);
        SPROF_T(l2);
        const bool emit = (o.flags & 1) && !(o.flags & 2) && o.hits > 0;
        int tot;
        const int at = hoff + wave_excl_scan_lk(emit ? (int)o.hits : 0, lane, tot);
        if (emit && at + (int)o.hits <= LK_HCAP) lk_emit(q, lo, ub, eb, p, slot, at, one, ent);
        hoff += tot;
#ifdef RSA_SEED_PROF
        SPROF_T(l3);
        acc_pick += l1 - l0; acc_coop += l2 - l1; acc_emit += l3 - l2;
#endif
    }
    SPROF_ADD(11, acc_pick); SPROF_ADD(12, acc_coop); SPROF_ADD(13, acc_emit); SPROF_ADD(14, acc_wait[0]); SPROF_ADD(15, acc_wait[1]); SPROF_ADD(16, acc_wait[2]); SPROF_ADD(17, acc_wait[3]); SPROF_ADD(18, acc_wait[4]); SPROF_ADD(19, acc_wait[5] + acc_wait[6]);
    SPROF_T(q2);
    ls.wave_sum();                                      // every lane holds the read's totals
    const float nonrep = ls.found > 0 ? (float)ls.good / (float)ls.found : 1.0f;   // nam.cpp:920
    const bool need = qw_mode == 2 ||
                      (qw_mode == 1 && (ls.hfind > SQ_BIG_HITS || (rescue_level > 1 && (ls.hfind == 0 || nonrep < 0.7f))));
    if (need) {                                         // wave-uniform
        const uint64_t base = qbase[r];
        for (int x = lane; x < nq; x += 64) {
            const bool rcx = x >= m;
            uint64_t h; uint32_t a, b;
            rs_pick(hs, sp, n, rcx ? x - m : x, rcx, len, p, h, a, b);
            rsa_query_randstrobe q;
            q.hash = h; q.start = a; q.end = b + (uint32_t)p.k; q.is_reverse = rcx ? 1 : 0; q.pad_ = 0;
            uint64_t lo, ub;
            const rsa_ref_randstrobe* eb;
            qrs[base + x] = q;
            qi[base + x] = lookup_one(q, p, lo, ub, eb);
        }
    }
    if (lane == 0) { qcnt[r] = (uint32_t)nq; st[r] = ls.to_stat(need ? 1u : 0u); }
    SPROF_T(q3);
    SPROF_ADD(0, q1 - q0); SPROF_ADD(1, q2 - q1); SPROF_ADD(2, q3 - q2); SPROF_ADD(3, 1);
}

// The query randstrobes and QrsInfo of read r on one lane, for a read the fused
// kernel did not write them for (a global-map or rescue read it did not predict):
// k_randstrobes' lane walk and lookup_one.  `sync` is scratch for the read's
// syncmers (len entries).  Marks the read written.
__device__ __noinline__ void query_lane(int r, const char* __restrict__ seq, const uint64_t* __restrict__ roff,
                                        const uint32_t* __restrict__ rlen, const uint64_t* __restrict__ qbase,
                                        const SeedIndexParams& p, SyncD* __restrict__ sm,
                                        rsa_query_randstrobe* __restrict__ qrs, QrsInfo* __restrict__ qi,
                                        ReadStat* __restrict__ st, SeedHdr* __restrict__ hdr) {
    const int len = (int)rlen[r];
    const uint64_t base = qbase[r];
    const int k = p.k;
    int cnt = 0;
    if (len >= p.w_max) {
        const int n = syncmers_lane<0>(seq + roff[r], len, p, sm);
        for (int o = 0; o < 2 && n > 0; ++o) {
            if (o == 1) {                                // the reverse complement's syncmers
                for (int i = 0, j = n - 1; i < j; ++i, --j) { const SyncD x = sm[i]; sm[i] = sm[j]; sm[j] = x; }
                for (int i = 0; i < n; ++i) sm[i].pos = (uint32_t)(len - (int)sm[i].pos - k);
            }
            for (int i = 0; i + p.w_min < n; ++i) {
                uint64_t h; uint32_t a, b;
                rs_get(sm, n, i, p, h, a, b);
                rsa_query_randstrobe q;
                q.hash = h; q.start = a; q.end = b + (uint32_t)k; q.is_reverse = (uint32_t)o; q.pad_ = 0;
                uint64_t lo, ub;
                const rsa_ref_randstrobe* eb;
                qrs[base + cnt] = q;
                qi[base + cnt] = lookup_one(q, p, lo, ub, eb);
                cnt++;
            }
        }
    }
    st[r].qw = 1;
    atomicAdd(&hdr->qfix, 1ull);
}

// ---------------------------------------------------------------------------
// robin_hood::unordered_flat_map<unsigned, ...> slot-layout emulation
// (robin_hood.h v3.11.1; same algorithm as oracle/rsa_oracle.c rh_*)
// ---------------------------------------------------------------------------
// AS = address space of the tables: 0 (generic: global scratch) or 3 (LDS,
// so every probe is a ds_read instead of a flat access)
template <int AS> struct AsTypes {
    typedef __attribute__((address_space(AS))) uint8_t U8;
    typedef __attribute__((address_space(AS))) uint32_t U32;
    typedef __attribute__((address_space(AS))) int32_t I32;
};
template <> struct AsTypes<0> { typedef uint8_t U8; typedef uint32_t U32; typedef int32_t I32; };

template <int AS>
struct DMapT {
    typedef typename AsTypes<AS>::U8 U8;
    typedef typename AsTypes<AS>::U32 U32;
    typedef typename AsTypes<AS>::I32 I32;
    U8* info; U32* keys; I32* vals;
    U8* info2; U32* keys2; I32* vals2;
    uint32_t cap;                          // slots per table
    uint64_t mult;
    uint32_t mask, num, max_allowed, nwb, info_inc, info_shift;
    int overflow;
};
using DMap = DMapT<0>;
using LMap = DMapT<3>;

__device__ __forceinline__ uint32_t rh_calc_max(uint32_t n) { return (uint32_t)((uint64_t)n * 80 / 100); }
__device__ __forceinline__ uint32_t rh_calc_nwb(uint32_t n) { uint32_t m = rh_calc_max(n); return n + (m < 255 ? m : 255); }

template <class M>
__device__ bool rh_init_data(M& m, uint32_t max_elements) {
    const uint32_t nwb = rh_calc_nwb(max_elements);
    const uint32_t span = (nwb + 16 + 3) & ~3u;      // info bytes zeroed as words
    if (span > m.cap) { m.overflow = 1; return false; }
    m.num = 0;
    m.mask = max_elements - 1;
    m.max_allowed = rh_calc_max(max_elements);
    m.nwb = nwb;
    for (uint32_t i = 0; i < span; i += 4) *(typename M::U32*)(m.info + i) = 0;
    m.info[nwb] = 1;
    m.info_inc = 32;
    m.info_shift = 0;
    return true;
}

template <class M>
__device__ __forceinline__ void rh_key_to_idx(const M& m, uint32_t key, uint32_t& idx, uint32_t& info) {
    uint64_t h = (uint64_t)key;
    h ^= h >> 33; h *= 0xff51afd7ed558ccdULL; h ^= h >> 33;
    h *= m.mult;
    h ^= h >> 33;
    info = m.info_inc + (uint32_t)((h & 31u) >> m.info_shift);
    idx = (uint32_t)(h >> 5) & m.mask;
}

template <class M>
__device__ void rh_shift_up(M& m, uint32_t start, uint32_t ins) {
    for (uint32_t i = start; i != ins; --i) { m.keys[i] = m.keys[i - 1]; m.vals[i] = m.vals[i - 1]; }
    for (uint32_t i = start; i != ins; --i) {
        m.info[i] = (uint8_t)(m.info[i - 1] + m.info_inc);
        if ((uint32_t)m.info[i] + m.info_inc > 0xFF) m.max_allowed = 0;
    }
}

template <class M>
__device__ bool rh_try_increase_info(M& m) {
    if (m.info_inc <= 2) return false;
    m.info_inc >>= 1;
    m.info_shift++;
    const uint32_t nwb = rh_calc_nwb(m.mask + 1);
    for (uint32_t i = 0; i < nwb; i += 8)
        for (uint32_t b = 0; b < 8; ++b) m.info[i + b] = (uint8_t)(m.info[i + b] >> 1);
    m.info[nwb] = 1;
    m.max_allowed = rh_calc_max(m.mask + 1);
    return true;
}

template <class M>
__device__ void rh_insert_move(M& m, uint32_t key, int32_t val) {
    if (m.max_allowed == 0 && !rh_try_increase_info(m)) { m.overflow = 2; return; }
    uint32_t idx, info;
    rh_key_to_idx(m, key, idx, info);
    while (info <= m.info[idx]) { idx++; info += m.info_inc; }
    const uint32_t ins = idx;
    const uint8_t ins_info = (uint8_t)info;
    if ((uint32_t)ins_info + m.info_inc > 0xFF) m.max_allowed = 0;
    while (m.info[idx] != 0) { idx++; info += m.info_inc; }
    if (idx != ins) rh_shift_up(m, idx, ins);
    m.keys[ins] = key; m.vals[ins] = val;
    m.info[ins] = ins_info;
    m.num++;
}

template <class M>
__device__ void rh_rehash(M& m, uint32_t nb) {
    if (!m.info2) { m.overflow = 1; m.max_allowed = 0xFFFFFFFFu; return; }   // (both fields stored: keeps the map in registers)
    typename M::U8* oi = m.info;
    typename M::U32* ok = m.keys;
    typename M::I32* ov = m.vals;
    const uint32_t onwb = rh_calc_nwb(m.mask + 1);
    m.info = m.info2; m.keys = m.keys2; m.vals = m.vals2;
    m.info2 = oi; m.keys2 = ok; m.vals2 = ov;
    if (!rh_init_data(m, nb)) return;
    if (onwb > 1)
        for (uint32_t i = 0; i < onwb; ++i)
            if (oi[i] != 0) rh_insert_move(m, ok[i], ov[i]);
}

template <class M>
__device__ void rh_increase_size(M& m) {
    const uint32_t maxa = rh_calc_max(m.mask + 1);
    if (m.num < maxa && rh_try_increase_info(m)) return;
    m.mult += 0xc4ceb9fe1a85ec54ULL;
    if (m.num * 2 < rh_calc_max(m.mask + 1)) rh_rehash(m, m.mask + 1);
    else rh_rehash(m, (m.mask + 1) * 2);
}

// default construction + reserve(100) (nam.cpp:913-914)
template <class M>
__device__ void rh_new_reserved(M& m) {
    m.mult = 0xc4ceb9fe1a85ec53ULL;
    m.overflow = 0;
    rh_init_data(m, 128);
}

// operator[]: returns the value of key, inserting new_val if absent
template <class M>
__device__ int32_t rh_get_or_insert(M& m, uint32_t key, int32_t new_val, bool& inserted) {
    inserted = false;
    for (int attempt = 0; attempt < 256 && !m.overflow; ++attempt) {
        uint32_t idx, info;
        rh_key_to_idx(m, key, idx, info);
        while (info < m.info[idx]) { idx++; info += m.info_inc; }
        while (info == m.info[idx]) {
            if (m.keys[idx] == key) return m.vals[idx];
            idx++; info += m.info_inc;
        }
        if (m.num >= m.max_allowed) { rh_increase_size(m); continue; }
        const uint32_t ins = idx, ins_info = info;
        if (ins_info + m.info_inc > 0xFF) m.max_allowed = 0;
        while (m.info[idx] != 0) { idx++; info += m.info_inc; }
        if (idx != ins) rh_shift_up(m, idx, ins);
        m.info[ins] = (uint8_t)ins_info;
        m.keys[ins] = key; m.vals[ins] = new_val;
        m.num++;
        inserted = true;
        return new_val;
    }
    m.overflow = 3;
    return -1;
}

// per-read map scratch: 2 maps x 2 tables x cap slots x (1 + 4 + 4 bytes)
__device__ __forceinline__ size_t map_stride(uint32_t cap) { return (size_t)cap * 9 * 4; }

__device__ void map_bind(DMap& m, uint8_t* base, uint32_t cap, int which) {
    uint8_t* b = base + (size_t)which * 2 * cap * 9;
    m.cap = cap;
    m.keys = (uint32_t*)b; m.vals = (int32_t*)(b + (size_t)cap * 4); m.info = b + (size_t)cap * 8;
    uint8_t* b2 = b + (size_t)cap * 9;
    m.keys2 = (uint32_t*)b2; m.vals2 = (int32_t*)(b2 + (size_t)cap * 4); m.info2 = b2 + (size_t)cap * 8;
}

// field-wise copies: structs in LDS (address space 3) and generic memory are
// different C++ types, so whole-struct assignment between them does not compile
template <class P>
__device__ __forceinline__ HitD ld_hit(P p) {
    HitD h;
    h.qs = p->qs; h.qe = p->qe; h.rs = p->rs; h.re = p->re; h.list = p->list; h.pad = p->pad;
    return h;
}
template <class P>
__device__ __forceinline__ void st_hit(P p, const HitD& h) {
    p->qs = h.qs; p->qe = h.qe; p->rs = h.rs; p->re = h.re; p->list = h.list; p->pad = h.pad;
}
template <class P>
__device__ __forceinline__ rsa_nam ld_nam(P p) {
    rsa_nam n;
    n.nam_id = p->nam_id; n.query_start = p->query_start; n.query_end = p->query_end;
    n.query_prev_hit_startpos = p->query_prev_hit_startpos; n.ref_start = p->ref_start; n.ref_end = p->ref_end;
    n.ref_prev_hit_startpos = p->ref_prev_hit_startpos; n.n_hits = p->n_hits; n.ref_id = p->ref_id;
    n.score = p->score; n.is_rc = p->is_rc;
    return n;
}
template <class P>
__device__ __forceinline__ void st_nam(P p, const rsa_nam& n) {
    p->nam_id = n.nam_id; p->query_start = n.query_start; p->query_end = n.query_end;
    p->query_prev_hit_startpos = n.query_prev_hit_startpos; p->ref_start = n.ref_start; p->ref_end = n.ref_end;
    p->ref_prev_hit_startpos = n.ref_prev_hit_startpos; p->n_hits = n.n_hits; p->ref_id = n.ref_id;
    p->score = n.score; p->is_rc = n.is_rc;
}

// ---------------------------------------------------------------------------
// NAM construction helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ float nam_score(const rsa_nam& n) {   // nam.cpp:456-460
    const int qspan = n.query_end - n.query_start, rspan = n.ref_end - n.ref_start;
    const int mx = qspan > rspan ? qspan : rspan, mn = qspan < rspan ? qspan : rspan;
    return (2 * mn - mx) > 0 ? (float)(n.n_hits * (2 * mn - mx)) : 1.0f;
}

template <class OutP>
__device__ __forceinline__ void nam_emit(OutP out, int& n_out, rsa_nam x) {
    x.score = nam_score(x);
    x.nam_id = n_out;
    st_nam(&out[n_out++], x);
}

__device__ __forceinline__ rsa_nam nam_from_hit(const HitD& h, int ref_id, int is_rc) {
    rsa_nam n;
    n.nam_id = 0;
    n.query_start = h.qs; n.query_end = h.qe; n.ref_start = h.rs; n.ref_end = h.re;
    n.query_prev_hit_startpos = h.qs; n.ref_prev_hit_startpos = h.rs;
    n.n_hits = 1; n.ref_id = ref_id; n.score = 0.0f; n.is_rc = is_rc;
    return n;
}

template <class OpenP, class OutP>
__device__ void flush_passed(OpenP open, int& n_open, int query_start, OutP out, int& n_out) {
    for (int i = 0; i < n_open; ++i)
        if (open[i].query_end < query_start) nam_emit(out, n_out, ld_nam(&open[i]));
    int w = 0;
    for (int i = 0; i < n_open; ++i)
        if (!(open[i].query_end < query_start)) { if (w != i) st_nam(&open[w], ld_nam(&open[i])); w++; }
    n_open = w;
}

// add_to_hits_per_ref (nam.cpp:68-85): appends hits of one query randstrobe
template <class M>
__device__ void add_hits(M& m, int orient, int qs, int qe, const SeedIndexParams& p, uint64_t pos, uint32_t count,
                         HitD* hits, int& n_hits, int& n_lists) {
    int min_diff = INT_MAX;
    for (uint64_t e = pos; e < pos + count; ++e) {
        const rsa_ref_randstrobe x = p.rs[e];
        const int rs = (int)x.position;
        const int re = rs + (int)(x.packed & 0xFF) + p.k;
        int d = (qe - qs) - (re - rs);
        d = d < 0 ? -d : d;
        if (d <= min_diff) {
            bool ins;
            const int32_t lid = rh_get_or_insert(m, x.packed >> 8, n_lists, ins);
            if (ins) n_lists++;
            HitD h;
            h.qs = qs; h.qe = qe; h.rs = rs; h.re = re; h.list = lid | (orient << 30); h.pad = 0;
            hits[n_hits++] = h;
            min_diff = d;
        }
    }
}

// next occupied slot >= slot (slot order = robin_hood iteration order), nwb if none
template <class M>
__device__ __forceinline__ uint32_t rh_next_slot(const M& m, uint32_t slot) {
    while (slot < m.nwb) {
        if ((slot & 3) == 0 && *(const typename M::U32*)(m.info + slot) == 0) { slot += 4; continue; }
        if (m.info[slot]) return slot;
        ++slot;
    }
    return m.nwb;
}

// merge_hits_into_nams (nam.cpp:370-536, sort=true) for one hit list (one
// ref_id x orientation): emits into out[0..), nam_id = local index
template <class HitP, class OpenP, class OutP>
__device__ void merge_one_list(int32_t lid, int ref_id, int orient, HitP hits, int n_hits, int k, OpenP open,
                               OutP out, int& n_out) {
    int n_open = 0;
    unsigned prev_q_start = 0;
    for (int hi = 0; hi < n_hits; ++hi) {
        const HitD x = ld_hit(&hits[hi]);
        if (x.list != lid) continue;
        bool added = false;
        for (int o = 0; o < n_open; ++o) {
            auto& on = open[o];
            if (on.query_prev_hit_startpos < x.qs && x.qs <= on.query_end && on.ref_prev_hit_startpos < x.rs &&
                x.rs <= on.ref_end) {
                if (x.qe > on.query_end && x.re > on.ref_end) {
                    on.query_end = x.qe; on.ref_end = x.re;
                    on.query_prev_hit_startpos = x.qs; on.ref_prev_hit_startpos = x.rs;
                    on.n_hits++; added = true; break;
                } else if (x.qe <= on.query_end && x.re <= on.ref_end) {
                    on.query_prev_hit_startpos = x.qs; on.ref_prev_hit_startpos = x.rs;
                    on.n_hits++; added = true; break;
                }
            }
        }
        if (!added) st_nam(&open[n_open++], nam_from_hit(x, ref_id, orient));
        if ((unsigned)x.qs > prev_q_start + (unsigned)k) {
            flush_passed(open, n_open, x.qs, out, n_out);
            prev_q_start = (unsigned)x.qs;
        }
    }
    for (int o = 0; o < n_open; ++o) nam_emit(out, n_out, ld_nam(&open[o]));
}

// all lists of one orientation, in robin_hood slot order
template <class M, class HitP, class OpenP, class OutP>
__device__ void merge_slow(const M& m, int orient, HitP hits, int n_hits, int k, OpenP open, OutP out, int& n_out) {
    for (uint32_t slot = rh_next_slot(m, 0); slot < m.nwb; slot = rh_next_slot(m, slot + 1))
        merge_one_list(m.vals[slot] | (orient << 30), (int)m.keys[slot], orient, hits, n_hits, k, open, out, n_out);
}

// merge_hits_into_nams_fast (nam.cpp:117-366, sort=false)
template <class M>
__device__ void merge_fast(const M& m, int orient, HitD* hits, int n_hits, int k, rsa_nam* open, uint8_t* added,
                           HitD* grp, rsa_nam* out, int& n_out) {
    for (uint32_t slot = rh_next_slot(m, 0); slot < m.nwb; slot = rh_next_slot(m, slot + 1)) {
        const int32_t lid = m.vals[slot] | (orient << 30);
        const int ref_id = (int)m.keys[slot];
        int n_open = 0;
        unsigned prev_q_start = 0;
        int hi = 0;
        // hits of this list, in insertion order, processed in query_start groups
        while (true) {
            while (hi < n_hits && hits[hi].list != lid) hi++;
            if (hi >= n_hits) break;
            const int qstart = hits[hi].qs;
            int gn = 0;
            for (int z = hi; z < n_hits; ++z) {
                if (hits[z].list != lid) continue;
                if (hits[z].qs != qstart) break;
                grp[gn++] = hits[z];
                hi = z + 1;
            }
            // sort group by (qs, rs): insertion sort on rs (qs equal)
            for (int a = 1; a < gn; ++a) {
                HitD x = grp[a]; int b = a - 1;
                while (b >= 0 && x.rs < grp[b].rs) { grp[b + 1] = grp[b]; --b; }
                grp[b + 1] = x;
            }
            for (int a = 0; a < gn; ++a) added[a] = 0;
            int cnt_done = 0;
            for (int o = 0; o < n_open; ++o) {
                rsa_nam& on = open[o];
                int lower = 0, upper = 0;
                while (lower < gn && grp[lower].rs < on.ref_prev_hit_startpos + 1) lower++;
                while (upper < gn && grp[upper].rs < on.ref_end + 1) upper++;
                for (int z = lower; z < upper; ++z) {
                    if (added[z]) continue;
                    if (qstart <= on.query_end) {
                        const HitD& x = grp[z];
                        if (on.ref_prev_hit_startpos < x.rs && x.rs <= on.ref_end) {
                            if (x.qe > on.query_end && x.re > on.ref_end) {
                                on.query_end = x.qe; on.ref_end = x.re;
                                on.query_prev_hit_startpos = x.qs; on.ref_prev_hit_startpos = x.rs;
                                on.n_hits++; added[z] = 1; cnt_done++; break;
                            } else if (x.qe <= on.query_end && x.re <= on.ref_end) {
                                on.query_prev_hit_startpos = x.qs; on.ref_prev_hit_startpos = x.rs;
                                on.n_hits++; added[z] = 1; cnt_done++; break;
                            }
                        }
                    }
                }
                if (cnt_done == gn) break;
            }
            for (int z = 0; z < gn; ++z)
                if (!added[z]) open[n_open++] = nam_from_hit(grp[z], ref_id, orient);
            if ((unsigned)qstart > prev_q_start + (unsigned)k) {
                flush_passed(open, n_open, qstart, out, n_out);
                prev_q_start = (unsigned)qstart;
            }
        }
        for (int o = 0; o < n_open; ++o) nam_emit(out, n_out, open[o]);
    }
}

// ---------------------------------------------------------------------------
// find_nams of one read (nam.cpp:771-926) given k_lookup's per-randstrobe
// results.  `ms` holds the read's two robin_hood maps (map_stride(map_cap));
// hits / open / out have room for the read's hits_find entries.
// ---------------------------------------------------------------------------
__device__ void find_nams_read(int r, const rsa_query_randstrobe* __restrict__ qrs, const QrsInfo* __restrict__ qi,
                               const uint32_t* __restrict__ qcnt, const uint64_t* __restrict__ qbase,
                               const ReadStat* __restrict__ st, const SeedIndexParams& p, HitD* __restrict__ hits,
                               rsa_nam* __restrict__ open, rsa_nam* __restrict__ out, uint8_t* ms, uint32_t map_cap,
                               uint32_t* __restrict__ ncnt, float* __restrict__ nonrep, uint32_t* __restrict__ flags) {
    const int nq = (int)qcnt[r];
    const uint64_t base = qbase[r];
    const ReadStat s = st[r];
    // nonrepetitive_fraction (nam.cpp:920)
    nonrep[r] = s.found > 0 ? (float)s.good / (float)s.found : 1.0f;
    DMap m[2];
    map_bind(m[0], ms, map_cap, 0);
    map_bind(m[1], ms, map_cap, 1);
    rh_new_reserved(m[0]);
    rh_new_reserved(m[1]);
    int n_hits = 0, n_lists = 0;
    for (int i = 0; i < nq; ++i) {
        const QrsInfo o = qi[base + i];
        if (!(o.flags & 1) || (o.flags & 2)) continue;
        const rsa_query_randstrobe q = qrs[base + i];
        const int orient = q.is_reverse ? 1 : 0;
        add_hits(m[orient], orient, (int)q.start, (int)q.end, p, o.pos, o.count, hits, n_hits, n_lists);
    }
    if (m[0].overflow || m[1].overflow) { flags[r] = 2; ncnt[r] = 0; return; }
    int n_out = 0;
    merge_slow(m[0], 0, hits, n_hits, p.k, open, out, n_out);
    merge_slow(m[1], 1, hits, n_hits, p.k, open, out, n_out);
    ncnt[r] = (uint32_t)n_out;
    flags[r] = 0;
}

#define FN_WAVES 4
#define FN_MAP_CAP 256

// ---------------------------------------------------------------------------
// k_find_nams_w2: one wavefront per read, maps and hits in LDS (≈8.7 KB a read,
// so a CU keeps ~18 reads in flight).
//   1. the read's hits, written by k_seed_query in add_to_hits_per_ref order
//      (nam.cpp:68-85, 781-905), are copied to LDS (and kept in registers, one a lane)
//   2. lane 0 (fwd) and lane 1 (rc) insert the keys into the two robin_hood
//      emulations (LDS) in hit order -- only the first hit of each run of equal
//      keys, found by ballots; the rest of a run copies its list id.  The occupied
//      slots, fwd map then rc map, give the list order merge_hits_into_nams walks
//      (nam.cpp:370-536)
//   3. the lists one after another, the whole wave on each (merge_list_wave):
//      NAMs in registers, one a lane, in creation order; they carry the
//      sequence number of their emission (flush of passed NAMs, then the final
//      sweep), which is their place in the output; the open set is "created
//      and not yet emitted", in creation order, exactly the reference's
//      open_nams vector.
// Reads with more than FN2_HCAP hits or whose maps would rehash past
// FN_MAP_CAP are flagged (flags = 2) for the global-scratch kernel above.
// ---------------------------------------------------------------------------
#define FN2_WAVES 2
#define FN2_HCAP 128
#define FN2_MAPB (2 * FN_MAP_CAP * 9)


#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))
typedef __attribute__((address_space(3))) HitD LHit;
typedef __attribute__((address_space(3))) int2 LInt2;

// a hit's fields on its lane (list = -1: no hit)
struct WaveHit { int qs, qe, rs, re, list; };
__device__ __forceinline__ WaveHit load_wave_hit(const LHit* hits, int h, int n_hits) {
    WaveHit x;
    x.qs = x.qe = x.rs = x.re = 0; x.list = -1;
    if (h < n_hits) { x.qs = hits[h].qs; x.qe = hits[h].qe; x.rs = hits[h].rs; x.re = hits[h].re; x.list = hits[h].list; }
    return x;
}

// a NAM under construction in a lane's registers (nam.hpp:11-38 fields); seq < 0: open
struct RegNam { int qs, qe, qprev, rs, re, rprev, n_hits, seq; };

// does hit x extend NAM a (the two accepting branches of nam.cpp merge_hits_into_nams)
__device__ __forceinline__ bool nam_takes(const RegNam& a, int xqs, int xqe, int xrs, int xre) {
    return a.seq < 0 && a.qprev < xqs && xqs <= a.qe && a.rprev < xrs && xrs <= a.re &&
           ((xqe > a.qe && xre > a.re) || (xqe <= a.qe && xre <= a.re));
}
__device__ __forceinline__ void nam_take(RegNam& a, int xqs, int xqe, int xrs, int xre) {
    if (xqe > a.qe && xre > a.re) { a.qe = xqe; a.re = xre; }
    a.qprev = xqs; a.rprev = xrs; a.n_hits++;
}
__device__ __forceinline__ void nam_open(RegNam& a, int xqs, int xqe, int xrs, int xre) {
    a.qs = xqs; a.qe = xqe; a.qprev = xqs; a.rs = xrs; a.re = xre; a.rprev = xrs; a.n_hits = 1; a.seq = -1;
}
__device__ __forceinline__ void nam_write(const RegNam& a, int base, int ref_id, int orient, rsa_nam* out) {
    rsa_nam x;
    x.nam_id = base + a.seq;                                // position in the read's NAM vector
    x.query_start = a.qs; x.query_end = a.qe; x.query_prev_hit_startpos = a.qprev;
    x.ref_start = a.rs; x.ref_end = a.re; x.ref_prev_hit_startpos = a.rprev;
    x.n_hits = a.n_hits; x.ref_id = ref_id; x.score = 0.0f; x.is_rc = orient;
    x.score = nam_score(x);
    out[x.nam_id] = x;
}

// merge_hits_into_nams for list `lid` on the whole wave; writes its NAMs at
// out[base + emission order] and returns their number
__device__ int merge_list_wave(int lid, const WaveHit& h0, const WaveHit& h1, int n_hits, int k, int lane, int ref_id,
                               rsa_nam* out, int base) {
    RegNam A, B;                                            // NAM lane (bank 0), lane + 64 (bank 1)
    nam_open(A, 0, 0, 0, 0); nam_open(B, 0, 0, 0, 0);
    int n_created = 0, n_out = 0;
    unsigned prev_q_start = 0;
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int c = 0; c < 2 && c * 64 < n_hits; ++c) {
        const WaveHit& hv = c ? h1 : h0;
        uint64_t mask = __ballot(hv.list == lid);
        while (mask) {
            const int h = __builtin_ctzll(mask);
            mask &= mask - 1;
            const int xqs = __builtin_amdgcn_readlane(hv.qs, h), xqe = __builtin_amdgcn_readlane(hv.qe, h);
            const int xrs = __builtin_amdgcn_readlane(hv.rs, h), xre = __builtin_amdgcn_readlane(hv.re, h);
            const bool inA = lane < n_created, inB = lane + 64 < n_created;
            const uint64_t mA = __ballot(inA && nam_takes(A, xqs, xqe, xrs, xre));
            if (mA) {
                if (lane == __builtin_ctzll(mA)) nam_take(A, xqs, xqe, xrs, xre);
            } else {
                const uint64_t mB = n_created > 64 ? __ballot(inB && nam_takes(B, xqs, xqe, xrs, xre)) : 0ull;
                if (mB) {
                    if (lane == __builtin_ctzll(mB)) nam_take(B, xqs, xqe, xrs, xre);
                } else {
                    if (n_created < 64) { if (lane == n_created) nam_open(A, xqs, xqe, xrs, xre); }
                    else if (lane + 64 == n_created) nam_open(B, xqs, xqe, xrs, xre);
                    n_created++;
                }
            }
            if ((unsigned)xqs > prev_q_start + (unsigned)k) {       // emit the NAMs the query has passed
                const bool eA = lane < n_created && A.seq < 0 && A.qe < xqs;
                const bool eB = lane + 64 < n_created && B.seq < 0 && B.qe < xqs;
                const uint64_t bA = __ballot(eA), bB = __ballot(eB);
                if (eA) A.seq = n_out + __popcll(bA & below);
                if (eB) B.seq = n_out + __popcll(bA) + __popcll(bB & below);
                n_out += __popcll(bA) + __popcll(bB);
                prev_q_start = (unsigned)xqs;
            }
        }
    }
    {                                                       // the final sweep, creation order
        const bool eA = lane < n_created && A.seq < 0, eB = lane + 64 < n_created && B.seq < 0;
        const uint64_t bA = __ballot(eA), bB = __ballot(eB);
        if (eA) A.seq = n_out + __popcll(bA & below);
        if (eB) B.seq = n_out + __popcll(bA) + __popcll(bB & below);
        n_out += __popcll(bA) + __popcll(bB);
    }
    const int orient = (lid >> 30) & 1;
    if (lane < n_created) nam_write(A, base, ref_id, orient, out);
    if (lane + 64 < n_created) nam_write(B, base, ref_id, orient, out);
    return n_out;
}

__global__ void __launch_bounds__(64 * FN2_WAVES)
k_find_nams_w2(const ReadStat* __restrict__ st, const HitD* __restrict__ hit_slots, int n_reads, SeedIndexParams p,
               rsa_nam* __restrict__ nam_buf, uint32_t* __restrict__ ncnt, float* __restrict__ nonrep,
               uint32_t* __restrict__ flags, uint64_t* __restrict__ nsrc, SeedHdr* __restrict__ hdr,
               uint32_t* __restrict__ big_list) {
    __shared__ __attribute__((aligned(16))) uint8_t s_map[FN2_WAVES][FN2_MAPB];   // maps, then NAMs
    __shared__ HitD s_hits[FN2_WAVES][FN2_HCAP];
    __shared__ int2 s_order[FN2_WAVES][FN2_HCAP];
    __shared__ int s_ctl[FN2_WAVES][4];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = blockIdx.x * FN2_WAVES + w;
    if (r >= n_reads) return;                           // whole wave
    const ReadStat rs = st[r];
    if (rs.hits_find > FN2_HCAP || rs.hits_find > LK_HCAP) {
        if (lane == 0) {
            nonrep[r] = rs.found > 0 ? (float)rs.good / (float)rs.found : 1.0f;
            flags[r] = 2; ncnt[r] = 0;
            big_list[atomicAdd(&hdr->big_count, 1u)] = (uint32_t)r;   // the global-map pass
        }
        return;
    }
    LHit* hits = LDS_PTR(HitD, s_hits[w]);
    SPROF_T(f0);
    // 1. the read's hits, written in add_to_hits_per_ref order by k_lookup
    const int n_hits = (int)rs.hits_find;
    const HitD* slot = hit_slots + (size_t)r * LK_HCAP;
    const bool v0 = lane < n_hits, v1 = lane + 64 < n_hits;
    HitD x0, x1;
    x0.list = x1.list = 0; x0.pad = x1.pad = 0;
    if (v0) { x0 = slot[lane]; st_hit(&hits[lane], x0); }
    if (v1) { x1 = slot[lane + 64]; st_hit(&hits[lane + 64], x1); }
    WSYNC_SEED();
    SPROF_T(f1);
    // 2. the two robin_hood maps (fwd, rc) in LDS
    LMap m0, m1;
    {
        uint8_t* b0 = s_map[w];
        uint8_t* b1 = s_map[w] + (size_t)FN_MAP_CAP * 9;
        m0.cap = m1.cap = FN_MAP_CAP;
        m0.keys = LDS_PTR(uint32_t, b0); m0.vals = LDS_PTR(int32_t, b0 + (size_t)FN_MAP_CAP * 4);
        m0.info = LDS_PTR(uint8_t, b0 + (size_t)FN_MAP_CAP * 8);
        m1.keys = LDS_PTR(uint32_t, b1); m1.vals = LDS_PTR(int32_t, b1 + (size_t)FN_MAP_CAP * 4);
        m1.info = LDS_PTR(uint8_t, b1 + (size_t)FN_MAP_CAP * 8);
        m0.info2 = m1.info2 = nullptr; m0.keys2 = m1.keys2 = nullptr; m0.vals2 = m1.vals2 = nullptr;  // rehash -> fallback
    }
    if (lane == 0) nonrep[r] = rs.found > 0 ? (float)rs.good / (float)rs.found : 1.0f;   // nam.cpp:920
    // operator[] on the key just looked up changes nothing (nam.cpp:68-85), so only
    // the first hit of each run of equal keys, in its orientation's hit order,
    // touches the map: the runs come from ballots, the map insertions stay in hit
    // order on one lane per map, and the rest of each run copies its list id
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint64_t M[2][2], S[2][2];                         // [orientation][hit chunk]: hits, run starts
#pragma unroll
    for (int o = 0; o < 2; ++o) {
        M[o][0] = __ballot(v0 && (int)x0.pad == o);
        M[o][1] = __ballot(v1 && (int)x1.pad == o);
    }
    uint32_t last0[2];                                  // key of each orientation's last hit in chunk 0
#pragma unroll
    for (int o = 0; o < 2; ++o)
        last0[o] = M[o][0] ? (uint32_t)__builtin_amdgcn_readlane(x0.list, 63 - __builtin_clzll(M[o][0])) : 0u;
    bool start0 = false, start1 = false;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const HitD& x = c ? x1 : x0;
        const bool v = c ? v1 : v0;
        const int o = (int)x.pad & 1;
        const uint64_t pm = (o ? M[1][c] : M[0][c]) & below;
        const uint32_t pk = (uint32_t)__shfl(x.list, pm ? 63 - __builtin_clzll(pm) : lane, 64);
        bool has_prev = pm != 0;
        uint32_t prevk = pk;
        if (c == 1 && !pm && (o ? M[1][0] : M[0][0])) { has_prev = true; prevk = last0[o]; }
        const bool st_ = v && (!has_prev || prevk != (uint32_t)x.list);
        S[0][c] = __ballot(st_ && o == 0);
        S[1][c] = __ballot(st_ && o == 1);
        if (c) start1 = st_; else start0 = st_;
    }
    if (lane < 2) {
        // each map sees its own keys in hit order, which fixes its slot layout; list
        // ids only have to be distinct, so each map numbers its lists itself: lane 0
        // fills the fwd map while lane 1 fills the rc map (each writes only its own
        // orientation's run starts).  The map is built by value per lane: picking m0
        // or m1 by reference would take their addresses (scratch).
        LMap m;
        uint8_t* bm = s_map[w] + (size_t)lane * FN_MAP_CAP * 9;
        m.cap = FN_MAP_CAP;
        m.keys = LDS_PTR(uint32_t, bm); m.vals = LDS_PTR(int32_t, bm + (size_t)FN_MAP_CAP * 4);
        m.info = LDS_PTR(uint8_t, bm + (size_t)FN_MAP_CAP * 8);
        m.info2 = nullptr; m.keys2 = nullptr; m.vals2 = nullptr;   // rehash -> fallback
        rh_new_reserved(m);
        int n_lists = 0;
        for (int c = 0; c < 2; ++c) {
            uint64_t mask = lane ? S[1][c] : S[0][c];
            while (mask) {
                const int h = 64 * c + (int)__builtin_ctzll(mask);
                mask &= mask - 1;
                bool ins;
                const int32_t lid = rh_get_or_insert(m, (uint32_t)hits[h].list, n_lists, ins);
                if (ins) n_lists++;
                hits[h].list = lid | (lane << 30);
            }
        }
        s_ctl[w][1 + lane] = (int)m.nwb;
        s_ctl[w][3 - lane * 3] = m.overflow ? 1 : 0;         // lane 0 -> [3], lane 1 -> [0]
    }
    WSYNC_SEED();
#pragma unroll
    for (int c = 0; c < 2; ++c) {                       // the rest of each run: its start's list id
        const HitD& x = c ? x1 : x0;
        const bool v = c ? v1 : v0;
        const int o = (int)x.pad & 1;
        if (v && !(c ? start1 : start0)) {
            const uint64_t sm = (o ? S[1][c] : S[0][c]) & below;
            const uint64_t s0 = o ? S[1][0] : S[0][0];
            const int st_h = sm ? 64 * c + 63 - __builtin_clzll(sm) : 63 - __builtin_clzll(s0);
            hits[64 * c + lane].list = hits[st_h].list;
        }
    }
    WSYNC_SEED();
    SPROF_T(f2);
    if (s_ctl[w][0] | s_ctl[w][3]) {
        if (lane == 0) {
            flags[r] = 2; ncnt[r] = 0;
            big_list[atomicAdd(&hdr->big_count, 1u)] = (uint32_t)r;
        }
        return;
    }
    // list order = occupied slots of the fwd map, then of the rc map (robin_hood iteration order);
    // every list holds at least one hit, so there are at most FN2_HCAP of them
    LInt2* order = LDS_PTR(int2, s_order[w]);
    int nl = 0;
#pragma unroll
    for (int o = 0; o < 2; ++o) {
        const LMap::U8* minfo = o ? m1.info : m0.info;
        const LMap::U32* mkeys = o ? m1.keys : m0.keys;
        const LMap::I32* mvals = o ? m1.vals : m0.vals;
        const int nwb = s_ctl[w][1 + o];
        const uint32_t word = lane * 4 < nwb ? ((const LMap::U32*)minfo)[lane] : 0u;
        uint64_t mk[4];
        int occ = 0;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
            const bool on = ((word >> (8 * bb)) & 0xFFu) != 0 && lane * 4 + bb < nwb;
            mk[bb] = __ballot(on);
            occ += __popcll(mk[bb]);
        }
        const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
        int rank = __popcll(mk[0] & lt) + __popcll(mk[1] & lt) + __popcll(mk[2] & lt) + __popcll(mk[3] & lt);
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
            if ((mk[bb] >> lane) & 1ull) {
                const int slot = lane * 4 + bb;
                if (nl + rank < FN2_HCAP) {
                    order[nl + rank].x = mvals[slot] | (o << 30);
                    order[nl + rank].y = (int)mkeys[slot];
                }
                rank++;
            }
        }
        nl += occ;
    }
    WSYNC_SEED();
    SPROF_T(f3);
    rsa_nam* out = nam_buf + (size_t)r * FN2_HCAP;          // a read's fixed NAM slot (NAMs <= hits)
    // 3. merge_hits_into_nams (nam.cpp:370-536), one list after another in list
    //    order, the whole wave on one list: hit h's fields sit on lane h % 64
    //    (bank h / 64) and come out by readlane in hit order; NAM o (creation
    //    order) lives in the registers of lane o % 64, bank o / 64.  "The first
    //    open NAM the hit extends" is the lowest set bit of a ballot, the flush
    //    of passed NAMs a ballot ranked by creation order.
    WaveHit h0 = load_wave_hit(hits, lane, n_hits), h1 = load_wave_hit(hits, lane + 64, n_hits);
    int obase = 0;
    for (int l = 0; l < nl; ++l) {
        const int lid = order[l].x, ref_id = order[l].y;
        const int n_out = merge_list_wave(lid, h0, h1, n_hits, p.k, lane, ref_id, out, obase);
        obase += n_out;
    }
    if (lane == 0) { ncnt[r] = (uint32_t)obase; flags[r] = 0; nsrc[r] = (uint64_t)r * FN2_HCAP; }
    SPROF_T(f4);
    SPROF_ADD(4, f1 - f0); SPROF_ADD(5, f2 - f1); SPROF_ADD(6, f3 - f2); SPROF_ADD(7, f4 - f3); SPROF_ADD(8, 1);
    SPROF_ADD(9, n_hits); SPROF_ADD(10, nl);
}

// ---------------------------------------------------------------------------
// The rare reads k_find_nams_w2 lists (more hits than its LDS holds, or maps
// that would rehash past the LDS tables): one lane per read, maps in global
// scratch, hits / open NAMs / NAMs from the call's pool (one bump allocation a
// read).  A single block works through the device list, so the host never
// waits for the list to know what to launch.
// ---------------------------------------------------------------------------
#define BIG_LANES 32
__global__ void __launch_bounds__(64)
k_find_nams_big(rsa_query_randstrobe* __restrict__ qrs, QrsInfo* __restrict__ qi,
                const uint32_t* __restrict__ qcnt, const uint64_t* __restrict__ qbase, ReadStat* __restrict__ st,
                const char* __restrict__ seq, const uint64_t* __restrict__ roff, const uint32_t* __restrict__ rlen,
                RescueScratch scr, SeedIndexParams p, SeedPool pool, uint8_t* __restrict__ map_scratch, uint32_t map_cap,
                uint32_t* __restrict__ ncnt, float* __restrict__ nonrep, uint32_t* __restrict__ flags,
                uint64_t* __restrict__ nsrc, SeedHdr* __restrict__ hdr, const uint32_t* __restrict__ big_list) {
    const int lane = threadIdx.x;
    if (lane >= BIG_LANES) return;
    const uint32_t nb = hdr->big_count;
    for (uint32_t t = lane; t < nb; t += BIG_LANES) {
        const int r = (int)big_list[t];
        const uint32_t hf = st[r].hits_find;
        const unsigned long long e = atomicAdd(&hdr->pool_used, (unsigned long long)hf);
        if (e + hf > pool.n) { atomicOr(&hdr->errors, SEED_E_POOL); ncnt[r] = 0; continue; }
        nsrc[r] = pool.arena_base + e;
        if (!st[r].qw) query_lane(r, seq, roff, rlen, qbase, p, scr.sync(qbase[r]), qrs, qi, st, hdr);
        find_nams_read(r, qrs, qi, qcnt, qbase, st, p, pool.hits + e, pool.open + e, pool.nams + e,
                       map_scratch + (size_t)lane * map_stride(map_cap), map_cap, ncnt, nonrep, flags);
        if (flags[r] & 2u) atomicOr(&hdr->errors, SEED_E_FIND);
    }
}

// ---------------------------------------------------------------------------
// k_rescue: find_nams_rescue for listed reads (one lane per read)
// ---------------------------------------------------------------------------

__device__ __forceinline__ bool rcmp1(const RescueD& a, const RescueD& b) {   // nam.cpp:943-946
    if (a.count != b.count) return a.count < b.count;
    if (a.qs != b.qs) return a.qs < b.qs;
    return a.qe < b.qe;
}

__device__ void rescue_read(int r, const rsa_query_randstrobe* __restrict__ qrs, const QrsInfo* __restrict__ qi,
                            const uint32_t* __restrict__ qcnt, const uint64_t* __restrict__ qbase,
                            const uint64_t* __restrict__ roff, const SeedIndexParams& p, uint32_t rescue_cutoff,
                            RescueD* __restrict__ rbuf, HitD* __restrict__ hits_buf, rsa_nam* __restrict__ open_buf,
                            rsa_nam* __restrict__ nam_buf, HitD* __restrict__ grp_buf, uint8_t* __restrict__ added_buf,
                            uint8_t* ms, uint32_t map_cap, uint32_t* __restrict__ ncnt, uint32_t* __restrict__ flags) {
    const int nq = (int)qcnt[r];
    const uint64_t base = qbase[r];
    RescueD* rv = rbuf + base;        // room for nq entries (both orientations)
    int nf = 0;
    for (int i = 0; i < nq; ++i) {    // forward first, then rc
        const QrsInfo o = qi[base + i];
        if (!(o.flags & 1)) continue;
        const rsa_query_randstrobe q = qrs[base + i];
        if (q.is_reverse) continue;
        RescueD x; x.pos = o.pos; x.count = o.count; x.qs = q.start; x.qe = q.end; x.pad = 0;
        rv[nf++] = x;
    }
    int nr = nf;
    for (int i = 0; i < nq; ++i) {
        const QrsInfo o = qi[base + i];
        if (!(o.flags & 1)) continue;
        const rsa_query_randstrobe q = qrs[base + i];
        if (!q.is_reverse) continue;
        RescueD x; x.pos = o.pos; x.count = o.count; x.qs = q.start; x.qe = q.end; x.pad = 0;
        rv[nr++] = x;
    }
    const int seg_a[2] = {0, nf}, seg_n[2] = {nf, nr - nf};
    DMap m[2];
    map_bind(m[0], ms, map_cap, 0);
    map_bind(m[1], ms, map_cap, 1);
    rh_new_reserved(m[0]);
    rh_new_reserved(m[1]);
    int taken[2];
    int n_lists = 0;
    for (int o = 0; o < 2; ++o) {
        RescueD* v = rv + seg_a[o];
        const int n = seg_n[o];
        for (int a = 1; a < n; ++a) {   // std::sort by cmp1: keys are unique
            RescueD x = v[a]; int b = a - 1;
            while (b >= 0 && rcmp1(x, v[b])) { v[b + 1] = v[b]; --b; }
            v[b + 1] = x;
        }
        int cnt = 0;
        for (int a = 0; a < n; ++a) {
            if ((v[a].count > rescue_cutoff && cnt >= 5) || v[a].count > 1000) break;
            // add_to_hits_per_ref_pre (nam.cpp:87-107): pre-insert keys
            int min_diff = INT_MAX;
            for (uint64_t e = v[a].pos; e < v[a].pos + v[a].count; ++e) {
                const rsa_ref_randstrobe x = p.rs[e];
                const int rs = (int)x.position, re = rs + (int)(x.packed & 0xFF) + p.k;
                int d = ((int)v[a].qe - (int)v[a].qs) - (re - rs);
                d = d < 0 ? -d : d;
                if (d <= min_diff) {
                    bool ins;
                    (void)rh_get_or_insert(m[o], x.packed >> 8, n_lists, ins);
                    if (ins) n_lists++;
                    min_diff = d;
                }
            }
            cnt++;
        }
        taken[o] = cnt;
        // re-sort the taken prefix by query_start (cmp2, nam.cpp:948-952)
        for (int a = 1; a < cnt; ++a) {
            RescueD x = v[a]; int b = a - 1;
            while (b >= 0 && x.qs < v[b].qs) { v[b + 1] = v[b]; --b; }
            v[b + 1] = x;
        }
    }
    HitD* hits = hits_buf + roff[r];
    int n_hits = 0;
    for (int o = 0; o < 2; ++o) {
        const RescueD* v = rv + seg_a[o];
        for (int a = 0; a < taken[o]; ++a)
            add_hits(m[o], o, (int)v[a].qs, (int)v[a].qe, p, v[a].pos, v[a].count, hits, n_hits, n_lists);
    }
    if (m[0].overflow || m[1].overflow) { flags[r] |= 4; ncnt[r] = 0; return; }
    rsa_nam* out = nam_buf + roff[r];
    rsa_nam* open = open_buf + roff[r];
    HitD* grp = grp_buf + roff[r];
    uint8_t* added = added_buf + roff[r];
    int n_out = 0;
    merge_fast(m[0], 0, hits, n_hits, p.k, open, added, grp, out, n_out);
    merge_fast(m[1], 1, hits, n_hits, p.k, open, added, grp, out, n_out);
    ncnt[r] = (uint32_t)n_out;
    flags[r] = (flags[r] & ~4u) | 8u;   // bit3: rescued result present
}

// The rescue decision (aln.cpp:1954-1962: rescue_level > 1 and no NAMs or
// nonrepetitive_fraction < 0.7) from k_find_nams' results, one thread a read:
// the reads that need find_nams_rescue are listed and take hits_all pool
// entries each (one atomic per rescued read; most reads take none).
__global__ void __launch_bounds__(256)
k_rescue_select(int n_reads, int32_t rescue_level, const ReadStat* __restrict__ st, const uint32_t* __restrict__ ncnt1,
                const float* __restrict__ nonrep, uint32_t* __restrict__ ncnt2, uint64_t* __restrict__ rbase,
                uint8_t* __restrict__ rescued, uint64_t pool_n, SeedHdr* __restrict__ hdr,
                uint32_t* __restrict__ rlist) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_reads) return;
    const bool need = rescue_level > 1 && (ncnt1[r] == 0 || nonrep[r] < 0.7f);
    rescued[r] = need ? 1 : 0;
    ncnt2[r] = 0;
    if (!need) return;
    const uint32_t ha = st[r].hits_all;
    const unsigned long long e = atomicAdd(&hdr->pool_used, (unsigned long long)ha);
    if (e + ha > pool_n) { atomicOr(&hdr->errors, SEED_E_POOL); return; }
    rbase[r] = e;
    rlist[atomicAdd(&hdr->rcount, 1u)] = (uint32_t)r;
}

// The rescued reads whose query randstrobes k_seed_query did not write (a read its
// prediction missed): query_lane makes them before k_rescue_w reads them.  One
// block walking the device list; normally it finds nothing to do.  (A separate
// launch: the call inside k_rescue_w put a stack frame into that kernel.)
__global__ void __launch_bounds__(64)
k_query_fix(const uint32_t* __restrict__ rlist, SeedHdr* __restrict__ hdr, const char* __restrict__ seq,
            const uint64_t* __restrict__ roff, const uint32_t* __restrict__ rlen, const uint64_t* __restrict__ qbase,
            SeedIndexParams p, RescueScratch scr, rsa_query_randstrobe* __restrict__ qrs, QrsInfo* __restrict__ qi,
            ReadStat* __restrict__ st) {
    const uint32_t nr = hdr->rcount;
    for (uint32_t t = threadIdx.x; t < nr; t += 64) {
        const int r = (int)rlist[t];
        if (!st[r].qw) query_lane(r, seq, roff, rlen, qbase, p, scr.sync(qbase[r]), qrs, qi, st, hdr);
    }
}

// ---------------------------------------------------------------------------
// find_nams_rescue of one read by a whole wave (k_rescue_w).  The same result as
// rescue_read, with the parallel parts spread over the lanes:
//  - the read's query randstrobes with a hit, per orientation in order (ballot
//    compaction), ranked by cmp1 (count, q_start, q_end; unique keys, so any
//    correct sort is std::sort's) -- at most RW_MAXS a side (reads up to ~330 bp),
//    else the whole read runs rescue_read on lane 0;
//  - the taken prefix (nam.cpp:982-988) from the ranks;
//  - every taken randstrobe's index entries, 64 a round: add_to_hits_per_ref_pre
//    and add_to_hits_per_ref keep an entry iff its |q span - r span| is <= the
//    minimum over the entries before it (an entry not kept never lowers the
//    running min_diff), so a wave prefix-minimum decides, and lane 0 inserts the
//    kept keys in order into the robin_hood map (nam.cpp:87-107).  Both passes
//    keep the same entries, and a key's list id is fixed at its insertion, so the
//    hits of the second pass are recorded in the first (as staged HitD);
//  - the hits in cmp2 (q_start) order of their randstrobes, then
//    merge_hits_into_nams_fast per map (merge_fast, lane 0).
// Before: lane 0 alone walked the entries one dependent load at a time, twice
// (k_rescue_w averaged 524 us a launch on PE 2x250).
// ---------------------------------------------------------------------------
#define RW_MAXS 64                                         // randstrobes a side the wave path ranks (one a lane)
struct RwStrobe { uint64_t pos; uint32_t count, qs, qe, stage_off, stage_cnt, pad; };

// exclusive prefix minimum over the wave (INT_MAX below lane 0)
__device__ __forceinline__ int wave_excl_min(int v, int lane, int& all) {
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x = min(x, y);
    }
    all = __shfl(x, 63, 64);
    const int e = __shfl_up(x, 1, 64);
    return lane == 0 ? INT_MAX : e;
}

__device__ void rescue_read_wave(int r, int lane, const rsa_query_randstrobe* __restrict__ qrs,
                                 const QrsInfo* __restrict__ qi, const uint32_t* __restrict__ qcnt,
                                 const uint64_t* __restrict__ qbase, const uint64_t* __restrict__ roff,
                                 const SeedIndexParams& p, uint32_t rescue_cutoff, RescueD* __restrict__ rbuf,
                                 const SeedPool& pool, uint8_t* ms, RwStrobe* sv, uint32_t* __restrict__ ncnt,
                                 uint32_t* __restrict__ flags) {
    const int nq = (int)qcnt[r];
    const uint64_t base = qbase[r];
    // 1. the randstrobes with a hit of each side, in order, into sv[side][..]
    int n_side[2] = {0, 0};
    for (int i0 = 0; i0 < nq; i0 += 64) {
        const int i = i0 + lane;
        bool hit = false, rev = false;
        RwStrobe x = {};
        if (i < nq) {
            const QrsInfo o = qi[base + i];
            const rsa_query_randstrobe q = qrs[base + i];
            hit = (o.flags & 1) != 0;
            rev = q.is_reverse != 0;
            x.pos = o.pos; x.count = o.count; x.qs = q.start; x.qe = q.end;
        }
#pragma unroll
        for (int o = 0; o < 2; ++o) {
            const bool take = hit && (rev == (o == 1));
            const uint64_t bm = __ballot(take);
            const int at = n_side[o] + __popcll(bm & (lane ? (~0ull >> (64 - lane)) : 0ull));
            if (take && at < RW_MAXS) sv[o * RW_MAXS + at] = x;
            n_side[o] += __popcll(bm);
        }
    }
    if (n_side[0] > RW_MAXS || n_side[1] > RW_MAXS) {      // a read this path does not rank: lane 0, as before
        if (lane == 0)
            rescue_read(r, qrs, qi, qcnt, qbase, roff, p, rescue_cutoff, rbuf, pool.hits, pool.open, pool.nams,
                        pool.grp, pool.added, ms, FN_MAP_CAP, ncnt, flags);
        return;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    DMap m[2];
    map_bind(m[0], ms, FN_MAP_CAP, 0);
    map_bind(m[1], ms, FN_MAP_CAP, 1);
    rh_new_reserved(m[0]);
    rh_new_reserved(m[1]);
    HitD* stage = pool.grp + roff[r];                      // kept hits in cmp1 order (room: hits_all)
    int n_stage = 0, n_lists = 0, taken[2] = {0, 0};
#pragma unroll
    for (int o = 0; o < 2; ++o) {
        RwStrobe* v = sv + o * RW_MAXS;
        const int n = n_side[o];
        // 2. cmp1 ranks (one element a lane), then the taken prefix of the sorted order
        RwStrobe e0 = {};
        if (lane < n) e0 = v[lane];
        int rk0 = 0;
        for (int j = 0; j < n; ++j) {
            const RwStrobe y = v[j];
            rk0 += (y.count != e0.count ? y.count < e0.count : (y.qs != e0.qs ? y.qs < e0.qs : y.qe < e0.qe)) ? 1 : 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (lane < n) v[rk0] = e0;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // taken = the first sorted index a with (count > rescue_cutoff && a >= 5) || count > 1000
        const bool stop_here = lane < n && ((v[lane].count > rescue_cutoff && lane >= 5) || v[lane].count > 1000);
        const uint64_t sm = __ballot(stop_here);
        const int stop = sm ? __builtin_ctzll(sm) : n;
        taken[o] = stop;
        // 3. the kept entries of each taken randstrobe: map keys in order (lane 0) and staged hits
        for (int a = 0; a < stop; ++a) {
            const RwStrobe x = v[a];
            const int qspan = (int)x.qe - (int)x.qs;
            int carry = INT_MAX;
            const int off = n_stage;
            for (uint32_t c0 = 0; c0 < x.count; c0 += 64) {
                const uint32_t i = c0 + lane;
                int d = INT_MAX, rs = 0, re = 0;
                uint32_t key = 0;
                if (i < x.count) {
                    const rsa_ref_randstrobe ent = p.rs[x.pos + i];
                    rs = (int)ent.position;
                    re = rs + (int)(ent.packed & 0xFF) + p.k;
                    d = qspan - (re - rs);
                    d = d < 0 ? -d : d;
                    key = ent.packed >> 8;
                }
                int all;
                const int before = min(carry, wave_excl_min(d, lane, all));
                carry = min(carry, all);
                uint64_t km = __ballot(i < x.count && d <= before);
                while (km) {
                    const int b = __builtin_ctzll(km);
                    km &= km - 1;
                    const uint32_t k_b = (uint32_t)__shfl((int)key, b, 64);
                    const int rs_b = __shfl(rs, b, 64), re_b = __shfl(re, b, 64);
                    if (lane == 0) {
                        bool ins;
                        const int32_t lid = rh_get_or_insert(m[o], k_b, n_lists, ins);
                        if (ins) n_lists++;
                        HitD h;
                        h.qs = (int)x.qs; h.qe = (int)x.qe; h.rs = rs_b; h.re = re_b; h.list = lid | (o << 30); h.pad = 0;
                        stage[n_stage] = h;
                    }
                    n_stage++;
                }
            }
            if (lane == 0) { v[a].stage_off = (uint32_t)off; v[a].stage_cnt = (uint32_t)(n_stage - off); }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    const int ovf = (lane == 0) ? ((m[0].overflow || m[1].overflow) ? 1 : 0) : 0;
    if (__shfl(ovf, 0, 64)) {
        if (lane == 0) { flags[r] |= 4; ncnt[r] = 0; }
        return;
    }
    // 4. the hits: taken randstrobes in q_start order (cmp2, nam.cpp:948-952; q_starts of a side
    //    are distinct), each one's staged hits in entry order
    HitD* hits = pool.hits + roff[r];
    int n_hits = 0;
#pragma unroll
    for (int o = 0; o < 2; ++o) {
        const RwStrobe* v = sv + o * RW_MAXS;
        const int n = taken[o];
        // the hit offset of each taken randstrobe = the staged hits of the taken ones with a smaller q_start
        RwStrobe e0 = {};
        if (lane < n) e0 = v[lane];
        int off0 = 0, tot = 0;
        for (int j = 0; j < n; ++j) {
            const RwStrobe y = v[j];
            off0 += y.qs < e0.qs ? (int)y.stage_cnt : 0;
            tot += (int)y.stage_cnt;
        }
        for (int a = 0; a < n; ++a) {                      // each randstrobe's run, lanes over its hits
            const int so = __shfl((int)e0.stage_off, a, 64), sc = __shfl((int)e0.stage_cnt, a, 64);
            const int d0 = __shfl(off0, a, 64);
            for (int h = lane; h < sc; h += 64) hits[n_hits + d0 + h] = stage[so + h];
        }
        n_hits += tot;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");       // lane 0 reads what every lane wrote
    __builtin_amdgcn_wave_barrier();
    if (lane != 0) return;
    rsa_nam* out = pool.nams + roff[r];
    rsa_nam* open = pool.open + roff[r];
    HitD* grp = pool.grp + roff[r];
    uint8_t* added = pool.added + roff[r];
    int n_out = 0;
    merge_fast(m[0], 0, hits, n_hits, p.k, open, added, grp, out, n_out);
    merge_fast(m[1], 1, hits, n_hits, p.k, open, added, grp, out, n_out);
    ncnt[r] = (uint32_t)n_out;
    flags[r] = (flags[r] & ~4u) | 8u;   // bit3: rescued result present
}

// find_nams_rescue (nam.cpp:955-1012) of the listed reads: one wave per read
// (rescue_read_wave), maps in LDS; a fixed grid walks the device list
#define RESCUE_GRID 256
__global__ void __launch_bounds__(64 * FN_WAVES)
k_rescue_w(const rsa_query_randstrobe* __restrict__ qrs, const QrsInfo* __restrict__ qi,
           const uint32_t* __restrict__ qcnt, const uint64_t* __restrict__ qbase, SeedIndexParams p,
           uint32_t rescue_cutoff, RescueD* __restrict__ rbuf, SeedPool pool, uint32_t* __restrict__ ncnt2,
           uint32_t* __restrict__ flags, const uint64_t* __restrict__ rbase, SeedHdr* __restrict__ hdr,
           const uint32_t* __restrict__ rlist, uint32_t* __restrict__ rbig_list) {
    __shared__ __attribute__((aligned(16))) uint8_t s_map[FN_WAVES][FN_MAP_CAP * 9 * 4];
    __shared__ __attribute__((aligned(16))) RwStrobe s_sv[FN_WAVES][2 * RW_MAXS];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t nr = hdr->rcount;
    for (uint32_t t = blockIdx.x * FN_WAVES + w; t < nr; t += gridDim.x * FN_WAVES) {
        const int r = (int)rlist[t];
        rescue_read_wave(r, lane, qrs, qi, qcnt, qbase, rbase, p, rescue_cutoff, rbuf, pool, s_map[w], s_sv[w], ncnt2,
                         flags);
        if (lane == 0 && (flags[r] & 4u)) rbig_list[atomicAdd(&hdr->rbig_count, 1u)] = (uint32_t)r;
    }
}

// the rescued reads whose maps outgrow LDS: one lane per read, global map scratch,
// the read's pool entries again
__global__ void __launch_bounds__(64)
k_rescue_big(const rsa_query_randstrobe* __restrict__ qrs, const QrsInfo* __restrict__ qi,
             const uint32_t* __restrict__ qcnt, const uint64_t* __restrict__ qbase, SeedIndexParams p,
             uint32_t rescue_cutoff, RescueD* __restrict__ rbuf, SeedPool pool, uint8_t* __restrict__ map_scratch,
             uint32_t map_cap, uint32_t* __restrict__ ncnt2, uint32_t* __restrict__ flags,
             const uint64_t* __restrict__ rbase, SeedHdr* __restrict__ hdr, const uint32_t* __restrict__ rbig_list) {
    const int lane = threadIdx.x;
    if (lane >= BIG_LANES) return;
    const uint32_t nb = hdr->rbig_count;
    for (uint32_t t = lane; t < nb; t += BIG_LANES) {
        const int r = (int)rbig_list[t];
        rescue_read(r, qrs, qi, qcnt, qbase, rbase, p, rescue_cutoff, rbuf, pool.hits, pool.open, pool.nams, pool.grp,
                    pool.added, map_scratch + (size_t)lane * map_stride(map_cap), map_cap, ncnt2, flags);
        if (flags[r] & 4u) atomicOr(&hdr->errors, SEED_E_RESCUE);
    }
}

// final NAM offsets: count[r] = rescued ? rescue NAMs : find NAMs, exclusive scan
// into ooff[0..n] and the total into the header, plus the call's statistics
// summed over the reads (LDS atomics, one global write each: k_lookup's 20 k
// waves adding to one address serialised).  One workgroup walks the reads in
// tiles of 4096, each thread 16 consecutive reads whose loads all issue before
// the tile's scan (a thread walking a private run of reads waited on one
// dependent load per read: 142 us a call).
#define SEED_NSTAT 14
// Final NAM offsets (exclusive scan of the per-read NAM counts) and the call's 14
// statistics, in two launches: k_seed_count -- one read a thread, a workgroup of SS_TPB
// reads -- scans within its workgroup, writes the workgroup's NAM total and adds its
// statistics to the header (14 atomics a workgroup); k_seed_scan (one workgroup) scans
// the totals into workgroup offsets; k_compact adds its read's workgroup offset and
// writes the final offset.  (The single-workgroup scan this replaces walked the batch
// in serial tiles: 89 us a call of 20000 reads; with the statistics summed in
// k_seed_scan instead, one serial load chain cost it 21 us.)
#define SS_TPB 256
#define SS_WAVES (SS_TPB / 64)
__global__ void __launch_bounds__(SS_TPB)
k_seed_count(int n_reads, const uint8_t* __restrict__ rescued, const uint32_t* __restrict__ ncnt1,
             const uint32_t* __restrict__ ncnt2, const uint32_t* __restrict__ qcnt, const ReadStat* __restrict__ st,
             uint32_t* __restrict__ loc, uint64_t* __restrict__ bsum, SeedHdr* __restrict__ hdr) {
    __shared__ uint32_t s_w[SS_WAVES];
    __shared__ unsigned long long s_stat[SEED_NSTAT];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int r = blockIdx.x * SS_TPB + t;
    if (t < SEED_NSTAT) s_stat[t] = 0;
    uint64_t v[SEED_NSTAT] = {0};    // qrs found good hits_find hits_all scan_find scan_all n1 n2 rr rq rscan rhits qw_q
    uint32_t cnt = 0;
    if (r < n_reads) {
        const bool rs = rescued[r] != 0;
        const uint32_t c1 = ncnt1[r], c2 = rs ? ncnt2[r] : 0, q = qcnt[r];
        const ReadStat x = st[r];
        cnt = rs ? c2 : c1;
        v[0] = q; v[1] = x.found; v[2] = x.good; v[3] = x.hits_find; v[4] = x.hits_all;
        v[5] = x.scan_find; v[6] = x.scan_all; v[7] = c1; v[8] = c2;
        if (rs) { v[9] = 1; v[10] = q; v[11] = x.scan_all; v[12] = x.hits_all; }
        if (x.qw) v[13] = q;
    }
    uint32_t x = cnt;                            // wave inclusive scan
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();                             // s_stat zeroed, s_w written
    uint32_t wpre = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < SS_WAVES; ++j) {
        wpre += j < w ? s_w[j] : 0;
        tot += s_w[j];
    }
    if (r < n_reads) loc[r] = wpre + x - cnt;
#pragma unroll
    for (int k = 0; k < SEED_NSTAT; ++k) {       // wave sums, one LDS atomic a wave
        uint64_t a = v[k];
        for (int o = 32; o >= 1; o >>= 1) a += __shfl_xor(a, o, 64);
        if (lane == 0 && a) atomicAdd(&s_stat[k], (unsigned long long)a);
    }
    __syncthreads();
    if (t == 0) bsum[blockIdx.x] = tot;
    if (t < SEED_NSTAT && s_stat[t]) {
        // qrs found good hits_find hits_all scan_find scan_all n1 n2 resc_reads resc_q resc_scan resc_hits qw_q
        unsigned long long* dst[SEED_NSTAT] = {&hdr->qrs, &hdr->found, &hdr->good, &hdr->hits_find, &hdr->hits_all,
                                               &hdr->scan_find, &hdr->scan_all, &hdr->n1, &hdr->n2, &hdr->resc_reads,
                                               &hdr->resc_q, &hdr->resc_scan, &hdr->resc_hits, &hdr->qw_q};
        atomicAdd(dst[t], s_stat[t]);
    }
}

__global__ void __launch_bounds__(SS_TPB)
k_seed_scan(int n_blocks, int n_reads, uint64_t* __restrict__ bsum, uint64_t* __restrict__ ooff,
            SeedHdr* __restrict__ hdr) {
    __shared__ uint64_t s_w[SS_WAVES];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint64_t carry = 0;
    for (int base = 0; base < n_blocks; base += SS_TPB) {   // block totals -> exclusive block offsets, in place
        const int b = base + t;
        const uint64_t mine = b < n_blocks ? bsum[b] : 0;
        uint64_t x = mine;
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        uint64_t wpre = 0, tot = 0;
#pragma unroll
        for (int j = 0; j < SS_WAVES; ++j) {
            wpre += j < w ? s_w[j] : 0;
            tot += s_w[j];
        }
        if (b < n_blocks) bsum[b] = carry + wpre + x - mine;
        carry += tot;
        __syncthreads();
    }
    if (t == 0) {
        ooff[n_reads] = carry;
        hdr->total = carry;
    }
}

// ---------------------------------------------------------------------------
// k_compact: final list per read = rescue list if rescued else find_nams list,
// from the NAM arena to the batch's output (at most `cap` NAMs: a batch with
// more is reported to the host, which asks again with room for them).
// by_score (RSA_NAMS_BY_SCORE): a list of 2..16 NAMs lands in the order the
// caller's std::sort(by_score) gives it (aln.cpp:1962-1964).  libstdc++ sorts
// such a list by insertion (no introsort pass at <= 16 elements), which is
// stable by descending score, so NAM i goes to its rank: the NAMs scoring
// higher, plus the equal ones before it.  One wave a read, scores by shuffle.
// ---------------------------------------------------------------------------
// complement of src/revcomp.hpp:10-27 (A/C/G/T/U either case, all else N)
__device__ __forceinline__ unsigned char rc_base(unsigned char c) {
    switch (c) {
        case 'A': case 'a': return 'T';
        case 'C': case 'c': return 'G';
        case 'G': case 'g': return 'C';
        case 'T': case 't': case 'U': case 'u': return 'A';
        default: return 'N';
    }
}

// What k_sites needs of a final NAM besides the NAM: where its read and its contig
// lie, and the slot of its site check (its read's list start + nam_id).  k_compact
// writes it with the NAM, so k_sites starts with one round of loads, not three.
struct SiteDesc {
    uint64_t read_off;        // the read in the call's sequence buffer
    uint64_t ref_off;         // the NAM's contig in the resident reference
    uint64_t slot;            // sites[] index; ~0: nam_id outside its read's list (a broken permutation)
    uint32_t read_len, ref_len;
};

// k_compact: reads (waves) a workgroup.  One: four (256-thread workgroups) ran 59 against 44 us
// a launch under the bench's kernel trace (profiles/r05k_rocprof.md vs r05j)
#define CP_WAVES 1
__global__ void __launch_bounds__(64 * CP_WAVES)
k_compact(int n_reads, const uint64_t* __restrict__ nsrc, const uint64_t* __restrict__ rbase,
          uint64_t arena_base, const uint32_t* __restrict__ ncnt1, const uint32_t* __restrict__ ncnt2,
          const uint8_t* __restrict__ rescued, const rsa_nam* __restrict__ arena, const uint32_t* __restrict__ loc,
          const uint64_t* __restrict__ boff, uint64_t* __restrict__ ooff, uint64_t cap, rsa_nam* __restrict__ out,
          SiteDesc* __restrict__ desc, const uint64_t* __restrict__ roff, const uint32_t* __restrict__ rlen,
          const uint64_t* __restrict__ coff, const char* __restrict__ seq, char* __restrict__ seq_rc, int by_score) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * CP_WAVES + (threadIdx.x >> 6);
    if (r >= n_reads) return;                                // whole wave
    const bool resc = rescued[r] != 0;
    const rsa_nam* src = arena + (resc ? arena_base + rbase[r] : nsrc[r]);
    const uint32_t n = resc ? ncnt2[r] : ncnt1[r];
    const uint64_t o = boff[r / SS_TPB] + loc[r];          // k_seed_count + k_seed_scan
    if (lane == 0) ooff[r] = o;
    if (desc && n) {                                         // the read's reverse complement for k_sites
        const uint64_t ro = roff[r];
        const uint32_t len = rlen[r];
        for (uint32_t i = lane; i < len; i += 64)
            seq_rc[ro + i] = (char)rc_base((unsigned char)seq[ro + len - 1 - i]);
    }
    if (o + n > cap) return;
    auto put = [&](uint64_t at, const rsa_nam& x) {
        out[at] = x;
        if (!desc) return;
        SiteDesc d;
        d.read_off = roff[r];
        d.read_len = rlen[r];
        const uint64_t c0 = coff[x.ref_id];
        d.ref_off = c0;
        d.ref_len = (uint32_t)(coff[x.ref_id + 1] - c0);
        d.slot = (x.nam_id >= 0 && (uint32_t)x.nam_id < n) ? o + (uint64_t)x.nam_id : ~0ull;
        desc[at] = d;
    };
    if (by_score && n >= 2 && n <= 16) {
        const int i = lane;
        const float si = i < (int)n ? src[i].score : 0.0f;
        int rank = 0;
        for (int j = 0; j < (int)n; ++j) {
            const float sj = __shfl(si, j, 64);
            rank += (sj > si || (sj == si && j < i)) ? 1 : 0;
        }
        if (i < (int)n) put(o + rank, src[i]);
        return;
    }
    for (uint32_t i = lane; i < n; i += 64) put(o + i, src[i]);
}

// ---------------------------------------------------------------------------
// k_sites: per-NAM site checks, 16 lanes per final NAM.
// reverse_nam_if_needed (src/aln.cpp:60-93): the NAM's first and last k-mers
// against the reference, as is or with the read reversed; then, for the
// (reversed) NAM, extend_seed_part's test (aln.cpp:374-431): a read-length
// projection gets its Hamming distance and, when hd / len < 0.05 (float
// quotient, double compare), its mismatch positions.  The host then builds
// hamming_align's result without touching the reference.
// ---------------------------------------------------------------------------

typedef const __attribute__((address_space(1))) u32x4 GU4;   // global loads, not flat ones
typedef const __attribute__((address_space(1))) unsigned char GU8;
// a read and its reverse complement (k_compact writes the latter into the call's rc
// buffer, at the read's offset)
struct SiteRead {
    const char* s;
    int64_t rc_delta;          // rc buffer - read buffer (the same for every read of a call)
    int64_t len;
    __device__ __forceinline__ const char* side(bool rc) const { return s + (rc ? rc_delta : 0); }
    __device__ __forceinline__ unsigned char at(bool rc, int64_t i) const { return (unsigned char)side(rc)[i]; }
};

// G lanes per NAM (8 by default: 8 NAMs per wave; RSA_SITES_G=16 selects 16 lanes, 4
// NAMs a wave): a lane compares every G-th byte of a k-mer and 256 / G consecutive
// window positions of every 256-position chunk, and the group combines its ballot bits
// (in position order, so mismatch positions come out sorted without a sort)
template <int G>
__device__ __forceinline__ uint32_t grp_ballot(bool v) {
    const uint64_t b = __ballot(v);
    return (uint32_t)(b >> (threadIdx.x & (64 - G))) & ((1u << G) - 1u);
}

// site_kmer_eq for k <= 32, in two steps so that every load of a NAM's checks is in
// flight at once: KmerLoad holds the clamped spans and the lane's 32 / G byte pairs
// (positions lg + G t; a position past the span reads its first byte, valid memory, and
// is not compared)
template <int G> struct KmerLoad { uint32_t rl, ql; unsigned char r[32 / G], q[32 / G]; };
template <int G>
__device__ __forceinline__ KmerLoad<G> kmer_load(const char* ref, int64_t rlen, int64_t rpos, const SiteRead& rd,
                                                 bool rc, int64_t qpos, int k, int lg) {
    const uint64_t rp = (uint64_t)rpos, qp = (uint64_t)qpos;
    const uint64_t ra = rp > (uint64_t)rlen ? (uint64_t)rlen : rp, qa = qp > (uint64_t)rd.len ? (uint64_t)rd.len : qp;
    KmerLoad<G> x;
    x.rl = (uint32_t)min((uint64_t)k, (uint64_t)rlen - ra);
    x.ql = (uint32_t)min((uint64_t)k, (uint64_t)rd.len - qa);
    GU8* rb = (GU8*)(ref + ra);
    GU8* qb = (GU8*)(rd.side(rc) + qa);
#pragma unroll
    for (int t = 0; t < 32 / G; ++t) {
        const uint32_t j = (uint32_t)(lg + G * t) < x.rl ? (uint32_t)(lg + G * t) : 0u;
        x.r[t] = rb[j];
        x.q[t] = qb[j];
    }
    return x;
}
template <int G>
__device__ __forceinline__ bool kmer_test(const KmerLoad<G>& x, int lg) {
    bool bad = x.rl != x.ql;
#pragma unroll
    for (int t = 0; t < 32 / G; ++t)
        if ((uint32_t)(lg + G * t) < x.rl) bad |= x.r[t] != x.q[t];
    return grp_ballot<G>(bad) == 0;
}

// sub(ref, rpos, k) == sub(read view, qpos, k) with std::string::substr clamping
// (a position past the end -- negative ints included, as size_t -- gives "")
template <int G>
__device__ bool site_kmer_eq(const char* ref, int64_t rlen, int64_t rpos, const SiteRead& rd, bool rc, int64_t qpos,
                             int k, int lg) {
    const uint64_t rp = (uint64_t)rpos, qp = (uint64_t)qpos;
    const uint64_t ra = rp > (uint64_t)rlen ? (uint64_t)rlen : rp, qa = qp > (uint64_t)rd.len ? (uint64_t)rd.len : qp;
    const uint64_t rl = min((uint64_t)k, (uint64_t)rlen - ra), ql = min((uint64_t)k, (uint64_t)rd.len - qa);
    bool bad = rl != ql;
    if (!bad)                                  // every byte's load issued before any compare
        for (uint64_t j = lg; j < rl; j += G) bad |= (unsigned char)ref[ra + j] != rd.at(rc, (int64_t)(qa + j));
    return grp_ballot<G>(bad) == 0;
}

// Mismatch mask of 16 window positions x0 .. x0 + 15 (bit b: x0 + b < n and the
// reference byte differs from the oriented read byte).  Each side is two aligned
// 16-byte loads and a byte funnel: the window lies inside its contig and the reference
// buffer has 64 bytes of padding past the last one; the read buffer has SEQ_PAD bytes
// of padding before the first read and after the last.
__device__ __forceinline__ void load16(const char* p, uint32_t out[4]) {   // bytes p[0 .. 16), any alignment
    const uintptr_t a = (uintptr_t)p;
    GU4* q = (GU4*)(a & ~(uintptr_t)15);
    const u32x4 x = q[0], y = q[1];
    const bool w2 = (a & 8) != 0, w1 = (a & 4) != 0;
    const uint32_t sh = (uint32_t)a & 3u;
    // words (a >> 2) & 3 .. + 4 of the 32 loaded bytes: shift by two words, then by one
    const uint32_t t0 = w2 ? x.z : x.x, t1 = w2 ? x.w : x.y, t2 = w2 ? y.x : x.z, t3 = w2 ? y.y : x.w,
                   t4 = w2 ? y.z : y.x, t5 = w2 ? y.w : y.y;
    const uint32_t u0 = w1 ? t1 : t0, u1 = w1 ? t2 : t1, u2 = w1 ? t3 : t2, u3 = w1 ? t4 : t3, u4 = w1 ? t5 : t4;
    out[0] = __builtin_amdgcn_alignbyte(u1, u0, sh);
    out[1] = __builtin_amdgcn_alignbyte(u2, u1, sh);
    out[2] = __builtin_amdgcn_alignbyte(u3, u2, sh);
    out[3] = __builtin_amdgcn_alignbyte(u4, u3, sh);
}
__device__ __forceinline__ uint32_t window_mask16(const char* ref_win, const SiteRead& rd, bool rc, int64_t x0,
                                                  int64_t n) {
    const int64_t xl = x0 < n ? x0 : 0;        // past the read: load in range, mask nothing
    uint32_t r[4], q[4];
    load16(ref_win + xl, r);
    load16(rd.side(rc) + xl, q);
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t x = r[k] ^ q[k];
#pragma unroll
        for (int b = 0; b < 4; ++b) m |= ((x >> (8 * b)) & 0xFFu) ? (1u << (4 * k + b)) : 0u;
    }
    const int64_t left = n - x0;               // positions past the read end do not count
    return left >= 16 ? m : left <= 0 ? 0u : m & ((1u << left) - 1u);
}
// the mask of a lane's 256 / G positions x0 .. (bit b: position x0 + b)
template <int G>
__device__ __forceinline__ uint32_t window_mask(const char* ref_win, const SiteRead& rd, bool rc, int64_t x0,
                                                int64_t n) {
    if (G == 16) return window_mask16(ref_win, rd, rc, x0, n);
    const uint32_t lo = window_mask16(ref_win, rd, rc, x0, n);
    const uint32_t hi = window_mask16(ref_win, rd, rc, x0 + 16, n);
    return lo | (hi << 16);
}

// reads over 1024 bp: masks past the four kept in registers, out of line
template <int G>
__device__ __forceinline__ uint32_t window_mask_far(const char* ref_win, const SiteRead& rd, bool rc, int64_t x0) {
    return window_mask<G>(ref_win, rd, rc, x0, rd.len);
}

// sums / exclusive prefix sums over a G-lane group
template <int G>
__device__ __forceinline__ uint32_t grp_sum(uint32_t v) {
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, G);
    return v;
}
template <int G>
__device__ __forceinline__ uint32_t grp_excl_scan(uint32_t v, int lg) {
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, G);
        if (lg >= o) x += y;
    }
    return x - v;
}

// G lanes a NAM, 256 / G NAMs a block of 256 threads, a fixed grid walking the batch's
// NAMs.  A NAM's loads come in two rounds: the NAM with its descriptor (k_compact), then
// -- together -- the two k-mers of the orientation test and the read-length window of
// the NAM as it stands (the common outcome, aln.cpp:60-93 finds most NAMs consistent as
// they are); a reversed NAM loads its window again.  The kernel waits on memory most of
// its cycles, so 8 lanes a NAM (8 NAMs a wave, two 16-position masks a lane) keeps twice
// the NAMs' loads in flight per wave as 16 lanes did.  Pool space is taken with one
// atomic a block: same-address atomics from every wave serialise (one a wave made the
// kernel 2.7x slower than one a 16-NAM block, profiles/r05/sites_ab).
#define SITES_TPB 256
// waves a SIMD the register budget is sized for (RSA_SITES_WAVES at build time: 5 = 92
// VGPRs, what the compiler picks unasked; 6 = 80 with a few spills, 8 = 64 with more)
#ifndef RSA_SITES_WAVES
#define RSA_SITES_WAVES 5
#endif
// 8 lanes a NAM hold twice the window bytes a lane: 4 waves a SIMD (128 VGPRs) keep it
// out of scratch (5 spilled 36 registers)
template <int G> struct SitesWaves { static constexpr int value = G == 8 ? 4 : RSA_SITES_WAVES; };
template <int G>
__global__ void __launch_bounds__(SITES_TPB) __attribute__((amdgpu_waves_per_eu(SitesWaves<G>::value)))
k_sites(const rsa_nam* __restrict__ nams, const SiteDesc* __restrict__ desc, SeedHdr* __restrict__ err_hdr,
        uint64_t cap, const char* __restrict__ seq, const char* __restrict__ seq_rc, SeedIndexParams p,
        rsa_nam_site* __restrict__ sites,
        uint16_t* __restrict__ pool, uint64_t pool_cap, unsigned long long* __restrict__ pool_used, int ham,
        int h_match, int h_mismatch, int h_bonus) {
    constexpr int NB = SITES_TPB / G;            // NAMs a block
    constexpr int PL = 256 / G;                  // positions a lane of each 256-position chunk
    // a batch whose NAMs overflow the output was not compacted whole (k_compact skips
    // the reads past `cap`, so their descriptors were never written): no site checks
    // then -- the host reports RSA_ERR_CAPACITY and the caller asks again
    __shared__ uint32_t s_need[NB], s_base[NB];
    __shared__ unsigned long long s_at;
    const uint64_t total = (uint64_t)err_hdr->total <= cap ? (uint64_t)err_hdr->total : 0;
    const int lg = threadIdx.x & (G - 1), grp = threadIdx.x / G;
#ifdef RSA_SEED_PROF
    unsigned long long sp_acc[6] = {0, 0, 0, 0, 0, 0};
#endif
    for (uint64_t blk = blockIdx.x; blk * NB < total; blk += gridDim.x) {
    SPROF_T(t0);
    const uint64_t g0 = blk * NB + grp;
    const bool valid = g0 < total;
    const uint64_t g = valid ? g0 : total - 1;             // idle groups shadow the last NAM (ballots stay uniform)
    const rsa_nam nam = nams[g];
    const SiteDesc d = desc[g];
    const char* ref = p.ref + d.ref_off;
    const int64_t ref_len = (int64_t)d.ref_len;
    const SiteRead rd{seq + d.read_off, seq_rc - seq, (int64_t)d.read_len};
    const int k = p.k;
    bool is_rc = nam.is_rc != 0;
    int64_t qs = nam.query_start, qe = nam.query_end;
    // projected_ref_start = max(0, ref_start - query_start); projected_ref_end =
    // min(ref_end + |read| - query_end, |contig|) (size_t arithmetic, aln.cpp:374-431)
    auto proj = [&](int64_t q_s, int64_t q_e, int64_t& ps) {
        ps = max((int64_t)0, (int64_t)nam.ref_start - q_s);
        const uint64_t pe = min((uint64_t)((int64_t)nam.ref_end + rd.len - q_e), (uint64_t)ref_len);
        return pe - (uint64_t)ps == (uint64_t)rd.len;
    };
    int64_t ps = 0;
    bool hamming = proj(qs, qe, ps);
    // the window as the NAM stands and the two k-mers: every load issued before any
    // test.  A window that is not tested is loaded from the read itself and dropped (the
    // read buffer is padded past its last read; a short last contig is not)
    uint32_t m0 = window_mask<G>(hamming ? ref + ps : rd.s, rd, is_rc, PL * lg, rd.len);
    uint32_t flags;
    bool fwd_ok;
    if (k <= 32) {
        const KmerLoad<G> a = kmer_load<G>(ref, ref_len, nam.ref_start, rd, is_rc, qs, k, lg);
        const KmerLoad<G> b = kmer_load<G>(ref, ref_len, (int64_t)nam.ref_end - k, rd, is_rc, qe - k, k, lg);
        __builtin_amdgcn_sched_barrier(0);                 // every load above issued before the first test
        fwd_ok = kmer_test<G>(a, lg) & kmer_test<G>(b, lg);
    } else {
        fwd_ok = site_kmer_eq<G>(ref, ref_len, nam.ref_start, rd, is_rc, qs, k, lg) &
                 site_kmer_eq<G>(ref, ref_len, (int64_t)nam.ref_end - k, rd, is_rc, qe - k, k, lg);
    }
    if (!hamming) m0 = 0u;
    if (fwd_ok) {
        flags = 0;
    } else {
        const int64_t qs2 = rd.len - nam.query_end, qe2 = rd.len - nam.query_start;
        bool rev_ok;
        if (k <= 32) {
            const KmerLoad<G> a = kmer_load<G>(ref, ref_len, nam.ref_start, rd, !is_rc, qs2, k, lg);
            const KmerLoad<G> b = kmer_load<G>(ref, ref_len, (int64_t)nam.ref_end - k, rd, !is_rc, qe2 - k, k, lg);
            __builtin_amdgcn_sched_barrier(0);
            rev_ok = kmer_test<G>(a, lg) & kmer_test<G>(b, lg);
        } else {
            rev_ok = site_kmer_eq<G>(ref, ref_len, nam.ref_start, rd, !is_rc, qs2, k, lg) &
                     site_kmer_eq<G>(ref, ref_len, (int64_t)nam.ref_end - k, rd, !is_rc, qe2 - k, k, lg);
        }
        if (rev_ok) {
            flags = 1;
            is_rc = !is_rc;
            qs = qs2;
            qe = qe2;
            hamming = proj(qs, qe, ps);
            m0 = hamming ? window_mask<G>(ref + ps, rd, is_rc, PL * lg, rd.len) : 0u;
        } else {
            flags = 2;
            hamming = false;
        }
    }
    SPROF_T(t1);
    const int n = (int)rd.len;
    uint32_t hd = 0, mm_off = 0;
    uint32_t m1 = 0, m2 = 0, m3 = 0;             // this lane's masks, positions c * 256 + PL * lg + b
    bool want = false;
    // the mask of chunk c (256 positions): registers for the first four, loads again beyond
    auto mask_of = [&](int c) -> uint32_t {
        if (c < 4) return c == 0 ? m0 : c == 1 ? m1 : c == 2 ? m2 : m3;
        return window_mask_far<G>(ref + ps, rd, is_rc, 256 * (int64_t)c + PL * lg);
    };
    if (hamming) {
        flags |= RSA_SITE_HAMMING;
        hd = __popc(m0);
        // reads over 256 bp: the masks of positions 256 .. 1023 into registers too
#pragma nounroll
        for (int c = 1; 256 * c < n; ++c) {
            const uint32_t mc = window_mask<G>(ref + ps, rd, is_rc, 256 * (int64_t)c + PL * lg, rd.len);
            m1 = c == 1 ? mc : m1;
            m2 = c == 2 ? mc : m2;
            m3 = c == 3 ? mc : m3;
            hd += __popc(mc);
        }
        hd = grp_sum<G>(hd);
        want = (double)((float)hd / (float)rd.len) < 0.05;
    }
    // the pool's u16 words hold positions and hamming_align's segment ends: longer reads
    // leave the accepted window to the host (RSA_SITE_POOL_FULL: it recomputes it)
    const bool fits = n <= 65535;
    // pool space: a block-wide prefix over its NAMs and one atomic a block (positions:
    // n_mm words; hamming_align's result: a 6-word header and at most 2 n_mm + 3 ops of 2 words)
    const uint32_t need = (want && valid && fits) ? (ham ? 12u + 4u * hd : hd) : 0u;
    SPROF_T(t2);
    if (lg == 0) s_need[grp] = need;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int j = 0; j < NB; ++j) { s_base[j] = acc; acc += s_need[j]; }
        s_at = acc ? atomicAdd(pool_used, (unsigned long long)acc) : 0ull;
    }
    __syncthreads();
    SPROF_T(t3);
    if (want) {
        const unsigned long long at = s_at + s_base[grp];
        if (!fits || at + need > pool_cap) {
            flags |= RSA_SITE_POOL_FULL;
        } else if (!ham) {
            flags |= RSA_SITE_POSITIONS;
            mm_off = (uint32_t)at;
            uint32_t m = 0;
            for (int c = 0; 256 * c < n && m < hd; ++c) {
                uint32_t bits = mask_of(c);
                const uint32_t cnt = __popc(bits);
                uint32_t o = m + grp_excl_scan<G>(cnt, lg);
                while (bits) {
                    const int b = __builtin_ctz(bits);
                    bits &= bits - 1;
                    if (valid) pool[at + o] = (uint16_t)(256 * c + PL * lg + b);
                    ++o;
                }
                m += grp_sum<G>(cnt);
            }
        } else {
            // hamming_align (aligner.cpp:219-302) over the window just tested: the group walks
            // the mismatch positions in order (per-lane ballots) twice, every lane computing the
            // same values; lane 0 writes the result
            flags |= RSA_SITE_POSITIONS | RSA_SITE_ALIGNED;
            mm_off = (uint32_t)at;
            // 1. highest_scoring_segment (aligner.cpp:219-252), run by run: between mismatches
            //    the score only grows, so each run of matches needs one check at its end
            //    Only the lanes' position blocks holding a mismatch are visited (a group ballot
            //    of the lanes' masks, in position order): the others change nothing here.
            int start = 0, best_start = 0, best_end = 0, i = 0;
            int score = h_bonus, best = 0;
            for (int c = 0; 256 * c < n; ++c) {
                const uint32_t mc = mask_of(c);
                uint32_t nz = grp_ballot<G>(mc != 0u);
                while (nz) {
                    // lane li of the group holds positions 256 c + PL li .. + PL - 1
                    const int li = __builtin_ctz(nz);
                    nz &= nz - 1;
                    const int i0 = 256 * c + PL * li;
                    uint32_t bits = (uint32_t)__shfl((int)mc, li, G);
                    while (bits) {
                        const int m = i0 + __builtin_ctz(bits);
                        bits &= bits - 1;
                        if (m > i) {
                            score += h_match * (m - i);
                            if (score > best) { best_start = start; best = score; best_end = m; }
                        }
                        score -= h_mismatch;
                        if (score < 0) { start = m + 1; score = 0; }
                        if (score > best) { best_start = start; best = score; best_end = m + 1; }
                        i = m + 1;
                    }
                }
            }
            if (n > i) {
                score += h_match * (n - i);
                if (score > best) { best_start = start; best = score; best_end = n; }
            }
            if (score + h_bonus > best) { best = score + h_bonus; best_end = n; best_start = start; }
            // 2. the CIGAR (S, =/X runs of the segment, S) with Cigar::push's merging, and the
            //    mismatches inside the segment
            uint32_t n_ops = 0, last = 0, ed = 0;
            bool have = false;
            auto push = [&](uint32_t op, uint32_t len) {
                if (have && (last & 0xf) == op) { last += len << 4; return; }
                if (have && lg == 0 && valid) {
                    pool[at + 6 + 2 * n_ops] = (uint16_t)(last & 0xFFFF);
                    pool[at + 7 + 2 * n_ops] = (uint16_t)(last >> 16);
                }
                n_ops += have ? 1 : 0;
                last = (len << 4) | op;
                have = true;
            };
            if (best_start > 0) push(4, (uint32_t)best_start);
            int cur = best_start;
            for (int c = best_start >> 8; 256 * c < best_end; ++c) {
                // this lane's positions in [best_start, best_end) only, blocks with a mismatch visited
                const int p0 = 256 * c + PL * lg;
                uint32_t mine = mask_of(c);
                const int lo = best_start - p0, hi = best_end - p0;
                if (lo >= PL || hi <= 0) mine = 0u;
                else {
                    if (lo > 0) mine &= ~((1u << lo) - 1u);
                    if (hi < PL) mine &= (1u << hi) - 1u;
                }
                uint32_t nz = grp_ballot<G>(mine != 0u);
                while (nz) {
                    const int li = __builtin_ctz(nz);
                    nz &= nz - 1;
                    const int i0 = 256 * c + PL * li;
                    uint32_t bits = (uint32_t)__shfl((int)mine, li, G);
                    while (bits) {
                        const int m = i0 + __builtin_ctz(bits);
                        bits &= bits - 1;
                        if (m > cur) push(7, (uint32_t)(m - cur));
                        push(8, 1);
                        ed++;
                        cur = m + 1;
                    }
                }
            }
            if (best_end > cur) push(7, (uint32_t)(best_end - cur));
            if (n - best_end > 0) push(4, (uint32_t)(n - best_end));
            if (have && lg == 0 && valid) {
                pool[at + 6 + 2 * n_ops] = (uint16_t)(last & 0xFFFF);
                pool[at + 7 + 2 * n_ops] = (uint16_t)(last >> 16);
            }
            n_ops += have ? 1 : 0;
            if (lg == 0 && valid) {
                pool[at + 0] = (uint16_t)((uint32_t)best & 0xFFFF);
                pool[at + 1] = (uint16_t)((uint32_t)best >> 16);
                pool[at + 2] = (uint16_t)best_start;
                pool[at + 3] = (uint16_t)best_end;
                pool[at + 4] = (uint16_t)ed;
                pool[at + 5] = (uint16_t)n_ops;
            }
        }
    }
    SPROF_T(t4);
    if (valid && lg == 0) {
        rsa_nam_site out;
        out.flags = (uint8_t)flags;
        out.orig_is_rc = (uint8_t)(nam.is_rc != 0);
        out.n_mm = (uint16_t)min(hd, 65535u);
        out.mm_offset = mm_off;
        out.orig_query_start = nam.query_start;
        out.orig_query_end = nam.query_end;
        // at the NAM's index in its read's list as found (nam_id; the NAMs may come sorted);
        // a nam_id outside the list would alias another NAM's slot: no write, the call fails
        if (d.slot != ~0ull) sites[d.slot] = out;
        else atomicOr(&err_hdr->errors, SEED_E_SITE);
    }
    __syncthreads();                             // s_need / s_base / s_at are reused next round
#ifdef RSA_SEED_PROF
    SPROF_T(t5);
    sp_acc[0] += t1 - t0; sp_acc[1] += t2 - t1; sp_acc[2] += t3 - t2; sp_acc[3] += t4 - t3; sp_acc[4] += t5 - t4;
    sp_acc[5] += 1;
#endif
    }
#ifdef RSA_SEED_PROF
    const int wv = (int)(threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096)
        for (int i = 0; i < 6; ++i) g_sites_prof[blockIdx.x * 4 + wv][i] = (unsigned int)sp_acc[i];
#endif
}

// lanes per NAM of k_sites (RSA_SITES_G=8/16 fixes it; read per call).  By default 8 for
// reads of <= 192 bp on average, 16 above: in-bench launches (profiles/r06/ab_setprio_sites*.json)
// 2 x 150 bp 211 -> 179 us with 8, 2 x 250 bp 371 -> 421 us (a wave's 8 groups walk more
// mismatches each in hamming_align, and the serial walks diverge)
static int sites_lanes(uint64_t bases, uint32_t n) {
    const char* e = getenv("RSA_SITES_G");
    if (e && (atoi(e) == 8 || atoi(e) == 16)) return atoi(e);
    return bases <= 192ull * n ? 8 : 16;
}

// ---------------------------------------------------------------------------
// k_bucket_lines: the BucketLine copy of the bucket table (rsa_seed.h), eight
// lanes a line, each writing 16 contiguous bytes (bounds, then entry slot - 1)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_bucket_lines(const uint64_t* __restrict__ starts, const rsa_ref_randstrobe* __restrict__ rs, uint64_t n_buckets,
               uint4* __restrict__ lines) {
    const uint64_t total = n_buckets * 8;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t bk = t >> 3;
        const uint32_t s = (uint32_t)(t & 7);
        const uint64_t a = starts[bk], e = starts[bk + 1];
        uint4 v = make_uint4(0, 0, 0, 0);
        if (s == 0) v = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)e, (uint32_t)(e >> 32));
        else if (e - a <= BL_CAP && s - 1 < e - a) v = ((const uint4*)rs)[a + s - 1];
        lines[t] = v;
    }
}

hipError_t bucket_lines_build(const uint64_t* starts, const rsa_ref_randstrobe* rs, int bits, BucketLine* lines,
                              hipStream_t st) {
    const uint64_t nb = (uint64_t)1 << bits;
    const uint64_t threads = nb * 8;
    const unsigned grid = (unsigned)std::min<uint64_t>((threads + 255) / 256, 8192);
    k_bucket_lines<<<grid, 256, 0, st>>>(starts, rs, nb, (uint4*)lines);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e;
}

// ---------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------
enum {
    B_SEQ, B_ROFF, B_RLEN, B_QBASE, B_QRS, B_QCNT, B_SYNC, B_QI, B_ST, B_X, B_ARENA, B_PHIT, B_POPEN, B_PGRP, B_PADD,
    B_NCNT1, B_FLAGS, B_MAP, B_NCNT2, B_NSRC, B_RBASE, B_BIGL, B_RBIGL, B_RBUF, B_OUT, B_SLOTS, B_SITES, B_POOL,
    B_NREAD, B_RSLIST, B_RLIST, B_LOC, B_BSUM, B_SEQRC
};
// every host side of a transfer is page-locked: a pageable one would make the copy synchronous
enum { H_X, H_QBASE, H_RSLIST };

void seed_bufs_release(SeedBufs& b) {
    for (int i = 0; i < SEED_NBUF; ++i) if (b.p[i]) (void)hipFree(b.p[i]);
    for (int i = 0; i < SEED_NHBUF; ++i) if (b.h[i]) (void)hipHostFree(b.h[i]);
    for (int i = 0; i < SEED_NBUF; ++i) { b.p[i] = nullptr; b.cap[i] = 0; }
    for (int i = 0; i < SEED_NHBUF; ++i) { b.h[i] = nullptr; b.hcap[i] = 0; }
    if (b.done) (void)hipEventDestroy(b.done);
    b.done = nullptr;
}

static hipError_t dens(SeedBufs& b, int i, size_t bytes) {
    bytes = std::max<size_t>(bytes, 64);
    if (bytes <= b.cap[i]) return hipSuccess;
    if (b.p[i]) (void)hipFree(b.p[i]);
    size_t n = std::max(bytes, b.cap[i] + b.cap[i] / 2);
    hipError_t e = hipMalloc(&b.p[i], n);
    if (e != hipSuccess) { b.p[i] = nullptr; b.cap[i] = 0; return e; }
    b.cap[i] = n;
    return rsa_poison(b.p[i], n);
}

static hipError_t hens(SeedBufs& b, int i, size_t bytes) {
    bytes = std::max<size_t>(bytes, 64);
    if (bytes <= b.hcap[i]) return hipSuccess;
    if (b.h[i]) (void)hipHostFree(b.h[i]);
    size_t n = std::max(bytes, b.hcap[i] + b.hcap[i] / 2);
    hipError_t e = hipHostMalloc(&b.h[i], n, hipHostMallocDefault);
    if (e != hipSuccess) { b.h[i] = nullptr; b.hcap[i] = 0; return e; }
    b.hcap[i] = n;
    return hipSuccess;
}

#define SCHK(x)                                                        \
    do {                                                               \
        hipError_t e_ = (x);                                           \
        if (e_ != hipSuccess) { err = std::string(#x) + ": " + hipGetErrorString(e_); return RSA_ERR_HIP; } \
    } while (0)
#define DP(i, T) ((T*)b.p[i])
// the reads sit SEQ_PAD bytes into B_SEQ, with as many after them: k_sites reads 16-byte
// windows by aligned dwords that may start or end up to 19 bytes outside a read
#define SEQ_PAD 64
#define D_SEQ ((char*)b.p[B_SEQ] + SEQ_PAD)
#define D_SEQRC ((char*)b.p[B_SEQRC] + SEQ_PAD)     // reverse complements, at the reads' offsets (k_compact)
#define HP(i, T) ((T*)b.h[i])

static const uint32_t MAP_BIG = 65536 + 512;

// Stage 1 (shared by rsa_randstrobes and rsa_seed): upload reads, run k_randstrobes.
int seed_stage_randstrobes(SeedBufs& b, hipStream_t st, const SeedIndexParams& p, const rsa_read_batch* rb,
                           std::vector<uint64_t>& qbase, std::string& err, KTimer* kt) {
    const uint32_t n = rb->n_reads;
    qbase.assign(n + 1, 0);
    uint64_t total_len = 0;
    for (uint32_t i = 0; i < n; ++i) {
        qbase[i + 1] = qbase[i] + 2ull * rb->lengths[i];
        total_len = std::max<uint64_t>(total_len, rb->offsets[i] + rb->lengths[i]);
    }
    SCHK(dens(b, B_SEQ, total_len + 2 * SEQ_PAD));
    SCHK(dens(b, B_ROFF, 8ull * n));
    SCHK(dens(b, B_RLEN, 4ull * n));
    SCHK(dens(b, B_QBASE, 8ull * (n + 1)));
    SCHK(dens(b, B_QRS, sizeof(rsa_query_randstrobe) * (qbase[n] + 1)));
    SCHK(dens(b, B_QCNT, 4ull * n));
    SCHK(hipMemcpyAsync(D_SEQ, rb->seq, total_len, hipMemcpyHostToDevice, st));
    SCHK(hipMemcpyAsync(b.p[B_ROFF], rb->offsets, 8ull * n, hipMemcpyHostToDevice, st));
    SCHK(hipMemcpyAsync(b.p[B_RLEN], rb->lengths, 4ull * n, hipMemcpyHostToDevice, st));
    SCHK(hens(b, H_QBASE, 8ull * (n + 1)));
    memcpy(b.h[H_QBASE], qbase.data(), 8ull * (n + 1));
    SCHK(hipMemcpyAsync(b.p[B_QBASE], b.h[H_QBASE], 8ull * (n + 1), hipMemcpyHostToDevice, st));
    // one wave per read (k_rs_wave); reads longer than RW_MAXLEN, and parameters
    // outside its window / k-mer limits, one lane per read (k_randstrobes)
    const bool wave_ok = p.k <= 32 && p.s <= 32 && p.s >= 1 && p.k - p.s + 1 <= RW_WMAX && p.k - p.s + 1 >= 1;
    uint32_t n_long = 0;
    for (uint32_t i = 0; i < n; ++i) n_long += rb->lengths[i] > RW_MAXLEN ? 1 : 0;
    const int* lane_list = nullptr;
    uint32_t n_lane = wave_ok ? n_long : n;
    if (wave_ok && n_long) {
        SCHK(hens(b, H_RSLIST, 4ull * n_long));
        int* hl = HP(H_RSLIST, int);
        uint32_t at = 0;
        for (uint32_t i = 0; i < n; ++i) if (rb->lengths[i] > RW_MAXLEN) hl[at++] = (int)i;
        SCHK(dens(b, B_RSLIST, 4ull * n_long));
        SCHK(hipMemcpyAsync(b.p[B_RSLIST], hl, 4ull * n_long, hipMemcpyHostToDevice, st));
        lane_list = DP(B_RSLIST, int);
    }
    if (kt) kt->begin(st, RSA_K_RANDSTROBES);
    if (wave_ok)
        hipLaunchKernelGGL(k_rs_wave, dim3((n + RW_WAVES - 1) / RW_WAVES), dim3(64 * RW_WAVES), 0, st, D_SEQ,
                           DP(B_ROFF, uint64_t), DP(B_RLEN, uint32_t), DP(B_QBASE, uint64_t), (int)n, p,
                           DP(B_QRS, rsa_query_randstrobe), DP(B_QCNT, uint32_t));
    if (n_lane) {
        SCHK(dens(b, B_SYNC, sizeof(SyncD) * (qbase[n] / 2 + 1)));
        if (p.k - p.s + 1 == 5)
            hipLaunchKernelGGL(k_randstrobes<5>, dim3((n_lane + 63) / 64), dim3(64), 0, st, D_SEQ,
                               DP(B_ROFF, uint64_t), DP(B_RLEN, uint32_t), DP(B_QBASE, uint64_t), (int)n_lane,
                               lane_list, p, DP(B_SYNC, SyncD), DP(B_QRS, rsa_query_randstrobe), DP(B_QCNT, uint32_t));
        else
            hipLaunchKernelGGL(k_randstrobes<0>, dim3((n_lane + 63) / 64), dim3(64), 0, st, D_SEQ,
                               DP(B_ROFF, uint64_t), DP(B_RLEN, uint32_t), DP(B_QBASE, uint64_t), (int)n_lane,
                               lane_list, p, DP(B_SYNC, SyncD), DP(B_QRS, rsa_query_randstrobe), DP(B_QCNT, uint32_t));
    }
    SCHK(hipGetLastError());
    if (kt) kt->end(st);
    return RSA_OK;
}

int seed_randstrobes_run(SeedBufs& b, hipStream_t st, const SeedIndexParams& p, const rsa_read_batch* rb,
                         rsa_randstrobe_batch* out, std::string& err) {
    const uint32_t n = rb->n_reads;
    std::vector<uint64_t> qbase;
    int rc = seed_stage_randstrobes(b, st, p, rb, qbase, err, nullptr);
    if (rc) return rc;
    std::vector<uint32_t> cnt(n);
    SCHK(hipMemcpyAsync(cnt.data(), b.p[B_QCNT], 4ull * n, hipMemcpyDeviceToHost, st));
    SCHK(stream_wait(st, b.done));
    uint64_t tot = 0;
    for (uint32_t i = 0; i < n; ++i) { out->offsets[i] = tot; tot += cnt[i]; }
    out->offsets[n] = tot;
    out->needed = tot;
    if (tot > out->capacity) { err = "rsa_randstrobes: output too small"; return RSA_ERR_CAPACITY; }
    std::vector<rsa_query_randstrobe> all(qbase[n] + 1);
    SCHK(hipMemcpyAsync(all.data(), b.p[B_QRS], sizeof(rsa_query_randstrobe) * qbase[n], hipMemcpyDeviceToHost, st));
    SCHK(stream_wait(st, b.done));
    for (uint32_t i = 0; i < n; ++i)
        memcpy(out->out + out->offsets[i], all.data() + qbase[i], sizeof(rsa_query_randstrobe) * cnt[i]);
    return RSA_OK;
}

// Byte layout of the call's packed device/host block B_X / H_X: the header and the
// read table go up in one copy, the header and the per-read results come down in one.
struct XLayout {
    size_t roff, rlen, qbase, rsl, up, ooff, nonrep, resc, down;
    XLayout(uint32_t n, uint32_t n_long) {
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        roff = al(sizeof(SeedHdr));
        rlen = al(roff + 8ull * n);
        qbase = al(rlen + 4ull * n);
        rsl = al(qbase + 8ull * (n + 1));
        up = rsl + 4ull * n_long;
        ooff = al(up);
        nonrep = al(ooff + 8ull * (n + 1));
        resc = al(nonrep + 4ull * n);
        down = resc + n;
    }
};

static const uint32_t MAP_BIG_LANES = BIG_LANES;

// rsa_seed: every kernel of the call is queued before the host waits once.  The
// per-read counts the kernels need from each other stay on the device (fixed NAM
// slots for k_find_nams_w2, device lists for the global-map passes, a pool for
// their variable-size scratch, a device scan for the final offsets); the host gets
// the header, offsets, NAMs, site checks and mismatch positions back in one round
// trip.  A second round trip is needed only when a guessed download size was too
// small; a pool that ran out is grown and the call runs again.
int seed_run(SeedBufs& b, hipStream_t st, KTimer& kt, const SeedIndexParams& p, const rsa_read_batch* rb,
             int32_t rescue_level, uint32_t rescue_cutoff, rsa_nam_batch* out, std::string& err, SeedCounters& c) {
    const uint32_t n = rb->n_reads;
    if (rsa_poison_every())                       // tests: nothing an earlier call wrote survives
        for (int i = 0; i < SEED_NBUF; ++i)
            if (b.p[i]) SCHK(hipMemsetAsync(b.p[i], 0xA5, b.cap[i], st));
    // reads longer than RW_MAXLEN (and parameters k_rs_wave cannot take) go one lane per read
    const bool wave_ok = p.k <= 32 && p.s <= 32 && p.s >= 1 && p.k - p.s + 1 <= RW_WMAX && p.k - p.s + 1 >= 1;
    uint32_t n_long = 0;
    uint64_t total_len = 0, bases = 0;
    for (uint32_t i = 0; i < n; ++i) {
        n_long += rb->lengths[i] > RW_MAXLEN ? 1 : 0;
        total_len = std::max<uint64_t>(total_len, rb->offsets[i] + rb->lengths[i]);
        bases += rb->lengths[i];
    }
    const uint32_t n_lane = wave_ok ? n_long : n;
    const XLayout X(n, wave_ok ? n_long : 0);
    // RSA_SEED_QW (tests): 1 = k_seed_query writes the randstrobes of the reads it predicts
    // the global-map / rescue passes need, 0 = of none (query_lane makes them), 2 = of all
    const char* qwv = getenv("RSA_SEED_QW");
    const int qw_mode = qwv ? atoi(qwv) : 1;
    SCHK(hens(b, H_X, X.down));
    char* hx = (char*)b.h[H_X];
    memcpy(hx + X.roff, rb->offsets, 8ull * n);
    memcpy(hx + X.rlen, rb->lengths, 4ull * n);
    uint64_t* hq = (uint64_t*)(hx + X.qbase);
    hq[0] = 0;
    for (uint32_t i = 0; i < n; ++i) hq[i + 1] = hq[i] + 2ull * rb->lengths[i];
    const uint64_t nq_cap = hq[n];
    if (wave_ok && n_long) {
        int* hl = (int*)(hx + X.rsl);
        uint32_t at = 0;
        for (uint32_t i = 0; i < n; ++i) if (rb->lengths[i] > RW_MAXLEN) hl[at++] = (int)i;
    }
    if (b.pool_n < 4ull * n + 65536) b.pool_n = 4ull * n + 65536;
    const uint64_t slots = (uint64_t)n * FN2_HCAP;
    const uint64_t cap = out->capacity;
    SCHK(dens(b, B_SEQ, total_len + 2 * SEQ_PAD));
    SCHK(dens(b, B_X, X.down));
    SCHK(dens(b, B_QRS, sizeof(rsa_query_randstrobe) * (nq_cap + 1)));
    SCHK(dens(b, B_QCNT, 4ull * n));
    SCHK(dens(b, B_QI, sizeof(QrsInfo) * (nq_cap + 1)));
    SCHK(dens(b, B_ST, sizeof(ReadStat) * n));
    SCHK(dens(b, B_SLOTS, sizeof(HitD) * LK_HCAP * (size_t)n));
    SCHK(dens(b, B_NCNT1, 4ull * n));
    SCHK(dens(b, B_NCNT2, 4ull * n));
    SCHK(dens(b, B_FLAGS, 4ull * n));
    SCHK(dens(b, B_NSRC, 8ull * n));
    SCHK(dens(b, B_RBASE, 8ull * n));
    SCHK(dens(b, B_BIGL, 4ull * n));
    SCHK(dens(b, B_RBIGL, 4ull * n));
    SCHK(dens(b, B_RLIST, 4ull * n));
    SCHK(dens(b, B_LOC, 4ull * n));                                        // k_seed_count: offsets in a workgroup
    SCHK(dens(b, B_BSUM, 8ull * ((n + SS_TPB - 1) / SS_TPB + 1)));          // workgroup totals -> offsets
    SCHK(dens(b, B_RBUF, sizeof(RescueD) * (nq_cap + 1)));
    SCHK(dens(b, B_MAP, (size_t)MAP_BIG * 9 * 4 * MAP_BIG_LANES));
    SCHK(dens(b, B_OUT, sizeof(rsa_nam) * (cap + 1)));
    if (out->sites) {
        SCHK(dens(b, B_NREAD, sizeof(SiteDesc) * (cap + 1)));       // per-NAM site descriptors
        SCHK(dens(b, B_SEQRC, total_len + 2 * SEQ_PAD));
        SCHK(dens(b, B_SITES, sizeof(rsa_nam_site) * (cap + 1)));
        SCHK(dens(b, B_POOL, 2 * std::max<uint64_t>(1, out->mm_capacity)));
    }
    char* dx = (char*)b.p[B_X];
    SeedHdr* dhdr = (SeedHdr*)dx;
    const uint64_t* d_roff = (const uint64_t*)(dx + X.roff);
    const uint32_t* d_rlen = (const uint32_t*)(dx + X.rlen);
    const uint64_t* d_qbase = (const uint64_t*)(dx + X.qbase);
    uint64_t* d_ooff = (uint64_t*)(dx + X.ooff);
    float* d_nonrep = (float*)(dx + X.nonrep);
    uint8_t* d_resc = (uint8_t*)(dx + X.resc);
    SCHK(hipMemcpyAsync(D_SEQ, rb->seq, total_len, hipMemcpyHostToDevice, st));
    SeedHdr hh;
    for (int attempt = 0;; ++attempt) {
        SCHK(dens(b, B_ARENA, sizeof(rsa_nam) * (slots + b.pool_n)));
        SCHK(dens(b, B_PHIT, sizeof(HitD) * b.pool_n));
        SCHK(dens(b, B_POPEN, sizeof(rsa_nam) * b.pool_n));
        SCHK(dens(b, B_PGRP, sizeof(HitD) * b.pool_n));
        SCHK(dens(b, B_PADD, b.pool_n));
        const SeedPool pool{DP(B_PHIT, HitD), DP(B_POPEN, rsa_nam), DP(B_ARENA, rsa_nam) + slots, DP(B_PGRP, HitD),
                            DP(B_PADD, uint8_t), b.pool_n, slots};
        memset(hx, 0, sizeof(SeedHdr));             // counters start at zero (a retry re-zeroes them)
        SCHK(hipMemcpyAsync(dx, hx, X.up, hipMemcpyHostToDevice, st));
        // 1. reads the fused kernel does not take (longer than RW_MAXLEN, or parameters
        //    outside its limits): randstrobes one lane per read (randstrobes.cpp:207-253)
        const int* lane_list = wave_ok ? (const int*)(dx + X.rsl) : nullptr;
        if (n_lane) {
            kt.begin(st, RSA_K_RANDSTROBES);
            SCHK(dens(b, B_SYNC, sizeof(SyncD) * (nq_cap / 2 + 1)));
            if (p.k - p.s + 1 == 5)
                hipLaunchKernelGGL(k_randstrobes<5>, dim3((n_lane + 63) / 64), dim3(64), 0, st, D_SEQ, d_roff,
                                   d_rlen, d_qbase, (int)n_lane, lane_list, p, DP(B_SYNC, SyncD),
                                   DP(B_QRS, rsa_query_randstrobe), DP(B_QCNT, uint32_t));
            else
                hipLaunchKernelGGL(k_randstrobes<0>, dim3((n_lane + 63) / 64), dim3(64), 0, st, D_SEQ, d_roff,
                                   d_rlen, d_qbase, (int)n_lane, lane_list, p, DP(B_SYNC, SyncD),
                                   DP(B_QRS, rsa_query_randstrobe), DP(B_QCNT, uint32_t));
            SCHK(hipGetLastError());
            kt.end(st);
        }
        // 2. randstrobes + lookups + the min_diff hits (randstrobes.cpp:207-253, index.hpp:57-93,
        //    nam.cpp:68-85): fused, one wave a read; the lane-walked reads through k_lookup
        kt.begin(st, RSA_K_LOOKUP);
        if (wave_ok)
            hipLaunchKernelGGL(k_seed_query, dim3((n + RW_WAVES - 1) / RW_WAVES), dim3(64 * RW_WAVES), 0, st,
                               D_SEQ, d_roff, d_rlen, d_qbase, (int)n, p, rescue_level, qw_mode,
                               DP(B_QRS, rsa_query_randstrobe), DP(B_QCNT, uint32_t), DP(B_QI, QrsInfo),
                               DP(B_ST, ReadStat), DP(B_SLOTS, HitD));
        if (n_lane)
            hipLaunchKernelGGL(k_lookup, dim3((n_lane + 3) / 4), dim3(256), 0, st, DP(B_QRS, rsa_query_randstrobe),
                               DP(B_QCNT, uint32_t), d_qbase, (int)n_lane, lane_list, p, DP(B_QI, QrsInfo),
                               DP(B_ST, ReadStat), DP(B_SLOTS, HitD));
        SCHK(hipGetLastError());
        kt.end(st);
        // 3. find_nams (nam.cpp:771-926): LDS maps, then the listed reads with global maps
        kt.begin(st, RSA_K_FIND_NAMS);
        hipLaunchKernelGGL(k_find_nams_w2, dim3((n + FN2_WAVES - 1) / FN2_WAVES), dim3(64 * FN2_WAVES), 0, st,
                           DP(B_ST, ReadStat), DP(B_SLOTS, HitD), (int)n, p, DP(B_ARENA, rsa_nam),
                           DP(B_NCNT1, uint32_t), d_nonrep, DP(B_FLAGS, uint32_t), DP(B_NSRC, uint64_t), dhdr,
                           DP(B_BIGL, uint32_t));
        hipLaunchKernelGGL(k_find_nams_big, dim3(1), dim3(64), 0, st, DP(B_QRS, rsa_query_randstrobe),
                           DP(B_QI, QrsInfo), DP(B_QCNT, uint32_t), d_qbase, DP(B_ST, ReadStat), D_SEQ, d_roff,
                           d_rlen, RescueScratch{DP(B_RBUF, RescueD)}, p, pool,
                           DP(B_MAP, uint8_t), MAP_BIG, DP(B_NCNT1, uint32_t), d_nonrep, DP(B_FLAGS, uint32_t),
                           DP(B_NSRC, uint64_t), dhdr, DP(B_BIGL, uint32_t));
        SCHK(hipGetLastError());
        kt.end(st);
        // 4. rescue (aln.cpp:1954-1962, nam.cpp:955-1012)
        kt.begin(st, RSA_K_RESCUE);
        hipLaunchKernelGGL(k_rescue_select, dim3((n + 255) / 256), dim3(256), 0, st, (int)n, rescue_level,
                           DP(B_ST, ReadStat), DP(B_NCNT1, uint32_t), d_nonrep, DP(B_NCNT2, uint32_t),
                           DP(B_RBASE, uint64_t), d_resc, b.pool_n, dhdr, DP(B_RLIST, uint32_t));
        if (wave_ok)
            hipLaunchKernelGGL(k_query_fix, dim3(1), dim3(64), 0, st, DP(B_RLIST, uint32_t), dhdr, D_SEQ, d_roff,
                               d_rlen, d_qbase, p, RescueScratch{DP(B_RBUF, RescueD)},
                               DP(B_QRS, rsa_query_randstrobe), DP(B_QI, QrsInfo), DP(B_ST, ReadStat));
        // the persistent rescue walk is sized from the lane's last call (rescue is rare on
        // most inputs -- a few reads a call on the headline -- and 256 idle 52-KB-LDS
        // workgroups still queue behind the other lanes' kernels); the grid-stride loop
        // takes any count
        const uint32_t resc_grid =
            b.resc_rate < 0 ? RESCUE_GRID
                            : (uint32_t)std::min<double>(RESCUE_GRID, std::max(8.0, std::ceil(1.5 * b.resc_rate * n / FN_WAVES)));
        hipLaunchKernelGGL(k_rescue_w, dim3(resc_grid), dim3(64 * FN_WAVES), 0, st, DP(B_QRS, rsa_query_randstrobe),
                           DP(B_QI, QrsInfo), DP(B_QCNT, uint32_t), d_qbase, p, rescue_cutoff, DP(B_RBUF, RescueD),
                           pool, DP(B_NCNT2, uint32_t), DP(B_FLAGS, uint32_t), DP(B_RBASE, uint64_t), dhdr,
                           DP(B_RLIST, uint32_t), DP(B_RBIGL, uint32_t));
        hipLaunchKernelGGL(k_rescue_big, dim3(1), dim3(64), 0, st, DP(B_QRS, rsa_query_randstrobe), DP(B_QI, QrsInfo),
                           DP(B_QCNT, uint32_t), d_qbase, p, rescue_cutoff, DP(B_RBUF, RescueD), pool,
                           DP(B_MAP, uint8_t), MAP_BIG, DP(B_NCNT2, uint32_t), DP(B_FLAGS, uint32_t),
                           DP(B_RBASE, uint64_t), dhdr, DP(B_RBIGL, uint32_t));
        SCHK(hipGetLastError());
        kt.end(st);
        // 5. final offsets and the NAM lists back to back
        kt.begin(st, RSA_K_COMPACT);
        const int n_sblk = (int)((n + SS_TPB - 1) / SS_TPB);
        hipLaunchKernelGGL(k_seed_count, dim3(std::max(1, n_sblk)), dim3(SS_TPB), 0, st, (int)n, d_resc,
                           DP(B_NCNT1, uint32_t), DP(B_NCNT2, uint32_t), DP(B_QCNT, uint32_t), DP(B_ST, ReadStat),
                           DP(B_LOC, uint32_t), DP(B_BSUM, uint64_t), dhdr);
        hipLaunchKernelGGL(k_seed_scan, dim3(1), dim3(SS_TPB), 0, st, n_sblk, (int)n, DP(B_BSUM, uint64_t), d_ooff,
                           dhdr);
        hipLaunchKernelGGL(k_compact, dim3(std::max<uint32_t>(1, (n + CP_WAVES - 1) / CP_WAVES)), dim3(64 * CP_WAVES), 0, st, (int)n, DP(B_NSRC, uint64_t), DP(B_RBASE, uint64_t),
                           slots, DP(B_NCNT1, uint32_t), DP(B_NCNT2, uint32_t), d_resc, DP(B_ARENA, rsa_nam),
                           DP(B_LOC, uint32_t), DP(B_BSUM, uint64_t), d_ooff,
                           cap, DP(B_OUT, rsa_nam), out->sites ? DP(B_NREAD, SiteDesc) : nullptr, d_roff, d_rlen,
                           p.coff, D_SEQ, D_SEQRC, out->order == RSA_NAMS_BY_SCORE ? 1 : 0);
        SCHK(hipGetLastError());
        kt.end(st);
        // 6. site checks (aln.cpp:60-93, 374-431)
        if (out->sites) {
            kt.begin(st, RSA_K_SITES);
            const int sg = sites_lanes(bases, n);
            const uint64_t nb = SITES_TPB / sg;
            const uint32_t grid = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(1, (cap + nb - 1) / nb), 4096);
            if (sg == 16)
                hipLaunchKernelGGL(k_sites<16>, dim3(grid), dim3(SITES_TPB), 0, st, DP(B_OUT, rsa_nam), DP(B_NREAD, SiteDesc),
                                   dhdr, cap, D_SEQ, D_SEQRC, p, DP(B_SITES, rsa_nam_site), DP(B_POOL, uint16_t),
                                   out->mm_capacity, &dhdr->mm_used, out->hamming_align ? 1 : 0, out->match,
                                   out->mismatch, out->end_bonus);
            else
                hipLaunchKernelGGL(k_sites<8>, dim3(grid), dim3(SITES_TPB), 0, st, DP(B_OUT, rsa_nam), DP(B_NREAD, SiteDesc),
                                   dhdr, cap, D_SEQ, D_SEQRC, p, DP(B_SITES, rsa_nam_site), DP(B_POOL, uint16_t),
                                   out->mm_capacity, &dhdr->mm_used, out->hamming_align ? 1 : 0, out->match,
                                   out->mismatch, out->end_bonus);
            SCHK(hipGetLastError());
            kt.end(st);
        }
        // 7. one download of the header + per-read results, and the outputs up to a guessed size
        SCHK(hipMemcpyAsync(hx, dx, X.down, hipMemcpyDeviceToHost, st));
        // the first download's size: 8 NAMs a read, or 1.15 x the lane's last call's rate
        const uint64_t guess =
            std::min<uint64_t>(cap, (uint64_t)((double)n * std::max(8.0, 1.15 * b.nam_rate)) + 1024);
        SCHK(hipMemcpyAsync(out->nams, b.p[B_OUT], sizeof(rsa_nam) * guess, hipMemcpyDeviceToHost, st));
        // pool words copied before the total is known: ~1 accepted site a read, n_mm words each,
        // or 12 + 4 n_mm with hamming_align's results (or 1.15 x the last call's words a NAM)
        const double mm_a_nam = std::max((double)(out->hamming_align ? 3 : 1), 1.15 * b.mm_rate);
        const uint64_t mm_guess =
            out->sites ? std::min<uint64_t>(out->mm_capacity, (uint64_t)(mm_a_nam * (double)guess)) : 0;
        if (out->sites) {
            SCHK(hipMemcpyAsync(out->sites, b.p[B_SITES], sizeof(rsa_nam_site) * guess, hipMemcpyDeviceToHost, st));
            if (mm_guess) SCHK(hipMemcpyAsync(out->mm_pool, b.p[B_POOL], 2 * mm_guess, hipMemcpyDeviceToHost, st));
        }
        SCHK(stream_wait(st, b.done));
        memcpy(&hh, hx, sizeof hh);
        if (hh.errors & SEED_E_FIND) { err = "rsa_seed: robin_hood emulation overflow"; return RSA_ERR_NOMEM; }
        if (hh.errors & SEED_E_RESCUE) { err = "rsa_seed: rescue map overflow"; return RSA_ERR_NOMEM; }
        if (hh.errors & SEED_E_SITE) { err = "rsa_seed: site check for a NAM outside its read's list"; return RSA_ERR_INTERNAL; }
        if (hh.errors & SEED_E_POOL) {          // grow the pool and run the call again
            if (attempt >= 8) { err = "rsa_seed: seeding pool exhausted"; return RSA_ERR_NOMEM; }
            b.pool_n = std::max<uint64_t>(2 * b.pool_n, hh.pool_used + 1024);
            kt.reset();
            continue;
        }
        const uint64_t total = hh.total;
        out->needed = total;
        memcpy(out->offsets, hx + X.ooff, 8ull * (n + 1));
        memcpy(out->nonrepetitive_fraction, hx + X.nonrep, 4ull * n);
        memcpy(out->rescued, hx + X.resc, n);
        if (total > cap) { err = "rsa_seed: NAM output too small"; return RSA_ERR_CAPACITY; }
        const uint64_t mm_used = out->sites ? std::min<uint64_t>(hh.mm_used, out->mm_capacity) : 0;
        if (out->sites) out->mm_used = mm_used;
        else out->mm_used = 0;
        if (n) b.nam_rate = (double)total / (double)n;
        if (n) b.resc_rate = (double)hh.resc_reads / (double)n;
        if (total) b.mm_rate = (double)mm_used / (double)total;
        if (total > guess || mm_used > mm_guess) {   // rare: a second round trip for the rest
            c.second_trip = 1;
            if (total > guess) {
                SCHK(hipMemcpyAsync(out->nams + guess, DP(B_OUT, rsa_nam) + guess, sizeof(rsa_nam) * (total - guess),
                                    hipMemcpyDeviceToHost, st));
                if (out->sites)
                    SCHK(hipMemcpyAsync(out->sites + guess, DP(B_SITES, rsa_nam_site) + guess,
                                        sizeof(rsa_nam_site) * (total - guess), hipMemcpyDeviceToHost, st));
            }
            if (mm_used > mm_guess)
                SCHK(hipMemcpyAsync(out->mm_pool + mm_guess, DP(B_POOL, uint16_t) + mm_guess, 2 * (mm_used - mm_guess),
                                    hipMemcpyDeviceToHost, st));
            SCHK(stream_wait(st, b.done));
        }
        break;
    }
#ifdef RSA_SEED_PROF
    {
        static std::atomic<int> calls{0};
        if (++calls % 20 == 0) {
            static std::vector<unsigned int> h((size_t)SPROF_READS * 20);
            unsigned long long v[20] = {};
            if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_seed_prof), 4ull * h.size()) == hipSuccess) {
                for (size_t i = 0; i < std::min<size_t>(n, SPROF_READS); ++i)
                    for (int j = 0; j < 20; ++j) v[j] += h[i * 20 + j];
                const double qw = v[3] ? (double)v[3] : 1.0, fw = v[8] ? (double)v[8] : 1.0;
                fprintf(stderr, "seedprof query/wave cycles: syncmers %.0f lookups %.0f tail %.0f | find_nams/wave: "
                        "copy %.0f maps %.0f order %.0f merge %.0f | hits/read %.1f lists/read %.1f | lookup: pick %.0f fetch %.0f "
                        "emit %.0f (line wait %.0f, ballots %.0f, search %.0f, count %.0f; to indices %.0f, issue %.0f)\n",
                        v[0] / qw, v[1] / qw, v[2] / qw, v[4] / fw, v[5] / fw, v[6] / fw, v[7] / fw, v[9] / fw, v[10] / fw,
                        v[11] / qw, v[12] / qw, v[13] / qw, v[14] / qw, v[15] / qw, v[16] / qw, v[17] / qw, v[18] / qw,
                        v[19] / qw);
                static std::vector<unsigned int> hs((size_t)4096 * 4 * 8);
                unsigned long long u[8] = {};
                if (hipMemcpyFromSymbol(hs.data(), HIP_SYMBOL(g_sites_prof), 4ull * hs.size()) == hipSuccess) {
                    for (size_t i = 0; i < (size_t)4096 * 4; ++i)
                        for (int j = 0; j < 8; ++j) u[j] += hs[i * 8 + j];
                    const double rr = u[5] ? (double)u[5] : 1.0;
                    fprintf(stderr, "seedprof k_sites per wave-round cycles: loads+kmers %.0f window %.0f sync %.0f "
                            "pool/align %.0f tail %.0f | rounds %.0f\n", u[0] / rr, u[1] / rr, u[2] / rr, u[3] / rr,
                            u[4] / rr, rr);
                }
            }
        }
    }
#endif
    // counters and algorithmic bytes (DESIGN.md "Kernels")
    const uint64_t total = hh.total;
    const double QRS = sizeof(rsa_query_randstrobe), QI = sizeof(QrsInfo), RS = sizeof(rsa_ref_randstrobe),
                 NAM = sizeof(rsa_nam), HIT = sizeof(HitD);
    c.reads = n; c.read_bases = bases; c.qrs = hh.qrs; c.found = hh.found; c.filtered = hh.found - hh.good;
    c.hits = hh.hits_find; c.nams = total; c.rescued = hh.resc_reads; c.qw = hh.qw_q; c.qfix = hh.qfix;
    // fused (k_seed_query): the read bases and read table, per query randstrobe its bucket bounds,
    // the found entries, the hits into the slots, the per-read results; the randstrobes and
    // QrsInfo stay in registers (the predicted rescue / global-map reads aside: hh.qw_q)
    c.alg_bytes[RSA_K_RANDSTROBES] = 0;
    c.alg_bytes[RSA_K_LOOKUP] = (double)bases + 24.0 * n + 16.0 * hh.qrs + 8.0 * hh.found + RS * hh.scan_all +
                                HIT * hh.hits_find + sizeof(ReadStat) * (double)n + (QRS + QI) * hh.qw_q;
    // the hits from the read's slot (k_lookup wrote them), the NAMs, the per-read results
    c.alg_bytes[RSA_K_FIND_NAMS] = HIT * hh.hits_find + NAM * hh.n1 + (16.0 + sizeof(ReadStat)) * n;
    c.alg_bytes[RSA_K_RESCUE] = (QRS + QI) * hh.resc_q + RS * hh.resc_scan + 2 * HIT * hh.resc_hits + NAM * hh.n2;
    c.alg_bytes[RSA_K_COMPACT] = 2 * NAM * total + 28.0 * n;
    // NAM + read bytes read, window bytes compared, site + positions written
    if (out->sites)
        c.alg_bytes[RSA_K_SITES] = (double)total * (sizeof(rsa_nam) + sizeof(rsa_nam_site) + 2.0 * 20 + 150) +
                                   2.0 * (double)out->mm_used;
    return RSA_OK;
}
