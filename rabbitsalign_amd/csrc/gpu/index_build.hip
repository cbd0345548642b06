// index_build.hip -- StrobemerIndex::populate (src/index.cpp:141-309) on gfx950.
//
// The reference builds the .sti on the host: one thread per contig runs the
// SyncmerIterator / RandstrobeGenerator (index.cpp:28-69, 244-309,
// randstrobes.cpp:57-202), pdqsort orders the 16-B RefRandstrobe AoS by
// (hash, position) (index.cpp:168) and one sequential pass writes the bucket
// table and the repetitive-hash counts (index.cpp:174-238).  Here:
//
//  k_seg_syncmers    one lane per reference segment of SEG bases.  A segment's
//                    syncmers are those whose last base lies in it; the lane
//                    replays the iterator from a warm-up point before the
//                    segment (see "Warm-up" below), counting (passes 0/1) or
//                    writing (pass 2) them.
//  k_ref_randstrobes one lane per syncmer: RandstrobeGenerator::next, i.e. the
//                    minimum popcount((h1 ^ h2) & q) over the w_min..w_max
//                    following syncmers within max_dist (first minimum wins).
//  radix sorts       stable hipcub passes: by position, then by hash, so equal
//                    (hash, position) keys of two contigs stay in contig order
//                    (the host build's stable merge sort does the same; the
//                    reference's pdqsort leaves that order unspecified).
//  k_bucket_table    one lane per entry: the reference's fill rule, including
//                    its quirk that the first hash run's bucket points past that
//                    run (randstrobe_start_indices is only pushed at a hash change).
//  k_run_counts      one lane per hash run: unique count and a histogram of run
//                    lengths clamped to 101 -- enough to reproduce the filter
//                    cutoff (sorted counts[index_cutoff], clamped to [30, 100]).
//
// Warm-up.  The iterator's state after base i is (rolling k-/s-mer words, the
// window of the last k-s+1 s-mer hashes, its minimum, the position of the
// tracked minimum).  All but the tracked position are functions of the last k
// bases.  The tracked position depends on history only among tied minima
// (leftmost after a first fill, rightmost after a rescan, oldest while equal
// values arrive).  So once a full window has a unique minimum -- or an N resets
// both runs -- a run started anywhere earlier is in the same state as the run
// from the contig start.  Each segment replays WARM bases before its start and
// reports whether that happened; a segment that did not converge (a tandem
// repeat longer than WARM) is replayed from the warm-up point of the nearest
// earlier segment that did.  Every segment's syncmers therefore equal the
// sequential iterator's.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rsa_dev.h"
#include "../../../include/rsa_gpu.h"
#include "rsa_seed.h"
#include "../host/sti_order.hpp"

namespace {

constexpr uint64_t END64 = 0xFFFFFFFFFFFFFFFFULL;
constexpr int SEG = 4096;        // bases per segment lane
constexpr int WARM = 512;        // warm-up bases replayed before a segment
constexpr int TPB = 256;

struct BuildParams {
    int k, s, t, w_min, w_max, max_dist;
    uint64_t q;
};

struct SyncmerOut { uint64_t hash; uint32_t pos; uint32_t pad; };

// SyncmerIterator (randstrobes.cpp:57-118) as an explicit state machine.
// WC > 0: the window holds exactly WC s-mer hashes in registers; WC == 0: any
// window up to 32 in a ring.
template <int WC>
struct SyncState {
    uint64_t win[WC > 0 ? WC : 32];
    int qn = 0, qh = 0;
    uint64_t min_val = END64;
    long long min_pos = -1;
    int l = 0;
    uint64_t xk0 = 0, xk1 = 0, xs0 = 0, xs1 = 0;

    __device__ __forceinline__ uint64_t at(int j) const {
        if constexpr (WC > 0) {
            uint64_t v = win[0];
#pragma unroll
            for (int x = 1; x < WC; ++x) if (j == x) v = win[x];
            return v;
        } else {
            return win[(qh + j) & 31];
        }
    }
    // push; true when the window was full (its oldest value dropped)
    __device__ __forceinline__ bool push(uint64_t h, int W) {
        if constexpr (WC > 0) {
            // always shift in at the end (no store at a variable index, which
            // would move the window out of registers); while filling, the
            // window is read only once it is full, when the order is right
#pragma unroll
            for (int x = 0; x + 1 < WC; ++x) win[x] = win[x + 1];
            win[WC - 1] = h;
            if (qn < WC) { qn++; return false; }
            return true;
        } else {
            win[(qh + qn) & 31] = h;
            if (qn < W) { qn++; return false; }
            qh = (qh + 1) & 31;
            return true;
        }
    }
    __device__ __forceinline__ void reset() {
        min_val = END64; min_pos = -1; l = 0; xk0 = xk1 = xs0 = xs1 = 0; qn = 0; qh = 0;
    }
    // one base at contig position i: 1 and the syncmer when one ends here, 0
    // otherwise, -1 on a reset (a base outside ACGTU)
    __device__ __forceinline__ int step(int c, long long i, const BuildParams& p, int W, uint64_t kmask,
                                        uint64_t smask, int kshift, int sshift, SyncmerOut& out) {
        if (c >= 4) { reset(); return -1; }
        xk0 = ((xk0 << 2) | (uint64_t)c) & kmask;
        xk1 = (xk1 >> 2) | ((uint64_t)(3 - c) << kshift);
        xs0 = ((xs0 << 2) | (uint64_t)c) & smask;
        xs1 = (xs1 >> 2) | ((uint64_t)(3 - c) << sshift);
        if (++l < p.s) return 0;
        const uint64_t hs = xxh64_u64(xs0 < xs1 ? xs0 : xs1);
        const bool popped = push(hs, W);
        if (!popped) {
            if (qn < W) return 0;
            // WC > 0: constant trip counts, so the window stays in registers
#pragma unroll
            for (int j = 0; j < (WC > 0 ? WC : W); ++j) {   // first fill: leftmost minimum
                const uint64_t v = at(j);
                if (v < min_val) { min_val = v; min_pos = i - p.k + j + 1; }
            }
        } else if (min_pos == i - p.k) {                 // the minimum left: rescan, rightmost wins
            min_val = END64;
            min_pos = i - p.s + 1;
#pragma unroll
            for (int j = (WC > 0 ? WC : W) - 1; j >= 0; --j) {
                const uint64_t v = at(j);
                if (v < min_val) { min_val = v; min_pos = i - p.k + j + 1; }
            }
        } else if (hs < min_val) {
            min_val = hs;
            min_pos = i - p.s + 1;
        }
        if (min_pos == i - p.k + p.t) {
            out.hash = xxh64_u64(xk0 < xk1 ? xk0 : xk1);
            out.pos = (uint32_t)(i - p.k + 1);
            return 1;
        }
        return 0;
    }
    // a full window with a unique minimum: the state no longer depends on history
    __device__ __forceinline__ bool converged(int W) const {
        if (qn < W) return false;
        int eq = 0;
#pragma unroll
        for (int j = 0; j < (WC > 0 ? WC : W); ++j) eq += at(j) == min_val;
        return eq == 1;
    }
};

struct SegTable {
    const uint32_t* contig;     // [n_seg] contig of the segment
    const uint64_t* begin;      // [n_seg] first base (contig coordinates)
    const uint64_t* replay;     // [n_seg] replay start (contig coordinates); pass 0: unused
    const uint64_t* coff;       // [n_contigs + 1] contig offsets in ref
    uint64_t n_seg;
};

// mode 0: warm-up probe (converged flag + syncmer count); 1: count from the
// replay start; 2: write the syncmers at out[off[seg]..].  The reference
// buffer is 256-B aligned with 64 bytes of slack past its end (aligned loads
// never leave the allocation).
//
// Memory shape: a wave's lanes walk 64 segments 4 KB apart, so every load and
// store instruction touches 64 lines.  The bases come from aligned 64-byte
// blocks held in eight registers (one block per 64 steps: a line is fetched
// once instead of once per 16-byte load when it drops out of L2 between two),
// and the records are staged in LDS and stored in runs that end on 128-byte
// boundaries (whole lines, instead of one 16-byte partial-line store per record).
constexpr int SEG_STAGE = 8;      // records staged per lane (one 128-B line)
template <int WC>
__global__ void __launch_bounds__(TPB)
k_seg_syncmers(const char* __restrict__ ref, SegTable st, BuildParams p, int mode, uint32_t* __restrict__ count,
               uint8_t* __restrict__ conv, const uint64_t* __restrict__ off, SyncmerOut* __restrict__ out) {
    __shared__ SyncmerOut s_stage[SEG_STAGE * TPB];        // [slot][lane]: consecutive lanes, consecutive banks
    const uint64_t sg = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (sg >= st.n_seg) return;
    const uint32_t c = st.contig[sg];
    const char* cs = ref + st.coff[c];
    const uint64_t clen = st.coff[c + 1] - st.coff[c];
    const uint64_t b = st.begin[sg];
    const uint64_t e = b + SEG < clen ? b + SEG : clen;
    uint64_t from;
    bool ok;
    if (mode == 0) { from = b > (uint64_t)WARM ? b - WARM : 0; ok = from == 0; }
    else { from = st.replay[sg]; ok = true; }
    const int W = p.k - p.s + 1;
    const uint64_t kmask = (p.k == 32) ? ~0ULL : ((1ULL << (2 * p.k)) - 1);
    const uint64_t smask = (p.s == 32) ? ~0ULL : ((1ULL << (2 * p.s)) - 1);
    const int kshift = (p.k - 1) * 2, sshift = (p.s - 1) * 2;
    SyncState<WC> S;
    SyncmerOut sm;
    // the base stream: words w0..w7 of the current 64-B block (w0 next), `cur` the
    // word being consumed with `nb` bases left in it.  Plain locals rotated with
    // constant indices: an array picked by a run-time index, or a lambda capturing
    // them by reference, put the state in scratch.
    uint64_t w0, w1, w2, w3, w4, w5, w6, w7, cur;
    int nb, nw;
    uint64_t nexta;
#define SEG_LOAD(a_)                                                                  \
    do {                                                                              \
        const ulonglong2* q_ = reinterpret_cast<const ulonglong2*>(ref + (a_));       \
        const ulonglong2 v0_ = q_[0], v1_ = q_[1], v2_ = q_[2], v3_ = q_[3];          \
        w0 = v0_.x; w1 = v0_.y; w2 = v1_.x; w3 = v1_.y;                                \
        w4 = v2_.x; w5 = v2_.y; w6 = v3_.x; w7 = v3_.y;                                \
    } while (0)
#define SEG_ROT() do { w0 = w1; w1 = w2; w2 = w3; w3 = w4; w4 = w5; w5 = w6; w6 = w7; } while (0)
    {
        const uint64_t g = (uint64_t)(cs - ref) + from, a = g & ~63ull;
        SEG_LOAD(a);
        nexta = a + 64;
        nw = 8;
        for (unsigned k = (unsigned)((g - a) >> 3); k > 0; --k) { SEG_ROT(); --nw; }
        cur = w0;
        SEG_ROT();
        --nw;
        cur >>= (g & 7) * 8;
        nb = 8 - (int)(g & 7);
    }
#define SEG_NEXT()                                                                    \
    ({                                                                                \
        if (nb == 0) {                                                                \
            if (nw == 0) { SEG_LOAD(nexta); nexta += 64; nw = 8; }                    \
            cur = w0;                                                                 \
            SEG_ROT();                                                                \
            --nw;                                                                     \
            nb = 8;                                                                   \
        }                                                                             \
        const int c_ = nt4_code((unsigned char)(cur & 0xFF));                         \
        cur >>= 8;                                                                    \
        --nb;                                                                         \
        c_;                                                                           \
    })
    uint64_t i = from;
    for (; i < b; ++i) {                                   // replay, no output
        const int r = S.step(SEG_NEXT(), (long long)i, p, W, kmask, smask, kshift, sshift, sm);
        if (mode == 0 && !ok) ok = r < 0 || S.converged(W);
    }
    uint32_t n = 0;
    if (mode == 2) {
        SyncmerOut* o = out + off[sg];
        const uint64_t g0 = off[sg];                       // record index of o[0] in `out`
        int k = 0;                                         // records staged
        for (; i < e; ++i) {
            if (S.step(SEG_NEXT(), (long long)i, p, W, kmask, smask, kshift, sshift, sm) == 1) {
                s_stage[k * TPB + threadIdx.x] = sm;
                ++k;
                ++n;
                if (((g0 + n) & (SEG_STAGE - 1)) == 0) {     // a 128-B line of `out` is complete
                    for (int j = 0; j < k; ++j) o[n - k + j] = s_stage[j * TPB + threadIdx.x];
                    k = 0;
                }
            }
        }
        for (int j = 0; j < k; ++j) o[n - k + j] = s_stage[j * TPB + threadIdx.x];
    } else {
        for (; i < e; ++i)
            if (S.step(SEG_NEXT(), (long long)i, p, W, kmask, smask, kshift, sshift, sm) == 1) n++;
        count[sg] = n;
        if (mode == 0) conv[sg] = ok ? 1 : 0;
    }
#undef SEG_NEXT
#undef SEG_ROT
#undef SEG_LOAD
}

// RandstrobeGenerator::next (randstrobes.cpp:173-202) + assign_randstrobes'
// packing (index.cpp:302-305), one lane per syncmer
__global__ void __launch_bounds__(TPB)
k_ref_randstrobes(const SyncmerOut* __restrict__ sm, uint64_t n_sync, const uint64_t* __restrict__ sync_begin,
                  const uint64_t* __restrict__ rs_begin, const uint8_t* __restrict__ emit, int n_contigs, BuildParams p,
                  rsa_ref_randstrobe* __restrict__ out) {
    const uint64_t g = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (g >= n_sync) return;
    int lo = 0, hi = n_contigs - 1;                      // contig: the last c with sync_begin[c] <= g
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (sync_begin[mid] <= g) lo = mid; else hi = mid - 1;
    }
    const int c = lo;
    if (!emit[c]) return;
    const uint64_t base = sync_begin[c], n = sync_begin[c + 1] - base, i = g - base;
    if (i + p.w_min >= n) return;                         // the last w_min syncmers start no randstrobe
    const uint64_t w_end = i + p.w_max < n - 1 ? i + p.w_max : n - 1;
    const SyncmerOut s1 = sm[g];
    const uint64_t max_position = (uint64_t)s1.pos + (unsigned)p.max_dist;
    uint64_t min_val = END64, h2 = s1.hash;
    uint32_t pos2 = s1.pos;
    for (uint64_t x = i + p.w_min; x <= w_end; ++x) {
        const SyncmerOut s2 = sm[base + x];
        if (s2.pos > max_position) break;
        const uint64_t res = (uint64_t)__popcll((s1.hash ^ s2.hash) & p.q);
        if (res < min_val) { min_val = res; h2 = s2.hash; pos2 = s2.pos; }
    }
    rsa_ref_randstrobe r;
    r.hash = s1.hash + h2;
    r.position = s1.pos;
    r.packed = ((uint32_t)c << 8) + (pos2 - s1.pos);
    out[rs_begin[c] + i] = r;
}

__global__ void __launch_bounds__(TPB)
k_split_keys(const rsa_ref_randstrobe* __restrict__ rs, uint64_t n, uint32_t* __restrict__ pos,
             uint32_t* __restrict__ idx) {
    const uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    pos[i] = rs[i].position;
    idx[i] = (uint32_t)i;
}

__global__ void __launch_bounds__(TPB)
k_gather_hash(const rsa_ref_randstrobe* __restrict__ rs, const uint32_t* __restrict__ idx, uint64_t n,
              uint64_t* __restrict__ hash) {
    const uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    hash[i] = rs[idx[i]].hash;
}

__global__ void __launch_bounds__(TPB)
k_gather_entries(const rsa_ref_randstrobe* __restrict__ rs, const uint32_t* __restrict__ idx, uint64_t n,
                 rsa_ref_randstrobe* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    out[i] = rs[idx[i]];
}

// randstrobe_start_indices (index.cpp:174-212): at every hash change at
// position i the buckets [size, top(hash[i])] receive i, where size is one
// past the top of the previous change (0 before the first change); after the
// loop the remaining buckets receive n.
__global__ void __launch_bounds__(TPB)
k_bucket_table(const rsa_ref_randstrobe* __restrict__ rs, uint64_t n, int bits, uint64_t* __restrict__ starts) {
    const uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (i == 0 || i >= n) return;
    const uint64_t h = rs[i].hash, hp = rs[i - 1].hash;
    if (h == hp) return;
    const uint64_t nb = 1ull << bits;
    const uint64_t top = h >> (64 - bits);
    const uint64_t lo = hp == rs[0].hash ? 0 : (hp >> (64 - bits)) + 1;
    for (uint64_t b = lo; b <= top; ++b) starts[b] = i;
    if (h == rs[n - 1].hash)                               // the last change: the tail gets n
        for (uint64_t b = top + 1; b <= nb; ++b) starts[b] = n;
}

__global__ void __launch_bounds__(TPB)
k_fill_u64(uint64_t* __restrict__ p, uint64_t n, uint64_t v) {
    const uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (i < n) p[i] = v;
}

// grid-stride over the entries; run starts count the unique hashes and
// histogram the run length (clamped to 101) of runs longer than one
// (index.cpp:186-224); bin 103 counts entries equal in (hash, position) to their
// predecessor (the ties whose order is pdqsort's).  One global atomic per block and bin.
constexpr int RC_BLOCKS = 2048;
constexpr int RC_BINS = 104;
__global__ void __launch_bounds__(TPB)
k_run_counts(const rsa_ref_randstrobe* __restrict__ rs, uint64_t n, unsigned long long* __restrict__ hist) {
    __shared__ unsigned long long lh[RC_BINS];
    for (int j = threadIdx.x; j < RC_BINS; j += TPB) lh[j] = 0;
    __syncthreads();
    unsigned long long starts = 0, ties = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * TPB) {
        const uint64_t h = rs[i].hash;
        if (i > 0 && rs[i - 1].hash == h && rs[i - 1].position == rs[i].position) ties++;
        if (i == 0 || rs[i - 1].hash != h) {
            starts++;
            if (i + 1 < n && rs[i + 1].hash == h) {          // a run longer than one
                uint64_t j = i + 2;
                while (j < n && j - i <= 100 && rs[j].hash == h) ++j;
                const uint64_t len = j - i;
                atomicAdd(&lh[len > 100 ? 101 : len], 1ull);
            }
        }
    }
    atomicAdd(&lh[102], starts);
    if (ties) atomicAdd(&lh[103], ties);
    __syncthreads();
    for (int j = threadIdx.x; j < RC_BINS; j += TPB)
        if (lh[j]) atomicAdd(&hist[j], lh[j]);
}

template <int WC>
void launch_seg(hipStream_t s, const char* ref, const SegTable& st, const BuildParams& p, int mode, uint32_t* count,
                uint8_t* conv, const uint64_t* off, SyncmerOut* out) {
    const unsigned grid = (unsigned)((st.n_seg + TPB - 1) / TPB);
    if (grid) k_seg_syncmers<WC><<<grid, TPB, 0, s>>>(ref, st, p, mode, count, conv, off, out);
}

void launch_seg_any(hipStream_t s, const char* ref, const SegTable& st, const BuildParams& p, int mode,
                    uint32_t* count, uint8_t* conv, const uint64_t* off, SyncmerOut* out) {
    if (p.k - p.s + 1 == 5) launch_seg<5>(s, ref, st, p, mode, count, conv, off, out);
    else launch_seg<0>(s, ref, st, p, mode, count, conv, off, out);
}

inline unsigned grid_of(uint64_t n) { return (unsigned)((n + TPB - 1) / TPB); }

}  // namespace

struct rsa_index_build {
    int device = 0;
    char* d_ref = nullptr;
    rsa_ref_randstrobe* d_rs = nullptr;      // sorted entries
    uint64_t* d_starts = nullptr;
    uint64_t n = 0;
    int bits = 0;
};

// shape of a build, read before a context takes it over (nothing changes hands)
void index_build_peek(const rsa_index_build* b, int* device, int* bits) {
    *device = b->device;
    *bits = b->bits;
}

// hands the device buffers of a build to a context (rsa_open_built) and frees the handle
void index_build_release(rsa_index_build* b, int* device, char** ref, rsa_ref_randstrobe** rs, uint64_t** starts,
                         uint64_t* n, int* bits) {
    *device = b->device;
    *ref = b->d_ref;
    *rs = b->d_rs;
    *starts = b->d_starts;
    *n = b->n;
    *bits = b->bits;
    delete b;
}

extern "C" {

void rsa_index_build_free(rsa_index_build* b) {
    if (!b) return;
    (void)hipSetDevice(b->device);
    if (b->d_ref) (void)hipFree(b->d_ref);
    if (b->d_rs) (void)hipFree(b->d_rs);
    if (b->d_starts) (void)hipFree(b->d_starts);
    delete b;
}

rsa_index_build* rsa_index_build_run(int device, const char* ref_seq, const uint64_t* coff_h, int32_t n_contigs,
                                     const rsa_index_build_params* bp, rsa_index_build_info* info, char* errbuf,
                                     size_t err_len) {
    const auto t_call = std::chrono::steady_clock::now();
    rsa_index_build* B = nullptr;
    std::vector<void*> tmp;                   // device temporaries, freed on every exit
    hipStream_t st = nullptr;
    std::vector<hipEvent_t> ev;
    auto cleanup = [&]() {
        if (st) (void)hipStreamSynchronize(st);
        for (void* x : tmp) if (x) (void)hipFree(x);
        tmp.clear();
        for (auto e : ev) (void)hipEventDestroy(e);
        ev.clear();
        if (st) (void)hipStreamDestroy(st);
        st = nullptr;
    };
    auto fail = [&](const std::string& s) -> rsa_index_build* {
        if (errbuf && err_len) snprintf(errbuf, err_len, "%s", s.c_str());
        cleanup();
        rsa_index_build_free(B);
        return nullptr;
    };
#define BCHK(x)                                                                                          \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) return fail(std::string("rsa_index_build: ") + #x + ": " + hipGetErrorString(e_)); \
    } while (0)
    auto dalloc = [&](void** p, size_t bytes) -> hipError_t {
        hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 64));
        if (e == hipSuccess) tmp.push_back(*p); else *p = nullptr;
        return e == hipSuccess ? rsa_poison(*p, std::max<size_t>(bytes, 64)) : e;
    };
    auto dfree = [&](void* p) {
        if (!p) return;
        (void)hipStreamSynchronize(st);
        (void)hipFree(p);
        for (auto& x : tmp) if (x == p) x = nullptr;
    };

    if (!bp || !coff_h || n_contigs < 0 || (n_contigs > 0 && !ref_seq)) return fail("rsa_index_build: bad arguments");
    if (bp->k > 32 || bp->s > 32 || bp->s > bp->k || bp->k - bp->s + 1 > 32 || bp->w_min > bp->w_max || bp->t_syncmer < 1)
        return fail("rsa_index_build: unsupported syncmer/randstrobe parameters");
    if (n_contigs >= (1 << 24)) return fail("rsa_index_build: at most 2^24 contigs");
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev == 0) return fail("rsa_index_build: no HIP device visible");
    if (device < 0 || device >= n_dev) return fail("rsa_index_build: bad device ordinal");
    BCHK(hipSetDevice(device));
    B = new rsa_index_build();
    B->device = device;
    BCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (int j = 0; j < 8; ++j) { hipEvent_t e; BCHK(hipEventCreate(&e)); ev.push_back(e); }
    const BuildParams P{bp->k, bp->s, bp->t_syncmer, bp->w_min, bp->w_max, bp->max_dist, bp->q};
    const uint64_t total = n_contigs ? coff_h[n_contigs] : 0;
    for (int c = 0; c < n_contigs; ++c)
        if (coff_h[c + 1] < coff_h[c] || coff_h[c + 1] - coff_h[c] >= (1ull << 32))
            return fail("rsa_index_build: contig offsets must be ascending and contigs shorter than 2^32");

    // pick_bits (index.cpp:135-139)
    int bits = bp->bits;
    if (bits < 0) {
        const size_t est = total / (size_t)(bp->k - bp->s + 1);
        bits = std::clamp((int)std::log2((double)est) - 1, 8, 31);
    }
    if (bits < 1 || bits > 31) return fail("rsa_index_build: bits must be in [1, 31]");
    B->bits = bits;

    // segment table (host): SEG-base segments, never crossing a contig
    std::vector<uint32_t> seg_c;
    std::vector<uint64_t> seg_b;
    seg_c.reserve(total / SEG + n_contigs + 1);
    seg_b.reserve(total / SEG + n_contigs + 1);
    for (int c = 0; c < n_contigs; ++c) {
        const uint64_t len = coff_h[c + 1] - coff_h[c];
        for (uint64_t b = 0; b < len; b += SEG) { seg_c.push_back((uint32_t)c); seg_b.push_back(b); }
    }
    const uint64_t n_seg = seg_c.size();

    BCHK(hipEventRecord(ev[0], st));
    BCHK(hipMalloc(&B->d_ref, total + 64));
    if (total) BCHK(hipMemcpyAsync(B->d_ref, ref_seq, total, hipMemcpyHostToDevice, st));
    BCHK(hipMemsetAsync(B->d_ref + total, 0, 64, st));        // the tail padding: zeros (rsa_open does the same)
    BCHK(hipEventRecord(ev[1], st));

    uint32_t *d_seg_c = nullptr, *d_count = nullptr;
    uint64_t *d_seg_b = nullptr, *d_replay = nullptr, *d_coff = nullptr, *d_off = nullptr;
    uint8_t* d_conv = nullptr;
    BCHK(dalloc((void**)&d_seg_c, 4 * n_seg));
    BCHK(dalloc((void**)&d_seg_b, 8 * n_seg));
    BCHK(dalloc((void**)&d_replay, 8 * n_seg));
    BCHK(dalloc((void**)&d_coff, 8 * ((size_t)n_contigs + 1)));
    BCHK(dalloc((void**)&d_count, 4 * n_seg));
    BCHK(dalloc((void**)&d_conv, n_seg));
    BCHK(dalloc((void**)&d_off, 8 * (n_seg + 1)));
    if (n_seg) {
        BCHK(hipMemcpyAsync(d_seg_c, seg_c.data(), 4 * n_seg, hipMemcpyHostToDevice, st));
        BCHK(hipMemcpyAsync(d_seg_b, seg_b.data(), 8 * n_seg, hipMemcpyHostToDevice, st));
    }
    BCHK(hipMemcpyAsync(d_coff, coff_h, 8 * ((size_t)n_contigs + 1), hipMemcpyHostToDevice, st));
    const SegTable T{d_seg_c, d_seg_b, d_replay, d_coff, n_seg};

    // pass 0: warm-up probe + counts
    launch_seg_any(st, B->d_ref, T, P, 0, d_count, d_conv, nullptr, nullptr);
    BCHK(hipGetLastError());
    std::vector<uint32_t> cnt(n_seg);
    std::vector<uint8_t> conv(n_seg);
    if (n_seg) {
        BCHK(hipMemcpyAsync(cnt.data(), d_count, 4 * n_seg, hipMemcpyDeviceToHost, st));
        BCHK(hipMemcpyAsync(conv.data(), d_conv, n_seg, hipMemcpyDeviceToHost, st));
    }
    BCHK(hipStreamSynchronize(st));
    // replay start of a segment: its own warm-up start if that converged, else
    // that of the nearest earlier segment that did (a contig's first segment
    // starts at the contig start and always converges)
    std::vector<uint64_t> replay(n_seg);
    uint64_t n_replayed = 0;
    for (uint64_t s = 0; s < n_seg; ++s) {
        const uint64_t own = seg_b[s] > (uint64_t)WARM ? seg_b[s] - WARM : 0;
        if (conv[s]) replay[s] = own;
        else { replay[s] = replay[s - 1]; n_replayed++; }
    }
    if (n_seg) BCHK(hipMemcpyAsync(d_replay, replay.data(), 8 * n_seg, hipMemcpyHostToDevice, st));
    if (n_replayed) {   // pass 1: recount from the replay starts (only the replayed segments change)
        launch_seg_any(st, B->d_ref, T, P, 1, d_count, nullptr, nullptr, nullptr);
        BCHK(hipGetLastError());
        BCHK(hipMemcpyAsync(cnt.data(), d_count, 4 * n_seg, hipMemcpyDeviceToHost, st));
        BCHK(hipStreamSynchronize(st));
    }
    // syncmer offsets per segment and per contig, randstrobe offsets per contig
    // (count_randstrobes index.cpp:28-41; contigs shorter than w_max emit none, 280-282)
    std::vector<uint64_t> off(n_seg + 1, 0);
    for (uint64_t s = 0; s < n_seg; ++s) off[s + 1] = off[s] + cnt[s];
    const uint64_t n_sync = off[n_seg];
    std::vector<uint64_t> sync_begin((size_t)n_contigs + 1, 0), rs_begin((size_t)n_contigs + 1, 0);
    std::vector<uint8_t> emit((size_t)std::max(1, n_contigs), 0);
    {
        uint64_t s = 0;
        for (int c = 0; c < n_contigs; ++c) {
            sync_begin[c] = off[s];
            while (s < n_seg && seg_c[s] == (uint32_t)c) ++s;
            const uint64_t nc = off[s] - sync_begin[c];
            const uint64_t len = coff_h[c + 1] - coff_h[c];
            emit[c] = len >= (uint64_t)bp->w_max;
            rs_begin[c + 1] = rs_begin[c] + (emit[c] && nc > (uint64_t)bp->w_min ? nc - bp->w_min : 0);
        }
        sync_begin[n_contigs] = n_sync;
    }
    const uint64_t n = rs_begin[n_contigs];
    B->n = n;
    if (n >= (1ull << 31)) return fail("rsa_index_build: more than 2^31 randstrobes");
    BCHK(hipMemcpyAsync(d_off, off.data(), 8 * (n_seg + 1), hipMemcpyHostToDevice, st));
    SyncmerOut* d_sync = nullptr;
    BCHK(dalloc((void**)&d_sync, sizeof(SyncmerOut) * (n_sync + 1)));
    launch_seg_any(st, B->d_ref, T, P, 2, nullptr, nullptr, d_off, d_sync);   // pass 2: write
    BCHK(hipGetLastError());
    BCHK(hipEventRecord(ev[2], st));

    // randstrobes in (contig, position) order
    uint64_t *d_sb = nullptr, *d_rb = nullptr;
    uint8_t* d_emit = nullptr;
    rsa_ref_randstrobe* d_raw = nullptr;
    BCHK(dalloc((void**)&d_sb, 8 * ((size_t)n_contigs + 1)));
    BCHK(dalloc((void**)&d_rb, 8 * ((size_t)n_contigs + 1)));
    BCHK(dalloc((void**)&d_emit, emit.size()));
    BCHK(dalloc((void**)&d_raw, sizeof(rsa_ref_randstrobe) * (n + 1)));
    BCHK(hipMemcpyAsync(d_sb, sync_begin.data(), 8 * ((size_t)n_contigs + 1), hipMemcpyHostToDevice, st));
    BCHK(hipMemcpyAsync(d_rb, rs_begin.data(), 8 * ((size_t)n_contigs + 1), hipMemcpyHostToDevice, st));
    BCHK(hipMemcpyAsync(d_emit, emit.data(), emit.size(), hipMemcpyHostToDevice, st));
    BCHK(hipEventRecord(ev[3], st));
    if (n_sync && n_contigs)
        k_ref_randstrobes<<<grid_of(n_sync), TPB, 0, st>>>(d_sync, n_sync, d_sb, d_rb, d_emit, n_contigs, P, d_raw);
    BCHK(hipGetLastError());
    BCHK(hipEventRecord(ev[4], st));
    dfree(d_sync);

    // sort by (hash, position): stable radix passes by position, then by hash
    uint32_t *d_pos0 = nullptr, *d_pos1 = nullptr, *d_idx0 = nullptr, *d_idx1 = nullptr;
    uint64_t *d_h0 = nullptr, *d_h1 = nullptr;
    BCHK(dalloc((void**)&d_pos0, 4 * n));
    BCHK(dalloc((void**)&d_pos1, 4 * n));
    BCHK(dalloc((void**)&d_idx0, 4 * n));
    BCHK(dalloc((void**)&d_idx1, 4 * n));
    const int nn = (int)n;
    size_t tb1 = 0, tb2 = 0;
    uint64_t max_len = 0;
    for (int c = 0; c < n_contigs; ++c) max_len = std::max<uint64_t>(max_len, coff_h[c + 1] - coff_h[c]);
    int pos_bits = 1;
    while (pos_bits < 32 && (1ull << pos_bits) <= max_len) ++pos_bits;
    BCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb1, d_pos0, d_pos1, d_idx0, d_idx1, nn, 0, pos_bits, st));
    BCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                            (const uint32_t*)d_idx1, d_idx0, nn, 0, 64, st));
    void* d_tmp = nullptr;
    BCHK(dalloc(&d_tmp, std::max(tb1, tb2)));
    if (n) {
        k_split_keys<<<grid_of(n), TPB, 0, st>>>(d_raw, n, d_pos0, d_idx0);
        BCHK(hipGetLastError());
    }
    uint32_t* idx_after_pos = d_idx0;
    if (n_contigs > 1 && n) {   // within one contig the entries are already in position order
        BCHK(hipcub::DeviceRadixSort::SortPairs(d_tmp, tb1, d_pos0, d_pos1, d_idx0, d_idx1, nn, 0, pos_bits, st));
        idx_after_pos = d_idx1;
    }
    dfree(d_pos0);
    dfree(d_pos1);
    BCHK(dalloc((void**)&d_h0, 8 * n));
    BCHK(dalloc((void**)&d_h1, 8 * n));
    uint32_t* idx_final = idx_after_pos == d_idx0 ? d_idx1 : d_idx0;
    if (n) {
        k_gather_hash<<<grid_of(n), TPB, 0, st>>>(d_raw, idx_after_pos, n, d_h0);
        BCHK(hipGetLastError());
        BCHK(hipcub::DeviceRadixSort::SortPairs(d_tmp, tb2, d_h0, d_h1, idx_after_pos, idx_final, nn, 0, 64, st));
    }
    dfree(d_h0);
    dfree(d_h1);
    dfree(d_tmp);
    BCHK(hipMalloc(&B->d_rs, sizeof(rsa_ref_randstrobe) * (n + 1)));
    // the entry past the last: all ones (a hash above every key), as in rsa_open
    BCHK(hipMemsetAsync(B->d_rs + n, 0xFF, sizeof(rsa_ref_randstrobe), st));
    if (n) {
        k_gather_entries<<<grid_of(n), TPB, 0, st>>>(d_raw, idx_final, n, B->d_rs);
        BCHK(hipGetLastError());
    }
    BCHK(hipEventRecord(ev[5], st));
    // d_raw (generation order) stays until the tie count is known: the replay starts from
    // it.  The counts run first, so without ties it is freed before the bucket table exists
    // (the peak is then entries + raw entries, not + the table)

    // run-length histogram (and the tie count, bin 103), then the bucket table
    unsigned long long* d_hist = nullptr;
    BCHK(dalloc((void**)&d_hist, 8 * RC_BINS));
    BCHK(hipMemsetAsync(d_hist, 0, 8 * RC_BINS, st));
    BCHK(hipEventRecord(ev[6], st));
    if (n) {
        k_run_counts<<<(unsigned)std::min<uint64_t>(RC_BLOCKS, grid_of(n)), TPB, 0, st>>>(B->d_rs, n, d_hist);
        BCHK(hipGetLastError());
    }
    unsigned long long hist[RC_BINS];
    BCHK(hipMemcpyAsync(hist, d_hist, sizeof hist, hipMemcpyDeviceToHost, st));
    BCHK(hipStreamSynchronize(st));
    const uint64_t ties = hist[103];
    if (!ties) {
        dfree(d_raw);
        d_raw = nullptr;
    }
    const uint64_t nb = 1ull << bits;
    BCHK(hipMalloc(&B->d_starts, 8 * (nb + 1)));
    // no hash change at all (n <= 1 or a single run): every bucket gets n (index.cpp:206-208)
    k_fill_u64<<<grid_of(nb + 1), TPB, 0, st>>>(B->d_starts, nb + 1, n);
    BCHK(hipGetLastError());
    if (n > 1) {
        k_bucket_table<<<grid_of(n), TPB, 0, st>>>(B->d_rs, n, bits, B->d_starts);
        BCHK(hipGetLastError());
    }
    BCHK(hipEventRecord(ev[7], st));
    BCHK(hipStreamSynchronize(st));

    // equal (hash, position) in two contigs: the reference's order of those entries is
    // what pdqsort_branchless's moves leave (index.cpp:168).  Replay that sort on the
    // host from generation order and put its result in place of the device sort's; keys
    // (and so the bucket table and the counts) are the same either way.
    double ms_ties = 0;
    if (ties) {
        const auto tr = std::chrono::steady_clock::now();
        std::vector<rsa_ref_randstrobe> h(n);
        BCHK(hipMemcpy(h.data(), d_raw, sizeof(rsa_ref_randstrobe) * n, hipMemcpyDeviceToHost));
        dfree(d_raw);
        d_raw = nullptr;
        // the caller's thread budget (the machine's, at most 64, when it gives none)
        const int threads = bp->threads > 0 ? bp->threads
                                            : (int)std::max(1u, std::min(64u, std::thread::hardware_concurrency()));
        rsa::sti_order::pdqsort_replay(h.data(), n, threads);
        BCHK(hipMemcpy(B->d_rs, h.data(), sizeof(rsa_ref_randstrobe) * n, hipMemcpyHostToDevice));
        ms_ties = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr).count();
    }

    // filter cutoff (index.cpp:214-238) from the clamped histogram: counts sorted
    // descending, the value at rank index_cutoff (or the smallest), clamped to [30, 100]
    const uint64_t unique_mers = hist[102];
    const uint64_t index_cutoff = (uint64_t)(unique_mers * bp->f);
    uint64_t n_counts = 0;
    for (int j = 2; j <= 101; ++j) n_counts += hist[j];
    int filter_cutoff = 30;
    if (n_counts) {
        unsigned v = 0;
        if (index_cutoff < n_counts) {
            uint64_t cum = 0;
            for (int j = 101; j >= 2; --j) {
                cum += hist[j];
                if (cum > index_cutoff) { v = (unsigned)j; break; }
            }
        } else {
            for (int j = 2; j <= 101; ++j) if (hist[j]) { v = (unsigned)j; break; }
        }
        v = std::max(30U, v);
        v = std::min(100U, v);
        filter_cutoff = (int)v;
    }
    if (info) {
        memset(info, 0, sizeof *info);
        info->n_randstrobes = n;
        info->n_syncmers = n_sync;
        info->unique_hashes = unique_mers;
        info->bits = bits;
        info->filter_cutoff = filter_cutoff;
        info->n_segments = n_seg;
        info->replayed_segments = n_replayed;
        info->position_ties = ties;
        info->ms_tie_replay = ms_ties;
        float t = 0;
        (void)hipEventElapsedTime(&t, ev[0], ev[1]); info->ms_upload = t;
        (void)hipEventElapsedTime(&t, ev[1], ev[2]); info->ms_syncmers = t;
        (void)hipEventElapsedTime(&t, ev[3], ev[4]); info->ms_randstrobes = t;
        (void)hipEventElapsedTime(&t, ev[4], ev[5]); info->ms_sort = t;
        (void)hipEventElapsedTime(&t, ev[6], ev[7]); info->ms_buckets = t;
    }
    cleanup();
    if (info)
        info->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count();
    return B;
#undef BCHK
}

int rsa_index_build_download(rsa_index_build* b, rsa_ref_randstrobe* randstrobes, uint64_t* bucket_starts) {
    if (!b) return RSA_ERR_ARG;
    if (hipSetDevice(b->device) != hipSuccess) return RSA_ERR_HIP;
    if (randstrobes && b->n &&
        hipMemcpy(randstrobes, b->d_rs, sizeof(rsa_ref_randstrobe) * b->n, hipMemcpyDeviceToHost) != hipSuccess)
        return RSA_ERR_HIP;
    if (bucket_starts &&
        hipMemcpy(bucket_starts, b->d_starts, 8 * ((1ull << b->bits) + 1), hipMemcpyDeviceToHost) != hipSuccess)
        return RSA_ERR_HIP;
    return RSA_OK;
}

}  // extern "C"
