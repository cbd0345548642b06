// aln.cpp -- mapping decisions around the hot path, restated from the
// reference's src/aln.cpp (part/last split of RabbitSAlign) and the per-job
// string building / result storing of src/pc.cpp.  Every function keeps the
// reference's arithmetic types (float vs double vs size_t) because they are
// observable in the SAM output.  Compile with -ffp-contract=off.
#include <algorithm>
#include <cassert>
#include <climits>
#include <cmath>
#include <math.h>
#include <unordered_set>

#include <emmintrin.h>
#include <tmmintrin.h>

#include "rsa_host.hpp"

// per-thread pairing scratch.  Dynamic TLS, never initial-exec: librsalign.so is
// dlopen'ed by FFI hosts (ctypes, torch processes) whose static-TLS surplus may
// already be spent, and initial-exec TLS in a dlopen'ed object fails to load then
// ("cannot allocate memory in static TLS block").  The library is built with TLS
// descriptors (-mtls-dialect=gnu2), so an access after the first is a short
// call that reads the thread's DTV, not a __tls_get_addr lookup.
#define RSA_TLS thread_local

namespace rsa {

// ------------------------------------------------------------ sequences ---
static const unsigned char* revcomp_table() {      // src/revcomp.hpp:10-27
    struct Table {
        unsigned char t[256];
        Table() {
            for (int i = 0; i < 256; ++i) t[i] = 'N';
            t['A'] = 'T'; t['C'] = 'G'; t['G'] = 'C'; t['T'] = 'A'; t['U'] = 'A';
            t['a'] = 'T'; t['c'] = 'G'; t['g'] = 'C'; t['t'] = 'A'; t['u'] = 'A';
        }
    };
    static const Table table;                       // thread-safe one-time init
    return table.t;
}

std::string reverse_complement(std::string_view s) {
    std::string r(s.size(), 'N');
    reverse_complement_into(s, r.data());
    return r;
}

// 16 bytes per step: pshufb complements by the low nibble (A=0x41 C=0x43
// G=0x47 T=0x54 are distinct there) and reverses the block; a block holding
// anything but upper-case ACGT takes the table.
__attribute__((target("ssse3"))) static void rc_ssse3(const char* s, size_t n, char* out) {
    const unsigned char* t = revcomp_table();
    const __m128i rev = _mm_setr_epi8(15, 14, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0);
    const __m128i lut = _mm_setr_epi8(0, 'T', 0, 'G', 'A', 0, 0, 'C', 0, 0, 0, 0, 0, 0, 0, 0);
    const __m128i lo = _mm_set1_epi8(0x0F);
    const __m128i cA = _mm_set1_epi8('A'), cC = _mm_set1_epi8('C'), cG = _mm_set1_epi8('G'), cT = _mm_set1_epi8('T');
    size_t i = 0;
    for (; i + 16 <= n; i += 16) {
        const char* src = s + n - i - 16;
        const __m128i v = _mm_loadu_si128((const __m128i*)src);
        const __m128i ok = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, cA), _mm_cmpeq_epi8(v, cC)),
                                        _mm_or_si128(_mm_cmpeq_epi8(v, cG), _mm_cmpeq_epi8(v, cT)));
        if (_mm_movemask_epi8(ok) == 0xFFFF) {
            const __m128i c = _mm_shuffle_epi8(lut, _mm_and_si128(v, lo));
            _mm_storeu_si128((__m128i*)(out + i), _mm_shuffle_epi8(c, rev));
        } else {
            for (int j = 0; j < 16; ++j) out[i + j] = (char)t[(unsigned char)src[15 - j]];
        }
    }
    for (; i < n; ++i) out[i] = (char)t[(unsigned char)s[n - 1 - i]];
}

__attribute__((target("ssse3"))) static void rev_ssse3(const char* s, size_t n, char* out) {
    const __m128i rev = _mm_setr_epi8(15, 14, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0);
    size_t i = 0;
    for (; i + 16 <= n; i += 16)
        _mm_storeu_si128((__m128i*)(out + i),
                         _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(s + n - i - 16)), rev));
    for (; i < n; ++i) out[i] = s[n - 1 - i];
}

static const bool g_ssse3 = __builtin_cpu_supports("ssse3");

void reverse_complement_into(std::string_view s, char* out) {
    const size_t n = s.size();
    if (g_ssse3) { rc_ssse3(s.data(), n, out); return; }
    const unsigned char* t = revcomp_table();
    for (size_t i = 0; i < n; ++i) out[i] = (char)t[(unsigned char)s[n - 1 - i]];
}

void reverse_into(std::string_view s, char* out) {
    const size_t n = s.size();
    if (g_ssse3) { rev_ssse3(s.data(), n, out); return; }
    for (size_t i = 0; i < n; ++i) out[i] = s[n - 1 - i];
}

void to_uppercase(std::string& s) {
    for (auto& c : s) c = (char)((unsigned char)c & ~32);
}

// std::string::substr semantics without the copy (throws never: pos <= size holds on every call site)
static inline std::string_view sub(std::string_view s, size_t pos, size_t len) {
    if (pos > s.size()) pos = s.size();
    return s.substr(pos, len);
}

// --------------------------------------------------------- estimators ---
void InsertSizeDistribution::update(int dist) {      // aln.cpp:1880-1903
    if (dist >= 2000) return;
    const float e = dist - mu;
    mu += e / sample_size;
    SSE += e * (dist - mu);
    if (sample_size > 1) V = SSE / (sample_size - 1.0);
    else V = SSE;
    sigma = std::sqrt(V);
    sample_size = sample_size + 1.0;
}

template <typename T>
static bool by_score(const T& a, const T& b) { return a.score > b.score; }

// std::sort(by_score) of a read's NAM list, the same permutation: libstdc++'s
// std::sort of <= 16 elements is exactly its (stable) insertion sort, done here
// with plain element moves instead of a memmove per shift; longer lists go to std::sort.
// dst = src[0 .. n) in std::sort(by_score) order: <= 16 NAMs sort (score, index)
// keys by the insertion sort and land in dst once, gathered
void load_sorted_nams(std::vector<Nam>& dst, const Nam* src, size_t n) {
    if (n > 16 || n < 2) {
        dst.assign(src, src + n);
        if (n > 16) std::sort(dst.begin(), dst.end(), by_score<Nam>);
        return;
    }
    float sc[16];
    uint8_t ix[16];
    for (size_t i = 0; i < n; ++i) { sc[i] = src[i].score; ix[i] = (uint8_t)i; }
    for (size_t i = 1; i < n; ++i) {
        if (!(sc[i] > sc[i - 1])) continue;
        const float xs = sc[i];
        const uint8_t xi = ix[i];
        size_t j = i;
        do { sc[j] = sc[j - 1]; ix[j] = ix[j - 1]; --j; } while (j > 0 && xs > sc[j - 1]);
        sc[j] = xs;
        ix[j] = xi;
    }
    dst.resize(n);
    for (size_t i = 0; i < n; ++i) dst[i] = src[ix[i]];
}

void sort_nams_by_score(NamSpan v) {
    const size_t n = v.size();
    if (n > 16) { std::sort(v.begin(), v.end(), by_score<Nam>); return; }
    if (n < 2) return;
    float sc[16];
    uint8_t ix[16];
    for (size_t i = 0; i < n; ++i) { sc[i] = v[i].score; ix[i] = (uint8_t)i; }
    bool moved = false;
    for (size_t i = 1; i < n; ++i) {
        if (!(sc[i] > sc[i - 1])) continue;
        moved = true;
        const float xs = sc[i];
        const uint8_t xi = ix[i];
        size_t j = i;
        do { sc[j] = sc[j - 1]; ix[j] = ix[j - 1]; --j; } while (j > 0 && xs > sc[j - 1]);
        sc[j] = xs;
        ix[j] = xi;
    }
    if (!moved) return;                    // already in order (the engine sorted it)
    Nam tmp[16];
    std::copy(v.begin(), v.end(), tmp);
    for (size_t i = 0; i < n; ++i) v[i] = tmp[ix[i]];
}

// ------------------------------------------------------------- NAM ops ---
// aln.cpp:60-93
static bool reverse_nam_if_needed(Nam& nam, const Read& read, const References& refs, int k) {
    const size_t read_len = read.size();
    if (const rsa_nam_site* st = read.site.find(nam)) {   // checked on the GPU (k_sites)
        const int o = st->flags & RSA_SITE_ORIENT_MASK;
        if (o != 1) return o == 0;
        if (nam.is_rc == st->orig_is_rc) {                  // not reversed yet (a second call keeps it)
            nam.is_rc = !st->orig_is_rc;
            nam.query_start = (int)read_len - st->orig_query_end;
            nam.query_end = (int)read_len - st->orig_query_start;
        }
        return true;
    }
    std::string_view ref = refs.seq(nam.ref_id);
    std::string_view ref_start_kmer = sub(ref, (size_t)nam.ref_start, (size_t)k);
    std::string_view ref_end_kmer = sub(ref, (size_t)(nam.ref_end - k), (size_t)k);
    std::string_view seq, seq_rc;
    if (nam.is_rc) { seq = read.rc; seq_rc = read.seq; }
    else { seq = read.seq; seq_rc = read.rc; }
    std::string_view read_start_kmer = sub(seq, (size_t)nam.query_start, (size_t)k);
    std::string_view read_end_kmer = sub(seq, (size_t)(nam.query_end - k), (size_t)k);
    if (ref_start_kmer == read_start_kmer && ref_end_kmer == read_end_kmer) return true;
    const int q_start_tmp = (int)read_len - nam.query_end;
    const int q_end_tmp = (int)read_len - nam.query_start;
    read_start_kmer = sub(seq_rc, (size_t)q_start_tmp, (size_t)k);
    read_end_kmer = sub(seq_rc, (size_t)(q_end_tmp - k), (size_t)k);
    if (ref_start_kmer == read_start_kmer && ref_end_kmer == read_end_kmer) {
        nam.is_rc = !nam.is_rc;
        nam.query_start = q_start_tmp;
        nam.query_end = q_end_tmp;
        return true;
    }
    return false;
}

static void shuffle_top_nams(NamSpan nams, std::minstd_rand& rng) {   // aln.cpp:1910-1925
    if (nams.empty()) return;
    const float best = nams[0].score;
    auto it = std::find_if(nams.begin(), nams.end(), [&](const Nam& n) { return n.score != best; });
    if (it != nams.end()) std::shuffle(nams.begin(), it, rng);
}

static float top_dropoff(const NamSpan& nams) {   // aln.cpp:1349-1360
    const Nam& n_max = nams[0];
    if (n_max.n_hits <= 2) return 1.0;
    if (nams.size() > 1) return (float)nams[1].n_hits / n_max.n_hits;
    return 0.0;
}

static uint8_t get_mapq(const NamSpan& nams, const Nam& n_max) {   // aln.cpp:493-503
    if (nams.size() <= 1) return 60;
    const float s1 = n_max.score;
    const float s2 = nams[1].score;
    const float min_matches = std::min(n_max.n_hits / 10.0, 1.0);
    const int uncapped_mapq = 40 * (1 - s2 / s1) * min_matches * log(s1);
    return std::min(uncapped_mapq, 60);
}

static bool is_proper_nam_pair(const Nam& nam1, const Nam& nam2, float mu, float sigma) {   // aln.cpp:552-569
    if (nam1.ref_id != nam2.ref_id || nam1.is_rc == nam2.is_rc) return false;
    int a = std::max(0, nam1.ref_start - nam1.query_start);
    int b = std::max(0, nam2.ref_start - nam2.query_start);
    bool r1_r2 = nam2.is_rc && (a <= b) && (b - a < mu + 10 * sigma);
    if (r1_r2) return true;
    bool r2_r1 = nam1.is_rc && (b <= a) && (a - b < mu + 10 * sigma);
    if (r2_r1) return true;
    return false;
}

struct NamPair { int score; Nam nam1; Nam nam2; };

// aln.cpp:583-918 (use_fast_loop3 variant)
// into `joint` (cleared first; the caller's per-thread vector, so no allocation per pair)
static void get_best_scoring_nam_pairs(std::vector<NamPair>& joint, const NamSpan& nams1,
                                       const NamSpan& nams2, float mu, float sigma) {
    joint.clear();
    if (nams1.empty() && nams2.empty()) return;
    joint.reserve(nams1.size() + nams2.size());
    // membership by nam_id (the NAM's index in its read's list) instead of a hash set
    RSA_TLS std::vector<uint8_t> added_n1, added_n2;
    auto reset_ids = [](std::vector<uint8_t>& v, const NamSpan& ns) {
        int mx = -1;
        for (const Nam& n : ns) mx = std::max(mx, n.nam_id);
        v.assign((size_t)(mx + 1), 0);
    };
    reset_ids(added_n1, nams1);
    reset_ids(added_n2, nams2);
    int best_joint_hits = 0;
    RSA_TLS std::vector<Nam> sorted2[2];
    sorted2[0].clear();
    sorted2[1].clear();
    for (const auto& n2 : nams2) sorted2[n2.is_rc ? 1 : 0].push_back(n2);
    for (int i = 0; i < 2; ++i)
        std::sort(sorted2[i].begin(), sorted2[i].end(), [](const Nam& a, const Nam& b) {
            int v1 = std::max(0, a.ref_start - a.query_start);
            int v2 = std::max(0, b.ref_start - b.query_start);
            return v1 < v2;
        });
    for (const auto& nam1 : nams1) {
        const int nam1_val = std::max(0, nam1.ref_start - nam1.query_start);
        if (nam1.is_rc == 1) {
            const float L_val = nam1_val - (mu + 10 * sigma);
            const float R_val = nam1_val;
            const auto& v = sorted2[0];
            int ll = 0, rr = (int)v.size() - 1, ans = (int)v.size();
            while (ll <= rr) {
                int mid = (ll + rr) / 2;
                int now = std::max(0, v[mid].ref_start - v[mid].query_start);
                if (now > L_val) { rr = mid - 1; ans = mid; }
                else ll = mid + 1;
            }
            for (int id = ans; id < (int)v.size(); ++id) {
                const Nam& nam2 = v[id];
                int joint_hits = nam1.n_hits + nam2.n_hits;
                if (nam1.ref_id != nam2.ref_id) continue;
                int a = std::max(0, nam1.ref_start - nam1.query_start);
                int b = std::max(0, nam2.ref_start - nam2.query_start);
                if (b > R_val - 1e-6) break;
                bool r2_r1 = (a - b >= 0) && (a - b < mu + 10 * sigma);
                if (r2_r1) {
                    joint.push_back(NamPair{joint_hits, nam1, nam2});
                    added_n1[nam1.nam_id] = 1;
                    added_n2[nam2.nam_id] = 1;
                }
            }
        } else {
            const float L_val = nam1_val;
            const float R_val = nam1_val + mu + 10 * sigma;
            const auto& v = sorted2[1];
            int ll = 0, rr = (int)v.size() - 1, ans = (int)v.size();
            while (ll <= rr) {
                int mid = (ll + rr) / 2;
                int now = std::max(0, v[mid].ref_start - v[mid].query_start);
                if (now >= L_val) { rr = mid - 1; ans = mid; }
                else ll = mid + 1;
            }
            for (int id = ans; id < (int)v.size(); ++id) {
                const Nam& nam2 = v[id];
                int joint_hits = nam1.n_hits + nam2.n_hits;
                if (nam1.ref_id != nam2.ref_id) continue;
                int a = std::max(0, nam1.ref_start - nam1.query_start);
                int b = std::max(0, nam2.ref_start - nam2.query_start);
                if (b >= R_val - 1e-6) break;
                bool r1_r2 = (b - a >= 0) && (b - a < mu + 10 * sigma);
                if (r1_r2) {
                    joint.push_back(NamPair{joint_hits, nam1, nam2});
                    added_n1[nam1.nam_id] = 1;
                    added_n2[nam2.nam_id] = 1;
                }
            }
        }
    }
    Nam dummy{};
    dummy.ref_start = -1;
    if (!nams1.empty()) {
        int best1 = best_joint_hits > 0 ? best_joint_hits : nams1[0].n_hits;
        for (const auto& nam1 : nams1) {
            if (nam1.n_hits < best1 / 2) break;
            if (added_n1[nam1.nam_id]) continue;
            joint.push_back(NamPair{nam1.n_hits, nam1, dummy});
        }
    }
    if (!nams2.empty()) {
        int best2 = best_joint_hits > 0 ? best_joint_hits : nams2[0].n_hits;
        for (const auto& nam2 : nams2) {
            if (nam2.n_hits < best2 / 2) break;
            if (added_n2[nam2.nam_id]) continue;
            joint.push_back(NamPair{nam2.n_hits, dummy, nam2});
        }
    }
    std::sort(joint.begin(), joint.end(), [](const NamPair& a, const NamPair& b) { return a.score > b.score; });
}

// ------------------------------------------------------------ hamming ---
// Mismatch positions of two equal-length strings, 16 bytes per SSE2 compare.
// Returns the mismatch count; the first `cap` positions are stored in pos.
static int mismatch_positions(const char* q, const char* r, size_t n, int* pos, int cap) {
    int cnt = 0;
    size_t i = 0;
    for (; i + 16 <= n; i += 16) {
        const __m128i a = _mm_loadu_si128((const __m128i*)(q + i));
        const __m128i b = _mm_loadu_si128((const __m128i*)(r + i));
        unsigned m = ~(unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(a, b)) & 0xFFFFu;
        while (m) {
            const int bit = __builtin_ctz(m);
            if (cnt < cap) pos[cnt] = (int)i + bit;
            cnt++;
            m &= m - 1;
        }
    }
    for (; i < n; ++i)
        if (q[i] != r[i]) { if (cnt < cap) pos[cnt] = (int)i; cnt++; }
    return cnt;
}

// highest_scoring_segment (aligner.cpp:219-252), evaluated run by run: between
// mismatches the score only grows, so the per-position updates of the
// reference collapse to one check at the end of each run of matches.
static void highest_scoring_segment(size_t n, const int* mm, int n_mm, int match, int mismatch, int end_bonus,
                                    size_t& bs, size_t& be, int& bsc) {
    size_t start = 0, best_start = 0, best_end = 0;
    int score = end_bonus, best_score = 0;
    size_t i = 0;
    for (int k = 0; k <= n_mm; ++k) {
        const size_t m = k < n_mm ? (size_t)mm[k] : n;
        if (m > i) {
            score += match * (int)(m - i);
            if (score > best_score) { best_start = start; best_score = score; best_end = m; }
        }
        if (k == n_mm) break;
        score -= mismatch;
        if (score < 0) { start = m + 1; score = 0; }
        if (score > best_score) { best_start = start; best_score = score; best_end = m + 1; }
        i = m + 1;
    }
    if (score + end_bonus > best_score) {
        best_score = score + end_bonus;
        best_end = n;
        best_start = start;
    }
    bs = best_start; be = best_end; bsc = best_score;
}

// hamming_align (aligner.cpp:254-302) from the mismatch positions
static AlignmentInfo hamming_align(size_t n, const int* mm, int n_mm, int match, int mismatch, int end_bonus) {
    AlignmentInfo aln;
    size_t s, e;
    int score;
    highest_scoring_segment(n, mm, n_mm, match, mismatch, end_bonus, s, e, score);
    Cigar cigar;
    cigar.ops.reserve(2 * (size_t)n_mm + 4);
    if (s > 0) cigar.push(C_S, (uint32_t)s);
    int mismatches = 0;
    size_t cur = s;
    for (int k = 0; k < n_mm; ++k) {
        const size_t m = (size_t)mm[k];
        if (m < s) continue;
        if (m >= e) break;
        if (m > cur) cigar.push(C_EQ, (uint32_t)(m - cur));
        cigar.push(C_X, 1);
        mismatches++;
        cur = m + 1;
    }
    if (e > cur) cigar.push(C_EQ, (uint32_t)(e - cur));
    int soft_right = (int)n - (int)e;
    if (soft_right > 0) cigar.push(C_S, (uint32_t)soft_right);
    aln.cigar = std::move(cigar);
    aln.sw_score = score;
    aln.edit_distance = (unsigned)mismatches;
    aln.ref_start = (unsigned)s; aln.ref_end = (unsigned)e;
    aln.query_start = (unsigned)s; aln.query_end = (unsigned)e;
    return aln;
}

// ------------------------------------------------------------- part ---
// extend_seed_part (aln.cpp:374-431)
static bool extend_seed_part(AlignTmpRes& res, const AlignmentParameters& ap, const Nam& nam, const References& refs,
                             const Read& read, bool consistent_nam) {
    std::string_view query = nam.is_rc ? std::string_view(read.rc) : std::string_view(read.seq);
    std::string_view ref = refs.seq(nam.ref_id);
    const auto projected_ref_start = std::max(0, nam.ref_start - nam.query_start);
    const auto projected_ref_end = std::min(nam.ref_end + query.size() - nam.query_end, ref.size());
    AlignmentInfo info;
    int result_ref_start = 0;
    bool gapped = true;
    const rsa_nam_site* st = consistent_nam ? read.site.find(nam) : nullptr;
    if (st && !(st->flags & RSA_SITE_POOL_FULL)) {         // the GPU checked this window (k_sites)
        if (st->flags & RSA_SITE_ALIGNED) {                   // ... and ran hamming_align on it
            const uint16_t* w = read.site.pool + st->mm_offset;
            info.sw_score = (int)((uint32_t)w[0] | ((uint32_t)w[1] << 16));
            info.ref_start = info.query_start = w[2];
            info.ref_end = info.query_end = w[3];
            info.edit_distance = w[4];
            const uint32_t n_ops = w[5];
            info.cigar.ops.reserve(n_ops);
            for (uint32_t k = 0; k < n_ops; ++k)
                info.cigar.ops.push_back((uint32_t)w[6 + 2 * k] | ((uint32_t)w[7 + 2 * k] << 16));
            result_ref_start = projected_ref_start + (int)info.ref_start;
            gapped = false;
        } else if (st->flags & RSA_SITE_POSITIONS) {
            int mm[64];
            std::vector<int> big;
            int* pos = mm;
            if (st->n_mm > 64) { big.resize(st->n_mm); pos = big.data(); }
            for (int i = 0; i < st->n_mm; ++i) pos[i] = read.site.pool[st->mm_offset + i];
            info = hamming_align(query.size(), pos, st->n_mm, ap.match, ap.mismatch, ap.end_bonus);
            result_ref_start = projected_ref_start + (int)info.ref_start;
            gapped = false;
        }
    } else if (projected_ref_end - projected_ref_start == query.size() && consistent_nam) {
        std::string_view segm = sub(ref, (size_t)projected_ref_start, query.size());
        int mm[64];
        const int hd = segm.size() == query.size()
                           ? mismatch_positions(query.data(), segm.data(), query.size(), mm, 64) : -1;
        if (hd >= 0 && (((float)hd / query.size()) < 0.05)) {
            if (hd > 64) {   // reads > 1280 bp only: positions beyond the buffer
                std::vector<int> all(hd);
                mismatch_positions(query.data(), segm.data(), query.size(), all.data(), hd);
                info = hamming_align(query.size(), all.data(), hd, ap.match, ap.mismatch, ap.end_bonus);
            } else {
                info = hamming_align(query.size(), mm, hd, ap.match, ap.mismatch, ap.end_bonus);
            }
            result_ref_start = projected_ref_start + (int)info.ref_start;
            gapped = false;
        }
    }
    res.todo_nams.push_back(nam);
    res.is_extend_seed.push_back(true);
    if (gapped) {
        res.done_align.push_back(false);
        res.align_res.push_back(Alignment());
    } else {
        res.done_align.push_back(true);
        int softclipped = (int)info.query_start + ((int)query.size() - (int)info.query_end);
        Alignment a;
        a.cigar = std::move(info.cigar);
        a.edit_distance = (int)info.edit_distance;
        a.global_ed = (int)info.edit_distance + softclipped;
        a.score = info.sw_score;
        a.ref_start = result_ref_start;
        a.length = info.ref_span();
        a.is_rc = nam.is_rc;
        a.is_unaligned = false;
        a.ref_id = nam.ref_id;
        a.gapped = gapped;
        res.align_res.push_back(std::move(a));
    }
    return gapped;
}

// has_shared_substring (aln.cpp:1000-1013)
bool has_shared_substring(std::string_view read_seq, std::string_view ref_seq, int k) {
    int sub_size = 2 * k / 3;
    int step_size = k / 3;
    for (size_t i = 0; i + sub_size < read_seq.size(); i += step_size) {
        if (ref_seq.find(read_seq.substr(i, sub_size)) != std::string_view::npos) return true;
    }
    return false;
}

// rescue window (aln.cpp:1029-1042 / pc.cpp:255-272): the mixed int/size_t/float arithmetic is kept
static void rescue_window(const Nam& nam, size_t read_len, float mu, float sigma, int ref_len_i, int& ref_start,
                          int& ref_end) {
    int a, b;
    if (nam.is_rc) {
        a = nam.ref_start - nam.query_start - (mu + 5 * sigma);
        b = nam.ref_start - nam.query_start + read_len / 2;
    } else {
        a = nam.ref_end + (read_len - nam.query_end) - read_len / 2;
        b = nam.ref_end + (read_len - nam.query_end) + (mu + 5 * sigma);
    }
    ref_start = std::max(0, std::min(a, ref_len_i));
    ref_end = std::min(ref_len_i, std::max(0, b));
}

// A rescue whose has_shared_substring test went to the engine with its SW job
// (SwJob::shared_k): the slot's edit distance until the result is stored
static constexpr int kSharedDeferred = INT_MIN;

// The engine makes the has_shared_substring test (RSA_SHARED_ON_ENGINE=0: the host
// always does).  Only once the insert-size estimate is frozen: the test's window is
// this call's (mu, sigma) and the SW job's is the one at job collection (pc.cpp:333-368),
// which are the same from then on, and within the device kernel's limits.
static bool shared_on_engine() {
    static const bool on = !(getenv("RSA_SHARED_ON_ENGINE") && getenv("RSA_SHARED_ON_ENGINE")[0] == '0');
    return on;
}

// rescue_mate_part (aln.cpp:1015-1076)
static bool rescue_mate_part(AlignTmpRes& res, const Nam& nam, const References& refs, const Read& read, float mu,
                             float sigma, int k, bool defer) {
    Alignment alignment;
    const size_t read_len = read.size();
    std::string_view r_tmp = nam.is_rc ? std::string_view(read.seq) : std::string_view(read.rc);
    const int ref_len = (int)refs.seq(nam.ref_id).size();
    int ref_start, ref_end;
    rescue_window(nam, read_len, mu, sigma, ref_len, ref_start, ref_end);
    res.todo_nams.push_back(nam);
    res.is_extend_seed.push_back(false);
    auto unaligned = [&]() {
        alignment.cigar = Cigar();
        alignment.edit_distance = (int)read_len;
        alignment.score = 0;
        alignment.ref_start = 0;
        alignment.is_rc = nam.is_rc;
        alignment.ref_id = nam.ref_id;
        alignment.is_unaligned = true;
        res.done_align.push_back(true);
        res.align_res.push_back(alignment);
        return true;
    };
    if (ref_end < ref_start + k) return unaligned();
    if (defer && read_len <= 1024 && ref_end - ref_start <= 4096 && k >= 3 && 2 * k / 3 <= 24) {
        alignment.edit_distance = kSharedDeferred;      // tested by the engine, stored by store_rescue
        res.done_align.push_back(false);
        res.align_res.push_back(alignment);
        return false;
    }
    std::string_view segm = sub(refs.seq(nam.ref_id), (size_t)ref_start, (size_t)(ref_end - ref_start));
    if (!has_shared_substring(r_tmp, segm, k)) return unaligned();
    res.done_align.push_back(false);
    res.align_res.push_back(alignment);
    return false;
}

// rescue_read_part (aln.cpp:1135-1176)
static void rescue_read_part(int flag, AlignTmpRes& res, const Read& read2, const Read& read1, const MapContext& mc,
                             NamSpan nams1, Details det[2], int k, float mu, float sigma, bool defer) {
    res.type = flag;
    const Nam n_max1 = nams1[0];
    int tries = 0;
    for (auto& nam : nams1) {
        float score_dropoff1 = (float)nam.n_hits / n_max1.n_hits;
        if (tries >= mc.mparams.max_tries || score_dropoff1 < mc.mparams.dropoff_threshold) break;
        const bool consistent = reverse_nam_if_needed(nam, read1, mc.refs, k);
        det[0].nam_inconsistent += !consistent;
        res.is_read1.push_back(flag == 1);
        bool gapped = extend_seed_part(res, mc.aparams, nam, mc.refs, read1, consistent);
        det[0].gapped += gapped;
        det[0].tried_alignment++;
        res.is_read1.push_back(flag != 1);
        (void)rescue_mate_part(res, nam, mc.refs, read2, mu, sigma, k, defer);
        tries++;
    }
}

// align_PE_part (aln.cpp:1372-1580)
static void align_PE_part(AlignTmpRes& res, const MapContext& mc, NamSpan nams1, NamSpan nams2,
                          const Read& read1, const Read& read2, int k, Details det[2], InsertSizeDistribution& isize) {
    const float mu = isize.mu, sigma = isize.sigma;
    const float dropoff = mc.mparams.dropoff_threshold;
    const unsigned max_tries = (unsigned)mc.mparams.max_tries;
    const bool defer = shared_on_engine() && isize.frozen();
    if (nams1.empty() && nams2.empty()) { res.type = 0; return; }
    if (!nams1.empty() && nams2.empty()) {
        rescue_read_part(1, res, read2, read1, mc, nams1, det, k, mu, sigma, defer);
        return;
    }
    if (nams1.empty() && !nams2.empty()) {
        rescue_read_part(2, res, read1, read2, mc, nams2, det, k, mu, sigma, defer);   // details unswapped (sic)
        return;
    }
    if (top_dropoff(nams1) < dropoff && top_dropoff(nams2) < dropoff && is_proper_nam_pair(nams1[0], nams2[0], mu, sigma)) {
        res.type = 3;
        Nam n_max1 = nams1[0], n_max2 = nams2[0];
        bool c1 = reverse_nam_if_needed(n_max1, read1, mc.refs, k);
        det[0].nam_inconsistent += !c1;
        bool c2 = reverse_nam_if_needed(n_max2, read2, mc.refs, k);
        det[1].nam_inconsistent += !c2;
        res.is_read1.push_back(true);
        bool g1 = extend_seed_part(res, mc.aparams, n_max1, mc.refs, read1, c1);
        det[0].tried_alignment++;
        det[0].gapped += g1;
        res.is_read1.push_back(false);
        bool g2 = extend_seed_part(res, mc.aparams, n_max2, mc.refs, read2, c2);
        det[1].tried_alignment++;
        det[1].gapped += g2;
        res.mapq1 = get_mapq(nams1, n_max1);
        res.mapq2 = get_mapq(nams2, n_max2);
        if (!g1 && !g2) {
            const size_t n = res.align_res.size();
            const Alignment& a1 = res.align_res[n - 2];
            const Alignment& a2 = res.align_res[n - 1];
            bool proper = is_proper_pair(a1, a2, mu, sigma);
            if ((isize.sample_size < 400) && (a1.edit_distance + a2.edit_distance < 3) && proper)
                isize.update(std::abs(a1.ref_start - a2.ref_start));
        }
        return;
    }
    res.type = 4;
    RSA_TLS std::vector<NamPair> joint;
    get_best_scoring_nam_pairs(joint, nams1, nams2, mu, sigma);
    // nam_id flags (the id is the NAM's index in its read's list) instead of hash sets
    RSA_TLS std::vector<uint8_t> aligned1, aligned2;
    auto reset_ids = [](std::vector<uint8_t>& v, const NamSpan& ns) {
        int mx = -1;
        for (const Nam& x : ns) mx = std::max(mx, x.nam_id);
        v.assign((size_t)(mx + 1), 0);
    };
    reset_ids(aligned1, nams1);
    reset_ids(aligned2, nams2);
    {
        Nam n1 = nams1[0];
        bool c1 = reverse_nam_if_needed(n1, read1, mc.refs, k);
        det[0].nam_inconsistent += !c1;
        res.is_read1.push_back(true);
        bool g1 = extend_seed_part(res, mc.aparams, n1, mc.refs, read1, c1);
        aligned1[n1.nam_id] = 1;
        det[0].tried_alignment++;
        det[0].gapped += g1;
        Nam n2 = nams2[0];
        bool c2 = reverse_nam_if_needed(n2, read2, mc.refs, k);
        det[1].nam_inconsistent += !c2;
        res.is_read1.push_back(false);
        bool g2 = extend_seed_part(res, mc.aparams, n2, mc.refs, read2, c2);
        aligned2[n2.nam_id] = 1;
        det[1].tried_alignment++;
        det[1].gapped += g2;
    }
    const int max_score = joint[0].score;
    res.type4_loop_size = 0;
    size_t n_high = 0;
    for (auto& jp : joint) {
        Nam& n1 = jp.nam1;
        Nam& n2 = jp.nam2;
        float score_dropoff = (float)jp.score / max_score;
        if (n_high >= max_tries || score_dropoff < dropoff) break;
        res.type4_nams.push_back(n1);
        res.type4_nams.push_back(n2);
        res.type4_loop_size++;
        if (n1.ref_start >= 0) {
            if (!aligned1[n1.nam_id]) {
                bool c = reverse_nam_if_needed(n1, read1, mc.refs, k);
                det[0].nam_inconsistent += !c;
                res.is_read1.push_back(true);
                bool g = extend_seed_part(res, mc.aparams, n1, mc.refs, read1, c);
                aligned1[n1.nam_id] = 1;
                det[0].tried_alignment++;
                det[0].gapped += g;
            }
        } else {
            det[1].nam_inconsistent += !reverse_nam_if_needed(n2, read2, mc.refs, k);
            res.is_read1.push_back(true);
            (void)rescue_mate_part(res, n2, mc.refs, read1, mu, sigma, k, defer);
            det[0].tried_alignment++;
        }
        if (n2.ref_start >= 0) {
            if (!aligned2[n2.nam_id]) {
                bool c = reverse_nam_if_needed(n2, read2, mc.refs, k);
                det[1].nam_inconsistent += !c;
                res.is_read1.push_back(false);
                bool g = extend_seed_part(res, mc.aparams, n2, mc.refs, read2, c);
                aligned2[n2.nam_id] = 1;
                det[1].tried_alignment++;
                det[1].gapped += g;
            }
        } else {
            det[0].nam_inconsistent += !reverse_nam_if_needed(n1, read1, mc.refs, k);
            res.is_read1.push_back(false);
            (void)rescue_mate_part(res, n1, mc.refs, read2, mu, sigma, k, defer);
            det[1].tried_alignment++;
        }
        n_high++;
    }
}

// align_PE_read_part (aln.cpp:1927-1981); the find_nams/rescue results come from the engine
void align_PE_read_part(AlignTmpRes& res, const RecView&, const RecView&, const Read& read1, const Read& read2,
                        NamSpan nams[2],
                        const bool rescued[2], AlignmentStatistics& stats, InsertSizeDistribution& isize,
                        const MapContext& mc, std::minstd_rand& rng, bool sorted) {
    Details det[2];
    for (int m = 0; m < 2; ++m) {
        if (mc.mparams.rescue_level > 1 && rescued[m]) det[m].nam_rescue = true;
        det[m].nams = nams[m].size();
        if (!sorted) sort_nams_by_score(nams[m]);
        shuffle_top_nams(nams[m], rng);
    }
    align_PE_part(res, mc, nams[0], nams[1], read1, read2, mc.iparams.k, det, isize);
    stats.add(det[0]);
    stats.add(det[1]);
}

// align_SE_part (aln.cpp:95-124)
void align_SE_read_part(AlignTmpRes& res, const RecView&, const Read& read, std::vector<Nam>& nams, bool rescued,
                        AlignmentStatistics& stats, const MapContext& mc, std::minstd_rand& rng) {
    Details det;
    if (mc.mparams.rescue_level > 1 && rescued) det.nam_rescue = true;
    det.nams = nams.size();
    sort_nams_by_score(nams);
    shuffle_top_nams(nams, rng);
    if (nams.empty()) {
        res.type = 0;
    } else {
        int tries = 0;
        const Nam n_max = nams[0];
        res.type = 4;
        for (auto& nam : nams) {
            float score_dropoff = (float)nam.n_hits / n_max.n_hits;
            if (tries >= mc.mparams.max_tries || score_dropoff < mc.mparams.dropoff_threshold) break;
            bool consistent = reverse_nam_if_needed(nam, read, mc.refs, mc.iparams.k);
            res.consistent_nam.push_back(consistent);
            res.is_read1.push_back(true);
            (void)extend_seed_part(res, mc.aparams, nam, mc.refs, read, consistent);
            tries++;
        }
    }
    stats.add(det);
}

// ------------------------------------------------------ SW job strings ---
// part2_extend_seed_get_str (pc.cpp:214-242): the window is the NAM's projection
// onto the reference widened by |ref span - query span| and up to 50 bases on
// each side (size_t arithmetic; std::string::substr clamps at the contig's end)
void extension_window(const Nam& nam, size_t read_len, size_t contig_len, uint32_t& start, uint32_t& len) {
    const auto projected_ref_start = std::max(0, nam.ref_start - nam.query_start);
    const int diff = std::abs((nam.ref_end - nam.ref_start) - (nam.query_end - nam.query_start));
    const int ext_left = std::min(50, projected_ref_start);
    const int ref_start = projected_ref_start - ext_left;
    const int ext_right = (int)std::min(std::size_t(50), contig_len - nam.ref_end);
    const size_t ref_segm_size = read_len + diff + ext_left + ext_right;
    start = (uint32_t)ref_start;
    len = (uint32_t)std::min(ref_segm_size, contig_len - (size_t)ref_start);
}

static void extend_job(const Nam& nam, const Read& read, const References& refs, std::vector<SwJob>& jobs) {
    std::string_view query = nam.is_rc ? std::string_view(read.rc) : std::string_view(read.seq);
    uint32_t start, len;
    extension_window(nam, read.size(), refs.seq(nam.ref_id).size(), start, len);
    jobs.push_back(SwJob{query, nam.ref_id, start, len});
}

// part2_rescue_mate_get_str (pc.cpp:333-368)
void rescue_mate_window(const Nam& nam, size_t read_len, float mu, float sigma, size_t contig_len, uint32_t& start,
                        uint32_t& len) {
    int ref_start, ref_end;
    rescue_window(nam, read_len, mu, sigma, (int)contig_len, ref_start, ref_end);
    const size_t s0 = std::min((size_t)ref_start, contig_len);
    start = (uint32_t)s0;
    len = (uint32_t)std::min((size_t)(ref_end - ref_start), contig_len - s0);
}

static void rescue_job(const Nam& nam, const Read& read, const References& refs, float mu, float sigma,
                       std::vector<SwJob>& jobs, int shared_k) {
    std::string_view r_tmp = nam.is_rc ? std::string_view(read.seq) : std::string_view(read.rc);
    uint32_t start, len;
    rescue_mate_window(nam, read.size(), mu, sigma, refs.seq(nam.ref_id).size(), start, len);
    jobs.push_back(SwJob{r_tmp, nam.ref_id, start, len, shared_k});
}
// the k of a rescue slot whose has_shared_substring test the engine makes, else 0
static inline int shared_k_of(const AlignTmpRes& res, size_t j, const MapContext& mc) {
    return res.align_res[j].edit_distance == kSharedDeferred ? mc.iparams.k : 0;
}

void collect_jobs_pe(AlignTmpRes& res, const RecView&, const RecView&, const Read& read1, const Read& read2,
                     const MapContext& mc, float mu, float sigma, std::vector<SwJob>& jobs) {
    const size_t n = res.todo_nams.size();
    auto rd = [&](size_t j) -> const Read& { return res.is_read1[j] ? read1 : read2; };
    if (res.type == 1 || res.type == 2) {
        for (size_t j = 0; j < n; j += 2) {
            if (!res.done_align[j]) extend_job(res.todo_nams[j], rd(j), mc.refs, jobs);
            if (!res.done_align[j + 1])
                rescue_job(res.todo_nams[j + 1], rd(j + 1), mc.refs, mu, sigma, jobs, shared_k_of(res, j + 1, mc));
        }
    } else if (res.type == 3) {
        if (!res.done_align[0]) extend_job(res.todo_nams[0], rd(0), mc.refs, jobs);
        if (!res.done_align[1]) extend_job(res.todo_nams[1], rd(1), mc.refs, jobs);
    } else if (res.type == 4) {
        for (size_t j = 0; j < n; ++j) {
            if (res.done_align[j]) continue;
            if (res.is_extend_seed[j]) extend_job(res.todo_nams[j], rd(j), mc.refs, jobs);
            else rescue_job(res.todo_nams[j], rd(j), mc.refs, mu, sigma, jobs, shared_k_of(res, j, mc));
        }
    }
}

// part2_extend_seed_store_res (pc.cpp:177-212): the alignment's reference start is
// the window start plus the aligner's; global_ed adds both soft clips
void extension_alignment(const Nam& nam, size_t read_len, AlignmentInfo& info, Alignment& a) {
    const auto projected_ref_start = std::max(0, nam.ref_start - nam.query_start);
    const int ext_left = std::min(50, projected_ref_start);
    const int ref_start = projected_ref_start - ext_left;
    int result_ref_start = ref_start + (int)info.ref_start;
    int softclipped = (int)info.query_start + ((int)read_len - (int)info.query_end);
    a.cigar = std::move(info.cigar);               // each result is stored exactly once
    a.edit_distance = (int)info.edit_distance;
    a.global_ed = (int)info.edit_distance + softclipped;
    a.score = info.sw_score;
    a.ref_start = result_ref_start;
    a.length = info.ref_span();
    a.is_rc = nam.is_rc;
    a.is_unaligned = false;
    a.ref_id = nam.ref_id;
    a.gapped = true;
}

static void store_extend(AlignTmpRes& res, size_t j, const Read& read, AlignmentInfo& info) {
    extension_alignment(res.todo_nams[j], read.size(), info, res.align_res[j]);
}

// part2_rescue_mate_store_res (pc.cpp:291-331): the mate lands on the other strand;
// an empty CIGAR (the aligner's sentinels) leaves it unaligned.  global_ed and
// gapped keep what part() left in the slot
void rescue_alignment(const Nam& nam, size_t read_len, float mu, float sigma, size_t contig_len, AlignmentInfo& info,
                      Alignment& a) {
    int ref_start, ref_end;
    rescue_window(nam, read_len, mu, sigma, (int)contig_len, ref_start, ref_end);
    a.is_unaligned = info.cigar.empty();
    a.cigar = std::move(info.cigar);               // each result is stored exactly once
    a.edit_distance = (int)info.edit_distance;
    a.score = info.sw_score;
    a.ref_start = ref_start + (int)info.ref_start;
    a.is_rc = !nam.is_rc;
    a.ref_id = nam.ref_id;
    a.length = info.ref_span();
}

static void store_rescue(AlignTmpRes& res, size_t j, const Read& read, const References& refs, float mu, float sigma,
                         AlignmentInfo& info) {
    const Nam& nam = res.todo_nams[j];
    if (info.no_shared) {                          // rescue_mate_part's unaligned result (aln.cpp:1060-1069)
        Alignment& a = res.align_res[j];
        a.cigar = Cigar();
        a.edit_distance = (int)read.size();
        a.score = 0;
        a.ref_start = 0;
        a.is_rc = nam.is_rc;
        a.ref_id = nam.ref_id;
        a.is_unaligned = true;
        return;
    }
    rescue_alignment(nam, read.size(), mu, sigma, refs.seq(nam.ref_id).size(), info, res.align_res[j]);
}

size_t store_results_pe(AlignTmpRes& res, const Read& read1, const Read& read2, const MapContext& mc, float mu,
                        float sigma, std::vector<AlignmentInfo>& infos, size_t pos) {
    const size_t n = res.todo_nams.size();
    auto rd = [&](size_t j) -> const Read& { return res.is_read1[j] ? read1 : read2; };
    if (res.type == 1 || res.type == 2) {
        for (size_t j = 0; j < n; j += 2) {
            if (!res.done_align[j]) store_extend(res, j, rd(j), infos[pos++]);
            if (!res.done_align[j + 1]) store_rescue(res, j + 1, rd(j + 1), mc.refs, mu, sigma, infos[pos++]);
        }
    } else if (res.type == 3) {
        if (!res.done_align[0]) store_extend(res, 0, rd(0), infos[pos++]);
        if (!res.done_align[1]) store_extend(res, 1, rd(1), infos[pos++]);
    } else if (res.type == 4) {
        for (size_t j = 0; j < n; ++j) {
            if (res.done_align[j]) continue;
            if (res.is_extend_seed[j]) store_extend(res, j, rd(j), infos[pos++]);
            else store_rescue(res, j, rd(j), mc.refs, mu, sigma, infos[pos++]);
        }
    }
    return pos;
}

void collect_jobs_se(AlignTmpRes& res, const Read& read, const MapContext& mc, std::vector<SwJob>& jobs) {
    if (res.type != 4) return;
    for (size_t j = 0; j < res.todo_nams.size(); ++j)
        if (!res.done_align[j] && res.is_extend_seed[j]) extend_job(res.todo_nams[j], read, mc.refs, jobs);
}

size_t store_results_se(AlignTmpRes& res, const Read& read, const MapContext& mc,
                        std::vector<AlignmentInfo>& infos, size_t pos) {
    if (res.type != 4) return pos;
    for (size_t j = 0; j < res.todo_nams.size(); ++j)
        if (!res.done_align[j] && res.is_extend_seed[j]) store_extend(res, j, read, infos[pos++]);
    return pos;
}

// -------------------------------------------------------------- last ---
// the alignments stay where they are (the pair's results, or the rescue lists):
// sorting and deduplicating the pairs moves two pointers, not two CIGARs
struct ScoredAlignmentPair { double score; const Alignment* alignment1; const Alignment* alignment2; };

static inline float normal_pdf(float x, float mu, float sigma) {   // aln.cpp:528-533
    static const float inv_sqrt_2pi = 0.3989422804014327;
    const float a = (x - mu) / sigma;
    return inv_sqrt_2pi / sigma * std::exp(-0.5f * a * a);
}

// aln.cpp:535-550
static void get_best_scoring_pairs(std::vector<ScoredAlignmentPair>& pairs, const std::vector<Alignment>& al1,
                                                               const std::vector<Alignment>& al2, float mu, float sigma) {
    pairs.clear();
    for (auto& a1 : al1) {
        for (auto& a2 : al2) {
            float dist = std::abs(a1.ref_start - a2.ref_start);
            double score = a1.score + a2.score;
            if ((a1.is_rc ^ a2.is_rc) && (dist < mu + 4 * sigma)) score += log(normal_pdf(dist, mu, sigma));
            else score -= 10;
            pairs.push_back(ScoredAlignmentPair{score, &a1, &a2});
        }
    }
}

static std::pair<int, int> joint_mapq_from_high_scores(const std::vector<ScoredAlignmentPair>& pairs) {  // aln.cpp:506-526
    if (pairs.size() <= 1) return {60, 60};
    auto score1 = pairs[0].score;
    auto score2 = pairs[1].score;
    if (score1 == score2) return {0, 0};
    int mapq;
    const int diff = score1 - score2;
    if (score1 > 0 && score2 > 0) mapq = std::min(60, diff);
    else if (score1 > 0 && score2 <= 0) mapq = 60;
    else mapq = 1;
    return {mapq, mapq};
}

static void deduplicate_scored_pairs(std::vector<ScoredAlignmentPair>& pairs) {   // aln.cpp:1082-1105
    int p1 = pairs[0].alignment1->ref_start, p2 = pairs[0].alignment2->ref_start;
    int i1 = pairs[0].alignment1->ref_id, i2 = pairs[0].alignment2->ref_id;
    size_t j = 1;
    for (size_t i = 1; i < pairs.size(); i++) {
        int s1 = pairs[i].alignment1->ref_start, s2 = pairs[i].alignment2->ref_start;
        int d1 = pairs[i].alignment1->ref_id, d2 = pairs[i].alignment2->ref_id;
        if (s1 != p1 || s2 != p2 || d1 != i1 || d2 != i2) {
            p1 = s1; p2 = s2; i1 = d1; i2 = d2;
            pairs[j] = pairs[i];
            j++;
        }
    }
    pairs.resize(j);
}

static void pick_random_top_pair(std::vector<ScoredAlignmentPair>& hs, std::minstd_rand& rng) {   // aln.cpp:1111-1127
    size_t i = 1;
    for (; i < hs.size(); ++i)
        if (hs[i].score != hs[0].score) break;
    if (i > 1) {
        size_t ri = std::uniform_int_distribution<>(0, i - 1)(rng);
        if (ri != 0) std::swap(hs[0], hs[ri]);
    }
}

// rescue_read_last (aln.cpp:1983-2081)
static void rescue_read_last(AlignTmpRes& res, const Read& read2, const Read& read1, const MapContext& mc,
                             Details det[2], float mu, float sigma, Sam& sam, const RecView& rec1, const RecView& rec2,
                             bool swap_r1r2, std::minstd_rand& rng) {
    RSA_TLS std::vector<Alignment> al1, al2;
    al1.clear();
    al2.clear();
    const size_t n = res.todo_nams.size();
    for (size_t i = 0; i < n; i += 2) {              // res is not read again: the alignments move
        det[1].mate_rescue += !res.align_res[i + 1].is_unaligned;
        al1.push_back(std::move(res.align_res[i]));
        al2.push_back(std::move(res.align_res[i + 1]));
    }
    std::sort(al1.begin(), al1.end(), by_score<Alignment>);
    std::sort(al2.begin(), al2.end(), by_score<Alignment>);
    RSA_TLS std::vector<ScoredAlignmentPair> hs;
    get_best_scoring_pairs(hs, al1, al2, mu, sigma);
    std::sort(hs.begin(), hs.end(), by_score<ScoredAlignmentPair>);
    deduplicate_scored_pairs(hs);
    pick_random_top_pair(hs, rng);
    auto [mapq1, mapq2] = joint_mapq_from_high_scores(hs);
    const double secondary_dropoff = 2 * mc.aparams.mismatch + mc.aparams.gap_open;
    if (mc.mparams.max_secondary == 0) {
        const Alignment& a1 = *hs[0].alignment1;
        const Alignment& a2 = *hs[0].alignment2;
        if (swap_r1r2) sam.add_pair(a2, a1, rec2, rec1, read2.rc, read1.rc, mapq2, mapq1, is_proper_pair(a2, a1, mu, sigma), true, det);
        else sam.add_pair(a1, a2, rec1, rec2, read1.rc, read2.rc, mapq1, mapq2, is_proper_pair(a1, a2, mu, sigma), true, det);
    } else {
        auto max_out = std::min(hs.size(), (size_t)mc.mparams.max_secondary);
        bool is_primary = true;
        auto s_max = hs[0].score;
        for (size_t i = 0; i < max_out; ++i) {
            if (i > 0) { is_primary = false; mapq1 = 0; mapq2 = 0; }
            const auto& ap = hs[i];
            if (s_max - ap.score < secondary_dropoff) {
                if (swap_r1r2) {
                    bool proper = is_proper_pair(*ap.alignment2, *ap.alignment1, mu, sigma);
                    Details sw[2] = {det[1], det[0]};
                    sam.add_pair(*ap.alignment2, *ap.alignment1, rec2, rec1, read2.rc, read1.rc, mapq2, mapq1, proper, is_primary, sw);
                } else {
                    bool proper = is_proper_pair(*ap.alignment1, *ap.alignment2, mu, sigma);
                    sam.add_pair(*ap.alignment1, *ap.alignment2, rec1, rec2, read1.rc, read2.rc, mapq1, mapq2, proper, is_primary, det);
                }
            } else break;
        }
    }
}

// align_PE_read_last (aln.cpp:2083-2306)
void align_PE_read_last(AlignTmpRes& res, const RecView& rec1, const RecView& rec2, const Read& read1, const Read& read2,
                        Sam& sam,
                        AlignmentStatistics& stats, const InsertSizeDistribution& isize, const MapContext& mc,
                        std::minstd_rand& rng) {
    Details det[2];
    const float mu = isize.mu, sigma = isize.sigma;
    if (res.type == 0) {
        sam.add_unmapped_pair(rec1, rec2);
    } else if (res.type == 1) {
        rescue_read_last(res, read2, read1, mc, det, mu, sigma, sam, rec1, rec2, false, rng);
    } else if (res.type == 2) {
        rescue_read_last(res, read1, read2, mc, det, mu, sigma, sam, rec2, rec1, true, rng);   // details unswapped (sic)
    } else if (res.type == 3) {
        const Alignment& a1 = res.align_res[0];
        const Alignment& a2 = res.align_res[1];
        bool proper = is_proper_pair(a1, a2, mu, sigma);
        sam.add_pair(a1, a2, rec1, rec2, read1.rc, read2.rc, (uint8_t)res.mapq1, (uint8_t)res.mapq2, proper, true, det);
    } else if (res.type == 4) {
        size_t pos = 0;
        // nam_id -> the alignment computed for it (small; linear lookup).  The cache and
        // the loop hold pointers into res.align_res, which does not change here, so an
        // alignment is copied once, into its scored pair
        RSA_TLS std::vector<std::pair<int, const Alignment*>> cache1, cache2;
        cache1.clear();
        cache2.clear();
        auto find_c = [](const std::vector<std::pair<int, const Alignment*>>& c, int id) -> const Alignment* {
            for (const auto& x : c) if (x.first == id) return x.second;
            return nullptr;
        };
        const Alignment* a1_indv_max = &res.align_res[pos];
        cache1.push_back({res.todo_nams[pos].nam_id, a1_indv_max});
        pos++;
        const Alignment* a2_indv_max = &res.align_res[pos];
        cache2.push_back({res.todo_nams[pos].nam_id, a2_indv_max});
        pos++;
        RSA_TLS std::vector<ScoredAlignmentPair> hs;
        hs.clear();
        for (int i = 0; i < res.type4_loop_size; ++i) {
            const Nam& n1 = res.type4_nams[2 * i];
            const Nam& n2 = res.type4_nams[2 * i + 1];
            const Alignment* p1;
            const Alignment* p2;
            if (n1.ref_start >= 0) {
                p1 = find_c(cache1, n1.nam_id);
                if (!p1) { p1 = &res.align_res[pos]; pos++; cache1.push_back({n1.nam_id, p1}); }
            } else {
                p1 = &res.align_res[pos]; pos++;
                det[0].mate_rescue += !p1->is_unaligned;
            }
            if (p1->score > a1_indv_max->score) a1_indv_max = p1;
            if (n2.ref_start >= 0) {
                p2 = find_c(cache2, n2.nam_id);
                if (!p2) { p2 = &res.align_res[pos]; pos++; cache2.push_back({n2.nam_id, p2}); }
            } else {
                p2 = &res.align_res[pos]; pos++;
                det[1].mate_rescue += !p2->is_unaligned;
            }
            if (p2->score > a2_indv_max->score) a2_indv_max = p2;
            const Alignment& a1 = *p1;
            const Alignment& a2 = *p2;
            bool r1_r2 = a2.is_rc && (a1.ref_start <= a2.ref_start) && ((a2.ref_start - a1.ref_start) < mu + 10 * sigma);
            bool r2_r1 = a1.is_rc && (a2.ref_start <= a1.ref_start) && ((a1.ref_start - a2.ref_start) < mu + 10 * sigma);
            double combined;
            if (r1_r2 || r2_r1) {
                float x = std::abs(a1.ref_start - a2.ref_start);
                combined = (double)a1.score + (double)a2.score + std::max(-20.0f + 0.001f, log(normal_pdf(x, mu, sigma)));
            } else {
                combined = (double)a1.score + (double)a2.score - 20;
            }
            hs.push_back(ScoredAlignmentPair{combined, p1, p2});
        }
        double combined = (double)a1_indv_max->score + (double)a2_indv_max->score - 20;
        hs.push_back(ScoredAlignmentPair{combined, a1_indv_max, a2_indv_max});
        std::sort(hs.begin(), hs.end(), by_score<ScoredAlignmentPair>);
        deduplicate_scored_pairs(hs);
        pick_random_top_pair(hs, rng);
        auto [mapq1, mapq2] = joint_mapq_from_high_scores(hs);
        const auto& best = hs[0];
        if (mc.mparams.max_secondary == 0) {
            bool proper = is_proper_pair(*best.alignment1, *best.alignment2, mu, sigma);
            sam.add_pair(*best.alignment1, *best.alignment2, rec1, rec2, read1.rc, read2.rc, mapq1, mapq2, proper, true, det);
        } else {
            auto max_out = std::min(hs.size(), (size_t)mc.mparams.max_secondary);
            float s_max = best.score;
            bool is_primary = true;
            const double sd = 2 * mc.aparams.mismatch + mc.aparams.gap_open;
            for (size_t i = 0; i < max_out; ++i) {
                const auto& ap = hs[i];
                float s_score = ap.score;
                if (i > 0) { is_primary = false; mapq1 = 255; mapq2 = 255; }
                if (s_max - s_score < sd) {
                    bool proper = is_proper_pair(*ap.alignment1, *ap.alignment2, mu, sigma);
                    sam.add_pair(*ap.alignment1, *ap.alignment2, rec1, rec2, read1.rc, read2.rc, mapq1, mapq2, proper, is_primary, det);
                } else break;
            }
        }
    }
    stats.add(det[0]);
    stats.add(det[1]);
}

// align_SE_read_last (aln.cpp:126-238)
void align_SE_read_last(AlignTmpRes& res, const RecView& rec, const Read& read, Sam& sam, AlignmentStatistics& stats,
                        const MapContext& mc, std::minstd_rand& rng) {
    Details det;
    if (res.type == 0) {
        sam.add_unmapped(rec);
        return;
    }
    std::vector<Alignment> alignments;
    int tries = 0;
    const Nam n_max = res.todo_nams[0];
    int best_edit_distance = INT_MAX, best_score = 0, second_best_score = 0, alignments_with_best_score = 0;
    size_t best_index = 0;
    Alignment best_alignment;
    best_alignment.is_unaligned = true;
    const int max_secondary = mc.mparams.max_secondary;
    for (size_t i = 0; i < res.todo_nams.size(); i++) {
        const Nam& nam = res.todo_nams[i];
        float score_dropoff = (float)nam.n_hits / n_max.n_hits;
        if (tries >= mc.mparams.max_tries || (tries > 1 && best_edit_distance == 0) ||
            score_dropoff < mc.mparams.dropoff_threshold) {
            for (size_t j = i; j < res.todo_nams.size(); j++)
                if (!res.done_align[j]) stats.tot_aligner_calls--;
            break;
        }
        bool consistent = res.consistent_nam[i];
        det.nam_inconsistent += !consistent;
        Alignment alignment = res.align_res[i];
        det.tried_alignment++;
        det.gapped += alignment.gapped;
        if (max_secondary > 0) alignments.emplace_back(alignment);
        if (alignment.score >= best_score) {
            second_best_score = best_score;
            bool update_best = false;
            if (alignment.score > best_score) {
                alignments_with_best_score = 1;
                update_best = true;
            } else {
                alignments_with_best_score++;
                std::uniform_int_distribution<> distrib(1, alignments_with_best_score);
                if (distrib(rng) == 1) update_best = true;
            }
            if (update_best) {
                best_score = alignment.score;
                best_alignment = std::move(alignment);
                best_index = (size_t)tries;
                if (max_secondary == 0) best_edit_distance = best_alignment.global_ed;
            }
        } else if (alignment.score > second_best_score) {
            second_best_score = alignment.score;
        }
        tries++;
    }
    // (60.0 * (best - second) + best - 1) / best as a double -> uint8_t (x86: via int32 truncation)
    const double mq = (60.0 * (best_score - second_best_score) + best_score - 1) / best_score;
    int32_t mq32 = (std::isnan(mq) || mq >= 2147483648.0 || mq < -2147483648.0) ? INT32_MIN : (int32_t)mq;
    uint8_t mapq = (uint8_t)mq32;
    sam.add(best_alignment, rec, read.rc, mapq, true, det);
    if (max_secondary == 0) {
        stats.add(det);
        return;
    }
    if (alignments.size() > 1) std::swap(alignments[best_index], alignments[alignments.size() - 1]);
    alignments.resize(alignments.size() - 1);
    std::sort(alignments.begin(), alignments.end(), [](const Alignment& a, const Alignment& b) { return a.score > b.score; });
    size_t n = 0;
    for (const auto& a : alignments) {
        if (n >= (size_t)max_secondary || a.score - best_score > 2 * mc.aparams.mismatch + mc.aparams.gap_open) break;
        sam.add(a, rec, read.rc, mapq, false, det);
        n++;
    }
    stats.add(det);
}

}  // namespace rsa
