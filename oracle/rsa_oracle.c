/*
 * rsa_oracle.c -- CPU restatement (parity oracle) of the RabbitSAlign hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see rsa_oracle.h).  Written from the semantics of
 * the reference, not copied: each block cites the reference file:line whose
 * behaviour it restates.  Pinned by tests/test_oracle_golden.py against vectors
 * emitted by the reference's own sources (oracle/_ref/refgen).
 */
#include "rsa_oracle.h"

#include <limits.h>
#include <stdlib.h>
#include <string.h>

/* ===================================================================== */
/* xxh64 of one u64 -- hash.hpp:105-118                                  */
/* ===================================================================== */
#define P1 0x9E3779B185EBCA87ULL
#define P2 0xC2B2AE3D27D4EB4FULL
#define P3 0x165667B19E3779F9ULL
#define P4 0x85EBCA77C2B2AE63ULL
#define P5 0x27D4EB2F165667C5ULL

static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

uint64_t ora_xxh64(uint64_t input) {
    uint64_t acc = P5 + 8;
    uint64_t k1 = rotl64(input * P2, 31) * P1;
    acc ^= k1;
    acc = rotl64(acc, 27) * P1 + P4;
    acc ^= acc >> 33;
    acc *= P2;
    acc ^= acc >> 29;
    acc *= P3;
    acc ^= acc >> 32;
    return acc;
}

/* ===================================================================== */
/* canonical open syncmers -- randstrobes.cpp:14-31 (nt4 table), 57-118   */
/* ===================================================================== */
static int nt4(unsigned char c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': case 'U': case 'u': return 3;
        default: return 4;
    }
}

typedef struct { uint64_t hash; uint32_t pos; } ora_syncmer;

/* Returns the number of syncmers.  The window of k-s+1 s-mer hashes is a ring;
 * min tracking follows randstrobes.cpp:77-102 exactly (first fill: leftmost
 * minimum; after popping the minimum: rescan right-to-left keeping the
 * rightmost minimum; a new strictly smaller value takes over). */
static int ora_syncmers(const char* seq, int len, const ora_params* p, ora_syncmer* out) {
    const int k = p->k, s = p->s, t = p->t_syncmer;
    const uint64_t kmask = (k == 32) ? ~0ULL : ((1ULL << (2 * k)) - 1);
    const uint64_t smask = (1ULL << (2 * s)) - 1;
    const int kshift = (k - 1) * 2, sshift = (s - 1) * 2;
    const int W = k - s + 1;
    uint64_t ring[64];
    int qn = 0, qhead = 0; /* ring holds qn values starting at qhead */
    uint64_t min_val = UINT64_MAX;
    long long min_pos = -1;
    int l = 0;
    uint64_t xk0 = 0, xk1 = 0, xs0 = 0, xs1 = 0;
    int n = 0;
    for (int i = 0; i < len; ++i) {
        int c = nt4((unsigned char)seq[i]);
        if (c < 4) {
            xk0 = ((xk0 << 2) | (uint64_t)c) & kmask;
            xk1 = (xk1 >> 2) | ((uint64_t)(3 - c) << kshift);
            xs0 = ((xs0 << 2) | (uint64_t)c) & smask;
            xs1 = (xs1 >> 2) | ((uint64_t)(3 - c) << sshift);
            if (++l < s) continue;
            uint64_t ys = xs0 < xs1 ? xs0 : xs1;
            uint64_t hs = ora_xxh64(ys);
            ring[(qhead + qn) & 63] = hs;
            qn++;
            if (qn < W) continue;
            if (qn == W) {
                for (int j = 0; j < qn; ++j) {
                    uint64_t v = ring[(qhead + j) & 63];
                    if (v < min_val) { min_val = v; min_pos = (long long)i - k + j + 1; }
                }
            } else {
                qhead = (qhead + 1) & 63; qn--;           /* pop_front */
                if (min_pos == (long long)i - k) {        /* popped the minimum: rescan */
                    min_val = UINT64_MAX;
                    min_pos = (long long)i - s + 1;
                    for (int j = qn - 1; j >= 0; --j) {
                        uint64_t v = ring[(qhead + j) & 63];
                        if (v < min_val) { min_val = v; min_pos = (long long)i - k + j + 1; }
                    }
                } else if (hs < min_val) {
                    min_val = hs;
                    min_pos = (long long)i - s + 1;
                }
            }
            if (min_pos == (long long)i - k + t) {
                uint64_t yk = xk0 < xk1 ? xk0 : xk1;
                out[n].hash = ora_xxh64(yk);
                out[n].pos = (uint32_t)(i - k + 1);
                n++;
            }
        } else {
            min_val = UINT64_MAX; min_pos = -1;
            l = 0; xs0 = xs1 = xk0 = xk1 = 0;
            qn = 0; qhead = 0;
        }
    }
    return n;
}

/* RandstrobeIterator::get -- randstrobes.cpp:148-171 */
static void ora_rs_get(const ora_syncmer* sm, int n, int i, const ora_params* p, uint64_t* hash,
                       uint32_t* pos1, uint32_t* pos2) {
    int w_end = i + p->w_max < n - 1 ? i + p->w_max : n - 1;
    uint64_t max_position = (uint64_t)sm[i].pos + (unsigned)p->max_dist;
    uint64_t min_val = UINT64_MAX;
    int best = i;
    for (int j = i + p->w_min; j <= w_end && sm[j].pos <= max_position; ++j) {
        uint64_t res = (uint64_t)__builtin_popcountll((sm[i].hash ^ sm[j].hash) & p->q);
        if (res < min_val) { min_val = res; best = j; }
    }
    *hash = sm[i].hash + sm[best].hash;
    *pos1 = sm[i].pos;
    *pos2 = sm[best].pos;
}

/* randstrobes_query -- randstrobes.cpp:207-253 */
int ora_randstrobes_query(const char* seq, int len, const ora_params* p, ora_qrs* out, int cap) {
    if (len < p->w_max) return 0;
    ora_syncmer* sm = (ora_syncmer*)malloc(sizeof(ora_syncmer) * (size_t)(len + 1));
    int n = ora_syncmers(seq, len, p, sm);
    int cnt = 0;
    if (n == 0) { free(sm); return 0; }
    for (int i = 0; i + p->w_min < n; ++i) {
        if (cnt >= cap) { free(sm); return -1; }
        uint64_t h; uint32_t a, b;
        ora_rs_get(sm, n, i, p, &h, &a, &b);
        out[cnt].hash = h; out[cnt].start = a; out[cnt].end = b + (uint32_t)p->k; out[cnt].is_reverse = 0;
        cnt++;
    }
    /* reverse complement: reuse syncmers, reversed, coordinates mirrored */
    for (int i = 0, j = n - 1; i < j; ++i, --j) { ora_syncmer t = sm[i]; sm[i] = sm[j]; sm[j] = t; }
    for (int i = 0; i < n; ++i) sm[i].pos = (uint32_t)(len - (int)sm[i].pos - p->k);
    for (int i = 0; i + p->w_min < n; ++i) {
        if (cnt >= cap) { free(sm); return -1; }
        uint64_t h; uint32_t a, b;
        ora_rs_get(sm, n, i, p, &h, &a, &b);
        out[cnt].hash = h; out[cnt].start = a; out[cnt].end = b + (uint32_t)p->k; out[cnt].is_reverse = 1;
        cnt++;
    }
    free(sm);
    return cnt;
}

/* ===================================================================== */
/* index lookups -- index.hpp:57-147                                     */
/* ===================================================================== */
#define ORA_END UINT64_MAX

/* StrobemerIndex::find (index.hpp:57-81) and its unrolled copy nam.cpp:779-905:
 * first index in the bucket whose hash equals key, else end(). */
static uint64_t ora_find(const ora_index* ix, uint64_t key) {
    uint64_t top = key >> (64 - ix->bits);
    uint64_t a = ix->starts[top], b = ix->starts[top + 1];
    /* linear scan (<4 entries) and lower_bound both return the first equal hash */
    uint64_t lo = a, hi = b;
    while (lo < hi) {
        uint64_t mid = lo + (hi - lo) / 2;
        if (ix->rs[mid].hash < key) lo = mid + 1; else hi = mid;
    }
    if (lo < b && ix->rs[lo].hash == key) return lo;
    return ORA_END;
}

static uint64_t ora_get_hash(const ora_index* ix, uint64_t pos) {
    return pos < ix->n ? ix->rs[pos].hash : ORA_END;   /* index.hpp:83-89 */
}

static int ora_is_filtered(const ora_index* ix, uint64_t pos) {   /* index.hpp:91-93 */
    return ora_get_hash(ix, pos) == ora_get_hash(ix, pos + ix->filter_cutoff);
}

static unsigned ora_get_count(const ora_index* ix, uint64_t pos) { /* index.hpp:115-147 */
    uint64_t key = ix->rs[pos].hash;
    unsigned c = 1;
    for (uint64_t p = pos + 1; p < ix->n && ix->rs[p].hash == key; ++p) c++;
    return c;
}

/* ===================================================================== */
/* robin_hood::unordered_flat_map<unsigned, ...> slot-order emulation     */
/* (ext/robin_hood.h v3.11.1: keyToIdx 1348-1360, hash_int 748-759,        */
/*  insertKeyPrepareEmptySpot 2331-2376, shiftUp 1377-1393,                */
/*  increase_size 2413-2442, try_increase_info 2382-2411,                  */
/*  rehashPowerOfTwo 2203-2234, insert_move 1453-1489, reserve 2179-2198)  */
/* Only the key->slot layout matters: iteration is in slot order.          */
/* ===================================================================== */
typedef struct rh_map {
    uint64_t mult;
    size_t mask, num, max_allowed, nwb;
    uint32_t info_inc, info_shift;
    uint8_t* info;      /* nwb + 8 bytes */
    uint32_t* keys;
    int32_t* vals;
} rh_map;

static size_t rh_calc_max(size_t n) { return n * 80 / 100; }
static size_t rh_calc_nwb(size_t n) { size_t m = rh_calc_max(n); return n + (m < 0xFF ? m : 0xFF); }

static void rh_init_data(rh_map* m, size_t max_elements) {
    m->num = 0;
    m->mask = max_elements - 1;
    m->max_allowed = rh_calc_max(max_elements);
    m->nwb = rh_calc_nwb(max_elements);
    m->info = (uint8_t*)calloc(m->nwb + 16, 1);
    m->keys = (uint32_t*)calloc(m->nwb + 16, sizeof(uint32_t));
    m->vals = (int32_t*)calloc(m->nwb + 16, sizeof(int32_t));
    m->info[m->nwb] = 1; /* sentinel */
    m->info_inc = 32;
    m->info_shift = 0;
}

static void rh_key_to_idx(const rh_map* m, uint32_t key, size_t* idx, uint32_t* info) {
    uint64_t h = (uint64_t)key;
    h ^= h >> 33; h *= 0xff51afd7ed558ccdULL; h ^= h >> 33;   /* hash_int */
    h *= m->mult;
    h ^= h >> 33;
    *info = m->info_inc + (uint32_t)((h & 31u) >> m->info_shift);
    *idx = (size_t)(h >> 5) & m->mask;
}

static void rh_shift_up(rh_map* m, size_t start, size_t ins) {
    for (size_t i = start; i != ins; --i) { m->keys[i] = m->keys[i - 1]; m->vals[i] = m->vals[i - 1]; }
    for (size_t i = start; i != ins; --i) {
        m->info[i] = (uint8_t)(m->info[i - 1] + m->info_inc);
        if ((uint32_t)m->info[i] + m->info_inc > 0xFF) m->max_allowed = 0;
    }
}

static int rh_try_increase_info(rh_map* m) {
    if (m->info_inc <= 2) return 0;
    m->info_inc >>= 1;
    m->info_shift++;
    size_t nwb = rh_calc_nwb(m->mask + 1);
    for (size_t i = 0; i < nwb; i += 8)
        for (size_t b = 0; b < 8; ++b) m->info[i + b] = (uint8_t)(m->info[i + b] >> 1);
    m->info[nwb] = 1;
    m->max_allowed = rh_calc_max(m->mask + 1);
    return 1;
}

static void rh_insert_move(rh_map* m, uint32_t key, int32_t val) {
    if (m->max_allowed == 0 && !rh_try_increase_info(m)) abort();
    size_t idx; uint32_t info;
    rh_key_to_idx(m, key, &idx, &info);
    while (info <= m->info[idx]) { idx++; info += m->info_inc; }
    size_t ins = idx; uint8_t ins_info = (uint8_t)info;
    if ((uint32_t)ins_info + m->info_inc > 0xFF) m->max_allowed = 0;
    while (m->info[idx] != 0) { idx++; info += m->info_inc; }
    if (idx != ins) rh_shift_up(m, idx, ins);
    m->keys[ins] = key; m->vals[ins] = val;
    m->info[ins] = ins_info;
    m->num++;
}

static void rh_rehash(rh_map* m, size_t nb) {
    uint8_t* oinfo = m->info; uint32_t* okeys = m->keys; int32_t* ovals = m->vals;
    size_t onwb = rh_calc_nwb(m->mask + 1);
    rh_init_data(m, nb);
    if (onwb > 1) {
        for (size_t i = 0; i < onwb; ++i)
            if (oinfo[i] != 0) rh_insert_move(m, okeys[i], ovals[i]);
    }
    free(oinfo); free(okeys); free(ovals);
}

static void rh_increase_size(rh_map* m) {
    if (m->mask == 0) { free(m->info); free(m->keys); free(m->vals); rh_init_data(m, 8); return; }
    size_t maxa = rh_calc_max(m->mask + 1);
    if (m->num < maxa && rh_try_increase_info(m)) return;
    m->mult += 0xc4ceb9fe1a85ec54ULL;
    if (m->num * 2 < rh_calc_max(m->mask + 1)) rh_rehash(m, m->mask + 1);
    else rh_rehash(m, (m->mask + 1) * 2);
}

/* default construction followed by reserve(100) (nam.cpp:913-914 / 960-961) */
static void rh_new_reserved(rh_map* m) {
    m->mult = 0xc4ceb9fe1a85ec53ULL;
    m->mask = 0; m->num = 0; m->max_allowed = 0;
    m->info = (uint8_t*)calloc(16, 1); m->keys = (uint32_t*)calloc(16, 4); m->vals = (int32_t*)calloc(16, 4);
    m->info[1] = 1;
    m->info_inc = 32; m->info_shift = 0;
    size_t ns = 8;
    while (rh_calc_max(ns) < 100) ns *= 2;
    if (ns > m->mask + 1) rh_rehash(m, ns);
}

static void rh_free(rh_map* m) { free(m->info); free(m->keys); free(m->vals); }

/* operator[] -> returns slot value pointer; *inserted tells whether it was new */
static int32_t* rh_get_or_insert(rh_map* m, uint32_t key, int32_t new_val) {
    for (int attempt = 0; attempt < 256; ++attempt) {
        size_t idx; uint32_t info;
        rh_key_to_idx(m, key, &idx, &info);
        while (info < m->info[idx]) { idx++; info += m->info_inc; }
        while (info == m->info[idx]) {
            if (m->keys[idx] == key) return &m->vals[idx];
            idx++; info += m->info_inc;
        }
        if (m->num >= m->max_allowed) { rh_increase_size(m); continue; }
        size_t ins = idx; uint32_t ins_info = info;
        if (ins_info + m->info_inc > 0xFF) m->max_allowed = 0;
        while (m->info[idx] != 0) { idx++; info += m->info_inc; }
        if (idx != ins) rh_shift_up(m, idx, ins);
        m->info[ins] = (uint8_t)ins_info;
        m->keys[ins] = key; m->vals[ins] = new_val;
        m->num++;
        return &m->vals[ins];
    }
    abort();
}

static int32_t rh_find(const rh_map* m, uint32_t key) {
    if (m->num == 0) return -1;
    size_t idx; uint32_t info;
    rh_key_to_idx(m, key, &idx, &info);
    for (;;) {
        if (info == m->info[idx] && m->keys[idx] == key) return m->vals[idx];
        idx++; info += m->info_inc;
        if (info > m->info[idx]) {
            if (info == m->info[idx] && m->keys[idx] == key) return m->vals[idx];
            break;
        }
    }
    /* fall back to a linear probe; only used to decide membership */
    for (size_t i = 0; i < m->nwb; ++i) if (m->info[i] && m->keys[i] == key) return m->vals[i];
    return -1;
}

/* ===================================================================== */
/* hit lists                                                              */
/* ===================================================================== */
typedef struct { int32_t qs, qe, rs, re; } ora_hit;   /* Hit (nam.cpp:16-32) */

typedef struct { ora_hit* v; int n, cap; } hit_list;

typedef struct {
    rh_map map;           /* ref_id -> list index */
    hit_list* lists;
    int n_lists, cap_lists;
} hits_per_ref_t;

static void hpr_init(hits_per_ref_t* h) {
    rh_new_reserved(&h->map);
    h->n_lists = 0; h->cap_lists = 8;
    h->lists = (hit_list*)calloc((size_t)h->cap_lists, sizeof(hit_list));
}

static void hpr_free(hits_per_ref_t* h) {
    for (int i = 0; i < h->n_lists; ++i) free(h->lists[i].v);
    free(h->lists);
    rh_free(&h->map);
}

static hit_list* hpr_get(hits_per_ref_t* h, uint32_t ref_id) {
    int32_t* slot = rh_get_or_insert(&h->map, ref_id, h->n_lists);
    if (*slot == h->n_lists) {
        if (h->n_lists == h->cap_lists) {
            h->cap_lists *= 2;
            h->lists = (hit_list*)realloc(h->lists, sizeof(hit_list) * (size_t)h->cap_lists);
        }
        h->lists[h->n_lists].v = NULL; h->lists[h->n_lists].n = 0; h->lists[h->n_lists].cap = 0;
        h->n_lists++;
    }
    return &h->lists[*slot];
}

static void hl_push(hit_list* l, ora_hit x) {
    if (l->n == l->cap) { l->cap = l->cap ? l->cap * 2 : 16; l->v = (ora_hit*)realloc(l->v, sizeof(ora_hit) * (size_t)l->cap); }
    l->v[l->n++] = x;
}

/* add_to_hits_per_ref (nam.cpp:68-85) */
static void add_to_hits_per_ref(hits_per_ref_t* h, int qs, int qe, const ora_index* ix, uint64_t pos) {
    int min_diff = INT_MAX;
    uint64_t hash = ora_get_hash(ix, pos);
    for (; ora_get_hash(ix, pos) == hash; ++pos) {
        int rs = (int)ix->rs[pos].position;
        int re = rs + (int)(ix->rs[pos].packed & 0xFF) + ix->k;
        int d = (qe - qs) - (re - rs);
        if (d < 0) d = -d;
        if (d <= min_diff) {
            ora_hit x = {qs, qe, rs, re};
            hl_push(hpr_get(h, ix->rs[pos].packed >> 8), x);
            min_diff = d;
        }
    }
}

/* add_to_hits_per_ref_pre (nam.cpp:87-107): only pre-inserts map keys */
static void add_to_hits_per_ref_pre(hits_per_ref_t* h, int qs, int qe, const ora_index* ix, uint64_t pos) {
    int min_diff = INT_MAX;
    uint64_t hash = ora_get_hash(ix, pos);
    for (; ora_get_hash(ix, pos) == hash; ++pos) {
        int rs = (int)ix->rs[pos].position;
        int re = rs + (int)(ix->rs[pos].packed & 0xFF) + ix->k;
        int d = (qe - qs) - (re - rs);
        if (d < 0) d = -d;
        if (d <= min_diff) {
            (void)hpr_get(h, ix->rs[pos].packed >> 8);
            min_diff = d;
        }
    }
}

static int hit_less(const ora_hit* a, const ora_hit* b) {   /* Hit::operator< (nam.cpp:21-24) */
    if (a->qs == b->qs) return a->rs < b->rs;
    return a->qs < b->qs;
}

static void hits_sort(ora_hit* v, int n) {  /* keys are unique per list: any correct sort matches std::sort */
    for (int i = 1; i < n; ++i) {
        ora_hit x = v[i]; int j = i - 1;
        while (j >= 0 && hit_less(&x, &v[j])) { v[j + 1] = v[j]; --j; }
        v[j + 1] = x;
    }
}

/* ===================================================================== */
/* NAM output vector                                                      */
/* ===================================================================== */
typedef struct { ora_nam* v; int n, cap; int overflow; } nam_out;

static float nam_score(const ora_nam* n) {   /* nam.cpp:456-460 */
    int qspan = n->query_end - n->query_start, rspan = n->ref_end - n->ref_start;
    int mx = qspan > rspan ? qspan : rspan, mn = qspan < rspan ? qspan : rspan;
    return (2 * mn - mx) > 0 ? (float)(n->n_hits * (2 * mn - mx)) : 1.0f;
}

static void nams_emit(nam_out* o, ora_nam n) {
    n.score = nam_score(&n);
    n.nam_id = o->n;
    if (o->n < o->cap) o->v[o->n] = n; else o->overflow = 1;
    o->n++;
}

typedef struct { ora_nam* v; int n, cap; } open_vec;
static void ov_push(open_vec* o, ora_nam x) {
    if (o->n == o->cap) { o->cap = o->cap ? o->cap * 2 : 16; o->v = (ora_nam*)realloc(o->v, sizeof(ora_nam) * (size_t)o->cap); }
    o->v[o->n++] = x;
}

static ora_nam nam_from_hit(const ora_hit* h, int ref_id, int is_rc) {
    ora_nam n;
    memset(&n, 0, sizeof n);
    n.query_start = h->qs; n.query_end = h->qe; n.ref_start = h->rs; n.ref_end = h->re;
    n.ref_id = ref_id; n.query_prev_hit_startpos = h->qs; n.ref_prev_hit_startpos = h->rs;
    n.n_hits = 1; n.is_rc = is_rc;
    return n;
}

/* flush open NAMs passed by query_start (nam.cpp:476-496) */
static void flush_passed(open_vec* open, int query_start, nam_out* out) {
    int w = 0;
    for (int i = 0; i < open->n; ++i)
        if (open->v[i].query_end < query_start) nams_emit(out, open->v[i]);
    for (int i = 0; i < open->n; ++i)
        if (!(open->v[i].query_end < query_start)) open->v[w++] = open->v[i];
    open->n = w;
}

/* map iteration in slot order */
static int rh_slot_order(const rh_map* m, int32_t* order) {
    int c = 0;
    for (size_t i = 0; i < m->nwb; ++i) if (m->info[i]) order[c++] = m->vals[i];
    return c;
}

/* merge_hits_into_nams (nam.cpp:370-536), sort = true */
static void merge_hits_into_nams(hits_per_ref_t* h, int k, int is_rc, nam_out* out) {
    int32_t* order = (int32_t*)malloc(sizeof(int32_t) * (size_t)(h->map.nwb + 1));
    int no = rh_slot_order(&h->map, order);
    for (int oi = 0; oi < no; ++oi) {
        int li = order[oi];
        uint32_t ref_id = 0;
        for (size_t i = 0; i < h->map.nwb; ++i) if (h->map.info[i] && h->map.vals[i] == li) { ref_id = h->map.keys[i]; break; }
        hit_list* l = &h->lists[li];
        hits_sort(l->v, l->n);
        open_vec open = {0, 0, 0};
        unsigned prev_q_start = 0;
        for (int hi = 0; hi < l->n; ++hi) {
            const ora_hit* x = &l->v[hi];
            int added = 0;
            for (int oi2 = 0; oi2 < open.n; ++oi2) {
                ora_nam* o = &open.v[oi2];
                if (o->query_prev_hit_startpos < x->qs && x->qs <= o->query_end &&
                    o->ref_prev_hit_startpos < x->rs && x->rs <= o->ref_end) {
                    if (x->qe > o->query_end && x->re > o->ref_end) {
                        o->query_end = x->qe; o->ref_end = x->re;
                        o->query_prev_hit_startpos = x->qs; o->ref_prev_hit_startpos = x->rs;
                        o->n_hits++; added = 1; break;
                    } else if (x->qe <= o->query_end && x->re <= o->ref_end) {
                        o->query_prev_hit_startpos = x->qs; o->ref_prev_hit_startpos = x->rs;
                        o->n_hits++; added = 1; break;
                    }
                }
            }
            if (!added) ov_push(&open, nam_from_hit(x, (int)ref_id, is_rc));
            if ((unsigned)x->qs > prev_q_start + (unsigned)k) {
                flush_passed(&open, x->qs, out);
                prev_q_start = (unsigned)x->qs;
            }
        }
        for (int i = 0; i < open.n; ++i) nams_emit(out, open.v[i]);
        free(open.v);
    }
    free(order);
}

/* merge_hits_into_nams_fast (nam.cpp:117-366), sort = false */
static void merge_hits_into_nams_fast(hits_per_ref_t* h, int k, int is_rc, nam_out* out) {
    int32_t* order = (int32_t*)malloc(sizeof(int32_t) * (size_t)(h->map.nwb + 1));
    int no = rh_slot_order(&h->map, order);
    for (int oi = 0; oi < no; ++oi) {
        int li = order[oi];
        uint32_t ref_id = 0;
        for (size_t i = 0; i < h->map.nwb; ++i) if (h->map.info[i] && h->map.vals[i] == li) { ref_id = h->map.keys[i]; break; }
        hit_list* l = &h->lists[li];
        ora_hit* hits = l->v;
        open_vec open = {0, 0, 0};
        unsigned prev_q_start = 0;
        for (int i = 0; i < l->n;) {
            int i_start = i, i_end = i + 1;
            while (i_end < l->n && hits[i_end].qs == hits[i].qs) i_end++;
            i = i_end;
            int i_size = i_end - i_start;
            char* is_added = (char*)calloc((size_t)i_size, 1);
            int query_start = hits[i_start].qs;
            int cnt_done = 0;
            hits_sort(hits + i_start, i_size);
            for (int oi2 = 0; oi2 < open.n; ++oi2) {
                ora_nam* o = &open.v[oi2];
                int lower = i_start, upper = i_start;
                while (lower < i_end && hits[lower].rs < o->ref_prev_hit_startpos + 1) lower++;
                while (upper < i_end && hits[upper].rs < o->ref_end + 1) upper++;
                for (int j = lower; j < upper; ++j) {
                    if (is_added[j - i_start]) continue;
                    if (query_start <= o->query_end) {
                        const ora_hit* x = &hits[j];
                        if (o->ref_prev_hit_startpos < x->rs && x->rs <= o->ref_end) {
                            if (x->qe > o->query_end && x->re > o->ref_end) {
                                o->query_end = x->qe; o->ref_end = x->re;
                                o->query_prev_hit_startpos = x->qs; o->ref_prev_hit_startpos = x->rs;
                                o->n_hits++; is_added[j - i_start] = 1; cnt_done++; break;
                            } else if (x->qe <= o->query_end && x->re <= o->ref_end) {
                                o->query_prev_hit_startpos = x->qs; o->ref_prev_hit_startpos = x->rs;
                                o->n_hits++; is_added[j - i_start] = 1; cnt_done++; break;
                            }
                        }
                    }
                }
                if (cnt_done == i_size) break;
            }
            for (int j = 0; j < i_size; ++j)
                if (!is_added[j]) ov_push(&open, nam_from_hit(&hits[i_start + j], (int)ref_id, is_rc));
            free(is_added);
            if ((unsigned)query_start > prev_q_start + (unsigned)k) {
                flush_passed(&open, query_start, out);
                prev_q_start = (unsigned)query_start;
            }
        }
        for (int j = 0; j < open.n; ++j) nams_emit(out, open.v[j]);
        free(open.v);
    }
    free(order);
}

/* find_nams -- nam.cpp:771-926 */
int ora_find_nams(const ora_index* ix, const ora_qrs* q, int nq, ora_nam* out, int cap, float* nonrep) {
    hits_per_ref_t h[2];
    hpr_init(&h[0]); hpr_init(&h[1]);
    int good = 0, total = 0;
    for (int i = 0; i < nq; ++i) {
        uint64_t pos = ora_find(ix, q[i].hash);
        if (pos == ORA_END) continue;
        total++;
        if (ora_is_filtered(ix, pos)) continue;
        good++;
        add_to_hits_per_ref(&h[q[i].is_reverse ? 1 : 0], (int)q[i].start, (int)q[i].end, ix, pos);
    }
    *nonrep = total > 0 ? (float)good / (float)total : 1.0f;
    nam_out o = {out, 0, cap, 0};
    merge_hits_into_nams(&h[0], ix->k, 0, &o);
    merge_hits_into_nams(&h[1], ix->k, 1, &o);
    hpr_free(&h[0]); hpr_free(&h[1]);
    return o.overflow ? -1 : o.n;
}

typedef struct { uint64_t position; unsigned count, qs, qe; } ora_rescue_hit;  /* nam.cpp:935-941 */

static int rh_cmp1(const ora_rescue_hit* a, const ora_rescue_hit* b) {   /* nam.cpp:943-946 */
    if (a->count != b->count) return a->count < b->count;
    if (a->qs != b->qs) return a->qs < b->qs;
    return a->qe < b->qe;
}

static void rescue_sort(ora_rescue_hit* v, int n, int by_qs_only) {
    for (int i = 1; i < n; ++i) {
        ora_rescue_hit x = v[i]; int j = i - 1;
        while (j >= 0 && (by_qs_only ? x.qs < v[j].qs : rh_cmp1(&x, &v[j]))) { v[j + 1] = v[j]; --j; }
        v[j + 1] = x;
    }
}

/* find_nams_rescue -- nam.cpp:955-1012 (#define pre_sort branch) */
int ora_find_nams_rescue(const ora_index* ix, const ora_qrs* q, int nq, unsigned rescue_cutoff,
                         ora_nam* out, int cap) {
    hits_per_ref_t h[2];
    hpr_init(&h[0]); hpr_init(&h[1]);
    ora_rescue_hit* hv[2];
    int hn[2] = {0, 0};
    hv[0] = (ora_rescue_hit*)malloc(sizeof(ora_rescue_hit) * (size_t)(nq + 1));
    hv[1] = (ora_rescue_hit*)malloc(sizeof(ora_rescue_hit) * (size_t)(nq + 1));
    for (int i = 0; i < nq; ++i) {
        uint64_t pos = ora_find(ix, q[i].hash);
        if (pos == ORA_END) continue;
        ora_rescue_hit r = {pos, ora_get_count(ix, pos), q[i].start, q[i].end};
        int o = q[i].is_reverse ? 1 : 0;
        hv[o][hn[o]++] = r;
    }
    ora_rescue_hit* rhs[2];
    int rn[2] = {0, 0};
    for (int o = 0; o < 2; ++o) {
        rescue_sort(hv[o], hn[o], 0);
        rhs[o] = (ora_rescue_hit*)malloc(sizeof(ora_rescue_hit) * (size_t)(hn[o] + 1));
        int cnt = 0;
        for (int i = 0; i < hn[o]; ++i) {
            ora_rescue_hit* r = &hv[o][i];
            if ((r->count > rescue_cutoff && cnt >= 5) || r->count > 1000) break;
            rhs[o][rn[o]++] = *r;
            add_to_hits_per_ref_pre(&h[o], (int)r->qs, (int)r->qe, ix, r->position);
            cnt++;
        }
    }
    for (int o = 0; o < 2; ++o) {
        rescue_sort(rhs[o], rn[o], 1);
        for (int i = 0; i < rn[o]; ++i)
            add_to_hits_per_ref(&h[o], (int)rhs[o][i].qs, (int)rhs[o][i].qe, ix, rhs[o][i].position);
    }
    nam_out no = {out, 0, cap, 0};
    merge_hits_into_nams_fast(&h[0], ix->k, 0, &no);
    merge_hits_into_nams_fast(&h[1], ix->k, 1, &no);
    for (int o = 0; o < 2; ++o) { free(hv[o]); free(rhs[o]); }
    hpr_free(&h[0]); hpr_free(&h[1]);
    return no.overflow ? -1 : no.n;
}

/* ===================================================================== */
/* SSW restatement                                                        */
/* ===================================================================== */
/* Score of a translated pair -- BuildSwScoreMatrix (ssw_cpp.cpp:27-52):
 * +match on the ACGT diagonal, -mismatch for everything else incl. N-N. */
static inline int sub_score(int a, int b, int match, int mismatch) {
    return (a == b && a < 4) ? match : -mismatch;
}

/* Striped local Gotoh in the order the SSE kernels visit the reference
 * (sw_sse2_byte ssw.c:197-386 / sw_sse2_word ssw.c:412-588), restated as a
 * scalar recurrence.  The query is cut into stripes of seg_len rows
 * (16 lanes x seg_len in byte mode, 8 lanes in word mode).  Within a stripe F
 * is carried in the main loop; across stripe boundaries it only arrives in the
 * Lazy_F loop, which raises H but does NOT update E (ssw.c:275-289).  So:
 *   Fw  = within-stripe F (reset to 0 at every stripe start)
 *   Hm  = max(0, diag + s, E, Fw)          -- main-loop H, feeds E and Fw
 *   H   = max(Hm, F)                       -- final H (F = exact vertical gap)
 *   E'  = max(E - gE, Hm - gO)             -- next column's E
 * All of E/F/Fw saturate at 0 (result-neutral).  Tie rules: the best column is
 * the first column (scan order) at which the running max strictly increases
 * to its final value; the best row is the smallest row of that column holding
 * it (0 if nothing scored, pvHmax is zero-filled); a scan stops at the first
 * column whose column max equals `terminate` (>0). */
typedef struct { int score; int ref; int read; } ora_end;

static ora_end sw_scan(const int8_t* ref, int dir, int ref_len, const int8_t* read, int read_len,
                       int match, int mismatch, int gap_o, int gap_e, int terminate, int init_ref,
                       int seg_len) {
    int* H = (int*)calloc((size_t)read_len + 1, sizeof(int));   /* previous column, final H */
    int* Hn = (int*)calloc((size_t)read_len + 1, sizeof(int));
    int* E = (int*)calloc((size_t)read_len + 1, sizeof(int));
    ora_end r = {0, init_ref, read_len - 1};
    int best = 0;
    int begin = 0, end = ref_len, step = 1;
    if (dir == 1) { begin = ref_len - 1; end = -1; step = -1; }
    for (int i = begin; i != end; i += step) {
        int F = 0, Fw = 0, colmax = 0;
        for (int j = 0; j < read_len; ++j) {
            if (j % seg_len == 0) Fw = 0;
            int diag = j == 0 ? 0 : H[j - 1];
            int hm = diag + sub_score(ref[i], read[j], match, mismatch);
            if (hm < 0) hm = 0;
            if (E[j] > hm) hm = E[j];
            if (Fw > hm) hm = Fw;
            int h = F > hm ? F : hm;
            Hn[j] = h;
            if (h > colmax) colmax = h;
            int ho = hm - gap_o; if (ho < 0) ho = 0;
            int e = E[j] - gap_e; if (e < 0) e = 0;
            E[j] = e > ho ? e : ho;
            int fw = Fw - gap_e; if (fw < 0) fw = 0;
            Fw = fw > ho ? fw : ho;
            int hfo = h - gap_o; if (hfo < 0) hfo = 0;
            int f = F - gap_e; if (f < 0) f = 0;
            F = f > hfo ? f : hfo;
        }
        int* t = H; H = Hn; Hn = t;
        if (colmax > best) {
            best = colmax;
            r.ref = i;
            r.read = read_len - 1;
            for (int j = 0; j < read_len; ++j) if (H[j] == best) { r.read = j; break; }
        }
        if (terminate > 0 && colmax == terminate) break;
    }
    r.score = best;
    if (best == 0 && read_len > 0) r.read = 0;
    free(H); free(Hn); free(E);
    return r;
}

static inline uint32_t to_cigar_int(uint32_t len, char op) {
    uint32_t code = 0;
    switch (op) {
        case 'M': code = 0; break; case 'I': code = 1; break; case 'D': code = 2; break;
        case 'N': code = 3; break; case 'S': code = 4; break; case 'H': code = 5; break;
        case 'P': code = 6; break; case '=': code = 7; break; case 'X': code = 8; break;
    }
    return (len << 4) | code;
}

/* banded_sw (ssw.c:590-774), restated literally: the band/array index
 * arithmetic (set_u/set_d, the per-row h_b[edge]=e_b[edge]=0 reset, e_b and
 * the direction buffer surviving band doubling) is part of the observable
 * result, so it is reproduced as-is.  Returns #ops (reversed order fixed up)
 * or -1 on a traceback error. */
#define SET_U(w, i, j) ({ int _x = (i) - (w); _x = _x > 0 ? _x : 0; (j) - _x + 1; })
#define SET_D(w, i, j, p) ({ int _x = (i) - (w); _x = _x > 0 ? _x : 0; _x = (j) - _x; _x * 3 + (p); })

static int banded_sw(const int8_t* ref, const int8_t* read, int ref_len, int read_len, int score,
                     int gap_o, int gap_e, int band_width, int match, int mismatch, uint32_t* out) {
    int len = ref_len > read_len ? ref_len : read_len;
    int s1 = 8;
    int64_t s2 = 1024;
    int* h_b = (int*)calloc((size_t)s1, sizeof(int));
    int* e_b = (int*)calloc((size_t)s1, sizeof(int));
    int* h_c = (int*)calloc((size_t)s1, sizeof(int));
    int8_t* direction = (int8_t*)calloc((size_t)s2, 1);
    int8_t* direction_line = direction;
    int max = 0, width, width_d;
    do {
        width = band_width * 2 + 3; width_d = band_width * 2 + 1;
        while (width >= s1) {
            int ns = s1 + 1;
            ns--; ns |= ns >> 1; ns |= ns >> 2; ns |= ns >> 4; ns |= ns >> 8; ns |= ns >> 16; ns++;
            h_b = (int*)realloc(h_b, sizeof(int) * (size_t)ns);
            e_b = (int*)realloc(e_b, sizeof(int) * (size_t)ns);
            h_c = (int*)realloc(h_c, sizeof(int) * (size_t)ns);
            for (int z = s1; z < ns; ++z) h_b[z] = e_b[z] = h_c[z] = 0;
            s1 = ns;
        }
        while ((int64_t)width_d * read_len * 3 >= s2) {
            int64_t ns = s2 + 1;
            ns--; ns |= ns >> 1; ns |= ns >> 2; ns |= ns >> 4; ns |= ns >> 8; ns |= ns >> 16; ns |= ns >> 32; ns++;
            direction = (int8_t*)realloc(direction, (size_t)ns);
            memset(direction + s2, 0, (size_t)(ns - s2));
            s2 = ns;
        }
        direction_line = direction;
        for (int j = 1; j < width - 1; j++) h_b[j] = 0;
        for (int i = 0; i < read_len; i++) {
            int beg = 0, end = ref_len - 1, u = 0, edge, f, j;
            j = i - band_width; beg = beg > j ? beg : j;
            j = i + band_width; end = end < j ? end : j;
            edge = end + 1 < width - 1 ? end + 1 : width - 1;
            f = h_b[0] = e_b[0] = h_b[edge] = e_b[edge] = h_c[0] = 0;
            direction_line = direction + (int64_t)width_d * i * 3;
            for (j = beg; j <= end; j++) {
                int b, e, e1, f1, d, de, df, dh, temp1, temp2;
                u = SET_U(band_width, i, j); e = SET_U(band_width, i - 1, j);
                b = SET_U(band_width, i, j - 1); d = SET_U(band_width, i - 1, j - 1);
                de = SET_D(band_width, i, j, 0); df = SET_D(band_width, i, j, 1); dh = SET_D(band_width, i, j, 2);
                temp1 = i == 0 ? -gap_o : h_b[e] - gap_o;
                temp2 = i == 0 ? -gap_e : e_b[e] - gap_e;
                e_b[u] = temp1 > temp2 ? temp1 : temp2;
                direction_line[de] = temp1 > temp2 ? 3 : 2;
                temp1 = h_c[b] - gap_o;
                temp2 = f - gap_e;
                f = temp1 > temp2 ? temp1 : temp2;
                direction_line[df] = temp1 > temp2 ? 5 : 4;
                e1 = e_b[u] > 0 ? e_b[u] : 0;
                f1 = f > 0 ? f : 0;
                temp1 = e1 > f1 ? e1 : f1;
                temp2 = h_b[d] + sub_score(ref[j], read[i], match, mismatch);
                h_c[u] = temp1 > temp2 ? temp1 : temp2;
                if (h_c[u] > max) max = h_c[u];
                if (temp1 <= temp2) direction_line[dh] = 1;
                else direction_line[dh] = e1 > f1 ? direction_line[de] : direction_line[df];
            }
            for (j = 1; j <= u; j++) h_b[j] = h_c[j];
        }
        band_width *= 2;
    } while (max < score && band_width <= len);
    band_width /= 2;

    /* traceback (ssw.c:685-753) */
    int i = read_len - 1, j = ref_len - 1, e = 0, l = 0, temp2 = 2;
    char op = 'M', prev_op = 'M';
    int ok = 1;
    uint32_t* c = out;
    while (i >= 0 && j > 0) {
        int temp1 = SET_D(band_width, i, j, temp2);
        int64_t at = (direction_line - direction) + temp1;
        if (at < 0 || at >= s2) { ok = 0; break; }
        switch (direction_line[temp1]) {
            case 1: --i; --j; temp2 = 2; direction_line -= width_d * 3; op = 'M'; break;
            case 2: --i; temp2 = 0; direction_line -= width_d * 3; op = 'I'; break;
            case 3: --i; temp2 = 2; direction_line -= width_d * 3; op = 'I'; break;
            case 4: --j; temp2 = 1; op = 'D'; break;
            case 5: --j; temp2 = 2; op = 'D'; break;
            default: ok = 0; break;
        }
        if (!ok) break;
        if (op == prev_op) ++e;
        else { ++l; c[l - 1] = to_cigar_int((uint32_t)e, prev_op); prev_op = op; e = 1; }
    }
    free(h_b); free(e_b); free(h_c); free(direction);
    if (!ok) return -1;
    if (op == 'M') { ++l; c[l - 1] = to_cigar_int((uint32_t)e + 1, op); }
    else { l += 2; c[l - 2] = to_cigar_int((uint32_t)e, op); c[l - 1] = to_cigar_int(1, 'M'); }
    for (int s = 0, t = l - 1; s < t; ++s, --t) { uint32_t x = c[s]; c[s] = c[t]; c[t] = x; }
    return l;
}

/* ssw_align (ssw.c:818-922) with flag 0x0f, filters 0, filterd 32767;
 * force_word: the word layout whatever the byte pass scores (the scan kernel's
 * certified path, ora_scan_certificate) */
static void ssw_align_impl(const int8_t* q, int qlen, const int8_t* r, int rlen, int match, int mismatch,
                           int gap_open, int gap_extend, ora_ssw_res* res, uint32_t* cigar, int force_word) {
    res->ref_begin1 = -1; res->read_begin1 = -1; res->flag = 0; res->n_cigar = 0;
    /* byte mode first (16 stripes, end_ref starts at -1); a max >= 255-bias
     * (bias = mismatch) overflows and the word kernel (8 stripes, end_ref
     * starts at 0) recomputes everything (ssw.c:838-850) */
    int word = 0;
    ora_end fwd = {0, -1, 0};
    if (!force_word)
        fwd = sw_scan(r, 0, rlen, q, qlen, match, mismatch, gap_open, gap_extend, 0, -1, (qlen + 15) / 16);
    if (force_word || fwd.score + mismatch >= 255) {
        word = 1;
        fwd = sw_scan(r, 0, rlen, q, qlen, match, mismatch, gap_open, gap_extend, 0, 0, (qlen + 7) / 8);
    }
    res->score1 = fwd.score;
    res->ref_end1 = fwd.ref;
    res->read_end1 = fwd.read;
    int8_t* rev = (int8_t*)malloc((size_t)res->read_end1 + 2);
    for (int j = 0; j <= res->read_end1; ++j) rev[j] = q[res->read_end1 - j];
    int rlen2 = res->read_end1 + 1;
    ora_end bwd = sw_scan(r, 1, res->ref_end1 + 1, rev, rlen2, match, mismatch, gap_open, gap_extend,
                          res->score1, word ? 0 : -1, word ? (rlen2 + 7) / 8 : (rlen2 + 15) / 16);
    free(rev);
    res->ref_begin1 = bwd.ref;
    res->read_begin1 = res->read_end1 - bwd.read;
    if (res->score1 > bwd.score) res->flag = 2;
    int ref_l = res->ref_end1 - res->ref_begin1 + 1;
    int read_l = res->read_end1 - res->read_begin1 + 1;
    int bw = abs(ref_l - read_l) + 1;
    /* ref + ref_begin1 may point before the buffer when score1 == 0 (UB in the
     * reference); we read it as an N. */
    int8_t* rbuf = (int8_t*)malloc((size_t)(ref_l > 0 ? ref_l : 1));
    for (int z = 0; z < ref_l; ++z) {
        int gi = res->ref_begin1 + z;
        rbuf[z] = (gi >= 0 && gi < rlen) ? r[gi] : 4;
    }
    int n = banded_sw(rbuf, q + res->read_begin1, ref_l, read_l, res->score1, gap_open, gap_extend, bw,
                      match, mismatch, cigar);
    free(rbuf);
    if (n < 0) res->flag = 1;
    else res->n_cigar = n;
}

void ora_ssw_align(const int8_t* q, int qlen, const int8_t* r, int rlen, int match, int mismatch,
                   int gap_open, int gap_extend, ora_ssw_res* res, uint32_t* cigar) {
    ssw_align_impl(q, qlen, r, rlen, match, mismatch, gap_open, gap_extend, res, cigar, 0);
}

/* The scan kernel's certificate (k_ext_scan_v).  SSW scores a job in
 * the byte layout and switches to the word layout when the byte max saturates
 * (score + bias >= 255, bias = mismatch, ssw.c:838-850).  The kernel runs the word
 * layout first and takes its result without the byte pass when the word score
 * reaches that bound AND the band path of the word result (banded_sw's traceback,
 * ssw.c:590-774) has no insertion next to a deletion: the two layouts differ only
 * where a cross-stripe F would open an E gap (an I directly followed by a D), so
 * such a path scores at least as high in the byte layout, whose max then saturates.
 * Returns 0: word score below the bound (not a candidate); 1: the path has an I
 * next to a D (the kernel re-runs the job exactly); 2: certified, and the byte
 * layout does saturate; -1: certified but the byte layout does not saturate (a
 * counterexample to the argument). */
int ora_scan_certificate(const int8_t* q, int qlen, const int8_t* r, int rlen, int match, int mismatch,
                         int gap_open, int gap_extend) {
    ora_end w = sw_scan(r, 0, rlen, q, qlen, match, mismatch, gap_open, gap_extend, 0, 0, (qlen + 7) / 8);
    if (w.score + mismatch < 255) return 0;
    uint32_t* cig = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(2 * (qlen + rlen) + 16));
    ora_ssw_res res;
    ssw_align_impl(q, qlen, r, rlen, match, mismatch, gap_open, gap_extend, &res, cig, 1);
    int adjacent = res.flag != 0;              /* a failed band pass is re-run as well */
    for (int i = 0; !adjacent && i + 1 < res.n_cigar; ++i) {
        const uint32_t a = cig[i] & 0xf, b = cig[i + 1] & 0xf;
        adjacent = (a == 1 && b == 2) || (a == 2 && b == 1);
    }
    free(cig);
    if (adjacent) return 1;
    ora_end b = sw_scan(r, 0, rlen, q, qlen, match, mismatch, gap_open, gap_extend, 0, -1, (qlen + 15) / 16);
    return b.score + mismatch >= 255 ? 2 : -1;
}

/* TranslateBase with kBaseTranslation (ssw_cpp.cpp:12-25, 352-363):
 * A/a->0 C/c->1 G/g->2 T/t->3, U/u->0 (sic), everything else 4 */
static int8_t translate(unsigned char c) {
    switch (c) {
        case 'A': case 'a': case 'U': case 'u': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return 4;
    }
}

typedef struct { uint32_t* v; int n; } cig;
static void cig_push_raw(cig* c, uint32_t x) { c->v[c->n++] = x; }
/* Cigar::push (cigar.hpp:52-59) merges equal adjacent ops */
static void cig_push(cig* c, uint32_t op, uint32_t len) {
    if (c->n == 0 || (c->v[c->n - 1] & 0xf) != op) c->v[c->n++] = (len << 4) | op;
    else c->v[c->n - 1] += len << 4;
}

typedef void (*ora_raw_fn)(const int8_t*, int, const int8_t*, int, int, int, int, int, ora_ssw_res*, uint32_t*);

void ora_aligner_align_with(const char* query, int qlen, const char* ref, int rlen, int match, int mismatch,
                            int gap_open, int gap_extend, int end_bonus, ora_aln_info* out, uint32_t* cigar,
                            ora_raw_fn raw_fn);

void ora_aligner_align(const char* query, int qlen, const char* ref, int rlen, int match, int mismatch,
                       int gap_open, int gap_extend, int end_bonus, ora_aln_info* out, uint32_t* cigar) {
    ora_aligner_align_with(query, qlen, ref, rlen, match, mismatch, gap_open, gap_extend, end_bonus, out, cigar,
                           ora_ssw_align);
}

/* Aligner::align with a pluggable raw ssw_align (ours, or the reference's ssw.c) */
void ora_aligner_align_with(const char* query, int qlen, const char* ref, int rlen, int match, int mismatch,
                            int gap_open, int gap_extend, int end_bonus, ora_aln_info* out, uint32_t* cigar,
                            ora_raw_fn raw_fn) {
    memset(out, 0, sizeof *out);
    if (rlen > 2000) {                       /* aligner.cpp:119-125 */
        out->edit_distance = 100000; out->ref_start = 0; out->sw_score = -1000000;
        return;
    }
    int8_t* tq = (int8_t*)malloc((size_t)qlen + 1);
    int8_t* tr = (int8_t*)malloc((size_t)rlen + 1);
    for (int i = 0; i < qlen; ++i) tq[i] = translate((unsigned char)query[i]);
    for (int i = 0; i < rlen; ++i) tr[i] = translate((unsigned char)ref[i]);
    uint32_t* raw = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(2 * (qlen + rlen) + 16));
    ora_ssw_res s;
    raw_fn(tq, qlen, tr, rlen, match, mismatch, gap_open, gap_extend, &s, raw);
    if (s.flag != 0) {                       /* aligner.cpp:131-136 */
        out->edit_distance = 100000; out->ref_start = 0; out->sw_score = -100000;
        free(tq); free(tr); free(raw);
        return;
    }
    /* ConvertAlignment + CalculateNumberMismatch (ssw_cpp.cpp:54-90, 126-210):
     * S(query_begin) + M split into =/X on translated bases + S(tail). */
    uint32_t* conv = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(2 * (qlen + rlen) + 16));
    cig c = {conv, 0};
    int mism = 0;
    if (s.read_begin1 > 0) cig_push_raw(&c, to_cigar_int((uint32_t)s.read_begin1, 'S'));
    /* ref_begin1 is -1 only when nothing scored (score1 == 0): the reference
     * then reads translated_ref[-1] (UB); we read it as an N, like banded_sw */
    int rpos = s.ref_begin1;
    const int8_t* qp = tq + s.read_begin1;
    int in_m = 0, in_x = 0; uint32_t len_m = 0, len_x = 0;
    for (int i = 0; i < s.n_cigar; ++i) {
        uint32_t op = raw[i] & 0xf, len = raw[i] >> 4;
        if (op == 0) {
            for (uint32_t j = 0; j < len; ++j) {
                int8_t rc = (rpos >= 0 && rpos < rlen) ? tr[rpos] : 4;
                if (rc != *qp) {
                    ++mism;
                    if (in_m) cig_push_raw(&c, to_cigar_int(len_m, '='));
                    len_m = 0; ++len_x; in_m = 0; in_x = 1;
                } else {
                    if (in_x) cig_push_raw(&c, to_cigar_int(len_x, 'X'));
                    ++len_m; len_x = 0; in_m = 1; in_x = 0;
                }
                ++rpos; ++qp;
            }
        } else if (op == 1 || op == 2) {
            if (op == 1) qp += len; else rpos += (int)len;
            mism += (int)len;
            if (in_m) cig_push_raw(&c, to_cigar_int(len_m, '='));
            else if (in_x) cig_push_raw(&c, to_cigar_int(len_x, 'X'));
            in_m = in_x = 0; len_m = len_x = 0;
            cig_push_raw(&c, raw[i]);
        }
    }
    if (in_m) cig_push_raw(&c, to_cigar_int(len_m, '='));
    else if (in_x) cig_push_raw(&c, to_cigar_int(len_x, 'X'));
    int tail = qlen - s.read_end1 - 1;
    if (tail > 0) cig_push_raw(&c, to_cigar_int((uint32_t)tail, 'S'));

    /* Aligner::align body (aligner.cpp:138-207) */
    uint32_t ed = (uint32_t)mism;
    int sw = s.score1;
    uint32_t rs = (uint32_t)s.ref_begin1, re = (uint32_t)s.ref_end1 + 1;
    uint32_t qs = (uint32_t)s.read_begin1, qe = (uint32_t)s.read_end1 + 1;
    /* left end bonus */
    {
        uint32_t q0 = qs, r0 = rs; int score = sw; uint32_t edits = ed;
        uint32_t* fb = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(qlen + 4));
        cig front = {fb, 0};
        while (q0 > 0 && r0 > 0) {
            q0--; r0--;
            if (query[q0] == ref[r0]) { score += match; cig_push(&front, 7, 1); }
            else { score -= mismatch; cig_push(&front, 8, 1); edits++; }
        }
        if (q0 == 0 && score + end_bonus > sw) {
            if (qs > 0) {
                /* drop leading soft clip, prepend reversed front extension */
                uint32_t* nb = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(c.n + front.n + 4));
                cig nc = {nb, 0};
                for (int z = front.n - 1; z >= 0; --z) cig_push(&nc, front.v[z] & 0xf, front.v[z] >> 4);
                for (int z = 1; z < c.n; ++z) cig_push(&nc, c.v[z] & 0xf, c.v[z] >> 4);
                memcpy(c.v, nb, sizeof(uint32_t) * (size_t)nc.n);
                c.n = nc.n;
                free(nb);
            }
            qs = 0; rs = r0; sw = score + end_bonus; ed = edits;
        }
        free(fb);
    }
    /* right end bonus */
    {
        uint32_t q1 = qe, r1 = re; int score = sw; uint32_t edits = ed;
        uint32_t* bb = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(qlen + 4));
        cig back = {bb, 0};
        while (q1 < (uint32_t)qlen && r1 < (uint32_t)rlen) {
            if (query[q1] == ref[r1]) { score += match; cig_push(&back, 7, 1); }
            else { score -= mismatch; cig_push(&back, 8, 1); edits++; }
            q1++; r1++;
        }
        if (q1 == (uint32_t)qlen && score + end_bonus > sw) {
            if (qe < (uint32_t)qlen) {
                c.n--;   /* pop trailing soft clip */
                for (int z = 0; z < back.n; ++z) cig_push(&c, back.v[z] & 0xf, back.v[z] >> 4);
            }
            qe = (uint32_t)qlen; re = r1; sw = score + end_bonus; ed = edits;
        }
        free(bb);
    }
    out->edit_distance = ed; out->ref_start = rs; out->ref_end = re;
    out->query_start = qs; out->query_end = qe; out->sw_score = sw;
    out->n_cigar = c.n;
    memcpy(cigar, c.v, sizeof(uint32_t) * (size_t)c.n);
    free(conv); free(tq); free(tr); free(raw);
}

/* ---- per-NAM site checks ------------------------------ */

/* revcomp_table + reverse_complement (revcomp.hpp:11-38): A->T, C->G, G->C,
 * T/U->A (either case, upper-case result), anything else -> N. */
void ora_reverse_complement(const char* s, int len, char* out) {
    for (int i = 0; i < len; ++i) {
        char o;
        switch (s[len - 1 - i]) {
            case 'A': case 'a': o = 'T'; break;
            case 'C': case 'c': o = 'G'; break;
            case 'G': case 'g': o = 'C'; break;
            case 'T': case 't': case 'U': case 'u': o = 'A'; break;
            default: o = 'N';
        }
        out[i] = o;
    }
}

/* a.substr(pa, k) == b.substr(pb, k) (std::string semantics: the substring is
 * cut at the end; a position past the end is treated as empty here -- the
 * reference's substr would throw there, which valid NAM coordinates never reach) */
static int sub_eq(const char* a, int64_t alen, int64_t pa, const char* b, int64_t blen, int64_t pb, int k) {
    if (pa < 0 || pa > alen) pa = alen;
    if (pb < 0 || pb > blen) pb = blen;
    int64_t na = alen - pa < k ? alen - pa : k, nb = blen - pb < k ? blen - pb : k;
    return na == nb && memcmp(a + pa, b + pb, (size_t)na) == 0;
}

/* reverse_nam_if_needed (aln.cpp:60-93) on a copy of the NAM, then
 * extend_seed_part's ungapped test (aln.cpp:374-395): projected window
 * [max(0, ref_start - query_start), min(ref_end + L - query_end, |contig|)),
 * Hamming distance when it is read-length and the NAM consistent
 * (hamming_distance, aligner.hpp:54-67), accepted when (float)hd / L < 0.05.
 * Returns rsa_nam_site flags: orientation 0 (as is) / 1 (reversed) / 2
 * (inconsistent), | 4 Hamming computed (*n_mm), | 8 accepted with the mismatch
 * positions (query coordinates of the oriented read) in mm_pos[0 .. *n_mm). */
int ora_nam_site(const ora_nam* nam, const char* read, const char* read_rc, int L, const char* contig, int64_t clen,
                 int k, uint16_t* mm_pos, int* n_mm) {
    int is_rc = nam->is_rc, qs = nam->query_start, qe = nam->query_end;
    const int rs = nam->ref_start, re = nam->ref_end;
    const char* seq = is_rc ? read_rc : read;
    const char* seq_rc = is_rc ? read : read_rc;
    int flags;
    *n_mm = 0;
    if (sub_eq(contig, clen, rs, seq, L, qs, k) && sub_eq(contig, clen, re - k, seq, L, qe - k, k)) {
        flags = 0;
    } else if (sub_eq(contig, clen, rs, seq_rc, L, L - qe, k) &&
               sub_eq(contig, clen, re - k, seq_rc, L, L - qs - k, k)) {
        const int t = qs;
        flags = 1; is_rc = !is_rc; qs = L - qe; qe = L - t;
    } else {
        return 2;
    }
    const char* q = is_rc ? read_rc : read;
    const int64_t ps = rs - qs > 0 ? rs - qs : 0;
    const int64_t pe0 = (int64_t)re + L - qe;
    const int64_t pe = pe0 < clen ? pe0 : clen;
    if (pe - ps != L) return flags;
    int hd = 0;
    for (int i = 0; i < L; ++i) if (contig[ps + i] != q[i]) hd++;
    flags |= 4;
    *n_mm = hd;
    if ((float)hd / (float)L < 0.05f) {
        int m = 0;
        for (int i = 0; i < L; ++i) if (contig[ps + i] != q[i]) mm_pos[m++] = (uint16_t)i;
        flags |= 8;
    }
    return flags;
}

/* hamming_align (src/aligner.cpp:254-302) with highest_scoring_segment
 * (aligner.cpp:219-252), restated per position as the reference runs them:
 * query and ref of equal length n.  Writes the CIGAR ops (len<<4|op, Cigar::push
 * merging) to cigar and returns their count; *score, *start, *end (the segment,
 * half-open) and *mismatches (inside it) as AlignmentInfo holds them. */
int ora_hamming_align(const char* query, const char* ref, int n, int match, int mismatch, int end_bonus,
                      int* score_out, int* start_out, int* end_out, int* mismatches_out, uint32_t* cigar) {
    int start = 0, score = end_bonus, best_start = 0, best_end = 0, best_score = 0;
    for (int i = 0; i < n; ++i) {
        if (query[i] == ref[i]) score += match;
        else score -= mismatch;
        if (score < 0) { start = i + 1; score = 0; }
        if (score > best_score) { best_start = start; best_score = score; best_end = i + 1; }
    }
    if (score + end_bonus > best_score) { best_score = score + end_bonus; best_end = n; best_start = start; }
    int nc = 0;
#define ORA_PUSH(op, len) do { uint32_t o_ = (op), l_ = (uint32_t)(len); \
        if (nc == 0 || (cigar[nc - 1] & 0xf) != o_) cigar[nc++] = (l_ << 4) | o_; else cigar[nc - 1] += l_ << 4; } while (0)
    if (best_start > 0) ORA_PUSH(4, best_start);
    int counter = 0, prev_is_match = 0, mismatches = 0, first = 1;
    for (int i = best_start; i < best_end; i++) {
        const int is_match = query[i] == ref[i];
        mismatches += is_match ? 0 : 1;
        if (!first && is_match != prev_is_match) {
            ORA_PUSH(prev_is_match ? 7 : 8, counter);
            counter = 0;
        }
        counter++;
        prev_is_match = is_match;
        first = 0;
    }
    if (!first) ORA_PUSH(prev_is_match ? 7 : 8, counter);
    if (n - best_end > 0) ORA_PUSH(4, n - best_end);
#undef ORA_PUSH
    *score_out = best_score;
    *start_out = best_start;
    *end_out = best_end;
    *mismatches_out = mismatches;
    return nc;
}
