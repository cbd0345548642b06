/*
 * sti.h -- .sti index reader for the oracle (TEST INFRASTRUCTURE ONLY).
 * Format: StrobemerIndex::write/read (src/index.cpp:73-132), io.hpp:12-27,
 * IndexParameters::write/read (src/indexparameters.cpp:87-108).
 */
#ifndef RSA_ORACLE_STI_H
#define RSA_ORACLE_STI_H
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "rsa_oracle.h"

typedef struct ora_sti {
    ora_index index;
    ora_params params;
    int canonical_read_length;
    ora_refrs* rs;
    uint64_t* starts;
} ora_sti;

static inline int ora_sti_load(const char* fn, ora_sti* s) {
    FILE* f = fopen(fn, "rb");
    if (!f) return -1;
    char magic[4];
    int32_t ver, fc, bits, prm[7];
    uint64_t reserved, n, ns;
    if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "STI\1", 4) != 0) { fclose(f); return -1; }
    if (fread(&ver, 4, 1, f) != 1 || ver != 2) { fclose(f); return -1; }
    if (fread(&reserved, 8, 1, f) != 1) { fclose(f); return -1; }
    fseek(f, (long)reserved, SEEK_CUR);
    if (fread(&fc, 4, 1, f) != 1 || fread(&bits, 4, 1, f) != 1 || fread(prm, 4, 7, f) != 7) { fclose(f); return -1; }
    if (fread(&n, 8, 1, f) != 1) { fclose(f); return -1; }
    s->rs = (ora_refrs*)malloc(sizeof(ora_refrs) * (size_t)(n + 1));
    if (fread(s->rs, sizeof(ora_refrs), (size_t)n, f) != (size_t)n) { fclose(f); return -1; }
    if (fread(&ns, 8, 1, f) != 1 || ns != (1ULL << bits) + 1) { fclose(f); return -1; }
    s->starts = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)ns);
    if (fread(s->starts, 8, (size_t)ns, f) != (size_t)ns) { fclose(f); return -1; }
    fclose(f);
    int k = prm[1], sp = prm[2], l = prm[3], u = prm[4], q = prm[5], md = prm[6];
    s->canonical_read_length = prm[0];
    s->params.k = k; s->params.s = sp; s->params.t_syncmer = (k - sp) / 2 + 1;
    int wm = k / (k - sp + 1) + l;
    s->params.w_min = wm > 0 ? wm : 0;
    s->params.w_max = k / (k - sp + 1) + u;
    s->params.max_dist = md;
    s->params.q = (uint64_t)q;
    s->index.rs = s->rs; s->index.n = n; s->index.starts = s->starts; s->index.bits = bits;
    s->index.filter_cutoff = (unsigned)fc; s->index.k = k;
    return 0;
}

static inline void ora_sti_free(ora_sti* s) { free(s->rs); free(s->starts); }
#endif
