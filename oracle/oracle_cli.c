/*
 * oracle_cli.c -- command-line front end of the C restatement (rsa_oracle.c).
 * TEST INFRASTRUCTURE ONLY.  Prints exactly the formats oracle/refgen.cpp
 * prints from the reference, so tests can diff the two byte for byte.
 *   seeds <sti> <reads.txt> <out> <R>
 *   ssw   <jobs.txt> <out>
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rsa_oracle.h"
#include "sti.h"

static void print_nam(FILE* o, const ora_nam* n) {
    fprintf(o, "%d %d %d %d %d %d %d %d %d %.9g %d\n", n->nam_id, n->query_start, n->query_end,
            n->query_prev_hit_startpos, n->ref_start, n->ref_end, n->ref_prev_hit_startpos, n->n_hits,
            n->ref_id, (double)n->score, n->is_rc);
}

static int cmd_seeds(int argc, char** argv) {
    if (argc < 6) { fprintf(stderr, "seeds <sti> <reads.txt> <out> <R>\n"); return 2; }
    ora_sti sti;
    if (ora_sti_load(argv[2], &sti) != 0) { fprintf(stderr, "bad sti %s\n", argv[2]); return 2; }
    int R = atoi(argv[5]);
    unsigned rescue_cutoff = R < 100 ? (unsigned)R * sti.index.filter_cutoff : 1000;
    FILE* in = fopen(argv[3], "r");
    FILE* o = fopen(argv[4], "w");
    if (!in || !o) return 2;
    char* line = NULL;
    size_t cap = 0;
    ssize_t len;
    int qcap = 4096, ncap = 1 << 16;
    ora_qrs* q = (ora_qrs*)malloc(sizeof(ora_qrs) * (size_t)qcap);
    ora_nam* nams = (ora_nam*)malloc(sizeof(ora_nam) * (size_t)ncap);
    while ((len = getline(&line, &cap, in)) > 0) {
        while (len > 0 && (line[len - 1] == '\n' || line[len - 1] == '\r')) line[--len] = 0;
        int nq = ora_randstrobes_query(line, (int)len, &sti.params, q, qcap);
        fprintf(o, "Q %d\n", nq);
        for (int i = 0; i < nq; ++i)
            fprintf(o, "%" PRIu64 " %u %u %u\n", q[i].hash, q[i].start, q[i].end, q[i].is_reverse);
        float nonrep;
        int nn = ora_find_nams(&sti.index, q, nq, nams, ncap, &nonrep);
        uint32_t bits;
        memcpy(&bits, &nonrep, 4);
        fprintf(o, "N %08x %d\n", bits, nn);
        for (int i = 0; i < nn; ++i) print_nam(o, &nams[i]);
        int nr = ora_find_nams_rescue(&sti.index, q, nq, rescue_cutoff, nams, ncap);
        fprintf(o, "R %d\n", nr);
        for (int i = 0; i < nr; ++i) print_nam(o, &nams[i]);
    }
    free(line); free(q); free(nams);
    fclose(in); fclose(o);
    ora_sti_free(&sti);
    return 0;
}

static int8_t tr(unsigned char c) {
    switch (c) {
        case 'A': case 'a': case 'U': case 'u': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return 4;
    }
}

static int cmd_ssw(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "ssw <jobs.txt> <out>\n"); return 2; }
    FILE* in = fopen(argv[2], "r");
    FILE* o = fopen(argv[3], "w");
    if (!in || !o) return 2;
    char* qb = (char*)malloc(1 << 16);
    char* rb = (char*)malloc(1 << 16);
    uint32_t* cig = (uint32_t*)malloc(sizeof(uint32_t) * (1 << 16));
    int8_t* tq = (int8_t*)malloc(1 << 16);
    int8_t* trr = (int8_t*)malloc(1 << 16);
    while (fscanf(in, "%65535s %65535s", qb, rb) == 2) {
        int ql = (int)strlen(qb), rl = (int)strlen(rb);
        for (int i = 0; i < ql; ++i) tq[i] = tr((unsigned char)qb[i]);
        for (int i = 0; i < rl; ++i) trr[i] = tr((unsigned char)rb[i]);
        ora_ssw_res r;
        ora_ssw_align(tq, ql, trr, rl, 2, 8, 12, 1, &r, cig);
        fprintf(o, "%s %s %d %d %d %d %d %d %d", qb, rb, r.score1, r.ref_begin1, r.ref_end1, r.read_begin1,
                r.read_end1, r.flag, r.n_cigar);
        for (int i = 0; i < r.n_cigar; ++i) fprintf(o, " %u", cig[i]);
        fprintf(o, "\n");
    }
    free(qb); free(rb); free(cig); free(tq); free(trr);
    fclose(in); fclose(o);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: oracle_cli seeds|ssw ...\n"); return 2; }
    if (!strcmp(argv[1], "seeds")) return cmd_seeds(argc, argv);
    if (!strcmp(argv[1], "ssw")) return cmd_ssw(argc, argv);
    fprintf(stderr, "unknown command\n");
    return 2;
}
