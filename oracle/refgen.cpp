// refgen.cpp -- golden-vector generator linked against the REFERENCE's own
// sources (compiled unmodified from /root/reference by oracle/Makefile into
// oracle/_ref/).  TEST INFRASTRUCTURE ONLY: this driver is our code; every
// number it prints is computed by the reference's functions:
//   index   : StrobemerIndex::populate + write      (src/index.cpp:73-242)
//   seeds   : randstrobes_query / find_nams / find_nams_rescue
//             (src/randstrobes.cpp:207-253, src/nam.cpp:771-1012)
//   ssw     : ssw_init + ssw_align                  (ext/ssw/ssw.c:789-922)
//   sam     : Sam::add / add_pair / add_unmapped*   (src/sam.cpp), reverse_complement (revcomp.hpp)
//   pdqsort : pdqsort_branchless over RefRandstrobe  (src/index.cpp:168, ext/pdqsort/pdqsort.h,
//             operator< of src/randstrobes.hpp:32-35) on a raw 16-byte entry file
// Only FASTA parsing (refs.cpp needs the un-vendored zstr) and the SSW base
// translation table (ssw_cpp.cpp includes a CUDA header) are restated here.
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "index.hpp"
#include "indexparameters.hpp"
#include "nam.hpp"
#include "randstrobes.hpp"
#include "refs.hpp"
#include "sam.hpp"
#include "revcomp.hpp"
#include <memory>
#include <array>
#include "ssw/ssw.h"
#include "pdqsort/pdqsort.h"

// refs.cpp:8-58 semantics: name cut at the first ' ', sequence uppercased with c & ~32
static References read_fasta(const std::string& fn) {
    std::ifstream in(fn);
    if (!in) { fprintf(stderr, "cannot open %s\n", fn.c_str()); exit(2); }
    std::vector<std::string> seqs, names;
    std::string line, seq, name;
    bool eof = false;
    do {
        eof = !bool(std::getline(in, line));
        if (eof || (!line.empty() && line[0] == '>')) {
            if (!seq.empty()) {
                for (auto& c : seq) c = (char)((unsigned char)c & ~32);
                seqs.push_back(seq);
                names.push_back(name);
            }
            if (!eof) name = line.substr(1, line.find(' ') - 1);
            seq.clear();
        } else {
            seq += line;
        }
    } while (!eof);
    return References(std::move(seqs), std::move(names));
}

static int cmd_index(int argc, char** argv) {
    if (argc < 5) { fprintf(stderr, "index <fasta> <read_len> <out.sti> [threads]\n"); return 2; }
    References refs = read_fasta(argv[2]);
    IndexParameters params = IndexParameters::from_read_length(atoi(argv[3]));
    StrobemerIndex index(refs, params);
    int threads = argc > 5 ? atoi(argv[5]) : 4;
    index.populate(0.0002f, threads);
    index.write(argv[4]);
    printf("bits=%d filter_cutoff=%u n=%zu\n", index.get_bits(), index.filter_cutoff, index.size());
    return 0;
}

static void print_nam(FILE* o, const Nam& n) {
    fprintf(o, "%d %d %d %d %d %d %d %d %d %.9g %d\n", n.nam_id, n.query_start, n.query_end,
            n.query_prev_hit_startpos, n.ref_start, n.ref_end, n.ref_prev_hit_startpos, n.n_hits,
            n.ref_id, (double)n.score, (int)n.is_rc);
}

// seeds <fasta> <sti> <read_len> <reads.txt> <out> <rescue_level>
static int cmd_seeds(int argc, char** argv) {
    if (argc < 8) { fprintf(stderr, "seeds <fasta> <sti> <read_len> <reads.txt> <out> <R>\n"); return 2; }
    References refs = read_fasta(argv[2]);
    IndexParameters params = IndexParameters::from_read_length(atoi(argv[4]));
    StrobemerIndex index(refs, params);
    index.read(argv[3]);
    unsigned rescue_cutoff = atoi(argv[7]) < 100 ? atoi(argv[7]) * index.filter_cutoff : 1000;
    std::ifstream in(argv[5]);
    FILE* o = fopen(argv[6], "w");
    std::string seq;
    while (std::getline(in, seq)) {
        auto q = randstrobes_query(seq, params);
        fprintf(o, "Q %zu\n", q.size());
        for (auto& r : q) fprintf(o, "%" PRIu64 " %u %u %d\n", r.hash, r.start, r.end, (int)r.is_reverse);
        auto [nonrep, nams] = find_nams(q, index);
        uint32_t bits;
        memcpy(&bits, &nonrep, 4);
        fprintf(o, "N %08x %zu\n", bits, nams.size());
        for (auto& n : nams) print_nam(o, n);
        auto rn = find_nams_rescue(q, index, rescue_cutoff);
        fprintf(o, "R %zu\n", rn.size());
        for (auto& n : rn) print_nam(o, n);
    }
    fclose(o);
    return 0;
}

// restated kBaseTranslation (ssw_cpp.cpp:12-25): U/u -> 0 (sic)
static int8_t tr(unsigned char c) {
    switch (c) {
        case 'A': case 'a': case 'U': case 'u': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return 4;
    }
}

static void run_ssw(FILE* o, const std::string& q, const std::string& r) {
    int8_t mat[25];
    int id = 0;
    for (int i = 0; i < 4; ++i) {   // BuildSwScoreMatrix (ssw_cpp.cpp:27-52) with A=2, B=8
        for (int j = 0; j < 4; ++j) mat[id++] = i == j ? 2 : -8;
        mat[id++] = -8;
    }
    for (int i = 0; i < 5; ++i) mat[id++] = -8;
    std::vector<int8_t> tq(q.size()), trf(r.size());
    for (size_t i = 0; i < q.size(); ++i) tq[i] = tr(q[i]);
    for (size_t i = 0; i < r.size(); ++i) trf[i] = tr(r[i]);
    int mask_len = std::max((int)q.size() / 2, 15);
    s_profile* p = ssw_init(tq.data(), (int)q.size(), mat, 5, 2);
    s_align* a = ssw_align(p, trf.data(), (int)r.size(), 12, 1, 0x0f, 0, 32767, mask_len);
    fprintf(o, "%s %s %d %d %d %d %d %d %d", q.c_str(), r.c_str(), a->score1, a->ref_begin1, a->ref_end1,
            a->read_begin1, a->read_end1, (int)a->flag, a->cigarLen);
    for (int i = 0; i < a->cigarLen; ++i) fprintf(o, " %u", a->cigar[i]);
    fprintf(o, "\n");
    align_destroy(a);
    init_destroy(p);
}

// ssw <jobs.txt> <out> : each line "query ref"
static int cmd_ssw(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "ssw <jobs.txt> <out>\n"); return 2; }
    std::ifstream in(argv[2]);
    FILE* o = fopen(argv[3], "w");
    std::string q, r;
    while (in >> q >> r) run_ssw(o, q, r);
    fclose(o);
    return 0;
}

// sswrand <seed> <n> <out> : random extension/rescue-shaped jobs (our generator)
static int cmd_sswrand(int argc, char** argv) {
    if (argc < 5) { fprintf(stderr, "sswrand <seed> <n> <out>\n"); return 2; }
    std::mt19937_64 rng(strtoull(argv[2], nullptr, 10));
    int n = atoi(argv[3]);
    FILE* o = fopen(argv[4], "w");
    const char* B = "ACGT";
    auto rnd = [&](int a, int b) { return a + (int)(rng() % (uint64_t)(b - a + 1)); };
    for (int it = 0; it < n; ++it) {
        int kind = rnd(0, 9);
        int L = kind < 6 ? 150 : (kind < 8 ? rnd(20, 300) : rnd(1, 60));
        int ref_len = L + rnd(0, 400);
        std::string ref(ref_len, 'A');
        int alph = kind == 9 ? 2 : 4;   // low-complexity
        for (auto& c : ref) c = B[rng() % alph];
        if (rng() % 10 == 0) for (int z = 0; z < rnd(1, 5); ++z) ref[rng() % ref.size()] = 'N';
        int off = rnd(0, ref_len - 1);
        std::string q;
        double sub = rnd(0, 8) / 100.0, ind = rnd(0, 4) / 100.0;
        for (int p = off; (int)q.size() < L; ++p) {
            char c = p < ref_len ? ref[p] : B[rng() % 4];
            double u = (rng() % 100000) / 100000.0;
            if (u < sub) q += B[rng() % 4];
            else if (u < sub + ind / 2) { /* deletion */ }
            else if (u < sub + ind) { q += c; q += B[rng() % 4]; }
            else q += c;
            if (rng() % 50 == 0) { int gl = rnd(1, 12); if (rng() % 2) p += gl; else for (int g = 0; g < gl; ++g) q += B[rng() % 4]; }
        }
        q.resize(L);
        if (rng() % 15 == 0) q[rng() % q.size()] = 'N';
        if (rng() % 7 == 0) std::swap(q, ref), (void)0;
        if (q.empty() || ref.empty()) continue;
        run_ssw(o, q, ref);
    }
    fclose(o);
    return 0;
}

// sam <fasta> <calls.txt> <out> : replay a list of Sam calls through the
// reference's Sam class (src/sam.cpp) -- the expected bytes of
// tests/golden/sam_calls.*; oracle/sam_replay.cpp replays the same list through
// the product's Sam (csrc/host/io.cpp).  One call per line, whitespace separated
// ("*" = empty string, "-" = empty read group):
//   S eqx rg_id output_unmapped details          new Sam (sam.hpp:72-92)
//   A name seq qual mapq primary <det> <aln>     add (sam.cpp:125-147)
//   P name1 seq1 qual1 name2 seq2 qual2 mapq1 mapq2 proper primary <det1> <det2> <aln1> <aln2>   add_pair
//   U name seq qual flags                        add_unmapped
//   UP name1 seq1 qual1 name2 seq2 qual2         add_unmapped_pair
//   UM name seq qual flags mate_ref mate_pos     add_unmapped_mate
//   det = nam_rescue nams nam_inconsistent mate_rescue tried_alignment gapped
//   aln = ref_id ref_start length edit_distance score is_rc is_unaligned ncig op...
// The reverse complements come from the reference's reverse_complement (revcomp.hpp).
static std::string tok(std::istream& s) {
    std::string t;
    s >> t;
    return t == "*" ? std::string() : t;
}

static Alignment parse_aln(std::istream& s) {
    Alignment a;
    int rc, un, nc;
    s >> a.ref_id >> a.ref_start >> a.length >> a.edit_distance >> a.score >> rc >> un >> nc;
    a.is_rc = rc; a.is_unaligned = un;
    std::vector<uint32_t> ops(nc);
    for (auto& x : ops) s >> x;
    a.cigar = Cigar(ops);
    return a;
}

static Details parse_det(std::istream& s) {
    Details d;
    int nr;
    s >> nr >> d.nams >> d.nam_inconsistent >> d.mate_rescue >> d.tried_alignment >> d.gapped;
    d.nam_rescue = nr;
    return d;
}

static klibpp::KSeq parse_rec(std::istream& s) {
    klibpp::KSeq r;
    r.name = tok(s);
    r.seq = tok(s);
    r.qual = tok(s);
    return r;
}

static int cmd_sam(int argc, char** argv) {
    if (argc < 5) { fprintf(stderr, "sam <fasta> <calls> <out>\n"); return 2; }
    References refs = read_fasta(argv[2]);
    std::ifstream in(argv[3]);
    std::string out;
    std::unique_ptr<Sam> sam;
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream s(line);
        std::string kind;
        s >> kind;
        if (kind == "S") {
            int eqx, unmapped, details;
            std::string rg;
            s >> eqx >> rg >> unmapped >> details;
            if (rg == "-") rg.clear();
            sam.reset(new Sam(out, refs, eqx ? CigarOps::EQX : CigarOps::M, rg, unmapped, details));
        } else if (kind == "A") {
            klibpp::KSeq r = parse_rec(s);
            int mapq, primary;
            s >> mapq >> primary;
            Details d = parse_det(s);
            Alignment a = parse_aln(s);
            sam->add(a, r, reverse_complement(r.seq), (uint8_t)mapq, primary, d);
        } else if (kind == "P") {
            klibpp::KSeq r1 = parse_rec(s), r2 = parse_rec(s);
            int m1, m2, proper, primary;
            s >> m1 >> m2 >> proper >> primary;
            std::array<Details, 2> det{parse_det(s), parse_det(s)};
            Alignment a1 = parse_aln(s), a2 = parse_aln(s);
            sam->add_pair(a1, a2, r1, r2, reverse_complement(r1.seq), reverse_complement(r2.seq), (uint8_t)m1,
                          (uint8_t)m2, proper, primary, det);
        } else if (kind == "U") {
            klibpp::KSeq r = parse_rec(s);
            int flags;
            s >> flags;
            sam->add_unmapped(r, (uint16_t)flags);
        } else if (kind == "UP") {
            klibpp::KSeq r1 = parse_rec(s), r2 = parse_rec(s);
            sam->add_unmapped_pair(r1, r2);
        } else if (kind == "UM") {
            klibpp::KSeq r = parse_rec(s);
            int flags;
            uint32_t pos;
            std::string ref;
            s >> flags >> ref >> pos;
            sam->add_unmapped_mate(r, (uint16_t)flags, ref, pos);
        } else if (!kind.empty()) {
            fprintf(stderr, "bad call line: %s\n", line.c_str());
            return 2;
        }
    }
    FILE* o = fopen(argv[4], "w");
    fwrite(out.data(), 1, out.size(), o);
    fclose(o);
    return 0;
}

// pdqsort IN OUT: IN holds RefRandstrobe entries (u64 hash, u32 position, u32 packed)
// back to back; OUT gets them in the order populate()'s sort leaves them
static int cmd_pdqsort(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: refgen pdqsort IN OUT\n"); return 2; }
    std::ifstream in(argv[2], std::ios::binary);
    std::vector<char> raw((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    static_assert(sizeof(RefRandstrobe) == 16, "the .sti entry layout");
    std::vector<RefRandstrobe> v(raw.size() / 16);
    if (!v.empty()) memcpy((void*)v.data(), raw.data(), 16 * v.size());   // the .sti payload layout (index.cpp:91-132)
    pdqsort_branchless(v.begin(), v.end());
    FILE* o = fopen(argv[3], "wb");
    if (!o) return 1;
    if (!v.empty()) fwrite((const void*)v.data(), 16, v.size(), o);
    fclose(o);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: refgen index|seeds|ssw|sswrand|sam|pdqsort ...\n"); return 2; }
    if (std::string(argv[1]) == "pdqsort") return cmd_pdqsort(argc, argv);
    std::string c = argv[1];
    if (c == "index") return cmd_index(argc, argv);
    if (c == "seeds") return cmd_seeds(argc, argv);
    if (c == "ssw") return cmd_ssw(argc, argv);
    if (c == "sswrand") return cmd_sswrand(argc, argv);
    if (c == "sam") return cmd_sam(argc, argv);
    fprintf(stderr, "unknown command %s\n", argv[1]);
    return 2;
}
