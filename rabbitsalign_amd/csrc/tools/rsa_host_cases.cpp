// rsa_host_cases -- runs the host pipeline's per-job arithmetic on cases read
// from stdin, for the hand-derived fixtures of tests/host_cases.py:
//   ext_window    qs qe rs re rc read_len contig_len
//   rescue_window qs qe rs re rc read_len contig_len mu sigma
//   ext_store     qs qe rs re rc read_len                    INFO
//   rescue_store  qs qe rs re rc read_len contig_len mu sigma INFO
// INFO = ref_start ref_end query_start query_end edit_distance sw_score n_ops op...
// (an AlignmentInfo as Aligner::align returns it).  Windows print "window START LEN",
// stores "aln ref_start length edit_distance global_ed score is_rc is_unaligned
// gapped n_ops op...".  mu / sigma are read as floats (strtof), as the pipeline
// holds them.  The functions are the product's own (rsa_host.hpp).
//
// `rsa_host_cases pdqsort IN OUT THREADS` instead sorts a raw 16-byte entry file
// (the .sti payload) with the product's replay of pdqsort_branchless
// (sti_order.hpp), for the comparison with the reference's own sort.
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <string>

#include "../host/rsa_host.hpp"
#include "../host/sti_order.hpp"

using namespace rsa;

static Nam read_nam(std::istringstream& in) {
    Nam n{};
    in >> n.query_start >> n.query_end >> n.ref_start >> n.ref_end >> n.is_rc;
    return n;
}

static AlignmentInfo read_info(std::istringstream& in) {
    AlignmentInfo a;
    size_t nops = 0;
    in >> a.ref_start >> a.ref_end >> a.query_start >> a.query_end >> a.edit_distance >> a.sw_score >> nops;
    for (size_t i = 0; i < nops; ++i) {
        uint32_t op = 0;
        in >> op;
        a.cigar.ops.push_back(op);
    }
    return a;
}

static float read_float(std::istringstream& in) {
    std::string t;
    in >> t;
    return strtof(t.c_str(), nullptr);
}

static void print_aln(const Alignment& a) {
    printf("aln %d %d %d %d %d %d %d %d %zu", a.ref_start, a.length, a.edit_distance, a.global_ed, a.score,
           a.is_rc ? 1 : 0, a.is_unaligned ? 1 : 0, a.gapped ? 1 : 0, a.cigar.ops.size());
    for (uint32_t x : a.cigar.ops) printf(" %u", x);
    printf("\n");
}

static int pdqsort_file(const char* in_path, const char* out_path, int threads) {
    FILE* f = fopen(in_path, "rb");
    if (!f) return 1;
    std::vector<rsa_ref_randstrobe> v;
    rsa_ref_randstrobe e;
    while (fread(&e, sizeof e, 1, f) == 1) v.push_back(e);
    fclose(f);
    sti_order::pdqsort_replay(v.data(), v.size(), threads);
    FILE* o = fopen(out_path, "wb");
    if (!o) return 1;
    if (!v.empty()) fwrite(v.data(), sizeof e, v.size(), o);
    return fclose(o) == 0 ? 0 : 1;
}

int main(int argc, char** argv) {
    if (argc >= 4 && std::string(argv[1]) == "pdqsort") return pdqsort_file(argv[2], argv[3], argc > 4 ? atoi(argv[4]) : 1);
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string kind;
        if (!(in >> kind)) continue;
        if (kind == "ext_window") {
            const Nam nam = read_nam(in);
            size_t read_len, contig_len;
            in >> read_len >> contig_len;
            uint32_t s, l;
            extension_window(nam, read_len, contig_len, s, l);
            printf("window %u %u\n", s, l);
        } else if (kind == "rescue_window") {
            const Nam nam = read_nam(in);
            size_t read_len, contig_len;
            in >> read_len >> contig_len;
            const float mu = read_float(in), sigma = read_float(in);
            uint32_t s, l;
            rescue_mate_window(nam, read_len, mu, sigma, contig_len, s, l);
            printf("window %u %u\n", s, l);
        } else if (kind == "ext_store") {
            const Nam nam = read_nam(in);
            size_t read_len;
            in >> read_len;
            AlignmentInfo info = read_info(in);
            Alignment a;
            extension_alignment(nam, read_len, info, a);
            print_aln(a);
        } else if (kind == "rescue_store") {
            const Nam nam = read_nam(in);
            size_t read_len, contig_len;
            in >> read_len >> contig_len;
            const float mu = read_float(in), sigma = read_float(in);
            AlignmentInfo info = read_info(in);
            Alignment a;
            rescue_alignment(nam, read_len, mu, sigma, contig_len, info, a);
            print_aln(a);
        } else {
            fprintf(stderr, "unknown case kind %s\n", kind.c_str());
            return 1;
        }
    }
    return 0;
}
