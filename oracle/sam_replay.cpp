// sam_replay.cpp -- replays a list of Sam calls (format: oracle/refgen.cpp
// cmd_sam) through the PRODUCT's SAM formatter (rabbitsalign_amd/csrc/host/io.cpp)
// and the product's reverse_complement.  TEST INFRASTRUCTURE ONLY: the output must
// equal, byte for byte, what the reference's own Sam class (src/sam.cpp) wrote for
// the same calls (tests/golden/sam_calls.golden.sam.gz, tests/test_sam_golden.py).
#include <cstdio>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>

#include "../rabbitsalign_amd/csrc/host/rsa_host.hpp"

using namespace rsa;

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
    for (int i = 0; i < nc; ++i) {
        uint32_t x;
        s >> x;
        a.cigar.ops.push_back(x);
    }
    return a;
}

static Details parse_det(std::istream& s) {
    Details d;
    int nr;
    s >> nr >> d.nams >> d.nam_inconsistent >> d.mate_rescue >> d.tried_alignment >> d.gapped;
    d.nam_rescue = nr;
    return d;
}

static Record parse_rec(std::istream& s) {
    Record r;
    r.name = tok(s);
    r.seq = tok(s);
    r.qual = tok(s);
    return r;
}

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "sam_replay <fasta> <calls> <out>\n"); return 2; }
    References refs = References::from_fasta(argv[1]);
    std::ifstream in(argv[2]);
    SamText out;
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
            sam.reset(new Sam(out, refs, eqx != 0, rg, unmapped != 0, details != 0));
        } else if (kind == "A") {
            Record r = parse_rec(s);
            int mapq, primary;
            s >> mapq >> primary;
            Details d = parse_det(s);
            Alignment a = parse_aln(s);
            const std::string rc = reverse_complement(r.seq);
            sam->add(a, r, rc, (uint8_t)mapq, primary != 0, d);
        } else if (kind == "P") {
            Record r1 = parse_rec(s), r2 = parse_rec(s);
            int m1, m2, proper, primary;
            s >> m1 >> m2 >> proper >> primary;
            Details det[2];
            det[0] = parse_det(s);
            det[1] = parse_det(s);
            Alignment a1 = parse_aln(s), a2 = parse_aln(s);
            const std::string rc1 = reverse_complement(r1.seq), rc2 = reverse_complement(r2.seq);
            sam->add_pair(a1, a2, r1, r2, rc1, rc2, (uint8_t)m1, (uint8_t)m2, proper != 0, primary != 0, det);
        } else if (kind == "U") {
            Record r = parse_rec(s);
            int flags;
            s >> flags;
            sam->add_unmapped(r, (uint16_t)flags);
        } else if (kind == "UP") {
            Record r1 = parse_rec(s), r2 = parse_rec(s);
            sam->add_unmapped_pair(r1, r2);
        } else if (kind == "UM") {
            Record r = parse_rec(s);
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
    FILE* o = fopen(argv[3], "w");
    if (!o) return 2;
    fwrite(out.data(), 1, out.size(), o);
    fclose(o);
    return 0;
}
