// engine_ref.cpp -- CPU path whose hot path is the REFERENCE's own code:
// randstrobes_query / find_nams / find_nams_rescue (src/randstrobes.cpp,
// src/nam.cpp) and ssw_init / ssw_align (ext/ssw/ssw.c), compiled unmodified
// from /root/reference into oracle/_ref/.  Around it runs the product's host
// pipeline (restated aln.cpp / pc.cpp / sam.cpp); the SSW C++ wrapper and the
// Aligner::align end-bonus step are restated in rsa_oracle.c because
// ext/ssw/ssw_cpp.cpp and src/aligner.cpp include a CUDA header and cannot be
// built here.  TEST INFRASTRUCTURE ONLY: end-to-end SAM parity reference and
// bench.py's cpu_baseline leg ("kind": "reference").
#include <cstring>
#include <stdexcept>

#include "index.hpp"
#include "indexparameters.hpp"
#include "nam.hpp"
#include "randstrobes.hpp"
#include "refs.hpp"
#include "ssw/ssw.h"

#include "../rabbitsalign_amd/csrc/host/rsa_host.hpp"
#include "rsa_oracle.h"

namespace {

// ssw_align on translated sequences through the reference's ssw.c; the
// translation / =X split / end bonus are the restated wrapper (rsa_oracle.c).
extern "C" void ora_aligner_align_with(const char* query, int qlen, const char* ref, int rlen, int match,
                                       int mismatch, int gap_open, int gap_extend, int end_bonus, ora_aln_info* out,
                                       uint32_t* cigar,
                                       void (*raw)(const int8_t*, int, const int8_t*, int, int, int, int, int,
                                                   ora_ssw_res*, uint32_t*));

void ref_ssw_raw(const int8_t* q, int qlen, const int8_t* r, int rlen, int match, int mismatch, int gap_open,
                 int gap_extend, ora_ssw_res* res, uint32_t* cigar) {
    int8_t mat[25];
    int id = 0;
    for (int i = 0; i < 4; ++i) {
        for (int j = 0; j < 4; ++j) mat[id++] = i == j ? (int8_t)match : (int8_t)-mismatch;
        mat[id++] = (int8_t)-mismatch;
    }
    for (int i = 0; i < 5; ++i) mat[id++] = (int8_t)-mismatch;
    int mask_len = std::max(qlen / 2, 15);
    s_profile* p = ssw_init(q, qlen, mat, 5, 2);
    s_align* a = ssw_align(p, r, rlen, (uint8_t)gap_open, (uint8_t)gap_extend, 0x0f, 0, 32767, mask_len);
    res->score1 = a->score1; res->ref_begin1 = a->ref_begin1; res->ref_end1 = a->ref_end1;
    res->read_begin1 = a->read_begin1; res->read_end1 = a->read_end1; res->flag = a->flag;
    res->n_cigar = a->cigarLen;
    for (int i = 0; i < a->cigarLen; ++i) cigar[i] = a->cigar[i];
    align_destroy(a);
    init_destroy(p);
}

class RefEngine final : public rsa::Engine {
public:
    RefEngine(const rsa::References& refs, const rsa::StiIndex& idx)
        : refs_(refs),
          ref_refs_(std::vector<std::string>(refs.seqs), std::vector<std::string>(refs.names)),
          params_(IndexParameters::from_read_length(idx.params.canonical_read_length)),
          index_(ref_refs_, params_, idx.bits) {
        index_.filter_cutoff = (unsigned)idx.filter_cutoff;
        index_.randstrobes.resize(idx.randstrobes.size());
        memcpy(index_.randstrobes.data(), idx.randstrobes.data(), idx.randstrobes.size() * sizeof(RefRandstrobe));
        index_.randstrobe_start_indices.assign(idx.bucket_starts.begin(), idx.bucket_starts.end());
    }
    const char* name() const override { return "cpu-reference"; }
    void seed(const std::vector<std::string_view>& reads, int rescue_level, unsigned rescue_cutoff,
              rsa::SeedBatchOut& out) override {
        const size_t n = reads.size();
        out.nams.clear();
        out.offsets.assign(n + 1, 0);
        out.nonrep.assign(n, 1.f);
        out.rescued.assign(n, 0);
        for (size_t i = 0; i < n; ++i) {
            auto q = randstrobes_query(reads[i], params_);
            auto [nonrep, nams] = find_nams(q, index_);
            out.nonrep[i] = nonrep;
            if (rescue_level > 1 && (nams.empty() || nonrep < 0.7)) {
                nams = find_nams_rescue(q, index_, rescue_cutoff);
                out.rescued[i] = 1;
            }
            for (auto& x : nams) {
                rsa_nam y;
                y.nam_id = x.nam_id; y.query_start = x.query_start; y.query_end = x.query_end;
                y.query_prev_hit_startpos = x.query_prev_hit_startpos; y.ref_start = x.ref_start;
                y.ref_end = x.ref_end; y.ref_prev_hit_startpos = x.ref_prev_hit_startpos; y.n_hits = x.n_hits;
                y.ref_id = x.ref_id; y.score = x.score; y.is_rc = x.is_rc;
                out.nams.push_back(y);
            }
            out.offsets[i + 1] = out.nams.size();
        }
    }
    void extend(const std::vector<rsa::SwJob>& jobs, const rsa::AlignmentParameters& p,
                std::vector<rsa::AlignmentInfo>& out) override {
        out.assign(jobs.size(), rsa::AlignmentInfo());
        std::vector<uint32_t> cig;
        for (size_t i = 0; i < jobs.size(); ++i) {
            const auto& j = jobs[i];
            const char* ref = refs_.concat.data() + refs_.offsets[j.ref_id] + j.ref_start;
            if (rsa::shared_check_fails(j, std::string_view(ref, j.ref_len))) { out[i].no_shared = true; continue; }
            cig.resize(2 * (j.query.size() + j.ref_len) + 16);
            ora_aln_info info;
            ora_aligner_align_with(j.query.data(), (int)j.query.size(), ref, (int)j.ref_len, p.match, p.mismatch,
                                   p.gap_open, p.gap_extend, p.end_bonus, &info, cig.data(), ref_ssw_raw);
            auto& o = out[i];
            o.sw_score = info.sw_score; o.edit_distance = info.edit_distance;
            o.ref_start = info.ref_start; o.ref_end = info.ref_end;
            o.query_start = info.query_start; o.query_end = info.query_end;
            o.cigar.ops.assign(cig.begin(), cig.begin() + info.n_cigar);
        }
    }
private:
    const rsa::References& refs_;
    References ref_refs_;
    IndexParameters params_;
    StrobemerIndex index_;
};

std::unique_ptr<rsa::Engine> make_ref_engine(const rsa::References& refs, const rsa::StiIndex& idx, int) {
    return std::unique_ptr<rsa::Engine>(new RefEngine(refs, idx));
}

}  // namespace

// engine of the CPU-path build of librsalign (capi.cpp)
namespace rsa {
std::unique_ptr<Engine> make_default_engine(const References& refs, const StiIndex& idx, int device) {
    return make_ref_engine(refs, idx, device);
}
}  // namespace rsa

#ifndef RSA_ENGINE_LIB
int main(int argc, char** argv) { return rsa::cli_main(argc, argv, make_ref_engine, "rsalign_ref"); }
#endif
