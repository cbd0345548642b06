// engine_cpu.cpp -- the CPU path: the product's host pipeline (restated
// aln.cpp/pc.cpp/sam.cpp) driven by the C restatement of the hot path
// (rsa_oracle.c) instead of the GPU.  TEST INFRASTRUCTURE ONLY: it is the
// parity reference for end-to-end SAM and bench.py's cpu_baseline leg.
#include <atomic>
#include <cstdio>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "../rabbitsalign_amd/csrc/host/rsa_host.hpp"
#include "rsa_oracle.h"

namespace {

class CpuEngine final : public rsa::Engine {
public:
    CpuEngine(const rsa::References& refs, const rsa::StiIndex& idx) : refs_(refs) {
        ix_.rs = (const ora_refrs*)idx.randstrobes.data();
        ix_.n = idx.randstrobes.size();
        ix_.starts = idx.bucket_starts.data();
        ix_.bits = idx.bits;
        ix_.filter_cutoff = (unsigned)idx.filter_cutoff;
        ix_.k = idx.params.k;
        p_.k = idx.params.k; p_.s = idx.params.s; p_.t_syncmer = idx.params.t;
        p_.w_min = (int)idx.params.w_min; p_.w_max = (int)idx.params.w_max; p_.max_dist = idx.params.max_dist;
        p_.q = (uint64_t)idx.params.q;
    }
    const char* name() const override { return "cpu-oracle"; }
    void seed(const std::vector<std::string_view>& reads, int rescue_level, unsigned rescue_cutoff,
              rsa::SeedBatchOut& out) override {
        const size_t n = reads.size();
        out.nams.clear();
        out.offsets.assign(n + 1, 0);
        out.nonrep.assign(n, 1.f);
        out.rescued.assign(n, 0);
        std::vector<ora_qrs> q;
        std::vector<ora_nam> nams(1 << 16);
        for (size_t i = 0; i < n; ++i) {
            const std::string_view s = reads[i];
            q.resize(2 * s.size() + 8);
            int nq = ora_randstrobes_query(s.data(), (int)s.size(), &p_, q.data(), (int)q.size());
            float nonrep = 1.f;
            int nn;
            while ((nn = ora_find_nams(&ix_, q.data(), nq, nams.data(), (int)nams.size(), &nonrep)) < 0) nams.resize(nams.size() * 2);
            out.nonrep[i] = nonrep;
            if (rescue_level > 1 && (nn == 0 || nonrep < 0.7f)) {
                while ((nn = ora_find_nams_rescue(&ix_, q.data(), nq, rescue_cutoff, nams.data(), (int)nams.size())) < 0)
                    nams.resize(nams.size() * 2);
                out.rescued[i] = 1;
            }
            for (int j = 0; j < nn; ++j) {
                rsa_nam x;
                static_assert(sizeof(rsa_nam) == sizeof(ora_nam), "layout");
                memcpy(&x, &nams[j], sizeof x);
                out.nams.push_back(x);
            }
            out.offsets[i + 1] = out.nams.size();
        }
    }
    void extend(const std::vector<rsa::SwJob>& jobs, const rsa::AlignmentParameters& p,
                std::vector<rsa::AlignmentInfo>& out) override {
        // fault injection for the pipeline's error path (tests only): RSA_TEST_FAIL_EXTEND=N
        // makes the N-th extend call throw, as a failed GPU call does in the product engine
        static const long fail_at = getenv("RSA_TEST_FAIL_EXTEND") ? atol(getenv("RSA_TEST_FAIL_EXTEND")) : 0;
        if (fail_at > 0 && ++calls_ == fail_at) throw std::runtime_error("injected extend failure");
        // job-shape histogram for kernel design (RSA_TEST_JOB_HIST=file; test infrastructure)
        static const char* hist_path = getenv("RSA_TEST_JOB_HIST");
        if (hist_path) {
            static std::mutex hm;
            std::lock_guard<std::mutex> g(hm);
            if (FILE* f = fopen(hist_path, "a")) {
                for (const auto& j : jobs) fprintf(f, "%zu %u\n", j.query.size(), (unsigned)j.ref_len);
                fclose(f);
            }
        }
        out.assign(jobs.size(), rsa::AlignmentInfo());
        std::vector<uint32_t> cig;
        for (size_t i = 0; i < jobs.size(); ++i) {
            const auto& j = jobs[i];
            const char* ref = refs_.concat.data() + refs_.offsets[j.ref_id] + j.ref_start;
            if (rsa::shared_check_fails(j, std::string_view(ref, j.ref_len))) { out[i].no_shared = true; continue; }
            cig.resize(2 * (j.query.size() + j.ref_len) + 16);
            ora_aln_info info;
            ora_aligner_align(j.query.data(), (int)j.query.size(), ref, (int)j.ref_len, p.match, p.mismatch,
                              p.gap_open, p.gap_extend, p.end_bonus, &info, cig.data());
            auto& o = out[i];
            o.sw_score = info.sw_score; o.edit_distance = info.edit_distance;
            o.ref_start = info.ref_start; o.ref_end = info.ref_end;
            o.query_start = info.query_start; o.query_end = info.query_end;
            o.cigar.ops.assign(cig.begin(), cig.begin() + info.n_cigar);
        }
    }
private:
    const rsa::References& refs_;
    std::atomic<long> calls_{0};
    ora_index ix_;
    ora_params p_;
};

std::unique_ptr<rsa::Engine> make_cpu_engine(const rsa::References& refs, const rsa::StiIndex& idx, int) {
    return std::unique_ptr<rsa::Engine>(new CpuEngine(refs, idx));
}

}  // namespace

// engine of the CPU-path build of librsalign (capi.cpp)
namespace rsa {
std::unique_ptr<Engine> make_default_engine(const References& refs, const StiIndex& idx, int device) {
    return make_cpu_engine(refs, idx, device);
}
}  // namespace rsa

#ifndef RSA_ENGINE_LIB
int main(int argc, char** argv) { return rsa::cli_main(argc, argv, make_cpu_engine, "rsalign_cpu"); }
#endif
