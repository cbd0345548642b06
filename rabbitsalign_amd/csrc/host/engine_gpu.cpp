// engine_gpu.cpp -- the product engine: every hot-path call goes through the
// HIP C-ABI (include/rsa_gpu.h, librsa_gpu.so).  There is no CPU fallback;
// a failed GPU call aborts the run with the library's error message.
#include <cstring>
#include <stdexcept>
#include <string>

#include "rsa_host.hpp"

namespace rsa {

namespace {

class GpuEngine final : public Engine {
public:
    GpuEngine(const References& refs, const StiIndex& idx, int device) {
        rsa_index_view v{};
        v.randstrobes = idx.randstrobes.data();
        v.n_randstrobes = idx.randstrobes.size();
        v.bucket_starts = idx.bucket_starts.data();
        v.bits = idx.bits;
        v.filter_cutoff = idx.filter_cutoff;
        v.k = idx.params.k; v.s = idx.params.s; v.t_syncmer = idx.params.t;
        v.w_min = (int)idx.params.w_min; v.w_max = (int)idx.params.w_max; v.max_dist = idx.params.max_dist;
        v.q = (uint64_t)idx.params.q;
        v.ref_seq = refs.concat.data();
        v.contig_offsets = refs.offsets.data();
        v.n_contigs = (int)refs.size();
        char err[512] = {0};
        ctx_ = rsa_open(device, &v, err, sizeof err);
        if (!ctx_) throw std::runtime_error(std::string("GPU engine: ") + err);
    }
    ~GpuEngine() override { rsa_close(ctx_); }
    const char* name() const override { return "hip-gfx950"; }

    void seed(const std::vector<const std::string*>& reads, int rescue_level, unsigned rescue_cutoff,
              SeedBatchOut& out) override {
        const size_t n = reads.size();
        std::string blob;
        size_t tot = 0;
        for (auto* r : reads) tot += r->size();
        blob.reserve(tot);
        std::vector<uint64_t> offs(n);
        std::vector<uint32_t> lens(n);
        for (size_t i = 0; i < n; ++i) { offs[i] = blob.size(); lens[i] = (uint32_t)reads[i]->size(); blob += *reads[i]; }
        rsa_read_batch rb{blob.data(), offs.data(), lens.data(), (uint32_t)n};
        out.offsets.assign(n + 1, 0);
        out.nonrep.assign(n, 0.f);
        out.rescued.assign(n, 0);
        size_t cap = std::max<size_t>(1024, 16 * n);
        for (;;) {
            out.nams.resize(cap);
            rsa_nam_batch nb{out.nams.data(), cap, out.offsets.data(), out.nonrep.data(), out.rescued.data(), 0};
            int rc = rsa_seed(ctx_, &rb, rescue_level, rescue_cutoff, &nb);
            if (rc == RSA_ERR_CAPACITY) { cap = nb.needed + 16; continue; }
            if (rc != RSA_OK) throw std::runtime_error(std::string("rsa_seed: ") + rsa_last_error(ctx_));
            out.nams.resize(nb.needed);
            break;
        }
    }

    void extend(const std::vector<SwJob>& jobs, const AlignmentParameters& p,
                std::vector<AlignmentInfo>& out) override {
        const size_t n = jobs.size();
        out.assign(n, AlignmentInfo());
        if (n == 0) return;
        std::string q;
        std::vector<rsa_job> js(n);
        for (size_t i = 0; i < n; ++i) {
            js[i].query_offset = q.size();
            js[i].query_len = (uint32_t)jobs[i].query.size();
            js[i].ref_id = jobs[i].ref_id;
            js[i].ref_start = jobs[i].ref_start;
            js[i].ref_len = jobs[i].ref_len;
            q += jobs[i].query;
        }
        rsa_job_batch jb{q.data(), q.size(), js.data(), (uint32_t)n, p.match, p.mismatch, p.gap_open,
                         p.gap_extend, p.end_bonus};
        const uint64_t bound = rsa_extend_cigar_bound(&jb);
        std::vector<rsa_aln> alns(n);
        std::vector<uint32_t> pool(bound + 1);
        rsa_aln_batch ab{alns.data(), pool.data(), bound + 1, 0};
        int rc = rsa_extend(ctx_, &jb, &ab);
        if (rc != RSA_OK) throw std::runtime_error(std::string("rsa_extend: ") + rsa_last_error(ctx_));
        for (size_t i = 0; i < n; ++i) {
            const rsa_aln& a = alns[i];
            AlignmentInfo& o = out[i];
            o.sw_score = a.sw_score;
            o.edit_distance = a.edit_distance;
            o.ref_start = a.ref_start; o.ref_end = a.ref_end;
            o.query_start = a.query_start; o.query_end = a.query_end;
            o.cigar.ops.assign(pool.begin() + (long)a.cigar_offset, pool.begin() + (long)(a.cigar_offset + a.cigar_len));
        }
    }

    bool kernel_stats(rsa_kernel_stats* out) override { return rsa_get_stats(ctx_, out) == RSA_OK; }
    void reset_kernel_stats() override { rsa_reset_stats(ctx_); }

private:
    rsa_ctx* ctx_ = nullptr;
};

}  // namespace

std::unique_ptr<Engine> make_gpu_engine(const References& refs, const StiIndex& index, int device) {
    return std::unique_ptr<Engine>(new GpuEngine(refs, index, device));
}

// engine of librsalign.so (capi.cpp)
std::unique_ptr<Engine> make_default_engine(const References& refs, const StiIndex& index, int device) {
    return make_gpu_engine(refs, index, device);
}

}  // namespace rsa
