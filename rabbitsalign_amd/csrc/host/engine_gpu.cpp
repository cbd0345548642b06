// engine_gpu.cpp -- the product engine: every hot-path call goes through the
// HIP C-ABI (include/rsa_gpu.h, librsa_gpu.so).  There is no CPU fallback;
// a failed GPU call aborts the run with the library's error message.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <mutex>
#include <string>
#include <vector>

#include "rsa_host.hpp"

namespace rsa {

namespace {

// Per-thread page-locked batch buffers (rsa_host_alloc), grown on demand and
// reused across chunks, so batch transfers run at DMA speed without staging.
struct Staging {
    enum { READS, ROFF, RLEN, NAMS, QUERIES, JOBS, ALNS, POOL, SITES, MMPOOL, N };
    void* p[N] = {};
    size_t cap[N] = {};
    template <class T> T* get(int k, size_t count) {
        const size_t bytes = std::max<size_t>(64, count * sizeof(T));
        if (bytes > cap[k]) {
            rsa_host_free(p[k]);
            const size_t nb = std::max(bytes, cap[k] + cap[k] / 2);
            p[k] = rsa_host_alloc(nb);
            if (!p[k]) { cap[k] = 0; throw std::runtime_error("rsa_host_alloc failed"); }
            cap[k] = nb;
        }
        return (T*)p[k];
    }
    ~Staging() { for (void* x : p) rsa_host_free(x); }
};

class GpuEngine final : public Engine {
public:
    GpuEngine(const References& refs, const StiIndex& idx, int device) {
        rsa_index_view v{};
        const bool adopt = idx.device_build && idx.device_build->handle && idx.randstrobes.empty();
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
        if (adopt) {   // the index built on this device stays where it is (no D2H + H2D)
            v.n_randstrobes = idx.n_device;
            ctx_ = rsa_open_built((rsa_index_build*)idx.device_build->handle, &v, err, sizeof err);
            if (ctx_) idx.device_build->handle = nullptr;
        } else {
            if (!idx.host_copy()) throw std::runtime_error("GPU engine: index has no host copy and no device build");
            ctx_ = rsa_open(device, &v, err, sizeof err);
        }
        if (!ctx_) throw std::runtime_error(std::string("GPU engine: ") + err);
    }
    bool download_index(StiIndex& idx) override {
        if (idx.host_copy()) return true;
        std::vector<rsa_ref_randstrobe> rs(idx.n_device);
        std::vector<uint64_t> st((1ull << idx.bits) + 1);
        if (rsa_index_download(ctx_, rs.data(), st.data()) != RSA_OK) return false;
        idx.randstrobes.swap(rs);
        idx.bucket_starts.swap(st);
        return true;
    }
    // a pipeline start sets them while seeding calls of another run on this engine may
    // read them: every seeding call takes one consistent snapshot under the lock
    void set_alignment_params(const AlignmentParameters& p) override {
        std::lock_guard<std::mutex> g(ap_m_);
        ap_ = p;
        ap_set_ = true;
    }

    ~GpuEngine() override {
        free_.clear();
        staging_.clear();                  // pinned buffers go before the context
        rsa_close(ctx_);
    }
    const char* name() const override { return "hip-gfx950"; }
    bool offloads() const override { return true; }

    const HostAllocFns* io_alloc() const override { return &pinned_fns(); }
    static const HostAllocFns& pinned_fns() {
        static const HostAllocFns f{rsa_host_alloc, rsa_host_free};
        return f;
    }

    void seed_packed(const char* blob, const uint64_t* offs, const uint32_t* lens, size_t n, int rescue_level,
                     unsigned rescue_cutoff, SeedBatchOut& out) override {
        rsa_read_batch rb{blob, offs, lens, (uint32_t)n};
        seed_batch(rb, rescue_level, rescue_cutoff, out);
    }

    void seed(const std::vector<std::string_view>& reads, int rescue_level, unsigned rescue_cutoff,
              SeedBatchOut& out) override {
        const size_t n = reads.size();
        const Lease ls = lease();
        Staging& sg = *ls.s;
        size_t tot = 0;
        for (auto r : reads) tot += r.size();
        char* blob = sg.get<char>(Staging::READS, tot + 16);
        uint64_t* offs = sg.get<uint64_t>(Staging::ROFF, n);
        uint32_t* lens = sg.get<uint32_t>(Staging::RLEN, n);
        size_t pos = 0;
        for (size_t i = 0; i < n; ++i) {
            if (i + 8 < n) {                       // scattered heap strings: request them ahead
                const char* a = reads[i + 8].data();
                for (size_t o = 0; o < reads[i + 8].size(); o += 64) __builtin_prefetch(a + o);
            }
            offs[i] = pos;
            lens[i] = (uint32_t)reads[i].size();
            memcpy(blob + pos, reads[i].data(), reads[i].size());
            pos += reads[i].size();
        }
        rsa_read_batch rb{blob, offs, lens, (uint32_t)n};
        seed_batch(rb, rescue_level, rescue_cutoff, out);
    }

    void seed_batch(const rsa_read_batch& rb, int rescue_level, unsigned rescue_cutoff, SeedBatchOut& out) {
        const size_t n = rb.n_reads;
        out.offsets.assign(n + 1, 0);
        out.nonrep.assign(n, 0.f);
        out.rescued.assign(n, 0);
        // the NAMs, site checks and mismatch positions come back by DMA straight into
        // the output vectors, whose storage is page-locked (no staging copy)
        const HostAllocFns& kPinned = pinned_fns();
        if (out.nams.get_allocator().fns != &kPinned) out.nams = decltype(out.nams)(HostAlloc<Nam>(&kPinned));
        if (out.sites.get_allocator().fns != &kPinned) out.sites = decltype(out.sites)(HostAlloc<rsa_nam_site>(&kPinned));
        if (out.mm_pool.get_allocator().fns != &kPinned) out.mm_pool = decltype(out.mm_pool)(HostAlloc<uint16_t>(&kPinned));
        // site checks on the device (k_sites): the host's NAM orientation and
        // Hamming windows then never read the reference
        static const bool want_sites = !(getenv("RSA_SITES") && getenv("RSA_SITES")[0] == '0');   // A/B switch
        // hamming_align on the device too (RSA_SITE_ALIGNED, RSA_SITE_ALIGN=0: positions only)
        static const bool align_env = !(getenv("RSA_SITE_ALIGN") && getenv("RSA_SITE_ALIGN")[0] == '0');
        AlignmentParameters hp;
        bool hp_set;
        {
            std::lock_guard<std::mutex> g(ap_m_);
            hp = ap_;
            hp_set = ap_set_;
        }
        const bool hamming_on = align_env && hp_set;
        size_t cap = std::max<size_t>(1024, 12 * n);
        for (;;) {
            // 12 + 4 n_mm words an accepted site at most (n_mm < 5 % of the read): overflow is
            // flagged per NAM and handled on the host
            const size_t mm_cap = (hamming_on ? 16 : 4) * cap;
            out.nams.resize(cap);
            out.sites.resize(want_sites ? cap : 0);
            out.mm_pool.resize(mm_cap);
            // lists of <= 16 NAMs come sorted (RSA_NAMS_BY_SCORE): part() works on them in place
            rsa_nam_batch nb{out.nams.data(), cap, out.offsets.data(), out.nonrep.data(), out.rescued.data(), 0,
                             want_sites ? out.sites.data() : nullptr, out.mm_pool.data(), mm_cap, 0,
                             RSA_NAMS_BY_SCORE, hamming_on ? 1u : 0u, hp.match, hp.mismatch, hp.end_bonus, 0};
            int rc = rsa_seed(ctx_, &rb, rescue_level, rescue_cutoff, &nb);
            if (rc == RSA_ERR_CAPACITY) { cap = nb.needed + 16; continue; }
            if (rc != RSA_OK) throw std::runtime_error(std::string("rsa_seed: ") + rsa_last_error(ctx_));
            out.nams.resize(nb.needed);
            out.by_score = true;
            if (want_sites) {
                out.sites.resize(nb.needed);
                out.mm_pool.resize(nb.mm_used);
            } else {
                out.sites.clear();
                out.mm_pool.clear();
            }
            break;
        }
    }

    // Extension calls from the pipeline's workers are combined: a caller that finds
    // fewer than ext_leaders() calls on the device takes every pending request (its
    // own and those that queued meanwhile, up to ext_batch_jobs() jobs) into one
    // rsa_extend; the others sleep until a leader has stored their results.  While
    // calls are in flight requests pile up, so the launches grow with the load
    // (k_ext_scan_g runs far below its throughput at one chunk's 7300 jobs, DESIGN.md
    // §3) and the results do not change: every job is aligned on its own.
    void extend(const std::vector<SwJob>& jobs, const AlignmentParameters& p,
                std::vector<AlignmentInfo>& out) override {
        out.assign(jobs.size(), AlignmentInfo());
        if (jobs.empty()) return;
        if (ext_leaders() <= 0) {
            ExtReq me{&jobs, &p, &out};
            ExtReq* one[1] = {&me};
            run_batch(one, 1);
            if (me.err) std::rethrow_exception(me.err);
            return;
        }
        ExtReq me{&jobs, &p, &out};
        std::unique_lock<std::mutex> l(ext_m_);
        ext_pending_.push_back(&me);
        while (!me.done) {
            // one more call than ext_leaders() while the queued jobs fill a whole batch: the
            // calls in flight cannot take the load (PE 2x250 calls run at the batch cap)
            size_t queued = 0;
            if (ext_active_ >= ext_leaders() && ext_active_ < ext_leaders() + ext_extra_leaders())
                for (const ExtReq* r : ext_pending_) queued += r->jobs->size();
            if ((ext_active_ < ext_leaders() || queued >= ext_batch_jobs()) && !ext_pending_.empty()) {
                ++ext_active_;
                std::vector<ExtReq*> batch;
                size_t n_jobs = 0;
                const AlignmentParameters& bp = *ext_pending_.front()->p;
                for (auto it = ext_pending_.begin(); it != ext_pending_.end();) {
                    ExtReq* r = *it;
                    const bool same = r->p->match == bp.match && r->p->mismatch == bp.mismatch &&
                                      r->p->gap_open == bp.gap_open && r->p->gap_extend == bp.gap_extend &&
                                      r->p->end_bonus == bp.end_bonus;
                    if (same && (batch.empty() || n_jobs + r->jobs->size() <= ext_batch_jobs())) {
                        batch.push_back(r);
                        n_jobs += r->jobs->size();
                        it = ext_pending_.erase(it);
                    } else {
                        ++it;
                    }
                }
                l.unlock();
                run_batch(batch.data(), batch.size());
                l.lock();
                for (ExtReq* r : batch) r->done = true;
                --ext_active_;
                ext_cv_.notify_all();
                continue;
            }
            ext_cv_.wait(l);
        }
        l.unlock();
        if (me.err) std::rethrow_exception(me.err);
    }

    bool kernel_stats(rsa_kernel_stats* out) override { return rsa_get_stats(ctx_, out) == RSA_OK; }
    void reset_kernel_stats() override { rsa_reset_stats(ctx_); }

private:
    struct ExtReq {
        const std::vector<SwJob>* jobs;
        const AlignmentParameters* p;
        std::vector<AlignmentInfo>* out;
        bool done = false;
        std::exception_ptr err;
    };
    // RSA_EXT_LEADERS: combined extension calls in flight at once (0 = every worker
    // calls rsa_extend for its own chunk); RSA_EXT_BATCH_JOBS: jobs a combined call takes
    static int ext_leaders() {
        static const int n = getenv("RSA_EXT_LEADERS") ? atoi(getenv("RSA_EXT_LEADERS")) : 2;
        return n;
    }
    // RSA_EXT_EXTRA_LEADERS: calls beyond ext_leaders() allowed while a full batch is queued
    static int ext_extra_leaders() {
        static const int n = getenv("RSA_EXT_EXTRA_LEADERS") ? std::max(0, atoi(getenv("RSA_EXT_EXTRA_LEADERS"))) : 1;
        return n;
    }
    static size_t ext_batch_jobs() {
        static const size_t n = getenv("RSA_EXT_BATCH_JOBS") ? (size_t)std::max(1, atoi(getenv("RSA_EXT_BATCH_JOBS")))
                                                             : 32768;
        return n;
    }
    // one rsa_extend over the jobs of several requests, results scattered back;
    // a failure is handed to every request of the batch
    void run_batch(ExtReq* const* reqs, size_t nr) {
        try {
            size_t n = 0, qtot = 0;
            for (size_t k = 0; k < nr; ++k) {
                n += reqs[k]->jobs->size();
                for (const auto& j : *reqs[k]->jobs) qtot += j.query.size();
            }
            const AlignmentParameters& p = *reqs[0]->p;
            const Lease ls = lease();
            Staging& sg = *ls.s;
            char* q = sg.get<char>(Staging::QUERIES, qtot + 16);
            rsa_job* js = sg.get<rsa_job>(Staging::JOBS, n);
            size_t pos = 0, i = 0;
            for (size_t k = 0; k < nr; ++k) {
                const std::vector<SwJob>& jobs = *reqs[k]->jobs;
                for (size_t t = 0; t < jobs.size(); ++t, ++i) {
                    if (t + 8 < jobs.size()) {
                        const char* a = jobs[t + 8].query.data();
                        for (size_t o = 0; o < jobs[t + 8].query.size(); o += 64) __builtin_prefetch(a + o);
                    }
                    js[i].query_offset = pos;
                    js[i].query_len = (uint32_t)jobs[t].query.size();
                    if (jobs[t].shared_k > 0)    // rescue_mate_part's pre-check on the device
                        js[i].query_len |= RSA_JOB_SHARED_CHECK | RSA_JOB_K(jobs[t].shared_k);
                    js[i].ref_id = jobs[t].ref_id;
                    js[i].ref_start = jobs[t].ref_start;
                    js[i].ref_len = jobs[t].ref_len;
                    memcpy(q + pos, jobs[t].query.data(), jobs[t].query.size());
                    pos += jobs[t].query.size();
                }
            }
            rsa_job_batch jb{q, qtot, js, (uint32_t)n, p.match, p.mismatch, p.gap_open, p.gap_extend, p.end_bonus};
            const uint64_t bound = rsa_extend_cigar_bound(&jb) + 1;
            rsa_aln* alns = sg.get<rsa_aln>(Staging::ALNS, n);
            uint32_t* pool = sg.get<uint32_t>(Staging::POOL, bound);
            rsa_aln_batch ab{alns, pool, bound, 0};
            int rc = rsa_extend(ctx_, &jb, &ab);
            if (rc != RSA_OK) throw std::runtime_error(std::string("rsa_extend: ") + rsa_last_error(ctx_));
            i = 0;
            for (size_t k = 0; k < nr; ++k) {
                std::vector<AlignmentInfo>& out = *reqs[k]->out;
                for (size_t t = 0; t < out.size(); ++t, ++i) {
                    const rsa_aln& a = alns[i];
                    AlignmentInfo& o = out[t];
                    o.sw_score = a.sw_score;
                    o.edit_distance = a.edit_distance;
                    o.ref_start = a.ref_start; o.ref_end = a.ref_end;
                    o.query_start = a.query_start; o.query_end = a.query_end;
                    o.no_shared = (a.flags & RSA_ALN_NO_SHARED) != 0;
                    o.cigar.ops.assign(pool + a.cigar_offset, pool + a.cigar_offset + a.cigar_len);
                }
            }
        } catch (...) {
            for (size_t k = 0; k < nr; ++k) reqs[k]->err = std::current_exception();
        }
    }
    std::mutex ext_m_;
    std::condition_variable ext_cv_;
    std::vector<ExtReq*> ext_pending_;
    int ext_active_ = 0;

    // staging sets are checked out per call (at most one per concurrent caller)
    struct Lease {
        GpuEngine* e;
        Staging* s;
        Lease(GpuEngine* e_, Staging* s_) : e(e_), s(s_) {}
        Lease(const Lease&) = delete;
        ~Lease() { std::lock_guard<std::mutex> g(e->staging_m_); e->free_.push_back(s); }
    };
    Lease lease() {
        std::lock_guard<std::mutex> g(staging_m_);
        if (free_.empty()) {
            staging_.emplace_back(new Staging());
            return Lease{this, staging_.back().get()};
        }
        Staging* s = free_.back();
        free_.pop_back();
        return Lease{this, s};
    }
    rsa_ctx* ctx_ = nullptr;
    std::mutex staging_m_;
    std::vector<std::unique_ptr<Staging>> staging_;
    std::mutex ap_m_;
    AlignmentParameters ap_;                    // hamming_align's scores (set_alignment_params)
    bool ap_set_ = false;
    std::vector<Staging*> free_;
};

}  // namespace

std::unique_ptr<Engine> make_gpu_engine(const References& refs, const StiIndex& index, int device) {
    return std::unique_ptr<Engine>(new GpuEngine(refs, index, device));
}

// StrobemerIndex::populate on the GPU (include/rsa_gpu.h rsa_index_build_run),
// downloaded into the host StiIndex (.sti writing, the host pipeline's
// parameters, a CPU engine opened on the same index)
void build_default_index(StiIndex& idx, const References& refs, const IndexParameters& p, int bits_override, float f,
                         int threads, int device, bool host_copy) {
    rsa_index_build_params bp{};
    bp.threads = threads;
    bp.k = p.k; bp.s = p.s; bp.t_syncmer = p.t;
    bp.w_min = (int)p.w_min; bp.w_max = (int)p.w_max; bp.max_dist = p.max_dist;
    bp.q = (uint64_t)p.q;
    bp.bits = bits_override;
    bp.f = f;
    rsa_index_build_info info{};
    char err[512] = {0};
    rsa_index_build* b = rsa_index_build_run(device, refs.concat.data(), refs.offsets.data(), (int)refs.size(), &bp,
                                             &info, err, sizeof err);
    if (!b) throw std::runtime_error(std::string("GPU index build: ") + err);
    idx.params = p;
    idx.bits = info.bits;
    idx.filter_cutoff = info.filter_cutoff;
    idx.randstrobes.clear();
    idx.bucket_starts.clear();
    idx.device_build.reset();
    idx.n_device = 0;
    if (host_copy) {
        idx.randstrobes.resize(info.n_randstrobes);
        idx.bucket_starts.resize((1ull << info.bits) + 1);
        const int rc = rsa_index_build_download(b, idx.randstrobes.data(), idx.bucket_starts.data());
        rsa_index_build_free(b);
        if (rc != RSA_OK) throw std::runtime_error("GPU index build: download failed");
    } else {
        idx.device_build = std::make_shared<StiIndex::DeviceBuild>();
        idx.device_build->handle = b;
        idx.device_build->release = [](void* h) { rsa_index_build_free((rsa_index_build*)h); };
        idx.n_device = info.n_randstrobes;
    }
    idx.built_on_device = true;
    const double ms[6] = {info.ms_upload, info.ms_syncmers, info.ms_randstrobes, info.ms_sort, info.ms_buckets,
                          info.ms_total};
    std::copy(ms, ms + 6, idx.device_build_ms);
    idx.replayed_segments = info.replayed_segments;
    idx.position_ties = info.position_ties;
    idx.ms_tie_replay = info.ms_tie_replay;
}

// engine of librsalign.so (capi.cpp)
std::unique_ptr<Engine> make_default_engine(const References& refs, const StiIndex& index, int device) {
    return make_gpu_engine(refs, index, device);
}

}  // namespace rsa
