// multi.cpp -- several engines (one per GPU) behind one Engine.
//
// The host pipeline keeps what makes the output independent of placement
// (SURVEY.md §8e): one chunk queue with the global chunk_index seeding
// minstd_rand (pc.cpp:1583, 1750), one insert-size estimate frozen in the
// sequential phase, one ordered writer (pc.cpp:119-135).  Seeding and
// extension calls are pure functions of their input, so each one can go to any
// device: it goes to the engine with the fewest calls in flight.  Every device
// holds a full replica of the index (no data-path collective).
#include <atomic>
#include <climits>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "rsa_host.hpp"

namespace rsa {

namespace {

void add_stats(rsa_kernel_stats& a, const rsa_kernel_stats& b) {
    for (int k = 0; k < RSA_K_COUNT; ++k) {
        a.kernel_ms[k] += b.kernel_ms[k];
        a.launches[k] += b.launches[k];
        a.alg_bytes[k] += b.alg_bytes[k];
    }
    uint64_t* au = &a.dp_cells_timed;
    const uint64_t* bu = &b.dp_cells_timed;
    const size_t nu = (size_t)(&a.scan_redo - &a.dp_cells_timed) + 1;  // dp_cells_timed .. scan_redo
    for (size_t i = 0; i < nu; ++i) au[i] += bu[i];
    for (int i = 0; i < 2; ++i) {
        a.call_ms[i] += b.call_ms[i];
        a.lane_wait_ms[i] += b.lane_wait_ms[i];
        a.device_wait_ms[i] += b.device_wait_ms[i];
    }
    a.query_written += b.query_written;
    a.query_fixed_reads += b.query_fixed_reads;
    a.shared_checks += b.shared_checks;
    a.no_shared += b.no_shared;
}

class MultiEngine final : public Engine {
public:
    explicit MultiEngine(std::vector<std::unique_ptr<Engine>> e)
        : e_(std::move(e)), inflight_(new std::atomic<int>[e_.size()]) {
        if (e_.empty()) throw std::runtime_error("no engines");
        for (size_t i = 0; i < e_.size(); ++i) inflight_[i] = 0;
        name_ = std::string(e_[0]->name()) + " x" + std::to_string(e_.size());
    }
    const char* name() const override { return name_.c_str(); }
    bool offloads() const override { return e_[0]->offloads(); }
    void seed(const std::vector<std::string_view>& reads, int rescue_level, unsigned rescue_cutoff,
              SeedBatchOut& out) override {
        Hold h(*this);
        e_[h.i]->seed(reads, rescue_level, rescue_cutoff, out);
    }
    void seed_packed(const char* blob, const uint64_t* offs, const uint32_t* lens, size_t n, int rescue_level,
                     unsigned rescue_cutoff, SeedBatchOut& out) override {
        Hold h(*this);
        e_[h.i]->seed_packed(blob, offs, lens, n, rescue_level, rescue_cutoff, out);
    }
    // every device's engine shares the process's page-locked allocator (or none): rsa_host_alloc
    // buffers are portable (hipHostMallocPortable), usable by any device's context
    const HostAllocFns* io_alloc() const override { return e_[0]->io_alloc(); }
    void extend(const std::vector<SwJob>& jobs, const AlignmentParameters& p,
                std::vector<AlignmentInfo>& out) override {
        Hold h(*this);
        e_[h.i]->extend(jobs, p, out);
    }
    bool kernel_stats(rsa_kernel_stats* out) override {
        memset(out, 0, sizeof *out);
        bool any = false;
        for (auto& e : e_) {
            rsa_kernel_stats s{};
            if (e->kernel_stats(&s)) { add_stats(*out, s); any = true; }
        }
        return any;
    }
    void reset_kernel_stats() override { for (auto& e : e_) e->reset_kernel_stats(); }
    bool download_index(StiIndex& idx) override { return e_[0]->download_index(idx); }
    void set_alignment_params(const AlignmentParameters& p) override {
        for (auto& e : e_) e->set_alignment_params(p);
    }

private:
    struct Hold {                       // the least busy engine, counted busy for the call
        MultiEngine& m;
        size_t i = 0;
        explicit Hold(MultiEngine& m_) : m(m_) {
            int best = INT_MAX;
            for (size_t k = 0; k < m.e_.size(); ++k) {
                const int v = m.inflight_[k].load(std::memory_order_relaxed);
                if (v < best) { best = v; i = k; }
            }
            m.inflight_[i].fetch_add(1);
        }
        ~Hold() { m.inflight_[i].fetch_sub(1); }
    };
    std::vector<std::unique_ptr<Engine>> e_;
    std::unique_ptr<std::atomic<int>[]> inflight_;
    std::string name_;
};

}  // namespace

std::unique_ptr<Engine> make_multi_engine(std::vector<std::unique_ptr<Engine>> engines) {
    if (engines.size() == 1) return std::move(engines[0]);
    return std::unique_ptr<Engine>(new MultiEngine(std::move(engines)));
}

std::unique_ptr<Engine> open_engines(EngineFactory factory, const References& refs, StiIndex& idx,
                                     const std::vector<int>& devices) {
    if (devices.empty()) throw std::runtime_error("no device given");
    std::vector<std::unique_ptr<Engine>> engines;
    engines.push_back(factory(refs, idx, devices[0]));
    if (devices.size() > 1) {
        // an index that lives only in the first device's HBM (GPU build, adopted by
        // its engine) comes to the host once; every other device uploads that copy
        if (!idx.host_copy() && !engines[0]->download_index(idx))
            throw std::runtime_error("multi-device: the index could not be copied to the host");
        std::vector<std::unique_ptr<Engine>> more(devices.size());
        std::vector<std::exception_ptr> errs(devices.size());
        std::vector<std::thread> ts;
        for (size_t i = 1; i < devices.size(); ++i)
            ts.emplace_back([&, i]() {
                try { more[i] = factory(refs, idx, devices[i]); } catch (...) { errs[i] = std::current_exception(); }
            });
        for (auto& t : ts) t.join();
        for (auto& e : errs) if (e) std::rethrow_exception(e);
        for (size_t i = 1; i < devices.size(); ++i) engines.push_back(std::move(more[i]));
    }
    return make_multi_engine(std::move(engines));
}

std::vector<int> parse_devices(const std::string& s) {
    std::vector<int> d;
    size_t a = 0;
    while (a <= s.size()) {
        const size_t b = s.find(',', a);
        const std::string t = s.substr(a, b == std::string::npos ? std::string::npos : b - a);
        if (t.empty()) throw std::runtime_error("bad device list '" + s + "'");
        size_t used = 0;
        const int v = std::stoi(t, &used);
        if (used != t.size() || v < 0) throw std::runtime_error("bad device list '" + s + "'");
        d.push_back(v);
        if (b == std::string::npos) break;
        a = b + 1;
    }
    return d;
}

}  // namespace rsa
