// host_prof.cpp -- host-pipeline cost isolation (profiling tool, not product).
//
// Maps a synthetic paired-end workload once with the reference CPU engine while
// recording every engine result, then re-maps it with a replay engine that
// returns the recorded results (cost of a vector copy).  The replay runs time
// exactly the host side of the pipeline (load, part, get_str, store, last, SAM,
// digest) at any thread count, without a GPU; built with -pg it gives a gprof
// profile of that host work alone.
//
//   host_prof <ref_len> <n_contigs> <pairs> <replays> <threads...>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <map>
#include <mutex>
#include <thread>

#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>

#include "../rabbitsalign_amd/csrc/host/rsa_host.hpp"
#include "../rabbitsalign_amd/csrc/host/synth.hpp"

namespace rsa {
std::unique_ptr<Engine> make_default_engine(const References& refs, const StiIndex& idx, int device);
}

std::atomic<uint64_t> g_news{0};
bool g_count_news = false;

namespace {

using namespace rsa;

uint64_t jobs_key(const std::vector<SwJob>& jobs) {
    uint64_t h = 1469598103934665603ULL ^ jobs.size();
    for (const SwJob& j : jobs) {
        uint64_t q = 0;
        memcpy(&q, j.query.data(), std::min<size_t>(8, j.query.size()));
        for (uint64_t v : {(uint64_t)j.ref_id, (uint64_t)j.ref_start, (uint64_t)j.ref_len, (uint64_t)j.query.size(), q})
            h = (h ^ v) * 1099511628211ULL;
    }
    return h;
}

class Recorder final : public Engine {
public:
    Engine* inner = nullptr;
    bool replay = false;
    std::mutex m;
    std::map<uint64_t, SeedBatchOut> seeds;
    std::map<uint64_t, std::vector<AlignmentInfo>> exts;
    double seed_ms = 0, ext_ms = 0;   // replay: emulated device latency per call (the thread sleeps)
    const char* name() const override { return replay ? "replay" : "record"; }
#ifndef HP_OLD_HOST
    bool offloads() const override { return replay && (seed_ms > 0 || ext_ms > 0); }
#endif
    static void nap(double ms) {
        if (ms > 0) std::this_thread::sleep_for(std::chrono::microseconds((long)(ms * 1000)));
    }
    void seed(const std::vector<std::string_view>& reads, int rl, unsigned rc, SeedBatchOut& out) override {
        // keyed by content: the pipeline recycles its chunk buffers, so addresses repeat
        uint64_t key = 1469598103934665603ULL ^ reads.size();
        for (size_t i = 0; i < reads.size(); i += std::max<size_t>(1, reads.size() / 64))
            for (char ch : reads[i]) key = (key ^ (unsigned char)ch) * 1099511628211ULL;
        if (replay) {
            nap(seed_ms);
            std::lock_guard<std::mutex> g(m);
            out = seeds.at(key);
            return;
        }
        inner->seed(reads, rl, rc, out);
        std::lock_guard<std::mutex> g(m);
        seeds[key] = out;
    }
    void extend(const std::vector<SwJob>& jobs, const AlignmentParameters& p, std::vector<AlignmentInfo>& out) override {
        const uint64_t key = jobs_key(jobs);
        if (replay) {
            nap(ext_ms);
            std::lock_guard<std::mutex> g(m);
            out = exts.at(key);
            return;
        }
        inner->extend(jobs, p, out);
        std::lock_guard<std::mutex> g(m);
        exts[key] = out;
    }
};

// PC sampler (HP_SAMPLE=file): ITIMER_PROF every 200 us, the interrupted PC of
// whichever thread took the signal; the histogram is symbolised offline
// (addr2line -f -i -C) since gprof misattributes inlined/static code.
uint64_t* g_pcs = nullptr;
std::atomic<size_t> g_npc{0};
constexpr size_t kMaxPcs = 1 << 22;
void on_prof(int, siginfo_t*, void* uc) {
    const size_t i = g_npc.fetch_add(1, std::memory_order_relaxed);
    if (i < kMaxPcs) g_pcs[i] = (uint64_t)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RIP];
}
void start_sampler() {
    g_pcs = new uint64_t[kMaxPcs];
    struct sigaction sa {};
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigaction(SIGPROF, &sa, nullptr);
    itimerval tv{{0, 200}, {0, 200}};
    setitimer(ITIMER_PROF, &tv, nullptr);
}
void stop_sampler(const char* path) {
    itimerval tv{};
    setitimer(ITIMER_PROF, &tv, nullptr);
    FILE* f = fopen(path, "w");
    const size_t n = std::min(g_npc.load(), kMaxPcs);
    std::map<uint64_t, uint64_t> h;
    for (size_t i = 0; i < n; ++i) h[g_pcs[i]]++;
    for (auto& kv : h) fprintf(f, "%llx %llu\n", (unsigned long long)kv.first, (unsigned long long)kv.second);
    fclose(f);
}

}  // namespace

uint64_t g_callers[1 << 20];
void* operator new(size_t n) {
    if (g_count_news) {
        const uint64_t i = g_news.fetch_add(1, std::memory_order_relaxed);
        if (i < (1 << 20)) g_callers[i] = (uint64_t)__builtin_return_address(0);
    }
    void* p = malloc(n ? n : 1);
    if (!p) throw std::bad_alloc();
    return p;
}
void operator delete(void* p) noexcept { free(p); }
void operator delete(void* p, size_t) noexcept { free(p); }

int main(int argc, char** argv) {
    if (argc < 6) {
        fprintf(stderr, "host_prof <ref_len> <n_contigs> <pairs> <replays> <threads...>\n");
        return 2;
    }
    const uint64_t ref_len = strtoull(argv[1], nullptr, 10);
    const int nc = atoi(argv[2]);
    const uint64_t pairs = strtoull(argv[3], nullptr, 10);
    const int replays = atoi(argv[4]);
    const int L = 150;
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());

    References refs;
    refs.seqs = synth::reference(1, ref_len, nc, hw);
    for (int c = 0; c < nc; ++c) refs.names.push_back("chr" + std::to_string(c + 1));
    refs.offsets.assign(1, 0);
    for (auto& s : refs.seqs) { refs.concat += s; refs.offsets.push_back(refs.concat.size()); }
#ifndef HP_OLD_HOST
    if (!getenv("HP_NO_HOT")) refs.make_hot();
#endif
    StiIndex idx;
    idx.build(refs, IndexParameters::from_read_length(L), -1, 0.0002f, hw);
    AlignmentParameters ap;
    MappingParameters mp;
    mp.r = L;
    mp.rescue_cutoff = mp.rescue_level < 100 ? mp.rescue_level * idx.filter_cutoff : 1000;
    MapContext mc{refs, idx.params, ap, mp};

    std::vector<Record> r1(pairs), r2(pairs);
    const std::string qual(L, 'I');
    for (uint64_t p = 0; p < pairs; ++p) {
        synth::Pair pr = synth::pair(refs.seqs, 7, p, L, 300.0, 30.0);
        const std::string nm = "r" + std::to_string(p);
        r1[p] = Record{nm + "/1", "", pr.a, qual};
        r2[p] = Record{nm + "/2", "", pr.b, qual};
    }

    auto inner = make_default_engine(refs, idx, 0);
    Recorder rec;
    rec.inner = inner.get();
    PipelineOptions po;
    po.threads = hw;
    po.digest = true;
    PipelineResult base = run_pipeline_pe(r1, r2, rec, mc, po, nullptr, nullptr);
    printf("record: %.3f s, digest %016llx, %zu seed calls, %zu extend calls\n", base.map_seconds,
           (unsigned long long)base.sam_digest.h, rec.seeds.size(), rec.exts.size());
    rec.replay = true;
    if (getenv("HP_SEED_MS")) rec.seed_ms = atof(getenv("HP_SEED_MS"));
    if (getenv("HP_EXT_MS")) rec.ext_ms = atof(getenv("HP_EXT_MS"));
    const char* sample = getenv("HP_SAMPLE");
    if (sample) start_sampler();
    for (int a = 5; a < argc; ++a) {
        po.threads = atoi(argv[a]);
        for (int k = 0; k < replays; ++k) {
            g_news = 0;
            g_count_news = getenv("HP_NEWS") != nullptr;
            PipelineResult r = run_pipeline_pe(r1, r2, rec, mc, po, nullptr, nullptr);
            g_count_news = false;
            const double n = (double)r.stats.n_reads;
            printf("  operator new per read: %.2f\n", (double)g_news.load() / n);
            if (getenv("HP_NEWS")) {
                FILE* f = fopen(getenv("HP_NEWS"), "w");
                std::map<uint64_t, uint64_t> h;
                for (uint64_t i = 0; i < std::min<uint64_t>(g_news.load(), 1 << 20); ++i) h[g_callers[i]]++;
                for (auto& kv : h) fprintf(f, "%llx %llu\n", (unsigned long long)kv.first, (unsigned long long)kv.second);
                fclose(f);
            }
            printf("replay T=%d: wall %.3f s = %.3f Mreads/s | per Mread thread-s: part %.3f collect %.3f last %.3f "
                   "load %.3f output %.3f | seq %.3f s | digest %s\n",
                   po.threads, r.map_seconds, n / r.map_seconds / 1e6, r.phases.part / n * 1e6,
                   r.phases.collect / n * 1e6, r.phases.last / n * 1e6, r.phases.load / n * 1e6,
                   r.phases.output / n * 1e6, r.phases.sequential,
                   r.sam_digest.h == base.sam_digest.h ? "same" : "DIFFERENT");
        }
    }
    if (sample) stop_sampler(sample);
    return 0;
}
