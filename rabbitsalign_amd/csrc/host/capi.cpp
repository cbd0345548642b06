// capi.cpp -- include/rsalign.h: the mapping path as a C library.
#include <atomic>
#include <chrono>
#include <map>

#include <dlfcn.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include "../../../include/rsalign.h"
#include "rsa_host.hpp"
#include "synth.hpp"

namespace rsa {
// provided by the engine translation unit linked into the library
std::unique_ptr<Engine> make_default_engine(const References& refs, const StiIndex& idx, int device);
}

using namespace rsa;

static thread_local std::string g_err;

// Host PC sampler for profiling the mapping on the GPU box (RSA_PC_SAMPLE=file):
// during rsam_map every pipeline worker (g_worker_start_hook) gets a timer on its
// own CPU clock firing every 500 us of CPU; the handler records the interrupted PC.
// Output: "pc count" lines and the process's executable mappings ("#map"), so
// scripts/pc_report.py can attribute and symbolise them offline.  Instrumentation only.
namespace {
constexpr size_t kMaxPcs = 1 << 22;
uint64_t* g_pcs = nullptr;
uint64_t* g_ras = nullptr;     // the word at the interrupted stack pointer: a leaf's return address
std::atomic<size_t> g_npc{0};
std::mutex g_tid_m;
void on_prof(int, siginfo_t*, void* uc) {
    const size_t i = g_npc.fetch_add(1, std::memory_order_relaxed);
    if (i >= kMaxPcs) return;
    const greg_t* r = ((ucontext_t*)uc)->uc_mcontext.gregs;
    g_pcs[i] = (uint64_t)r[REG_RIP];
    g_ras[i] = *(const uint64_t*)r[REG_RSP];
}
std::vector<timer_t> g_timers;
// a CPU-time timer per worker (CLOCK_THREAD_CPUTIME_ID, signal to that thread):
// samples land only where the worker spends CPU, blocked waits never show up
void register_worker() {
    sigevent sev{};
    sev.sigev_notify = SIGEV_THREAD_ID;
    sev.sigev_signo = SIGPROF;
    sev._sigev_un._tid = (pid_t)syscall(SYS_gettid);
    timer_t t;
    if (timer_create(CLOCK_THREAD_CPUTIME_ID, &sev, &t) != 0) return;
    itimerspec its{{0, 500000}, {0, 500000}};
    timer_settime(t, 0, &its, nullptr);
    std::lock_guard<std::mutex> g(g_tid_m);
    g_timers.push_back(t);
}
struct PcSampler {
    const char* path = getenv("RSA_PC_SAMPLE");
    PcSampler() {
        if (!path) return;
        if (!g_pcs) g_pcs = new uint64_t[kMaxPcs];
        if (!g_ras) g_ras = new uint64_t[kMaxPcs];
        g_npc = 0;
        struct sigaction sa{};
        sa.sa_sigaction = on_prof;
        sa.sa_flags = SA_SIGINFO | SA_RESTART;
        sigaction(SIGPROF, &sa, nullptr);
        rsa::g_worker_start_hook = register_worker;
    }
    ~PcSampler() {
        if (!path) return;
        rsa::g_worker_start_hook = nullptr;
        {
            std::lock_guard<std::mutex> g(g_tid_m);
            for (timer_t t : g_timers) timer_delete(t);
            g_timers.clear();
        }
        Dl_info di{};
        dladdr((void*)&on_prof, &di);
        const uint64_t base = (uint64_t)di.dli_fbase;
        std::map<uint64_t, uint64_t> h;
        const size_t n = std::min(kMaxPcs, g_npc.load());
        for (size_t i = 0; i < n; ++i) h[g_pcs[i]]++;
        FILE* f = fopen(path, "a");
        if (!f) return;
        fprintf(f, "# base %lx lib %s samples %zu\n", (unsigned long)base, di.dli_fname ? di.dli_fname : "?", n);
        for (auto& kv : h) fprintf(f, "%lx %lu\n", (unsigned long)kv.first, (unsigned long)kv.second);
        std::map<std::pair<uint64_t, uint64_t>, uint64_t> hr;
        for (size_t i = 0; i < n; ++i) hr[{g_pcs[i], g_ras[i]}]++;
        for (auto& kv : hr)
            fprintf(f, "#ra %lx %lx %lu\n", (unsigned long)kv.first.first, (unsigned long)kv.first.second,
                    (unsigned long)kv.second);
        if (FILE* mp = fopen("/proc/self/maps", "r")) {      // to attribute PCs to libraries offline
            char line[1024];
            while (fgets(line, sizeof line, mp))
                if (strstr(line, " r-xp ") || strstr(line, " r--p ")) fprintf(f, "#map %s", line);
            fclose(mp);
        }
        fclose(f);
    }
};
}  // namespace

struct rsam {
    References refs;
    StiIndex idx;
    std::unique_ptr<Engine> eng;
    AlignmentParameters ap;
    MappingParameters mp;
    double index_seconds = 0, upload_seconds = 0;
    int read_len = 150;
    bool digest = true;                // rsam_set_sam_digest
};

struct rsam_reads {
    std::vector<Record> r1, r2;
    bool paired = false;
    std::vector<Record> interleaved;   // rsam_reads_load_interleaved: paired up per chunk size in rsam_map
};

static void finish_refs(References& r) {
    r.offsets.assign(1, 0);
    size_t tot = 0;
    for (auto& s : r.seqs) { tot += s.size(); r.offsets.push_back(tot); }
    r.concat.clear();
    r.concat.reserve(tot);
    for (auto& s : r.seqs) r.concat += s;
    r.make_hot();
}

static void setup_params(rsam* m) {
    m->mp.r = m->read_len;
    m->mp.rescue_cutoff = m->mp.rescue_level < 100 ? m->mp.rescue_level * m->idx.filter_cutoff : 1000;
}

// Open mappers of the process.  When the last one closes, the pipeline's pooled
// threads are joined and its pooled (page-locked) buffers freed while that
// mapper's engine is still open: nothing of the library then runs or stays
// allocated, so the process can unload it or exit without a destructor touching
// a torn-down HIP runtime.
static std::mutex g_open_m;
static int g_open = 0;

static rsam* open_common(rsam* m, int device, char* err, size_t err_len) {
    try {
        setup_params(m);
        auto t = std::chrono::steady_clock::now();
        m->eng = make_default_engine(m->refs, m->idx, device);
        {
            std::lock_guard<std::mutex> g(g_open_m);
            ++g_open;
        }
        m->upload_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
        return m;
    } catch (const std::exception& e) {
        if (err && err_len) snprintf(err, err_len, "%s", e.what());
        g_err = e.what();
        delete m;
        return nullptr;
    }
}

extern "C" {

rsam* rsam_open_files(const char* ref_fa, const char* sti, int read_len, int device, int threads, char* err,
                      size_t err_len) {
    tune_malloc();
    rsam* m = new rsam();
    try {
        m->read_len = read_len;
        m->refs = References::from_fasta(ref_fa);
        auto t = std::chrono::steady_clock::now();
        IndexParameters ip = IndexParameters::from_read_length(read_len);
        if (sti && *sti) {
            m->idx.read(sti);
            if (!(m->idx.params == ip)) throw std::runtime_error("index parameters differ from the read length profile");
        } else {
            build_default_index(m->idx, m->refs, ip, -1, 0.0002f, std::max(1, threads), device, false);
        }
        m->index_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
    } catch (const std::exception& e) {
        if (err && err_len) snprintf(err, err_len, "%s", e.what());
        g_err = e.what();
        delete m;
        return nullptr;
    }
    return open_common(m, device, err, err_len);
}

rsam* rsam_open_synthetic(uint64_t seed, uint64_t ref_len, int n_contigs, int read_len, int device, int threads,
                          char* err, size_t err_len) {
    tune_malloc();
    rsam* m = new rsam();
    try {
        m->read_len = read_len;
        m->refs.seqs = synth::reference(seed, ref_len, n_contigs, std::max(1, threads));
        if (const char* dup = getenv("RSA_SYNTH_DUP")) {
            // a PAR-like duplicated region (measurement of the index build's tie path)
            const uint64_t len = strtoull(dup, nullptr, 10), at = 1u << 20;
            if (len && n_contigs > 1 && m->refs.seqs[0].size() >= at + len && m->refs.seqs[1].size() >= at + len)
                m->refs.seqs[1].replace(at, len, m->refs.seqs[0], at, len);
        }
        for (int c = 0; c < n_contigs; ++c) m->refs.names.push_back("chr" + std::to_string(c + 1));
        finish_refs(m->refs);
        auto t = std::chrono::steady_clock::now();
        build_default_index(m->idx, m->refs, IndexParameters::from_read_length(read_len), -1, 0.0002f,
                            std::max(1, threads), device, false);
        m->index_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
    } catch (const std::exception& e) {
        if (err && err_len) snprintf(err, err_len, "%s", e.what());
        g_err = e.what();
        delete m;
        return nullptr;
    }
    return open_common(m, device, err, err_len);
}

rsam* rsam_open_like(const rsam* o, int device, int threads, char* err, size_t err_len) {
    tune_malloc();
    (void)threads;
    rsam* m = new rsam();
    m->read_len = o->read_len;
    m->refs = o->refs;
    // an index that lives only in the other mapper's HBM comes to the host first
    if (!o->idx.host_copy() && !(o->eng && o->eng->download_index(const_cast<StiIndex&>(o->idx)))) {
        g_err = "rsam_open_like: the index has no host copy";
        if (err && err_len) snprintf(err, err_len, "%s", g_err.c_str());
        delete m;
        return nullptr;
    }
    m->idx = o->idx;
    m->index_seconds = o->index_seconds;
    return open_common(m, device, err, err_len);
}

void rsam_close(rsam* m) {
    if (!m) return;
    bool last = false;
    {
        std::lock_guard<std::mutex> g(g_open_m);
        last = --g_open == 0;
    }
    if (last) release_pipeline_resources();
    delete m;
}

int rsam_get_info(const rsam* m, rsam_info* out) {
    if (!m || !out) return -1;
    out->ref_bases = m->refs.concat.size();
    out->n_randstrobes = m->idx.size();
    out->n_contigs = (int32_t)m->refs.size();
    out->bits = m->idx.bits;
    out->filter_cutoff = m->idx.filter_cutoff;
    out->k = m->idx.params.k;
    out->canonical_read_length = m->idx.params.canonical_read_length;
    out->index_seconds = m->index_seconds;
    out->upload_seconds = m->upload_seconds;
    out->device_resident_bytes = m->refs.concat.size() + m->idx.size() * sizeof(rsa_ref_randstrobe) +
                                 (((size_t)1 << m->idx.bits) + 1) * 8;
    out->index_on_device = m->idx.built_on_device ? 1 : 0;
    out->pad_ = 0;
    for (int i = 0; i < 6; ++i) out->index_device_ms[i] = m->idx.device_build_ms[i];
    out->index_replayed_segments = m->idx.replayed_segments;
    out->index_position_ties = m->idx.position_ties;
    out->index_ms_tie_replay = m->idx.ms_tie_replay;
    return 0;
}

rsam_reads* rsam_reads_load(const char* fq1, const char* fq2) {
    tune_malloc();
    try {
        std::unique_ptr<rsam_reads> r(new rsam_reads());
        if (fq2 && *fq2) {
            FastxReader::read_pair(fq1, fq2, r->r1, r->r2);
            r->paired = true;
            if (r->r1.size() != r->r2.size()) throw std::runtime_error("read files have different record counts");
        } else {
            r->r1 = FastxReader::read_all(fq1);
        }
        return r.release();
    } catch (const std::exception& e) {
        g_err = e.what();
        return nullptr;
    }
}

rsam_reads* rsam_reads_load_interleaved(const char* fq) {
    tune_malloc();
    try {
        std::unique_ptr<rsam_reads> r(new rsam_reads());
        r->interleaved = FastxReader::read_all(fq);
        r->paired = true;
        return r.release();
    } catch (const std::exception& e) {
        g_err = e.what();
        return nullptr;
    }
}

rsam_reads* rsam_reads_synthetic(const rsam* m, uint64_t seed, uint64_t first, uint64_t n, int read_len, double mu,
                                 double sigma, int paired) {
    tune_malloc();
    auto* r = new rsam_reads();
    r->paired = paired != 0;
    r->r1.resize(n);
    if (paired) r->r2.resize(n);
    const std::string qual((size_t)read_len, 'I');
    const int T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> ws;
    for (int t = 0; t < T; ++t)
        ws.emplace_back([&, t]() {
            for (uint64_t i = (uint64_t)t; i < n; i += (uint64_t)T) {
                const uint64_t p = first + i;
                synth::Pair pr = synth::pair(m->refs.seqs, seed, p, read_len, mu, sigma);
                const std::string nm = "r" + std::to_string(p);
                r->r1[i] = Record{paired ? nm + "/1" : nm, "", pr.a, qual};
                if (paired) r->r2[i] = Record{nm + "/2", "", pr.b, qual};
            }
        });
    for (auto& w : ws) w.join();
    return r;
}

int rsam_reads_write_fastq(const rsam_reads* r, const char* fq1, const char* fq2) {
    if (!r || !fq1) return -1;
    auto write = [](const std::vector<Record>& v, const char* path) -> bool {
        FILE* f = fopen(path, "wb");
        if (!f) return false;
        std::string buf;
        buf.reserve(1 << 22);
        for (const Record& x : v) {
            buf += '@'; buf += x.name;
            if (!x.comment.empty()) { buf += ' '; buf += x.comment; }
            buf += '\n'; buf += x.seq; buf += "\n+\n"; buf += x.qual; buf += '\n';
            if (buf.size() > (1 << 22)) { fwrite(buf.data(), 1, buf.size(), f); buf.clear(); }
        }
        fwrite(buf.data(), 1, buf.size(), f);
        return fclose(f) == 0;
    };
    if (!write(r->r1, fq1)) { g_err = std::string("cannot write ") + fq1; return -1; }
    if (r->paired && fq2 && !write(r->r2, fq2)) { g_err = std::string("cannot write ") + fq2; return -1; }
    return 0;
}

uint64_t rsam_reads_count(const rsam_reads* r) {
    return r ? r->r1.size() + r->r2.size() + r->interleaved.size() : 0;
}
void rsam_reads_free(rsam_reads* r) { delete r; }

struct SinkState {
    FILE* f = nullptr;
    ~SinkState() { if (f) fclose(f); }   // an error path; the normal one closes and checks
};

static void sink_fn(void* user, const char* chunk, size_t bytes) {
    auto* s = (SinkState*)user;
    if (s->f) fwrite(chunk, 1, bytes, s->f);
}

static void fill_stats(const PipelineResult& res, rsam_stats* out) {
    if (!out) return;
    out->n_reads = res.stats.n_reads;
    out->sam_bytes = res.sam_bytes;
    out->sam_hash = res.sam_digest.h;
    out->sw_calls = res.stats.tot_aligner_calls;
    out->tried = res.stats.tot_all_tried;
    out->nam_rescue = res.stats.nam_rescue;
    out->mate_rescue = res.stats.tot_rescued;
    out->inconsistent = res.stats.inconsistent_nams;
    out->map_seconds = res.map_seconds;
    out->t_seed = res.phases.seed;
    out->t_extend = res.phases.extend;
    out->t_part = res.phases.part;
    out->t_collect = res.phases.collect;
    out->t_last = res.phases.last;
    out->t_sequential = res.phases.sequential;
    out->t_first_seeded = res.phases.first_seeded;
    out->t_last_start = res.phases.last_start;
    out->t_last_put = res.phases.last_put;
    out->t_workers_done = res.phases.workers_done;
    out->t_first_out = res.phases.first_out;
    out->t_first_ext_begin = res.phases.first_ext_begin;
    out->t_first_ext_end = res.phases.first_ext_end;
    out->replayed_chunks = res.phases.replayed;
}

// the pipeline over `src` with the SAM (header + body) to sam_path, or kept in memory
// only when sam_path is empty; map_seconds covers opening the output to the last byte
// `first_chunk` / `header`: a rank's part (rsam_map_files_part)
static int map_source(rsam* m, ReadSource& src, int threads, int chunk_size, const char* sam_path, rsam_stats* out,
                      std::chrono::steady_clock::time_point t0, size_t first_chunk = 0, bool header = true,
                      size_t end_chunk = SIZE_MAX) {
    PcSampler sampler;
    SinkState st;
    if (sam_path && *sam_path) {
        st.f = fopen(sam_path, "wb");
        if (!st.f) throw std::runtime_error(std::string("cannot open ") + sam_path);
        if (header) {
            std::string hdr = sam_header(m->refs, "", {}, "rsalign (library)");
            fwrite(hdr.data(), 1, hdr.size(), st.f);
        }
    }
    MapContext mc{m->refs, m->idx.params, m->ap, m->mp};
    PipelineOptions po;
    po.threads = threads;
    po.chunk_size = chunk_size;
    po.digest = m->digest;
    po.first_chunk = first_chunk;
    po.end_chunk = end_chunk;
    SamSink sk = st.f ? sink_fn : nullptr;
    PipelineResult res = src.paired() ? run_pipeline_pe(src, *m->eng, mc, po, sk, &st)
                                      : run_pipeline_se(src, *m->eng, mc, po, sk, &st);
    if (st.f) {
        FILE* f = st.f;
        st.f = nullptr;
        const bool bad = ferror(f) != 0;
        if (fclose(f) != 0 || bad) throw std::runtime_error(std::string("write failed: ") + sam_path);
    }
    res.map_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    fill_stats(res, out);
    return 0;
}

int rsam_map(rsam* m, const rsam_reads* reads, int threads, int chunk_size, const char* sam_path, rsam_stats* out) {
    tune_malloc();
    if (!m || !reads) return -1;
    try {
        const auto t0 = std::chrono::steady_clock::now();
        const size_t chunk = (size_t)std::max(1, chunk_size);
        // views into the read set: interleaved records are paired per chunk of
        // 2 x chunk_size records (pc.cpp:38-107) as each chunk is taken, no copy
        std::unique_ptr<ReadSource> src =
            !reads->interleaved.empty() ? make_interleaved_vector_source(&reads->interleaved, chunk)
                                        : make_vector_source(&reads->r1, reads->paired ? &reads->r2 : nullptr, chunk);
        return map_source(m, *src, threads, chunk_size, sam_path, out, t0);
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

int rsam_map_files(rsam* m, const char* fq1, const char* fq2, int interleaved, int threads, int chunk_size,
                   const char* sam_path, rsam_stats* out) {
    tune_malloc();
    if (!m || !fq1) return -1;
    try {
        const auto t0 = std::chrono::steady_clock::now();
        std::unique_ptr<ReadSource> src = open_fastq_source(fq1, fq2 ? fq2 : "", interleaved != 0,
                                                            (size_t)std::max(1, chunk_size));
        return map_source(m, *src, threads, chunk_size, sam_path, out, t0);
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

static void to_c(const PartPlan& p, rsam_part* o) {
    o->rank = p.rank;
    o->world = p.world;
    o->chunk_size = p.chunk_size;
    o->total_pairs = p.total_records;
    o->n_chunks = p.n_chunks;
    o->first_chunk = p.first_chunk;
    o->end_chunk = p.end_chunk;
    o->first_pair = p.first_record;
    o->n_pairs = p.n_records;
    o->offset1 = p.offset1;
    o->offset2 = p.offset2;
    o->flags = (p.by_record1 ? RSAM_PART_RECORDS1 : 0u) | (p.by_record2 ? RSAM_PART_RECORDS2 : 0u);
    o->reserved = 0;
}

static PartPlan from_c(const rsam_part& o) {
    PartPlan p;
    p.rank = o.rank;
    p.world = o.world;
    p.chunk_size = o.chunk_size;
    p.total_records = o.total_pairs;
    p.n_chunks = o.n_chunks;
    p.first_chunk = o.first_chunk;
    p.end_chunk = o.end_chunk;
    p.first_record = o.first_pair;
    p.n_records = o.n_pairs;
    p.offset1 = o.offset1;
    p.offset2 = o.offset2;
    p.by_record1 = (o.flags & RSAM_PART_RECORDS1) != 0;
    p.by_record2 = (o.flags & RSAM_PART_RECORDS2) != 0;
    return p;
}

int rsam_part_count(const char* path, int rank, int world, int threads, uint64_t* counts) {
    if (!path || !counts) return -1;
    try {
        const std::vector<uint64_t> c = count_part_lines(path, rank, world, threads);
        std::copy(c.begin(), c.end(), counts);
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

int rsam_part_plan(const char* fq1, const char* fq2, int rank, int world, int chunk_size, const uint64_t* counts1,
                   const uint64_t* counts2, int threads, rsam_part* out) {
    if (!fq1 || !out) return -1;
    try {
        const size_t nb = (size_t)std::max(0, world) * RSAM_PART_BLOCKS;
        const bool se = !fq2 || !*fq2;
        std::vector<uint64_t> c1, c2;
        if (counts1) c1.assign(counts1, counts1 + nb);
        if (counts2 && !se) c2.assign(counts2, counts2 + nb);
        to_c(plan_part(fq1, se ? "" : fq2, rank, world, (size_t)std::max(1, chunk_size), c1, c2, threads), out);
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

int rsam_map_files_part(rsam* m, const char* fq1, const char* fq2, const rsam_part* part, int threads,
                        const char* sam_path, rsam_stats* out) {
    tune_malloc();
    if (!m || !fq1 || !part) return -1;
    try {
        const auto t0 = std::chrono::steady_clock::now();
        const PartPlan pl = from_c(*part);
        validate_part(fq1, fq2 ? fq2 : "", pl);     // a stale or hand-built part maps nothing
        const bool header = pl.rank == 0;
        if (pl.n_records == 0) {              // more ranks than chunks: an empty part
            rsam_reads empty;
            auto src = make_vector_source(&empty.r1, (fq2 && *fq2) ? &empty.r2 : nullptr, 1);
            return map_source(m, *src, threads, (int)pl.chunk_size, sam_path, out, t0, 0, header);
        }
        std::unique_ptr<ReadSource> src = open_fastq_part_source(fq1, fq2 ? fq2 : "", pl);
        return map_source(m, *src, threads, (int)pl.chunk_size, sam_path, out, t0, (size_t)pl.first_chunk, header,
                          (size_t)pl.end_chunk);
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

int rsam_set_sam_digest(rsam* m, int on) {
    if (!m) return -1;
    m->digest = on != 0;
    return 0;
}

int rsam_add_devices(rsam* m, const int* devices, int n) {
    if (!m || !m->eng || n < 0 || (n > 0 && !devices)) return -1;
    try {
        if (n == 0) return 0;
        // a device-only index comes to the host once; every added device uploads it
        if (!m->idx.host_copy() && !m->eng->download_index(m->idx))
            throw std::runtime_error("rsam_add_devices: the index could not be copied to the host");
        std::vector<std::unique_ptr<Engine>> more((size_t)n);
        std::vector<std::exception_ptr> errs((size_t)n);
        std::vector<std::thread> ts;
        for (int i = 0; i < n; ++i)
            ts.emplace_back([&, i]() {
                try { more[i] = make_default_engine(m->refs, m->idx, devices[i]); }
                catch (...) { errs[i] = std::current_exception(); }
            });
        for (auto& t : ts) t.join();
        for (auto& e : errs) if (e) std::rethrow_exception(e);
        std::vector<std::unique_ptr<Engine>> all;
        all.push_back(std::move(m->eng));
        for (auto& e : more) all.push_back(std::move(e));
        m->eng = make_multi_engine(std::move(all));
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

int rsam_kernel_stats(rsam* m, rsa_kernel_stats* out) {
    if (!m || !out) return -1;
    memset(out, 0, sizeof *out);
    return m->eng->kernel_stats(out) ? 0 : 1;
}

void rsam_reset_kernel_stats(rsam* m) { if (m) m->eng->reset_kernel_stats(); }

const char* rsam_engine_name(const rsam* m) { return m ? m->eng->name() : ""; }

const char* rsam_last_error(void) { return g_err.c_str(); }

}  // extern "C"
