// pipeline.cpp -- chunk pipeline with the reference's single-worker semantics.
//
// The reference (src/pc.cpp:1522-1887, perform_task_async_pe) interleaves per
// worker: part(N-1) ... get_str(N-1) | part(N) | SW(N-1) | store(N-1), last(N-1).
// Two pieces of state make results depend on that order:
//  * the insert-size estimate (updated inside part() until 400 samples), read by
//    get_str/store/last at different times (pc.cpp:1620, 1798, 1861);
//  * minstd_rand seeded with the chunk index (pc.cpp:1583, 1750), consumed by
//    part() (shuffle_top_nams) and then by last() (pick_random_top_pair).
// We replay the exact single-worker timeline until the estimate is frozen; from
// then on chunks are independent and run in parallel on the host workers, each
// calling the GPU engine (seeding + extension) for its own chunk.
#include <sys/mman.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <cstring>
#include <deque>
#include <map>
#include <set>
#include <mutex>
#include <stdexcept>
#include <thread>

#include <malloc.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "rsa_host.hpp"

namespace rsa {

void (*g_worker_start_hook)() = nullptr;

namespace {

using Clock = std::chrono::steady_clock;
inline double since(Clock::time_point t) { return std::chrono::duration<double>(Clock::now() - t).count(); }

// CPU slots: at most `threads` workers compute at once.  With an offloading
// engine the pipeline runs extra workers, and a worker gives its slot back
// while it sleeps on the GPU (or on another chunk), so the host cores stay busy
// while seeding/extension run on the device.  A freed slot goes to the waiting
// worker with the lowest chunk index: the SAM writer takes chunks in order, so
// the oldest chunk in flight is the one it may be waiting for, while the newest
// are only being seeded ahead (RSA_SLOT_ORDER=0: first come, first served).
struct CpuSlots {
    static constexpr uint64_t kIdle = UINT64_MAX;   // a worker with no chunk yet
    std::mutex m;
    int free = 0;
    struct Waiter {
        uint64_t prio, seq;
        std::condition_variable cv;
        bool granted = false;
    };
    struct ByPrio {
        bool operator()(const Waiter* a, const Waiter* b) const {
            return a->prio != b->prio ? a->prio < b->prio : a->seq < b->seq;
        }
    };
    std::set<Waiter*, ByPrio> waiters;
    uint64_t seq = 0;
    static bool ordered() {
        static const bool on = !(getenv("RSA_SLOT_ORDER") && getenv("RSA_SLOT_ORDER")[0] == '0');
        return on;
    }
    void acquire(uint64_t prio = kIdle) {
        std::unique_lock<std::mutex> g(m);
        if (free > 0 && waiters.empty()) { --free; return; }
        Waiter w;
        w.prio = ordered() ? prio : 0;
        w.seq = seq++;
        waiters.insert(&w);
        w.cv.wait(g, [&] { return w.granted; });       // release() handed its slot over
    }
    void release() {
        std::lock_guard<std::mutex> g(m);
        if (waiters.empty()) { ++free; return; }
        Waiter* w = *waiters.begin();
        waiters.erase(waiters.begin());
        w->granted = true;
        w->cv.notify_one();                              // under the lock: w lives on its waiter's stack
    }
};
struct SlotHold {                 // a slot for the lifetime of a worker
    CpuSlots& s;
    explicit SlotHold(CpuSlots& s_) : s(s_) { s.acquire(); }
    ~SlotHold() { s.release(); }
};
struct Unslot {                   // the slot handed back for a blocking section (chunk `prio` waits)
    CpuSlots& s;
    bool on;
    uint64_t prio;
    Unslot(CpuSlots& s_, bool on_, uint64_t prio_ = CpuSlots::kIdle) : s(s_), on(on_), prio(prio_) {
        if (on) s.release();
    }
    ~Unslot() { if (on) s.acquire(prio); }
};

// extra workers beyond the compute slots (RSA_WAIT_WORKERS; default: three
// quarters as many as the slots when the engine offloads -- A/B on 16 cores:
// +0 9.0/8.8, +8 9.4, +16 8.3 Mreads/s; on the r26 code +4 14.4/14.8, +8
// 15.7/15.5, +12 15.8/16.3; r27: +12 17.2/17.6, +16 15.9/16.1, +20 15.9/15.7
// -- none for an engine computing in-thread)

static int wait_workers(const Engine& eng, int threads, bool has_sink) {
    const char* e = getenv("RSA_WAIT_WORKERS");
    if (e) return std::max(0, atoi(e));
    // 3/4 of the threads (12 of 16) for an in-memory run; 3/8 (6 of 16) when the SAM goes
    // to a sink, whose writer and readers need the cores the parked workers take when they
    // wake.  Round 5, alternating runs on two boxes (profiles/r05/wait_workers_ab.txt):
    // PE 2x150 streamed 21.35/22.00/21.42/21.15 with 6 against 19.77/20.04/21.18/20.10 with
    // 12, 0.46-0.54 against 0.50-0.59 core-us a read; PE 2x250 streamed 11.74/12.30 against
    // 11.25/11.80.  In memory 12 stays ahead (24.1 against 23.2 mean).
    if (!eng.offloads()) return 0;
    return has_sink ? (3 * threads) / 8 : (3 * threads) / 4;
}

// Chunks' SAM text in chunk order (OutputBuffer::output_records, pc.cpp:119-135).
// One writer thread of its own hands the text to the sink, so no worker blocks on
// the output file behind other chunks and nobody contends for it: the page-cache
// writes of one file are serialised by the kernel anyway (the inode lock), and
// parallel pwrite()s only spun on that lock.  Workers wait only when
// more than kMaxQueued bytes are waiting for the writer.

struct OrderedSink {
    SamSink sink;
    void* user;
    bool digest = false;
    static constexpr size_t kMaxQueued = 768u << 20;
    std::mutex m;
    std::condition_variable cv, room_cv;
    // a chunk's text may come in pieces (PeChunk SAM pieces, pe_store_last): the
    // writer takes the pieces of the next chunk in order as they come, so it can
    // start on a chunk while the rest of it is still being formatted
    struct Entry {
        std::deque<std::pair<SamText, SamDigest>> pieces;
        bool done = false;                    // its last piece is in
    };
    std::map<size_t, Entry> pending;
    std::deque<SamText> queue;                // in chunk order, for the writer
    size_t queued_bytes = 0;
    double first_out = 0;                     // s after opening: the first text reached the writer
    size_t next = 0;
    const size_t first;                       // the first chunk this sink writes
    uint64_t bytes = 0;
    SamDigest total;
    bool closing = false;
    std::thread writer;
    // RSA_SINK_TRACE=<file>: one line a write (instrumentation): seconds since the sink opened
    // at the call and at the return, bytes, bytes still queued, W
    FILE* trace = nullptr;
    Clock::time_point t_open = Clock::now();
    // `first`: the first chunk index this sink writes (a rank's part starts later)
    OrderedSink(SamSink s, void* u, bool d, size_t first_ = 0)
        : sink(s), user(u), digest(d), next(first_), first(first_) {
        static const char* trace_path = getenv("RSA_SINK_TRACE");
        if (sink && trace_path) trace = fopen(trace_path, "a");
        if (sink) writer = std::thread([this] { write_loop(); });
    }
    ~OrderedSink() {
        close();
        if (trace) fclose(trace);
    }
    // every chunk written (the writer drained and stopped)
    void close() {
        {
            std::lock_guard<std::mutex> g(m);
            closing = true;
        }
        cv.notify_all();
        if (writer.joinable()) writer.join();
    }
    // written chunks' buffers, kept at capacity for the next chunks (and the next
    // mapping calls): a fresh ~10 MB buffer per chunk is memory the first write
    // page-faults in
    struct Spares {
        std::mutex m;
        std::vector<SamText> v;
    };
    static Spares& spares() {
        static Spares* p = new Spares();     // never destroyed: no exit-time teardown
        return *p;
    }
    static void clear_spares() {
        std::vector<SamText> v;
        std::lock_guard<std::mutex> g(spares().m);
        v.swap(spares().v);
    }
    SamText take() {
        static const bool off = getenv("RSA_SAM_REUSE") && atoi(getenv("RSA_SAM_REUSE")) == 0;
        Spares& sp = spares();
        std::lock_guard<std::mutex> g(sp.m);
        if (off || sp.v.empty()) return SamText();
        SamText s = std::move(sp.v.back());
        sp.v.pop_back();
        return s;
    }
    void give_back(SamText& s) {
        Spares& sp = spares();
        std::lock_guard<std::mutex> g(sp.m);
        if (sp.v.size() >= 48) return;
        s.clear();
        sp.v.push_back(std::move(s));
    }
    // `made`: the chunk's digest, folded in while its text was written (Sam::digest_into)
    void put(size_t idx, SamText&& s, const SamDigest* made = nullptr) { put_piece(idx, std::move(s), made, true); }
    // the next piece of chunk idx's text (`last`: the chunk is complete with it)
    void put_piece(size_t idx, SamText&& s, const SamDigest* made, bool last) {
        SamDigest d;
        if (digest) d = made ? *made : SamDigest::of(s.data(), s.size());   // in the calling worker
        std::unique_lock<std::mutex> g(m);
        Entry& e = pending[idx];
        e.pieces.emplace_back(std::move(s), d);
        e.done = last;
        bool moved = false;
        for (auto it = pending.find(next); it != pending.end(); it = pending.find(next)) {
            for (auto& pc : it->second.pieces) {
                bytes += pc.first.size();
                total.append(pc.second);
                if (!first_out) first_out = since(t_open);
                if (sink) {
                    queued_bytes += pc.first.size();
                    queue.push_back(std::move(pc.first));
                    moved = true;
                } else {
                    give_back(pc.first);
                }
            }
            it->second.pieces.clear();
            if (!it->second.done) break;          // more of this chunk to come
            pending.erase(it);
            next++;
        }
        if (moved) cv.notify_one();
        room_cv.wait(g, [&] { return queued_bytes <= kMaxQueued; });
    }
    void write_loop() {
        if (g_worker_start_hook) g_worker_start_hook();
        std::unique_lock<std::mutex> g(m);
        for (;;) {
            cv.wait(g, [&] { return closing || !queue.empty(); });
            if (queue.empty()) break;           // closing and drained
            SamText t = std::move(queue.front());
            queue.pop_front();
            const size_t behind = queued_bytes;
            g.unlock();
            const double ta = since(t_open);
            sink(user, t.data(), t.size());
            if (trace) fprintf(trace, "%.4f %.4f %zu %zu W\n", ta, since(t_open), t.size(), behind);
            const size_t n = t.size();
            give_back(t);
            g.lock();
            queued_bytes -= n;
            room_cv.notify_all();
        }
        if (trace) fprintf(trace, "end %.4f\n", since(t_open));
    }
};

void release_sam_spares() { OrderedSink::clear_spares(); }

struct PeChunk {
    InputChunk in;                            // the source's records; in.r1/in.r2[i].seq upper-cased by pe_load
    size_t size() const { return in.r1.size(); }
    // both mates' upper-cased sequences (pc.cpp:1586-1587) back to back, read 2i + m at
    // seqoff[2i + m]; in memory the engine can DMA from (Engine::io_alloc) when it has one,
    // and the seeding call then takes them as is
    std::vector<char, HostAlloc<char>> seqbuf;
    std::vector<uint64_t> seqoff;
    std::vector<uint32_t> seqlen;
    SamText rcbuf;                            // reverse complements of both mates, computed once (resize: no fill):
    std::vector<uint64_t> rcoff;              // read i mate m at rcoff[2i+m] (length = read length)
    std::string_view rc(size_t i, int m) const {
        const RecView& r = m ? in.r2[i] : in.r1[i];
        return std::string_view(rcbuf.data() + rcoff[2 * i + m], r.seq.size());
    }
    std::vector<AlignTmpRes> res;
    SeedBatchOut seeds;                       // engine output of pe_seed
    std::minstd_rand rng;
    AlignmentStatistics stats;
    PhaseTimes times;
};

struct ChunkPool {
    std::mutex m;
    std::vector<std::unique_ptr<PeChunk>> free;
    static constexpr size_t kCap = 96;        // > the prefetch window of 24 workers
    std::unique_ptr<PeChunk> take() {
        std::lock_guard<std::mutex> g(m);
        if (free.empty()) return nullptr;
        auto c = std::move(free.back());
        free.pop_back();
        return c;
    }
    void clear() {
        std::vector<std::unique_ptr<PeChunk>> v;
        {
            std::lock_guard<std::mutex> g(m);
            v.swap(free);
        }
    }
    void put(std::unique_ptr<PeChunk> c) {
        if (!c) return;
        {
            std::lock_guard<std::mutex> g(m);
            if (free.size() < kCap) { free.push_back(std::move(c)); return; }
        }
        c.reset();                              // over the cap: freed by this worker, outside the lock
    }
};
// A worker's SW job and result lists, kept at capacity across mapping calls
// (each bench step is one call, with new worker threads) like the chunks.
struct WorkerScratch {
    std::vector<SwJob> jobs;
    std::vector<AlignmentInfo> infos;
};
struct ScratchLease {
    std::unique_ptr<WorkerScratch> s;
    static std::mutex& mu() {
        static std::mutex* m = new std::mutex();
        return *m;
    }
    static std::vector<std::unique_ptr<WorkerScratch>>& pool() {
        static auto* p = new std::vector<std::unique_ptr<WorkerScratch>>();   // never destroyed
        return *p;
    }
    ScratchLease() {
        {
            std::lock_guard<std::mutex> g(mu());
            if (!pool().empty()) { s = std::move(pool().back()); pool().pop_back(); }
        }
        if (!s) s.reset(new WorkerScratch());
    }
    ~ScratchLease() {
        std::lock_guard<std::mutex> g(mu());
        if (pool().size() < 64) pool().push_back(std::move(s));
    }
    static void clear() {
        std::vector<std::unique_ptr<WorkerScratch>> v;
        std::lock_guard<std::mutex> g(mu());
        v.swap(pool());
    }
};

// Worker threads outlive the mapping calls (each bench step is one call, and
// creating ~30 threads a call cost their stacks' mmap/mprotect, TLS setup and
// teardown on every step): run(n, f) runs f on n pool threads and returns when
// all are done.  Jobs never block on each other through the pool itself.
class WorkerPool {
public:
    void run(int n, const std::function<void()>& f) {
        // one mapping call at a time uses the pool; a concurrent one gets its own threads
        std::unique_lock<std::mutex> busy(run_m_, std::try_to_lock);
        if (!busy.owns_lock()) {
            std::vector<std::thread> ws;
            for (int t = 0; t < n; ++t) ws.emplace_back(f);
            for (auto& w : ws) w.join();
            return;
        }
        std::unique_lock<std::mutex> g(m_);
        while ((int)threads_.size() < n) threads_.emplace_back([this] { loop(); });
        pending_ = n;
        job_ = &f;
        generation_++;
        cv_.notify_all();
        done_cv_.wait(g, [&] { return pending_ == 0 && running_ == 0; });
        job_ = nullptr;
    }
    static WorkerPool& get() {
        static WorkerPool* p = new WorkerPool();     // never destroyed: no exit-time teardown
        return *p;
    }
    // every pool thread ended and joined (no mapping call may be running); the next run()
    // starts new ones
    void shutdown() {
        std::lock_guard<std::mutex> busy(run_m_);
        std::vector<std::thread> ts;
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            ts.swap(threads_);
        }
        cv_.notify_all();
        for (auto& t : ts) t.join();
        std::lock_guard<std::mutex> g(m_);
        stop_ = false;
    }

private:
    void loop() {
        uint64_t seen = 0;         // a thread made by run() takes part in that run's generation
        std::unique_lock<std::mutex> g(m_);
        for (;;) {
            cv_.wait(g, [&] { return stop_ || (generation_ != seen && pending_ > 0); });
            if (stop_) return;
            seen = generation_;
            pending_--;
            running_++;
            const std::function<void()>* f = job_;
            g.unlock();
            (*f)();
            g.lock();
            running_--;
            if (pending_ == 0 && running_ == 0) done_cv_.notify_all();
        }
    }
    std::mutex run_m_, m_;
    std::condition_variable cv_, done_cv_;
    std::vector<std::thread> threads_;
    const std::function<void()>* job_ = nullptr;
    int pending_ = 0, running_ = 0;
    uint64_t generation_ = 0;
    bool stop_ = false;
};

ChunkPool& chunk_pool() {
    static ChunkPool* p = new ChunkPool();     // never destroyed: no exit-time teardown
    return *p;
}

// Each read's name, sequence and qualities may sit anywhere (a caller's heap
// strings, a mapped file): loading a chunk (sequences) and writing its SAM
// records (all three) request them a few pairs ahead.
// Cores the mapping workers leave to the SAM writer and the FASTQ readers when the
// output goes to a sink (RSA_IO_CORES).  The writer is the streamed path's critical
// path at the end of a call: it must copy every chunk into the page cache in chunk
// order, and with all cores' worth of workers runnable it got a share of a core.
static int io_cores(bool has_sink, int threads) {
    static const int n = getenv("RSA_IO_CORES") ? atoi(getenv("RSA_IO_CORES")) : 1;
    return has_sink && threads > 2 ? std::max(0, n) : 0;
}
// RSA_WORKER_NICE=n: mapping workers run at nice n (default 0), so the SAM writer and the
// FASTQ readers -- the streamed path's serial stages -- win the host cores they compete for
static void worker_priority() {
    static const int n = getenv("RSA_WORKER_NICE") ? atoi(getenv("RSA_WORKER_NICE")) : 0;
    thread_local int set = 0;
    if (n > 0 && set != n) {
        (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), n);
        set = n;
    }
}
static bool prefetch_on() {                // RSA_PREFETCH=0 turns the software prefetches off (A/B)
    static const bool on = !(getenv("RSA_PREFETCH") && atoi(getenv("RSA_PREFETCH")) == 0);
    return on;
}
static size_t rec_ahead() {                 // RSA_PREFETCH_AHEAD, default 4 pairs
    static const size_t d = getenv("RSA_PREFETCH_AHEAD") ? (size_t)std::max(1, atoi(getenv("RSA_PREFETCH_AHEAD"))) : 4;
    return d;
}
static inline void prefetch_str(std::string_view s) {
    const char* p = s.data();
    for (size_t o = 0; o < s.size(); o += 64) __builtin_prefetch(p + o);
}
static inline void prefetch_record(const RecView& r) {
    prefetch_str(r.name);
    prefetch_str(r.qual);
}
static inline void prefetch_bytes(const void* p, size_t bytes) {
    const char* c = (const char*)p;
    bytes = std::min<size_t>(bytes, 2048);
    for (size_t o = 0; o < bytes; o += 64) __builtin_prefetch(c + o);
}
template <class T>
static inline void prefetch_vec(const std::vector<T>& v) {
    const char* p = (const char*)v.data();
    const size_t n = std::min<size_t>(v.size() * sizeof(T), 1024);
    for (size_t o = 0; o < n; o += 64) __builtin_prefetch(p + o);
}
template <class T>
static inline void prefetch_vec_w(const std::vector<T>& v) {   // the storage past size() too: it is about to be written
    const char* p = (const char*)v.data();
    const size_t n = std::min<size_t>(std::max(v.size(), (size_t)4) * sizeof(T), std::min<size_t>(v.capacity() * sizeof(T), 1024));
    for (size_t o = 0; o < n; o += 64) __builtin_prefetch(p + o, 1);
}
// the pool entries (mismatch positions / hamming_align results) of read r's first site
// checks; the sites themselves must be in cache by now (prefetched further ahead)
static inline void prefetch_site_pool(const SeedBatchOut& so, size_t r) {
    if (so.sites.empty()) return;
    const size_t a = so.offsets[r], b = std::min<size_t>(so.offsets[r + 1], so.offsets[r] + 8);
    for (size_t k = a; k < b; ++k) {
        const rsa_nam_site& st = so.sites[k];
        if (!(st.flags & RSA_SITE_POSITIONS) || (st.flags & RSA_SITE_POOL_FULL)) continue;
        const size_t words = (st.flags & RSA_SITE_ALIGNED) ? 12 + 4 * (size_t)st.n_mm : (size_t)st.n_mm;
        prefetch_bytes(so.mm_pool.data() + st.mm_offset, 2 * words);
    }
}
// the object itself (a pair's AlignTmpRes): its vector headers must be in cache before
// prefetch_res / prefetch_res_w read them, so this goes one distance further ahead
template <class T>
static inline void prefetch_obj(const T& x, int rw = 0) {
    const char* p = (const char*)&x;
    for (size_t o = 0; o < sizeof(T); o += 64) rw ? __builtin_prefetch(p + o, 1) : __builtin_prefetch(p + o);
    __builtin_prefetch(p + sizeof(T) - 1);
}
static inline void prefetch_res_w(const AlignTmpRes& r) {
    prefetch_vec_w(r.align_res);
    prefetch_vec_w(r.todo_nams);
    __builtin_prefetch(&r, 1);
}
// a pair's alignments and NAM lists, written by part() and extend, read back when stored
static inline void prefetch_res(const AlignTmpRes& r) {
    prefetch_vec(r.align_res);
    prefetch_vec(r.todo_nams);
    prefetch_vec(r.type4_nams);
}

// rescue jobs whose has_shared_substring test failed in the engine: no aligner call
// in the reference (rescue_mate_part returns before it)
static inline uint64_t no_shared_count(const std::vector<AlignmentInfo>& infos) {
    uint64_t n = 0;
    for (const AlignmentInfo& i : infos) n += i.no_shared ? 1 : 0;
    return n;
}

// to_uppercase (refs.cpp:10-16, c & ~32) of n bytes into dst
static inline void upper_into(const char* src, size_t n, char* dst) {
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, src + i, 8);
        w &= ~0x2020202020202020ULL;
        memcpy(dst + i, &w, 8);
    }
    for (; i < n; ++i) dst[i] = (char)((unsigned char)src[i] & ~32);
}

// Chunk idx from the source, with both mates' sequences upper-cased into one
// buffer (the chunk's record views then point there) and their reverse
// complements computed once.  False past the end of the input.
bool pe_load(PeChunk& c, ReadSource& src, size_t idx, const HostAllocFns* io) {
    c.stats = AlignmentStatistics();
    c.times = PhaseTimes();
    if (!src.get(idx, c.in)) return false;
    const size_t n = c.size();
    size_t tot = 0;
    for (size_t i = 0; i < n; ++i) tot += c.in.r1[i].seq.size() + c.in.r2[i].seq.size();
    c.rcbuf.resize(tot);
    c.rcoff.resize(2 * n);
    if (c.seqbuf.get_allocator().fns != io) c.seqbuf = decltype(c.seqbuf)(HostAlloc<char>(io));
    c.seqbuf.resize(tot + 16);
    c.seqoff.resize(2 * n);
    c.seqlen.resize(2 * n);
    size_t at = 0;
    const size_t ahead = rec_ahead();
    // one pass: the reverse complement is taken while the sequence is in cache
    for (size_t i = 0; i < n; ++i) {
        if (i + ahead < n) {
            prefetch_str(c.in.r1[i + ahead].seq);
            prefetch_str(c.in.r2[i + ahead].seq);
        }
        for (int m = 0; m < 2; ++m) {
            RecView& r = m ? c.in.r2[i] : c.in.r1[i];
            const size_t len = r.seq.size();
            char* up = c.seqbuf.data() + at;
            upper_into(r.seq.data(), len, up);
            r.seq = std::string_view(up, len);
            c.seqoff[2 * i + m] = at;
            c.seqlen[2 * i + m] = (uint32_t)len;
            c.rcoff[2 * i + m] = at;
            reverse_complement_into(r.seq, &c.rcbuf[at]);
            at += len;
        }
    }
    // recycled chunk: per-pair vectors keep their capacity; part() empties each pair's
    // results as it reaches it (a pass over every cold pair here cost its own misses)
    if (c.res.size() > n) c.res.resize(n);
    c.res.resize(n);
    return true;
}

// Seeding of a loaded chunk (randstrobes + find_nams + rescue on the engine).
// Independent of the insert-size state, so it can run ahead of part().
void pe_seed(PeChunk& c, Engine& eng, const MapContext& mc, CpuSlots& slots) {
    const size_t n = c.size();
    if (n == 0) { c.seeds.clear(); return; }
    const auto t = Clock::now();
    if (eng.io_alloc()) {                     // packed by pe_load in DMA-able memory
        Unslot u(slots, eng.offloads(), c.in.index);
        eng.seed_packed(c.seqbuf.data(), c.seqoff.data(), c.seqlen.data(), 2 * n, mc.mparams.rescue_level,
                        (unsigned)mc.mparams.rescue_cutoff, c.seeds);
        c.times.seed += since(t);
        return;
    }
    std::vector<std::string_view> reads;
    reads.reserve(2 * n);
    for (size_t i = 0; i < n; ++i) { reads.push_back(c.in.r1[i].seq); reads.push_back(c.in.r2[i].seq); }
    Unslot u(slots, eng.offloads(), c.in.index);
    eng.seed(reads, mc.mparams.rescue_level, (unsigned)mc.mparams.rescue_cutoff, c.seeds);
    c.times.seed += since(t);
}

// part() of every pair in chunk order (pc.cpp:1739-1766) on the seeded chunk
// on_frozen (sequential phase only) runs once, right after the pair whose
// sample freezes the insert-size estimate: from there on no later chunk depends
// on this one's remaining pairs, so the other workers can start.
// `replay_only`: a chunk before a rank's part (PipelineOptions::first_chunk), parted
// only for the insert-size estimate: nothing of it is used once the estimate froze.
template <class OnFrozen>
void pe_part(PeChunk& c, const MapContext& mc, InsertSizeDistribution& isize, OnFrozen&& on_frozen,
             bool replay_only = false) {
    bool was_frozen = isize.frozen();
    c.rng.seed((unsigned)c.in.index);
    const size_t n = c.size();
    if (n == 0) return;
    SeedBatchOut& so = c.seeds;
    const auto t = Clock::now();
    // an engine that sorted the lists (RSA_NAMS_BY_SCORE) leaves only those over 16
    // NAMs to sort, and part() works on its download in place; otherwise each list
    // is gathered into a reused vector in std::sort order
    std::vector<Nam> copies[2];
    const size_t ahead = rec_ahead();
    for (size_t i = 0; i < n; ++i) {
        if (prefetch_on()) {   // the NAMs, site checks and pool came by DMA: not in any cache
            if (i + 2 * ahead < n) {
                const size_t a = so.offsets[2 * (i + 2 * ahead)], b = so.offsets[2 * (i + 2 * ahead) + 2];
                prefetch_bytes(so.nams.data() + a, (b - a) * sizeof(Nam));
                if (!so.sites.empty()) prefetch_bytes(so.sites.data() + a, (b - a) * sizeof(rsa_nam_site));
                prefetch_obj(c.res[i + 2 * ahead], 1);
                if (i + 4 * ahead < n) __builtin_prefetch(&so.offsets[2 * (i + 4 * ahead)]);
            }
            if (i + ahead < n) {
                prefetch_site_pool(so, 2 * (i + ahead));       // sites read here came in `ahead` pairs ago
                prefetch_site_pool(so, 2 * (i + ahead) + 1);
                prefetch_res_w(c.res[i + ahead]);   // part() appends to the pair's lists (storage kept from the last chunk)
            }
        }
        bool rescued[2];
        NamSpan nams[2];
        for (int m = 0; m < 2; ++m) {
            const size_t r = 2 * i + m;
            Nam* src = so.nams.data() + so.offsets[r];
            const size_t cnt = so.offsets[r + 1] - so.offsets[r];
            if (so.by_score) {
                nams[m] = NamSpan(src, cnt);
                if (cnt > 16) sort_nams_by_score(nams[m]);
            } else {
                load_sorted_nams(copies[m], src, cnt);
                nams[m] = NamSpan(copies[m]);
            }
            rescued[m] = so.rescued[r] != 0;
        }
        Read read1(c.in.r1[i].seq, c.rc(i, 0)), read2(c.in.r2[i].seq, c.rc(i, 1));
        read1.site = so.site_view(2 * i, c.in.r1[i].seq.size());
        read2.site = so.site_view(2 * i + 1, c.in.r2[i].seq.size());
        c.res[i].reset();
        align_PE_read_part(c.res[i], c.in.r1[i], c.in.r2[i], read1, read2, nams, rescued, c.stats, isize, mc, c.rng,
                           true);
        c.stats.n_reads += 2;
        if (!was_frozen && isize.frozen()) {
            was_frozen = true;
            on_frozen(c);
        }
        if (replay_only && was_frozen) break;
    }
    c.seeds.clear();
    c.times.part += since(t);
}

void pe_part(PeChunk& c, const MapContext& mc, InsertSizeDistribution& isize) {
    pe_part(c, mc, isize, [](PeChunk&) {});
}

// appends the chunk's SW jobs (pc.cpp:214-242, 333-368) to `jobs`
void pe_get_str(PeChunk& c, const MapContext& mc, float mu, float sigma, std::vector<SwJob>& jobs) {
    const auto t = Clock::now();
    const size_t n = c.size(), ahead = rec_ahead();
    for (size_t i = 0; i < n; ++i) {
        if (i + 2 * ahead < n) prefetch_obj(c.res[i + 2 * ahead]);
        if (i + ahead < n) prefetch_vec(c.res[i + ahead].todo_nams);   // written by part(), cold by now
        const Read read1(c.in.r1[i].seq, c.rc(i, 0)), read2(c.in.r2[i].seq, c.rc(i, 1));
        collect_jobs_pe(c.res[i], c.in.r1[i], c.in.r2[i], read1, read2, mc, mu, sigma, jobs);
    }
    c.times.collect += since(t);
}

// pairs per piece of a chunk's SAM text handed to the writer (RSA_SAM_PIECE; 0 = the
// whole chunk at once, the default): with pieces the writer starts on a chunk while its
// last() runs on.  Measured (profiles/r06/ab_pieces.json, 16 alternating steps each):
// pieces of 2000 pairs bring the first SAM text to the writer 3 ms earlier a step (10.8
// against 14.0 ms) but the streamed rate falls from 19.7 to 18.7 Mreads/s
// RSA_SAM_PIECE_FIRST: the same for the run's first chunk only (the writer's first bytes wait
// for it; the other chunks stay whole)
static size_t sam_piece_pairs(bool first_chunk) {
    const char* e = getenv("RSA_SAM_PIECE");        // per chunk (A/B runs change it between calls)
    const char* f = first_chunk ? getenv("RSA_SAM_PIECE_FIRST") : nullptr;
    return f ? (size_t)atol(f) : e ? (size_t)atol(e) : 0;
}

// the chunk's extension results start at infos[pos]; its SAM text goes to `os` in pieces
void pe_store_last(PeChunk& c, const MapContext& mc, const InsertSizeDistribution& isize,
                   std::vector<AlignmentInfo>& infos, size_t pos, const std::string& rg_id, OrderedSink& os) {
    const auto t = Clock::now();
    const size_t n = c.size();
    const bool pf = prefetch_on();
    const size_t ahead = rec_ahead();
    for (size_t i = 0; i < n; ++i) {
        if (pf && i + 2 * ahead < n) prefetch_obj(c.res[i + 2 * ahead]);
        if (pf && i + ahead < n) prefetch_res(c.res[i + ahead]);
        const Read read1(c.in.r1[i].seq, c.rc(i, 0)), read2(c.in.r2[i].seq, c.rc(i, 1));
        pos = store_results_pe(c.res[i], read1, read2, mc, isize.mu, isize.sigma, infos, pos);
    }
    const size_t pp = sam_piece_pairs(c.in.index == os.first);
    const size_t piece = pp ? pp : std::max<size_t>(n, 1);
    double t_out = 0;
    for (size_t a = 0; a < n || a == 0; a += piece) {
        const size_t b = std::min(n, a + piece);
        SamText out = os.take();
        out.reserve(7 * (size_t)mc.mparams.r * (b - a));
        Sam sam(out, mc.refs, mc.mparams.cigar_eqx, rg_id, mc.mparams.output_unmapped, mc.mparams.details);
        SamDigest dg;
        if (os.digest) sam.digest_into(&dg);
        for (size_t i = a; i < b; ++i) {
            if (pf && i + 2 * ahead < n) {
                prefetch_obj(c.res[i + 2 * ahead]);
                prefetch_obj(c.in.r1[i + 2 * ahead]);
                prefetch_obj(c.in.r2[i + 2 * ahead]);
            }
            if (pf && i + ahead < n) {
                prefetch_record(c.in.r1[i + ahead]);
                prefetch_record(c.in.r2[i + ahead]);
                prefetch_res(c.res[i + ahead]);
                // SEQ comes from the chunk's upper-cased copy or its reverse complement,
                // both written at load time and long out of cache
                prefetch_str(c.in.r1[i + ahead].seq);
                prefetch_str(c.in.r2[i + ahead].seq);
                prefetch_str(c.rc(i + ahead, 0));
                prefetch_str(c.rc(i + ahead, 1));
            }
            const Read read1(c.in.r1[i].seq, c.rc(i, 0)), read2(c.in.r2[i].seq, c.rc(i, 1));
            align_PE_read_last(c.res[i], c.in.r1[i], c.in.r2[i], read1, read2, sam, c.stats, isize, mc, c.rng);
        }
        const auto tp = Clock::now();
        os.put_piece(c.in.index, std::move(out), os.digest ? &dg : nullptr, b >= n);
        t_out += since(tp);
        if (n == 0) break;
    }
    c.times.output += t_out;
    c.times.last += since(t) - t_out;
}

}  // namespace

bool huge_buffers_on() {
    static const bool on = [] {
        const char* v = getenv("RSA_HUGE_BUFFERS");
        return !v || atoi(v) != 0;
    }();
    return on;
}

void* huge_buffer_alloc(size_t bytes) {
    const size_t len = (bytes + kHugeBufferMin - 1) & ~(kHugeBufferMin - 1);
    // over-map by 2 MB and trim, so the buffer starts on a huge-page boundary
    void* m = mmap(nullptr, len + kHugeBufferMin, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) throw std::bad_alloc();
    const uintptr_t a = ((uintptr_t)m + kHugeBufferMin - 1) & ~(uintptr_t)(kHugeBufferMin - 1);
    if (a > (uintptr_t)m) munmap(m, a - (uintptr_t)m);
    const uintptr_t end = (uintptr_t)m + len + kHugeBufferMin;
    if (end > a + len) munmap((void*)(a + len), end - (a + len));
    (void)madvise((void*)a, len, MADV_HUGEPAGE);
    return (void*)a;
}

void huge_buffer_free(void* p, size_t bytes) {
    munmap(p, (bytes + kHugeBufferMin - 1) & ~(kHugeBufferMin - 1));
}

void tune_malloc() {
    static std::once_flag once;
    std::call_once(once, [] {
        mallopt(M_TRIM_THRESHOLD, 1 << 30);
        mallopt(M_TOP_PAD, 64 << 20);
        mallopt(M_MMAP_THRESHOLD, 256 << 20);
    });
}

// Chunks flow through three stages:
//   load + seed   any order, any worker, up to `window` chunks ahead (needs no
//                 insert-size state, so it also fills the sequential phase)
//   sequential    the reference's single-worker timeline (part(N) between
//                 get_str(N-1) and store(N-1)) until the estimate freezes
//   parallel      part, get_str, extend, store, last per chunk on any worker
// Chunks are claimed in index order; how many there are is known only once a
// claim runs past the end of the input (a streamed source reads while mapping).
// Every GPU wait sleeps, so a worker waiting on the engine leaves its core to the
// others.
PipelineResult run_pipeline_pe(ReadSource& src, Engine& eng, const MapContext& mc, const PipelineOptions& opt,
                               SamSink sink, void* user) {
    const auto t0 = Clock::now();
    PipelineResult result;
    eng.set_alignment_params(mc.aparams);     // hamming_align with the site checks (GPU engine)
    // a rank's part: chunks below `first` are replayed for the insert-size estimate only
    const size_t first = opt.first_chunk, end = opt.end_chunk;
    if (first >= end) {                     // an empty part (more ranks than chunks)
        result.map_seconds = since(t0);
        return result;
    }
    auto rel = [first](size_t i) { return i >= first ? i - first : i; };   // position among the run's own chunks
    auto mine = [first, end](size_t i) { return i >= first && i < end; };
    OrderedSink os(sink, user, opt.digest, first);
    const int T = std::max(1, opt.threads);
    const bool offl = eng.offloads();
    const int W = T + wait_workers(eng, T, sink != nullptr);
    CpuSlots slots;
    slots.free = std::max(1, T - io_cores(sink != nullptr, T));
    // prefetch depth (RSA_PREFETCH chunks, default 2W+2; 0 = every worker seeds its own chunk)
    const char* pf_env = getenv("RSA_PREFETCH");
    const size_t window = pf_env ? (size_t)atol(pf_env) : 2 * (size_t)W + 2;
    // until the first chunk's extension call has returned, the prefetch stays this many
    // chunks ahead (RSA_EARLY_WINDOW; 0 = the full window from the start): the first
    // chunk's extension -- on the path to the first SAM byte -- then shares the GPU with
    // a few seeding calls, not with the whole window's
    const char* ew_env = getenv("RSA_EARLY_WINDOW");
    const size_t early_window = ew_env ? (size_t)atol(ew_env) : 0;
    bool first_extended = false;

    std::mutex m;
    std::condition_variable cv;
    std::map<size_t, std::unique_ptr<PeChunk>> seeded;   // stage 1 done
    std::deque<uint8_t> claimed;                         // stage 1 taken by some worker
    auto is_claimed = [&](size_t i) { return i < claimed.size() && claimed[i]; };
    auto claim = [&](size_t i) {
        if (i >= claimed.size()) claimed.resize(i + 1, 0);
        claimed[i] = 1;
    };
    // the next chunk to prefetch: unclaimed, and never a replay chunk past 0 (those are
    // loaded by the leader when the estimate needs them)
    size_t next_seed = 0;          // every chunk below is claimed (or a replay chunk)
    auto skip_claimed = [&] {
        for (;;) {
            if (next_seed > 0 && next_seed < first) next_seed = first;
            else if (is_claimed(next_seed)) next_seed++;
            else break;
        }
    };
    size_t n_chunks = end;         // chunks of the input (of the part), once a claim has run past its end
    size_t consumed = 0;           // chunks handed past stage 1
    bool frozen = false, done = false;
    bool early = false;            // the parallel stage opened from inside part() (early_freeze)
    bool leader_busy = true;       // the leader may still hand a chunk over: nobody ends the run before
    // chunks 1..RSA_EARLY_SEEDS (default 2) are seeded alongside chunk 0: the writer needs them
    // right after it, and a few calls do not crowd chunk 0's seeding out of the GPU
    const size_t early_seeds = getenv("RSA_EARLY_SEEDS") ? (size_t)atoi(getenv("RSA_EARLY_SEEDS")) : 2;
    bool lead_seeded = false;      // other prefetch waits until chunk 0 is seeded: it would only queue
                                   // other chunks' seeding ahead of the single-worker timeline
    size_t next_par = 0;           // next chunk for the parallel stage (valid once frozen)
    // while the leader replays chunks before a rank's part (the estimate still open after
    // chunk 0), the other workers seed the next kReplayAhead of them ahead of it
    static constexpr size_t kReplayAhead = 2;
    size_t lead_next = 0;          // the replay chunk after the leader's (0: no replay prefetch)
    std::unique_ptr<PeChunk> handed;                     // part() done in the sequential phase
    InsertSizeDistribution isize, frozen_isize;
    std::exception_ptr failure;
    AlignmentStatistics stats_all;
    PhaseTimes phases_all;

    // finished chunks are recycled (process-wide, across runs), so the per-pair
    // result vectors stop allocating and no run ends by freeing them one by one;
    // the source gets the chunk's input storage back first
    std::atomic<uint64_t> singletons{0};
    auto recycle = [&](std::unique_ptr<PeChunk> c) {
        if (!c) return;
        singletons += c->in.singletons;
        src.release(c->in);
        chunk_pool().put(std::move(c));
    };
    // load + seed chunk idx; null when the input ends before it (n_chunks is then known)
    auto stage1 = [&](size_t idx) -> std::unique_ptr<PeChunk> {
        std::unique_ptr<PeChunk> c = chunk_pool().take();
        if (!c) c = std::make_unique<PeChunk>();
        const auto t = Clock::now();
        if (!pe_load(*c, src, idx, eng.io_alloc())) {
            chunk_pool().put(std::move(c));
            std::lock_guard<std::mutex> g(m);
            n_chunks = std::min(n_chunks, idx);
            cv.notify_all();
            return nullptr;
        }
        c->times.load += since(t);
        pe_seed(*c, eng, mc, slots);
        return c;
    };
    // chunk idx after stage 1: from the prefetch map, or loaded + seeded here.
    // Null past the end of the input or after a failure (`failure` set).
    auto acquire = [&](size_t idx) -> std::unique_ptr<PeChunk> {
        std::unique_lock<std::mutex> g(m);
        if (!is_claimed(idx)) {                 // nobody claimed it yet
            claim(idx);
            skip_claimed();
            g.unlock();
            auto c = stage1(idx);
            g.lock();
            if (c && idx >= first) consumed++;
            cv.notify_all();
            return c;
        }
        auto ready = [&] { return seeded.count(idx) || failure || idx >= n_chunks; };
        if (!ready()) {
            g.unlock();
            Unslot u(slots, true, idx);
            g.lock();
            cv.wait(g, ready);
            g.unlock();          // the slot comes back without the lock held
        }
        if (!g.owns_lock()) g.lock();
        if (failure || !seeded.count(idx)) return nullptr;
        auto c = std::move(seeded[idx]);
        seeded.erase(idx);
        if (idx >= first) consumed++;
        cv.notify_all();
        return c;
    };
    // SW jobs of a parted chunk in one engine call, then store + last
    auto finish = [&](PeChunk& c, const InsertSizeDistribution& est, std::vector<SwJob>& jobs,
                      std::vector<AlignmentInfo>& infos) {
        jobs.clear();
        pe_get_str(c, mc, est.mu, est.sigma, jobs);
        c.stats.tot_aligner_calls += jobs.size();
        const auto te = Clock::now();
        if (c.in.index == first) c.times.first_ext_begin = since(t0);
        {
            Unslot u(slots, offl, c.in.index);
            eng.extend(jobs, mc.aparams, infos);
        }
        if (c.in.index == first) {
            c.times.first_ext_end = since(t0);
            std::lock_guard<std::mutex> g(m);
            first_extended = true;
            cv.notify_all();
        }
        c.stats.tot_aligner_calls -= no_shared_count(infos);   // the reference aligns none of those
        c.times.extend += since(te);
        pe_store_last(c, mc, est, infos, 0, opt.rg_id, os);
    };

    auto worker = [&](bool leader) {
        if (g_worker_start_hook) g_worker_start_hook();
        worker_priority();
        ScratchLease scratch;
        std::vector<SwJob>& jobs = scratch.s->jobs;
        std::vector<AlignmentInfo>& infos = scratch.s->infos;
        AlignmentStatistics local;
        PhaseTimes lt;
        std::unique_ptr<SlotHold> hold(new SlotHold(slots));
        try {
            // inside the leader's part(): the estimate just froze, so chunks after the one being
            // parted no longer depend on the sequential timeline -- open the parallel stage now
            auto early_freeze = [&](PeChunk& cur_chunk) {
                std::lock_guard<std::mutex> g(m);
                frozen = true;
                frozen_isize = isize;
                next_par = std::max(cur_chunk.in.index + 1, first);
                early = true;
                cv.notify_all();
            };
            if (leader) {
                // ---- single-worker timeline until the insert-size estimate freezes ----
                auto pre = acquire(0);
                lt.first_seeded = since(t0);
                bool lost = false;
                {
                    std::lock_guard<std::mutex> g(m);
                    lost = failure != nullptr;
                    lead_seeded = pre != nullptr;
                    cv.notify_all();
                }
                if (lost) return;
                if (pre) pe_part(*pre, mc, isize, early_freeze, !mine(pre->in.index));
                size_t next = 1;
                while (pre && !isize.frozen() && pre->in.index < end) {
                    const bool own = mine(pre->in.index);         // else replayed for the estimate only
                    jobs.clear();
                    if (own) pe_get_str(*pre, mc, isize.mu, isize.sigma, jobs);
                    if (next < first) {
                        std::lock_guard<std::mutex> g(m);
                        lead_next = next + 1;
                        cv.notify_all();
                    }
                    std::unique_ptr<PeChunk> cur = acquire(next);
                    if (!cur) {
                        std::lock_guard<std::mutex> g(m);
                        if (failure) return;
                    }
                    if (cur) pe_part(*cur, mc, isize, early_freeze, !mine(cur->in.index));
                    next++;
                    if (!own) {
                        lt.replayed++;
                        recycle(std::move(pre));
                        pre = std::move(cur);
                        continue;
                    }
                    const auto te = Clock::now();
                    if (pre->in.index == first) pre->times.first_ext_begin = since(t0);
                    {
                        Unslot u(slots, offl, pre->in.index);
                        eng.extend(jobs, mc.aparams, infos);
                    }
                    if (pre->in.index == first) {
                        pre->times.first_ext_end = since(t0);
                        std::lock_guard<std::mutex> g(m);
                        first_extended = true;
                        cv.notify_all();
                    }
                    pre->times.extend += since(te);
                    pre->stats.tot_aligner_calls += jobs.size() - no_shared_count(infos);
                    pe_store_last(*pre, mc, isize, infos, 0, opt.rg_id, os);
                    local.add(pre->stats);
                    lt.add(pre->times);
                    recycle(std::move(pre));
                    pre = std::move(cur);
                }
                lt.sequential = since(t0);
                if (pre && !mine(pre->in.index)) {     // replayed only
                    lt.replayed++;
                    recycle(std::move(pre));
                }
                std::lock_guard<std::mutex> g(m);
                frozen = true;
                frozen_isize = isize;
                handed = std::move(pre);                 // may be null: everything was sequential
                leader_busy = false;
                if (!early) next_par = std::max(next, first);
                if (next_par >= n_chunks && !handed) done = true;
                cv.notify_all();
            }
            // ---- shared loop: parallel stage first, prefetch when it has nothing ----
            for (;;) {
                std::unique_ptr<PeChunk> c;
                size_t idx = SIZE_MAX, pf = SIZE_MAX;
                {
                    std::unique_lock<std::mutex> g(m);
                    for (;;) {
                        if (failure || done) break;
                        if (frozen && handed) { c = std::move(handed); break; }
                        if (frozen && next_par < n_chunks) { idx = next_par++; break; }
                        if (!frozen && lead_next) {       // replay chunks just ahead of the leader
                            for (size_t r = lead_next; r < std::min(first, lead_next + kReplayAhead); ++r)
                                if (!is_claimed(r)) { pf = r; claim(r); break; }
                            if (pf != SIZE_MAX) break;
                        }
                        skip_claimed();
                        const size_t win = first_extended || !early_window ? window : std::min(window, early_window);
                        if ((lead_seeded || rel(next_seed) <= early_seeds) && next_seed < n_chunks &&
                            rel(next_seed) < consumed + win) {
                            pf = next_seed;
                            claim(pf);
                            skip_claimed();
                            break;
                        }
                        if (frozen && next_par >= n_chunks && !leader_busy) { done = true; cv.notify_all(); break; }
                        g.unlock();
                        {
                            Unslot u(slots, true);
                            g.lock();
                            cv.wait(g);
                            g.unlock();
                        }
                        g.lock();
                    }
                }
                if (!c && idx != SIZE_MAX) {
                    c = acquire(idx);
                    if (!c) {
                        std::lock_guard<std::mutex> g(m);
                        if (failure) break;
                        continue;                        // past the end: n_chunks is known now
                    }
                    InsertSizeDistribution est = frozen_isize;
                    pe_part(*c, mc, est);
                }
                if (c) {
                    lt.last_start = std::max(lt.last_start, since(t0));
                    finish(*c, frozen_isize, jobs, infos);
                    lt.last_put = std::max(lt.last_put, since(t0));
                    local.add(c->stats);
                    lt.add(c->times);
                    recycle(std::move(c));
                    continue;
                }
                if (pf != SIZE_MAX) {
                    auto s1 = stage1(pf);
                    std::lock_guard<std::mutex> g(m);
                    if (s1) seeded.emplace(pf, std::move(s1));
                    cv.notify_all();
                    continue;
                }
                break;
            }
        } catch (...) {
            {
                std::lock_guard<std::mutex> g(m);
                if (!failure) failure = std::current_exception();
                cv.notify_all();
            }
            src.cancel();        // workers waiting on input (a stalled pipe) give up too
        }
        hold.reset();
        std::lock_guard<std::mutex> g(m);
        stats_all.add(local);
        phases_all.add(lt);
    };
    std::atomic<bool> lead_taken{false};
    WorkerPool::get().run(W, [&] { worker(!lead_taken.exchange(true)); });
    phases_all.workers_done = since(t0);
    // chunks seeded ahead but never mapped (a failure): their input goes back to the source
    for (auto& kv : seeded) recycle(std::move(kv.second));
    if (handed) recycle(std::move(handed));
    os.close();                                  // the last SAM byte is with the sink
    if (failure) std::rethrow_exception(failure);
    result.stats = stats_all;
    result.phases = phases_all;
    result.phases.first_out = os.first_out;
    result.singletons = singletons.load();
    result.map_seconds = since(t0);
    result.sam_bytes = os.bytes;
    result.sam_digest = os.total;
    return result;
}

PipelineResult run_pipeline_pe(const std::vector<Record>& r1, const std::vector<Record>& r2, Engine& eng,
                               const MapContext& mc, const PipelineOptions& opt, SamSink sink, void* user) {
    auto src = make_vector_source(&r1, &r2, (size_t)std::max(1, opt.chunk_size));
    return run_pipeline_pe(*src, eng, mc, opt, sink, user);
}

// a single-end worker's storage, kept across chunks and mapping calls: the seeding
// output (page-locked under the GPU engine, expensive to allocate: a fresh one per
// worker per call put page locking into every call) and the per-read results,
// reverse complements and NAM list, which keep their capacity
struct SeScratch {
    InputChunk in;
    SeedBatchOut so;
    std::vector<AlignTmpRes> res;
    std::vector<std::string> rcs;
    std::vector<Nam> nams;
    std::vector<std::string_view> reads;
};
struct SeScratchPool {
    std::mutex m;
    std::vector<std::unique_ptr<SeScratch>> v;
    static SeScratchPool& get() {
        static SeScratchPool* p = new SeScratchPool();   // never destroyed: no exit-time teardown
        return *p;
    }
    std::unique_ptr<SeScratch> take() {
        std::lock_guard<std::mutex> g(m);
        if (v.empty()) return std::make_unique<SeScratch>();
        auto x = std::move(v.back());
        v.pop_back();
        return x;
    }
    void put(std::unique_ptr<SeScratch> x) {
        std::lock_guard<std::mutex> g(m);
        if (v.size() < 64) v.push_back(std::move(x));
    }
    void clear() {
        std::vector<std::unique_ptr<SeScratch>> d;
        std::lock_guard<std::mutex> g(m);
        d.swap(v);
    }
};

// Every thread and pooled buffer the pipeline keeps between mapping calls: the
// worker pool's threads end (joined), and the recycled chunks, scratch and SAM
// buffers -- page-locked ones included, which go back through the engine's
// allocator -- are freed.  The caller guarantees no mapping call is running and
// that the engine whose allocator made them is still open (rsam_close: before the
// last engine goes).
void release_pipeline_resources() {
    WorkerPool::get().shutdown();
    chunk_pool().clear();
    ScratchLease::clear();
    SeScratchPool::get().clear();
    release_sam_spares();
}

// Single-end: perform_task_async_se (pc.cpp:814-1096).  No insert-size state;
// records are NOT upper-cased on this path; chunks are independent from the start.
PipelineResult run_pipeline_se(ReadSource& src, Engine& eng, const MapContext& mc, const PipelineOptions& opt,
                               SamSink sink, void* user) {
    auto t0 = std::chrono::steady_clock::now();
    PipelineResult result;
    eng.set_alignment_params(mc.aparams);
    OrderedSink os(sink, user, opt.digest, opt.first_chunk);
    std::atomic<size_t> next{opt.first_chunk};      // chunks are independent: a part starts at its own
    std::mutex stat_m;
    const int T = std::max(1, opt.threads);
    const bool offl = eng.offloads();
    CpuSlots slots;
    slots.free = T;
    std::exception_ptr failure;
    std::atomic<bool> failed{false};
    auto worker = [&]() {
        if (g_worker_start_hook) g_worker_start_hook();
        worker_priority();
        std::unique_ptr<SlotHold> hold(new SlotHold(slots));
        ScratchLease scratch;
        std::vector<SwJob>& jobs = scratch.s->jobs;
        std::vector<AlignmentInfo>& infos = scratch.s->infos;
        AlignmentStatistics local;
        std::unique_ptr<SeScratch> se = SeScratchPool::get().take();
        InputChunk& in = se->in;
        SeedBatchOut& so = se->so;                   // the worker's, reused chunk after chunk and across calls
        std::vector<AlignTmpRes>& res = se->res;
        std::vector<std::string>& rcs = se->rcs;
        std::vector<Nam>& nams = se->nams;
        std::vector<std::string_view>& reads = se->reads;
        try {
        for (;;) {
            if (failed.load()) break;
            const size_t idx = next.fetch_add(1);
            if (!src.get(idx, in)) break;
            const size_t n = in.r1.size();
            const RecView* recs = in.r1.data();
            AlignmentStatistics st;
            std::minstd_rand rng;
            rng.seed((unsigned)idx);
            reads.clear();
            for (size_t i = 0; i < n; ++i) reads.push_back(recs[i].seq);
            so.clear();
            if (n) {
                Unslot u(slots, offl, idx);
                eng.seed(reads, mc.mparams.rescue_level, (unsigned)mc.mparams.rescue_cutoff, so);
            }
            if (res.size() > n) res.resize(n);
            for (auto& x : res) x.reset();
            res.resize(n);
            rcs.resize(n);
            for (size_t r = 0; r < n; ++r) {
                rcs[r].resize(recs[r].seq.size());
                reverse_complement_into(recs[r].seq, rcs[r].data());
            }
            const size_t ahead = rec_ahead();
            for (size_t r = 0; r < n; ++r) {
                if (prefetch_on()) {
                    if (r + 2 * ahead < n && !so.sites.empty()) {
                        const size_t a = so.offsets[r + 2 * ahead], b = so.offsets[r + 2 * ahead + 1];
                        prefetch_bytes(so.sites.data() + a, (b - a) * sizeof(rsa_nam_site));
                    }
                    if (r + ahead < n) prefetch_site_pool(so, r + ahead);
                }
                nams.assign(so.nams.begin() + (long)so.offsets[r], so.nams.begin() + (long)so.offsets[r + 1]);
                Read read(recs[r].seq, rcs[r]);
                read.site = so.site_view(r, recs[r].seq.size());
                align_SE_read_part(res[r], recs[r], read, nams, so.rescued[r] != 0, st, mc, rng);
                st.n_reads++;
            }
            jobs.clear();
            for (size_t r = 0; r < n; ++r) {
                const Read read(recs[r].seq, rcs[r]);
                collect_jobs_se(res[r], read, mc, jobs);
            }
            {
                Unslot u(slots, offl, idx);
                eng.extend(jobs, mc.aparams, infos);
            }
            st.tot_aligner_calls += jobs.size();
            size_t pos = 0;
            for (size_t r = 0; r < n; ++r) {
                const Read read(recs[r].seq, rcs[r]);
                pos = store_results_se(res[r], read, mc, infos, pos);
            }
            SamText out = os.take();
            out.reserve(7 * (size_t)mc.mparams.r * n);
            Sam sam(out, mc.refs, mc.mparams.cigar_eqx, opt.rg_id, mc.mparams.output_unmapped, mc.mparams.details);
            SamDigest dg;
            if (os.digest) sam.digest_into(&dg);
            for (size_t r = 0; r < n; ++r) {
                if (r + rec_ahead() < n) prefetch_record(recs[r + rec_ahead()]);
                const Read read(recs[r].seq, rcs[r]);
                align_SE_read_last(res[r], recs[r], read, sam, st, mc, rng);
            }
            src.release(in);
            os.put(idx, std::move(out), os.digest ? &dg : nullptr);
            local.add(st);
        }
        } catch (...) {
            // an engine error on any worker ends the run: the others stop at their next
            // chunk and rsam_map / the CLI report it (an exception escaping a std::thread
            // would terminate the process)
            {
                std::lock_guard<std::mutex> g(stat_m);
                if (!failure) failure = std::current_exception();
                failed = true;
            }
            src.cancel();        // workers waiting on input (a stalled pipe) give up too
        }
        hold.reset();
        so.clear();
        src.release(in);
        SeScratchPool::get().put(std::move(se));
        std::lock_guard<std::mutex> g(stat_m);
        result.stats.add(local);
    };
    WorkerPool::get().run(T + wait_workers(eng, T, sink != nullptr), worker);
    os.close();                                  // the last SAM byte is with the sink
    if (failure) std::rethrow_exception(failure);
    result.map_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    result.sam_bytes = os.bytes;
    result.sam_digest = os.total;
    return result;
}

PipelineResult run_pipeline_se(const std::vector<Record>& r, Engine& eng, const MapContext& mc,
                               const PipelineOptions& opt, SamSink sink, void* user) {
    auto src = make_vector_source(&r, nullptr, (size_t)std::max(1, opt.chunk_size));
    return run_pipeline_se(*src, eng, mc, opt, sink, user);
}

}  // namespace rsa
