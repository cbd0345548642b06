// input.cpp -- read sources of the pipeline: records streamed from FASTQ/FASTA
// files while mapping runs, or records already in memory.
//
// The reference's workers pull chunks of 10000 pairs from one InputBuffer under
// a mutex (src/pc.cpp:74-107, called at pc.cpp:1574) while the other workers
// map.  Here each input file has a reader thread that parses blocks of records
// ahead of the pipeline (bounded: a few blocks past the last chunk asked for),
// so resident memory is set by the pipeline's window, not by the input size.
//
// Uncompressed files in the plain 4-line layout (header / one sequence line /
// '+' line / one quality line of the same length) are mapped and split in place:
// a record is four views into the mapping, no byte is copied, and the mapping's
// pages are dropped again when the chunk's SAM is written (ReadSource::release).
// The first record that is not in that layout switches the file to FastxReader
// (kseq++ semantics, io.cpp) from that record on: the plain records before it
// are exactly what kseq returns for them, and kseq restarts cleanly at a record
// header.  gzip input, pipes and FASTA go through FastxReader from the start.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <exception>
#include <map>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "rsa_host.hpp"

namespace rsa {

bool same_name(std::string_view n1, std::string_view n2) {      // pc.cpp:23-35
    if (n1.length() != n2.length()) return false;
    if (n1.length() <= 2) return n1 == n2;
    size_t i = 0;
    for (; i < n1.length() - 1; ++i)
        if (n1[i] != n2[i]) return false;
    if (n1[i - 1] == '/' && n1[i] == '1' && n2[i] == '2') return true;
    return n1[i] == n2[i];
}

// distribute_interleaved (pc.cpp:38-72) on one block; lookahead1 is never set there
size_t distribute_interleaved(const RecView* block, size_t n, std::vector<RecView>& r1, std::vector<RecView>& r2) {
    size_t singles = 0;
    for (size_t i = 0; i < n; ++i) {
        if (i + 1 < n && same_name(block[i].name, block[i + 1].name)) {
            r1.push_back(block[i]);
            r2.push_back(block[i + 1]);
            ++i;
        } else {
            singles++;
        }
    }
    return singles;
}

namespace {

// ------------------------------------------------------- records in memory --
class VectorSource final : public ReadSource {
public:
    VectorSource(const std::vector<Record>* r1, const std::vector<Record>* r2, size_t chunk)
        : r1_(r1), r2_(r2), chunk_(std::max<size_t>(1, chunk)) {
        if (r2_ && r2_->size() != r1_->size()) throw std::runtime_error("read files have different record counts");
    }
    bool paired() const override { return r2_ != nullptr; }
    bool get(size_t idx, InputChunk& out) override {
        out.clear();
        out.index = idx;
        const size_t b = idx * chunk_;
        if (b >= r1_->size()) return false;
        const size_t e = std::min(r1_->size(), b + chunk_);
        out.r1.assign(r1_->begin() + (long)b, r1_->begin() + (long)e);
        if (r2_) out.r2.assign(r2_->begin() + (long)b, r2_->begin() + (long)e);
        return true;
    }
private:
    const std::vector<Record>* r1_;
    const std::vector<Record>* r2_;
    size_t chunk_;
};

class InterleavedVectorSource final : public ReadSource {
public:
    InterleavedVectorSource(const std::vector<Record>* recs, size_t chunk)
        : recs_(recs), block_(2 * std::max<size_t>(1, chunk)) {}
    bool paired() const override { return true; }
    bool get(size_t idx, InputChunk& out) override {
        out.clear();
        out.index = idx;
        const size_t b = idx * block_;
        if (b >= recs_->size()) return false;
        const size_t e = std::min(recs_->size(), b + block_);
        std::vector<RecView>& tmp = scratch();
        tmp.assign(recs_->begin() + (long)b, recs_->begin() + (long)e);
        out.singletons = distribute_interleaved(tmp.data(), tmp.size(), out.r1, out.r2);
        return true;
    }
private:
    static std::vector<RecView>& scratch() {
        static thread_local std::vector<RecView> v;
        return v;
    }
    const std::vector<Record>* recs_;
    size_t block_;
};

// ------------------------------------------------------------ FASTQ files --
struct MappedFile {
    const char* p = nullptr;
    size_t n = 0;
    int fd = -1;
    ~MappedFile() { reset(); }
    void reset() {
        if (p && n) munmap((void*)p, n);
        if (fd >= 0) close(fd);
        p = nullptr;
        n = 0;
        fd = -1;
    }
    // a regular, uncompressed, non-empty file; false leaves the caller on the sequential reader
    bool open_map(const std::string& path) {
        if (path == "-") return false;
        fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) return false;
        struct stat st;
        if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode) || st.st_size < 2) return false;
        void* q = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (q == MAP_FAILED) return false;
        p = (const char*)q;
        n = (size_t)st.st_size;
        if ((unsigned char)p[0] == 0x1f && (unsigned char)p[1] == 0x8b) return false;   // gzip
        return true;
    }
};

inline std::string_view strip_cr(std::string_view l) {
    if (!l.empty() && l.back() == '\r') l.remove_suffix(1);
    return l;
}

// Newlines of [p, end) in order, 64 bytes at a time: four SSE2 compares give a
// 64-bit mask of the block's '\n' bytes, the set bits are taken one by one.  A
// record's four line ends cost a few instructions each instead of a memchr call.
// The block containing `end` is read with a scalar loop (no read past the mapping).
struct NlIter {
    const char* blk;                            // current 64-byte block
    const char* end;
    uint64_t mask;                              // newlines of blk not yet taken
    NlIter(const char* p, const char* e) : blk(p), end(e) { mask = load(blk); }
    uint64_t load(const char* q) const {
        if (q + 64 <= end) {
            const __m128i nl = _mm_set1_epi8('\n');
            const uint64_t m0 = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)q), nl));
            const uint64_t m1 = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)(q + 16)), nl));
            const uint64_t m2 = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)(q + 32)), nl));
            const uint64_t m3 = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)(q + 48)), nl));
            return m0 | m1 << 16 | m2 << 32 | m3 << 48;
        }
        uint64_t m = 0;
        for (const char* x = q; x < end; ++x)
            if (*x == '\n') m |= 1ull << (x - q);
        return m;
    }
    // the next '\n' at or after the current position, or `end` when there is none
    const char* next() {
        while (!mask) {
            blk += 64;
            if (blk >= end) { blk = end; return end; }
            mask = load(blk);
        }
        const char* r = blk + __builtin_ctzll(mask);
        mask &= mask - 1;
        return r;
    }
};

// One record of the plain layout starting at p (`it` positioned at p), as views;
// false when the bytes at p are anything else (`it` then undefined: the caller
// keeps a copy).  The conditions are those under which kseq's record
// (FastxReader::next) is exactly header / sequence line / quality line:
//  - the record starts with '@' and has four lines;
//  - the third line starts with '+';
//  - the sequence line is not empty and does not start with '>', '@', '+' or '\r'
//    (kseq would end the sequence there); kseq strips one '\r' from the line after
//    its first byte, then trailing blanks;
//  - the quality line (one '\r' stripped) is as long as the sequence, so kseq
//    stops reading quality after it.
inline bool plain_record(const char*& p, const char* end, NlIter& it, RecView& r) {
    if (p >= end || *p != '@') return false;
    const char* e0 = it.next();
    const char* e1 = it.next();
    const char* e2 = it.next();
    if (e2 >= end) return false;                // fewer than four lines
    const char* e3 = it.next();
    const char* l1 = e0 + 1;
    const char* l2 = e1 + 1;
    const char* l3 = e2 + 1;
    if (l2 >= e2 || *l2 != '+') return false;
    std::string_view sq(l1, (size_t)(e1 - l1));
    if (sq.empty()) return false;
    if (sq.size() >= 2 && sq.back() == '\r') sq.remove_suffix(1);
    const char c0 = sq[0];
    if (c0 == '>' || c0 == '@' || c0 == '+' || c0 == '\r') return false;
    while (!sq.empty() && (sq.back() == ' ' || sq.back() == '\t')) sq.remove_suffix(1);
    const std::string_view ql = strip_cr(std::string_view(l3, (size_t)(e3 - l3)));
    if (sq.empty() || ql.size() != sq.size()) return false;
    std::string_view h = strip_cr(std::string_view(p + 1, (size_t)(e0 - p - 1)));
    size_t ws = 0;
    while (ws < h.size() && h[ws] != ' ' && h[ws] != '\t' && h[ws] != '\v' && h[ws] != '\f' && h[ws] != '\r') ++ws;
    r.name = h.substr(0, ws);
    size_t cs = ws;
    while (cs < h.size() && (h[cs] == ' ' || h[cs] == '\t' || h[cs] == '\v' || h[cs] == '\f' || h[cs] == '\r')) ++cs;
    r.comment = h.substr(cs);
    r.seq = sq;
    r.qual = ql;
    p = e3 < end ? e3 + 1 : end;
    return true;
}

struct Block {
    std::vector<RecView> recs;
    std::vector<Record> owned;                  // records of the sequential reader (recs view them)
};

// The blocks of `per_block` records of one file, read by a thread of its own at
// most `ahead` blocks past the highest block asked for.  Mapped mode: the reader
// asks the kernel to map the next window of the file in one call
// (MADV_POPULATE_READ) instead of taking a page fault every few pages, and the
// pages of blocks whose chunks are done leave the process again in 64 MB steps.
//
// The reader's state is shared with its thread: a FileBlocks given up before the
// end of its input (a mapping error) stops the reader, and a reader that does not
// stop within kStopWait -- blocked in a read of a pipe or a terminal whose writer
// has stalled -- is detached with the state it holds, so the error path never
// waits on a slow producer.
class FileBlocks {
    struct State {
        std::string path;
        size_t per_block, ahead;
        MappedFile mf;
        size_t pos = 0;                             // mapped mode: next record's offset
        uint64_t left = UINT64_MAX;                 // records still to read (a rank's part ends early)
        uint64_t skip = 0;                          // records before a part planned by records (PartPlan)
        bool plain_only = false;                    // a rank's part: no kseq fallback (see PartPlan)
        size_t populated = 0;                       // mapped bytes already in the page table
        std::unique_ptr<FastxReader> seq;           // sequential mode
        std::mutex m;
        std::condition_variable cv;
        std::map<size_t, Block> blocks;
        size_t produced = 0, horizon = 0;
        bool finished = false, stop = false, exited = false, cancelled = false;
        std::exception_ptr err;
        std::vector<uint8_t> released;              // per produced block: its chunk is done
        std::vector<size_t> ends;                   // per produced block: mapped offset it ends at
        size_t prefix = 0, dropped = 0;

        void run() {
            if (g_worker_start_hook) g_worker_start_hook();
            try {
                // a part planned by records: the records before it are parsed and dropped
                while (skip > 0) {
                    {
                        std::lock_guard<std::mutex> g(m);
                        if (stop) break;
                    }
                    Block b;
                    const size_t got = fill_block(b, (size_t)std::min<uint64_t>(per_block, skip));
                    if (got == 0) throw std::runtime_error(path + ": fewer records than the part plan skips");
                    skip -= got;
                }
                for (;;) {
                    {
                        std::unique_lock<std::mutex> g(m);
                        cv.wait(g, [&] { return stop || produced < horizon + ahead; });
                        if (stop) break;
                    }
                    Block b;
                    const size_t end_off = read_block(b);
                    std::lock_guard<std::mutex> g(m);
                    if (b.recs.empty()) {
                        finished = true;
                        break;
                    }
                    released.push_back(0);
                    ends.push_back(end_off);
                    blocks.emplace(produced++, std::move(b));
                    cv.notify_all();
                }
            } catch (...) {
                std::lock_guard<std::mutex> g(m);
                err = std::current_exception();
            }
            std::lock_guard<std::mutex> g(m);
            exited = true;
            cv.notify_all();
        }
        // the mapped bytes from `pos` on are in this process's page table at least `want` ahead
        void populate(size_t want) {
#ifdef MADV_POPULATE_READ
            constexpr size_t kStep = 32u << 20;
            if (populated >= mf.n || populated >= pos + want) return;
            const size_t from = std::max(populated, pos) & ~(size_t)4095;
            const size_t to = std::min(mf.n, from + kStep);
            if (madvise((void*)(mf.p + from), to - from, MADV_POPULATE_READ) != 0) populated = mf.n;   // not supported
            else populated = to;
#else
            (void)want;
#endif
        }
        // returns the mapped offset the block ends at (0 in sequential mode)
        size_t read_block(Block& b) {
            const size_t cap = (size_t)std::min<uint64_t>(per_block, left);
            const size_t got = fill_block(b, cap);
            left -= got;
            return pos;
        }
        size_t fill_block(Block& b, size_t cap) {
            b.recs.reserve(cap);
            if (!seq) {
                populate(16u << 20);
                const char* end = mf.p + mf.n;
                const char* p = mf.p + pos;
                NlIter it(p, end);
                RecView r;
                while (b.recs.size() < cap && p < end) {
                    const NlIter save = it;
                    const char* at = p;
                    if (!plain_record(p, end, it, r)) {
                        it = save;
                        p = at;
                        break;
                    }
                    b.recs.push_back(r);
                }
                pos = (size_t)(p - mf.p);
                if (b.recs.size() == cap || p >= end) return b.recs.size();
                if (plain_only)
                    throw std::runtime_error(path + ": the record at byte " + std::to_string(pos) +
                                             " is not in the plain four-line FASTQ layout, which a rank's part of "
                                             "the input needs (map the file in one process instead)");
                // not the plain layout from here on: kseq over the rest of the mapped bytes
                seq.reset(new FastxReader(p, (size_t)(end - p)));
            }
            const size_t want = cap - b.recs.size();
            b.owned.reserve(want);
            Record r;
            while (b.owned.size() < want && seq->next(r)) {
                b.owned.push_back(std::move(r));
                r = Record();
            }
            for (const Record& x : b.owned) b.recs.push_back(RecView(x));
            return b.recs.size();
        }
    };

public:
    // `start` / `max_records` / `plain_only`: a rank's part of a mapped file (PartPlan);
    // `skip_records`: a rank's part of a file planned by records (gzip and other layouts)
    FileBlocks(const std::string& path, size_t per_block, size_t ahead, uint64_t start = 0,
               uint64_t max_records = UINT64_MAX, bool plain_only = false, uint64_t skip_records = 0)
        : st_(std::make_shared<State>()) {
        State& s = *st_;
        s.path = path;
        s.per_block = std::max<size_t>(1, per_block);
        s.ahead = std::max<size_t>(1, ahead);
        s.left = max_records;
        s.plain_only = plain_only;
        s.skip = skip_records;
        if (!s.mf.open_map(s.path)) {
            s.mf.reset();
            if (start || plain_only)
                throw std::runtime_error(path + ": a rank's part of the input needs a regular, uncompressed file");
            s.seq.reset(new FastxReader(s.path));   // throws when the file cannot be opened
        }
        if (start > s.mf.n) throw std::runtime_error(path + ": part offset past the end of the file");
        s.pos = (size_t)start;
        s.populated = (size_t)start;
        s.dropped = (size_t)start & ~(size_t)4095;
        std::shared_ptr<State> keep = st_;
        th_ = std::thread([keep] { keep->run(); });
    }
    ~FileBlocks() {
        static constexpr auto kStopWait = std::chrono::seconds(2);
        State& s = *st_;
        std::unique_lock<std::mutex> g(s.m);
        s.stop = true;
        s.cv.notify_all();
        const bool out = s.cv.wait_for(g, kStopWait, [&] { return s.exited; });
        g.unlock();
        if (out) th_.join();
        else th_.detach();                       // the thread keeps the state alive
    }
    // block idx, waiting for the reader; false past the end of the file
    bool take(size_t idx, Block& out) {
        State& s = *st_;
        std::unique_lock<std::mutex> g(s.m);
        if (idx + 1 > s.horizon) {
            s.horizon = idx + 1;
            s.cv.notify_all();
        }
        s.cv.wait(g, [&] {
            return s.err || s.cancelled || s.blocks.count(idx) || (s.finished && idx >= s.produced);
        });
        if (s.err) std::rethrow_exception(s.err);
        auto it = s.blocks.find(idx);
        if (it == s.blocks.end()) {
            if (s.finished) return false;
            throw std::runtime_error("input of " + s.path + " abandoned after an earlier failure");
        }
        out = std::move(it->second);
        s.blocks.erase(it);
        return true;
    }
    // the summed sequence length of the file's first `n` records (fewer at the end of
    // the file) and their count, before any block is taken: the records stay queued
    // for the pipeline, so a stream is read once (readlen.cpp:16-29 over the same
    // records the first chunk maps, as the reference's RewindableFile replays them)
    void peek_lengths(size_t n, uint64_t& tot, uint64_t& num) {
        State& s = *st_;
        std::unique_lock<std::mutex> g(s.m);
        for (;;) {
            tot = num = 0;
            for (size_t b = 0; b < s.produced && num < n; ++b) {
                auto it = s.blocks.find(b);
                if (it == s.blocks.end()) throw std::logic_error("read-length estimate after mapping started");
                for (const RecView& r : it->second.recs) {
                    if (num == n) break;
                    tot += r.seq.size();
                    num++;
                }
            }
            if (num >= n) return;
            if (s.err) std::rethrow_exception(s.err);
            if (s.finished) return;
            if (s.produced + 1 > s.horizon) {             // let the reader go past its lookahead
                s.horizon = s.produced + 1;
                s.cv.notify_all();
            }
            const size_t seen = s.produced;
            s.cv.wait(g, [&] { return s.err || s.finished || s.produced > seen; });
        }
    }
    void cancel() {
        std::lock_guard<std::mutex> g(st_->m);
        st_->cancelled = true;
        st_->cv.notify_all();
    }
    // block idx is no longer used: once every block before it is done too, the
    // mapped bytes up to its end are dropped from this process (64 MB at a time;
    // the file stays mapped, and the page cache keeps the data)
    void done(size_t idx) {
        State& s = *st_;
        if (!s.mf.p) return;
        static const bool keep = getenv("RSA_INPUT_DROP") && getenv("RSA_INPUT_DROP")[0] == '0';   // A/B
        size_t from = 0, to = 0;
        {
            std::lock_guard<std::mutex> g(s.m);
            if (idx >= s.released.size()) return;
            s.released[idx] = 1;
            while (s.prefix < s.released.size() && s.released[s.prefix]) s.prefix++;
            if (s.prefix == 0 || keep) return;
            const size_t off = s.ends[s.prefix - 1] & ~(size_t)4095;
            if (off < s.dropped + (64u << 20)) return;
            from = s.dropped;
            to = off;
            s.dropped = off;
        }
        madvise((void*)(s.mf.p + from), to - from, MADV_DONTNEED);
    }

private:
    std::shared_ptr<State> st_;
    std::thread th_;
};

// block idx of one file (single-end) or of both mate files, as chunk `index`
bool take_chunk(FileBlocks& f1, FileBlocks* f2, bool interleaved, size_t block, size_t index, InputChunk& out) {
    out.clear();
    out.index = index;
    Block b1, b2;
    const bool h1 = f1.take(block, b1);
    if (f2) {
        const bool h2 = f2->take(block, b2);
        if (h1 != h2 || b1.recs.size() != b2.recs.size())
            throw std::runtime_error("read files have different record counts");
        if (!h1) return false;
        out.r1 = std::move(b1.recs);
        out.r2 = std::move(b2.recs);
        out.owned1 = std::move(b1.owned);   // the vectors' buffers move, the records stay put
        out.owned2 = std::move(b2.owned);
        return true;
    }
    if (!h1) return false;
    if (interleaved) {
        out.singletons = distribute_interleaved(b1.recs.data(), b1.recs.size(), out.r1, out.r2);
    } else {
        out.r1 = std::move(b1.recs);
    }
    out.owned1 = std::move(b1.owned);
    return true;
}

// readlen.cpp:16-29 over InputBuffer::read_records(.., 500) (pc.cpp:74-107): the
// first 500 records of each file, or the first 1000 records of an interleaved
// file; 150 when the first file has none
int estimate_from(FileBlocks& f1, FileBlocks* f2, bool interleaved) {
    uint64_t tot1 = 0, n1 = 0, tot2 = 0, n2 = 0;
    f1.peek_lengths(interleaved ? 1000 : 500, tot1, n1);
    if (n1 == 0) return 150;
    if (f2) f2->peek_lengths(500, tot2, n2);
    return (int)((tot1 + tot2) / (n1 + n2));
}

class FastqSource final : public ReadSource {
public:
    FastqSource(const std::string& p1, const std::string& p2, bool interleaved, size_t chunk)
        : interleaved_(interleaved && p2.empty()) {
        const size_t per = (interleaved_ ? 2 : 1) * std::max<size_t>(1, chunk);
        static const size_t kAhead = getenv("RSA_READ_AHEAD") ? (size_t)atol(getenv("RSA_READ_AHEAD")) : 4;
        f1_.reset(new FileBlocks(p1, per, kAhead));
        if (!p2.empty()) f2_.reset(new FileBlocks(p2, per, kAhead));
    }
    bool paired() const override { return f2_ != nullptr || interleaved_; }
    bool get(size_t idx, InputChunk& out) override { return take_chunk(*f1_, f2_.get(), interleaved_, idx, idx, out); }
    void release(InputChunk& c) override {
        f1_->done(c.index);
        if (f2_) f2_->done(c.index);
        c.clear();
    }
    void cancel() override {
        f1_->cancel();
        if (f2_) f2_->cancel();
    }
    int estimate_read_length() override { return estimate_from(*f1_, f2_.get(), interleaved_); }

private:
    bool interleaved_;
    std::unique_ptr<FileBlocks> f1_, f2_;
};

// ------------------------------------------------------- a rank's part --
class PartSource final : public ReadSource {
public:
    PartSource(const std::string& p1, const std::string& p2, const PartPlan& plan)
        : p1_(p1), p2_(p2), plan_(plan) {
        static const size_t kAhead = getenv("RSA_READ_AHEAD") ? (size_t)atol(getenv("RSA_READ_AHEAD")) : 4;
        const size_t per = (size_t)std::max<uint64_t>(1, plan.chunk_size);
        // paired: one chunk past the part when there is one (the pipeline's insert-size replay
        // may part() it, PipelineOptions::end_chunk)
        const uint64_t tail = p2.empty() ? 0 : std::min<uint64_t>(per, plan.total_records - plan.first_record -
                                                                            plan.n_records);
        const uint64_t n = plan.n_records ? plan.n_records + tail : 0;
        // a file planned by bytes starts at its offset and must keep the plain layout; one
        // planned by records (gzip, other layouts) is parsed from its start, the records
        // before the part dropped
        auto open = [&](const std::string& p, bool by_record, uint64_t off) {
            return by_record ? new FileBlocks(p, per, kAhead, 0, n, false, plan.first_record)
                             : new FileBlocks(p, per, kAhead, off, n, true);
        };
        if (n) {                        // an empty part (an empty input, more ranks than chunks) reads nothing
            r1_.reset(open(p1, plan.by_record1, plan.offset1));
            if (!p2.empty()) r2_.reset(open(p2, plan.by_record2, plan.offset2));
        }
        if (plan.first_chunk > 0 && !p2.empty()) open_prefix();
    }
    bool paired() const override { return !p2_.empty(); }
    bool get(size_t idx, InputChunk& out) override {
        if (idx < plan_.first_chunk) {
            if (!f1_) throw std::logic_error("a chunk before the part asked for without the insert-size replay");
            return take_chunk(*f1_, f2_.get(), false, idx, idx, out);
        }
        if (!r1_ || idx > plan_.end_chunk || (idx == plan_.end_chunk && !paired())) {
            out.clear();
            out.index = idx;
            return false;
        }
        return take_chunk(*r1_, r2_.get(), false, idx - plan_.first_chunk, idx, out);
    }
    void release(InputChunk& c) override {
        if (c.index < plan_.first_chunk) {
            if (f1_) f1_->done(c.index);
            if (f2_) f2_->done(c.index);
        } else if (r1_) {
            r1_->done(c.index - plan_.first_chunk);
            if (r2_) r2_->done(c.index - plan_.first_chunk);
        }
        c.clear();
    }
    void cancel() override {
        for (FileBlocks* f : {f1_.get(), f2_.get(), r1_.get(), r2_.get()})
            if (f) f->cancel();
    }
    // from the file start, as one process estimates it (called before mapping starts)
    int estimate_read_length() override {
        if (!f1_) open_prefix();
        return estimate_from(*f1_, f2_.get(), false);
    }

private:
    // the files from their start: chunks 0 .. first_chunk - 1, read one block ahead
    void open_prefix() {
        const size_t per = (size_t)std::max<uint64_t>(1, plan_.chunk_size);
        f1_.reset(new FileBlocks(p1_, per, 1));
        if (!p2_.empty()) f2_.reset(new FileBlocks(p2_, per, 1));
    }
    std::string p1_, p2_;
    PartPlan plan_;
    std::unique_ptr<FileBlocks> f1_, f2_;          // from the file start (insert-size replay, estimate)
    std::unique_ptr<FileBlocks> r1_, r2_;          // the part
};

struct Fd {
    int fd = -1;
    explicit Fd(const std::string& path) : fd(::open(path.c_str(), O_RDONLY)) {
        if (fd < 0) throw std::runtime_error("cannot open " + path);
    }
    ~Fd() { if (fd >= 0) close(fd); }
    uint64_t size() const {
        struct stat st;
        if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode))
            throw std::runtime_error("a rank's part of the input needs regular files");
        return (uint64_t)st.st_size;
    }
};

inline uint64_t block_at(uint64_t size, uint64_t nb, uint64_t b) {
    return (uint64_t)((unsigned __int128)size * b / nb);
}

// '\n' bytes of [p, p + n): SSE2 compares, a popcount per 64 bytes
inline uint64_t count_nl(const char* p, size_t n) {
    uint64_t c = 0;
    size_t i = 0;
    const __m128i nl = _mm_set1_epi8('\n');
    for (; i + 64 <= n; i += 64) {
        const uint64_t m0 = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)(p + i)), nl));
        const uint64_t m1 = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)(p + i + 16)), nl));
        const uint64_t m2 = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)(p + i + 32)), nl));
        const uint64_t m3 = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)(p + i + 48)), nl));
        c += (uint64_t)__builtin_popcountll(m0 | m1 << 16 | m2 << 32 | m3 << 48);
    }
    for (; i < n; ++i) c += p[i] == '\n';
    return c;
}

// newline counts of blocks [b0, b0 + nblk) of nb, read with pread (no mapping: the
// page cache copies straight into a per-thread buffer)
std::vector<uint64_t> count_blocks(const std::string& path, uint64_t nb, uint64_t b0, uint64_t nblk, int threads) {
    Fd f(path);
    const uint64_t size = f.size();
    std::vector<uint64_t> out(nblk, 0);
    std::atomic<uint64_t> next{0};
    std::exception_ptr err;
    std::mutex em;
    auto work = [&] {
        std::vector<char> buf(4u << 20);
        try {
            for (uint64_t j; (j = next.fetch_add(1)) < nblk;) {
                uint64_t a = block_at(size, nb, b0 + j);
                const uint64_t e = block_at(size, nb, b0 + j + 1);
                uint64_t c = 0;
                while (a < e) {
                    const ssize_t got = pread(f.fd, buf.data(), (size_t)std::min<uint64_t>(buf.size(), e - a), (off_t)a);
                    if (got <= 0) throw std::runtime_error("read failed: " + path);
                    c += count_nl(buf.data(), (size_t)got);
                    a += (uint64_t)got;
                }
                out[j] = c;
            }
        } catch (...) {
            std::lock_guard<std::mutex> g(em);
            if (!err) err = std::current_exception();
        }
    };
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(1, threads), nblk));
    std::vector<std::thread> ws;
    for (int t = 1; t < T; ++t) ws.emplace_back(work);
    work();
    for (auto& w : ws) w.join();
    if (err) std::rethrow_exception(err);
    return out;
}

// byte offset just past newline number k (1-based) of a file whose nb blocks hold `lines`
uint64_t after_newline(const std::string& path, const std::vector<uint64_t>& lines, uint64_t k) {
    Fd f(path);
    const uint64_t size = f.size(), nb = lines.size();
    uint64_t before = 0, b = 0;
    while (b < nb && before + lines[b] < k) before += lines[b++];
    if (b == nb) throw std::runtime_error(path + ": fewer lines than the part plan needs");
    uint64_t a = block_at(size, nb, b);
    const uint64_t e = block_at(size, nb, b + 1);
    uint64_t want = k - before;
    std::vector<char> buf(1u << 20);
    while (a < e) {
        const ssize_t got = pread(f.fd, buf.data(), (size_t)std::min<uint64_t>(buf.size(), e - a), (off_t)a);
        if (got <= 0) throw std::runtime_error("read failed: " + path);
        for (ssize_t i = 0; i < got; ++i)
            if (buf[(size_t)i] == '\n' && --want == 0) return a + (uint64_t)i + 1;
        a += (uint64_t)got;
    }
    throw std::runtime_error(path + ": newline count changed while planning");
}

// records of a plain four-line FASTQ from its block counts (a last line without '\n'
// counts; empty lines at the end do not, as kseq skips them); UINT64_MAX when the line
// count does not fit four lines a record (the file is then planned by records)
uint64_t records_of(const std::string& path, const std::vector<uint64_t>& lines) {
    Fd f(path);
    const uint64_t size = f.size();
    uint64_t n = 0;
    for (uint64_t c : lines) n += c;
    if (size) {
        char tail[256];
        const size_t k = (size_t)std::min<uint64_t>(size, sizeof tail);
        if (pread(f.fd, tail, k, (off_t)(size - k)) != (ssize_t)k) throw std::runtime_error("read failed: " + path);
        if (tail[k - 1] != '\n') {
            ++n;
        } else {
            size_t j = k - 1;                   // "\n\n...": every '\n' after the first ends an empty line
            while (j > 0 && (tail[j - 1] == '\n' || tail[j - 1] == '\r') && n > 0) {
                if (tail[j - 1] == '\n') --n;
                --j;
            }
        }
    }
    return n % 4 ? UINT64_MAX : n / 4;
}

bool check_record_start(const std::string& path, uint64_t off) {
    Fd f(path);
    char c = 0;
    return pread(f.fd, &c, 1, (off_t)off) == 1 && c == '@';
}

bool is_gzip(const std::string& path) {
    Fd f(path);
    unsigned char m[2] = {0, 0};
    return pread(f.fd, m, 2, 0) == 2 && m[0] == 0x1f && m[1] == 0x8b;
}

// records of a file as kseq++ reads them (FastxReader): gzip, wrapped lines, FASTA
uint64_t count_records_kseq(const std::string& path) {
    FastxReader rd(path);
    Record r;
    uint64_t n = 0;
    while (rd.next(r)) ++n;
    return n;
}

void part_bounds(PartPlan& pl) {
    pl.n_chunks = (pl.total_records + pl.chunk_size - 1) / pl.chunk_size;
    pl.first_chunk = pl.n_chunks * (uint64_t)pl.rank / (uint64_t)pl.world;
    pl.end_chunk = pl.n_chunks * (uint64_t)(pl.rank + 1) / (uint64_t)pl.world;
    pl.first_record = std::min(pl.total_records, pl.first_chunk * pl.chunk_size);
    pl.n_records = std::min(pl.total_records, pl.end_chunk * pl.chunk_size) - pl.first_record;
}

}  // namespace

std::vector<uint64_t> count_part_lines(const std::string& path, int rank, int world, int threads) {
    if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("bad rank/world");
    if (is_gzip(path)) return std::vector<uint64_t>(kPartBlocks, 0);   // planned by records: not used
    return count_blocks(path, (uint64_t)world * kPartBlocks, (uint64_t)rank * kPartBlocks, kPartBlocks, threads);
}

PartPlan plan_part(const std::string& p1, const std::string& p2, int rank, int world, size_t chunk_size,
                   std::vector<uint64_t> lines1, std::vector<uint64_t> lines2, int threads) {
    if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("bad rank/world");
    const uint64_t nb = (uint64_t)world * kPartBlocks;
    const bool gz1 = is_gzip(p1), gz2 = !p2.empty() && is_gzip(p2);
    if (lines1.empty() && !gz1) lines1 = count_blocks(p1, nb, 0, nb, threads);
    if (!p2.empty() && lines2.empty() && !gz2) lines2 = count_blocks(p2, nb, 0, nb, threads);
    if ((!gz1 && lines1.size() != nb) || (!p2.empty() && !gz2 && lines2.size() != nb))
        throw std::runtime_error("part plan: expected world * 64 block counts per file");
    PartPlan pl;
    pl.rank = rank;
    pl.world = world;
    pl.chunk_size = std::max<size_t>(1, chunk_size);
    // the same decision on every rank: it rests on the file's first bytes and on the
    // all-gathered counts only
    uint64_t n1 = gz1 ? UINT64_MAX : records_of(p1, lines1);
    uint64_t n2 = p2.empty() ? 0 : gz2 ? UINT64_MAX : records_of(p2, lines2);
    pl.by_record1 = n1 == UINT64_MAX;
    pl.by_record2 = !p2.empty() && n2 == UINT64_MAX;
    {
        std::thread t2;
        std::exception_ptr e2;
        if (pl.by_record2) t2 = std::thread([&] { try { n2 = count_records_kseq(p2); } catch (...) { e2 = std::current_exception(); } });
        if (pl.by_record1) n1 = count_records_kseq(p1);
        if (t2.joinable()) t2.join();
        if (e2) std::rethrow_exception(e2);
    }
    pl.total_records = n1;
    if (!p2.empty() && n2 != pl.total_records) throw std::runtime_error("read files have different record counts");
    part_bounds(pl);
    if (pl.n_records) {
        auto offset = [&](const std::string& p, bool by_record, const std::vector<uint64_t>& lines) -> uint64_t {
            if (by_record) return pl.first_record;
            const uint64_t off = pl.first_record ? after_newline(p, lines, 4 * pl.first_record) : 0;
            if (!check_record_start(p, off))
                throw std::runtime_error(p + ": no FASTQ record starts at byte " + std::to_string(off) +
                                         " (a rank's part of an uncompressed file needs the plain four-line layout)");
            return off;
        };
        pl.offset1 = offset(p1, pl.by_record1, lines1);
        if (!p2.empty()) pl.offset2 = offset(p2, pl.by_record2, lines2);
    }
    return pl;
}

void validate_part(const std::string& p1, const std::string& p2, const PartPlan& plan) {
    auto bad = [](const std::string& why) { throw std::runtime_error("inconsistent part: " + why); };
    if (plan.world < 1 || plan.rank < 0 || plan.rank >= plan.world) bad("rank/world");
    if (plan.chunk_size < 1) bad("chunk size");
    PartPlan want = plan;
    part_bounds(want);
    if (want.n_chunks != plan.n_chunks || want.first_chunk != plan.first_chunk || want.end_chunk != plan.end_chunk)
        bad("chunks [" + std::to_string(plan.first_chunk) + ", " + std::to_string(plan.end_chunk) + ") of " +
            std::to_string(plan.n_chunks) + " for rank " + std::to_string(plan.rank) + " of " +
            std::to_string(plan.world) + " over " + std::to_string(plan.total_records) + " records");
    if (want.first_record != plan.first_record || want.n_records != plan.n_records)
        bad("records [" + std::to_string(plan.first_record) + ", +" + std::to_string(plan.n_records) +
            ") for its chunks");
    if (!plan.n_records) return;
    auto check = [&](const std::string& p, bool by_record, uint64_t off) {
        if (by_record ? off != plan.first_record : !check_record_start(p, off))
            bad(p + ": no record " + std::to_string(plan.first_record) + " at " + (by_record ? "record " : "byte ") +
                std::to_string(off));
    };
    check(p1, plan.by_record1, plan.offset1);
    if (!p2.empty()) check(p2, plan.by_record2, plan.offset2);
}

std::unique_ptr<ReadSource> open_fastq_part_source(const std::string& p1, const std::string& p2, const PartPlan& plan) {
    return std::unique_ptr<ReadSource>(new PartSource(p1, p2, plan));
}

std::unique_ptr<ReadSource> make_vector_source(const std::vector<Record>* r1, const std::vector<Record>* r2,
                                               size_t chunk_size) {
    return std::unique_ptr<ReadSource>(new VectorSource(r1, r2, chunk_size));
}

std::unique_ptr<ReadSource> make_interleaved_vector_source(const std::vector<Record>* recs, size_t chunk_size) {
    return std::unique_ptr<ReadSource>(new InterleavedVectorSource(recs, chunk_size));
}

std::unique_ptr<ReadSource> open_fastq_source(const std::string& path1, const std::string& path2, bool interleaved,
                                              size_t chunk_size) {
    return std::unique_ptr<ReadSource>(new FastqSource(path1, path2, interleaved, chunk_size));
}

}  // namespace rsa
