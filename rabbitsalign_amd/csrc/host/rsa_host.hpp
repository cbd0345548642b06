// rsa_host.hpp -- host side of the MI355X seed-and-extend path.
//
// Restates, byte-exactly, the reference's host logic around the hot path
// (mapping decisions src/aln.cpp, chunk pipeline src/pc.cpp, SAM src/sam.cpp,
// CIGAR src/cigar.{hpp,cpp}, FASTA src/refs.cpp, .sti src/index.cpp).  The
// hot path itself (seeding, find_nams, SW extension) is reached only through
// the Engine interface; the product engine is the HIP C-ABI (include/rsa_gpu.h).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <random>
#include <stdexcept>
#include <string>
#include <string_view>
#include <atomic>
#include <vector>

#include "../../../include/rsa_gpu.h"

namespace rsa {

// ---------------------------------------------------------------- CIGAR ---
enum CigarOp : uint8_t { C_M = 0, C_I = 1, C_D = 2, C_N = 3, C_S = 4, C_H = 5, C_P = 6, C_EQ = 7, C_X = 8 };

// The std::vector<uint32_t> subset a CIGAR needs, with the first kInline ops
// stored in the object: a read's alignments (usually a handful of =/X/S ops)
// are built, copied and moved without touching the heap.
class OpVec {
public:
    static constexpr uint32_t kInline = 12;
    OpVec() = default;
    OpVec(const OpVec& o) { copy_from(o); }
    OpVec(OpVec&& o) noexcept { steal(o); }
    OpVec& operator=(const OpVec& o) {
        if (this != &o) copy_from(o);
        return *this;
    }
    OpVec& operator=(OpVec&& o) noexcept {
        if (this != &o) { release(); steal(o); }
        return *this;
    }
    ~OpVec() { release(); }
    bool empty() const { return n_ == 0; }
    size_t size() const { return n_; }
    uint32_t* data() { return p_ ? p_ : buf_; }
    const uint32_t* data() const { return p_ ? p_ : buf_; }
    uint32_t* begin() { return data(); }
    uint32_t* end() { return data() + n_; }
    const uint32_t* begin() const { return data(); }
    const uint32_t* end() const { return data() + n_; }
    uint32_t& operator[](size_t i) { return data()[i]; }
    uint32_t operator[](size_t i) const { return data()[i]; }
    uint32_t& back() { return data()[n_ - 1]; }
    uint32_t back() const { return data()[n_ - 1]; }
    void clear() { n_ = 0; }
    void reserve(size_t c) { if (c > cap()) grow(c); }
    void push_back(uint32_t v) {
        if (n_ == cap()) grow(2 * (size_t)cap());
        data()[n_++] = v;
    }
    template <class It> void assign(It first, It last) {
        const size_t n = (size_t)(last - first);
        n_ = 0;
        reserve(n);
        uint32_t* d = data();
        for (size_t i = 0; i < n; ++i) d[i] = (uint32_t)first[i];
        n_ = (uint32_t)n;
    }
private:
    uint32_t cap() const { return p_ ? cap_ : kInline; }
    void grow(size_t c) {
        uint32_t* q = new uint32_t[c];
        memcpy(q, data(), sizeof(uint32_t) * n_);
        delete[] p_;
        p_ = q;
        cap_ = (uint32_t)c;
    }
    void release() { delete[] p_; p_ = nullptr; n_ = 0; }
    // inline contents move as one fixed-size block (no libc memcpy call for a
    // variable length; the bytes past n_ are never read)
    void copy_from(const OpVec& o) {
        if (!o.p_ && !p_) {
            memcpy(buf_, o.buf_, sizeof(buf_));
            n_ = o.n_;
        } else {
            n_ = 0;
            assign(o.begin(), o.end());
        }
    }
    void steal(OpVec& o) {
        n_ = o.n_;
        if (o.p_) { p_ = o.p_; cap_ = o.cap_; o.p_ = nullptr; }
        else memcpy(buf_, o.buf_, sizeof(buf_));
        o.n_ = 0;
    }
    uint32_t* p_ = nullptr;                     // heap storage once past kInline
    uint32_t n_ = 0, cap_ = 0;
    uint32_t buf_[kInline];
};

struct Cigar {                                  // src/cigar.hpp:23-93
    OpVec ops;
    bool empty() const { return ops.empty(); }
    void push(uint32_t op, uint32_t len) {
        if (ops.empty() || (ops.back() & 0xf) != op) ops.push_back(len << 4 | op);
        else ops.back() += len << 4;
    }
    void append(const Cigar& o) { for (uint32_t x : o.ops) push(x & 0xf, x >> 4); }
    Cigar to_m() const;
    void to_string(std::string& out) const;
    void to_m_string(std::string& out) const;   // to_m().to_string(out) without the temporary
};

// ---------------------------------------------------------------- types ---
using Nam = rsa_nam;                            // src/nam.hpp:11-38

struct AlignmentInfo {                          // src/aligner.hpp:20-30
    Cigar cigar;
    unsigned edit_distance = 0, ref_start = 0, ref_end = 0, query_start = 0, query_end = 0;
    int sw_score = 0;
    bool no_shared = false;                     // a job with SwJob::shared_k: has_shared_substring was false
    int ref_span() const { return (int)(ref_end - ref_start); }
};

struct Alignment {                              // src/sam.hpp:12-25
    int ref_id = 0;
    int ref_start = 0;
    Cigar cigar;
    int edit_distance = 0;
    int global_ed = 0;
    int score = 0;
    int length = 0;
    bool is_rc = false;
    bool is_unaligned = false;
    bool gapped = false;
};

// std::vector<bool> semantics for the per-pair flag lists of AlignTmpRes,
// inline for up to 128 entries (2 x max_tries + 2 with the default -M 20), so
// a pair's bookkeeping does not allocate; longer lists spill to the heap.
class BitVec {
public:
    void push_back(bool b) {
        if (n_ < 128) { if (b) w_[n_ >> 6] |= 1ull << (n_ & 63); else w_[n_ >> 6] &= ~(1ull << (n_ & 63)); }
        else spill_.push_back(b);
        n_++;
    }
    bool operator[](size_t i) const { return i < 128 ? (w_[i >> 6] >> (i & 63)) & 1 : spill_[i - 128]; }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    void clear() { n_ = 0; spill_.clear(); }
private:
    uint64_t w_[2] = {0, 0};
    size_t n_ = 0;
    std::vector<bool> spill_;
};

struct AlignTmpRes {                            // src/sam.hpp:27-45
    int type = 0;
    int mapq1 = 0, mapq2 = 0;
    int type4_loop_size = 0;
    BitVec is_extend_seed, consistent_nam, is_read1;
    std::vector<Nam> type4_nams, todo_nams;
    BitVec done_align;
    std::vector<Alignment> align_res;
    // empty again, keeping the vectors' capacity (the pipeline recycles chunks)
    void reset() {
        type = 0; mapq1 = mapq2 = 0; type4_loop_size = 0;
        is_extend_seed.clear(); consistent_nam.clear(); is_read1.clear(); done_align.clear();
        type4_nams.clear(); todo_nams.clear(); align_res.clear();
    }
};

struct Details {                                // src/sam.hpp:60-67
    bool nam_rescue = false;
    uint64_t nams = 0, nam_inconsistent = 0, mate_rescue = 0, tried_alignment = 0, gapped = 0;
};

struct AlignmentParameters { int match = 2, mismatch = 8, gap_open = 12, gap_extend = 1, end_bonus = 10; };

struct MappingParameters {                      // src/aln.hpp:58-74
    int r = 150;
    int max_secondary = 0;
    float dropoff_threshold = 0.5f;
    int rescue_level = 2;
    int max_tries = 20;
    int rescue_cutoff = 0;
    bool cigar_eqx = false;
    bool output_unmapped = true;
    bool details = false;
};

struct InsertSizeDistribution {                 // src/aln.hpp:79-90, aln.cpp:1880-1903
    float sample_size = 1, mu = 300, sigma = 100, V = 10000, SSE = 10000;
    void update(int dist);
    bool frozen() const { return !(sample_size < 400); }
};

struct AlignmentStatistics {
    uint64_t n_reads = 0, tot_aligner_calls = 0, tot_rescued = 0, tot_all_tried = 0, inconsistent_nams = 0,
             nam_rescue = 0;
    void add(const Details& d) {
        nam_rescue += d.nam_rescue; tot_rescued += d.mate_rescue; tot_all_tried += d.tried_alignment;
        inconsistent_nams += d.nam_inconsistent;
    }
    void add(const AlignmentStatistics& o) {
        n_reads += o.n_reads; tot_aligner_calls += o.tot_aligner_calls; tot_rescued += o.tot_rescued;
        tot_all_tried += o.tot_all_tried; inconsistent_nams += o.inconsistent_nams; nam_rescue += o.nam_rescue;
    }
};

struct Record { std::string name, comment, seq, qual; };   // klibpp::KSeq fields used

// A record as the pipeline and the SAM writer read it: views into storage that
// outlives the chunk (a mapped FASTQ file, a chunk's parsed records, a caller's
// Record vector).  Chunks of the mapped 4-line layout are never copied.
struct RecView {
    std::string_view name, comment, seq, qual;
    RecView() = default;
    RecView(const Record& r) : name(r.name), comment(r.comment), seq(r.seq), qual(r.qual) {}   // NOLINT: implicit
};

std::string reverse_complement(std::string_view s);
void reverse_complement_into(std::string_view s, char* out);   // out holds s.size() bytes
void reverse_into(std::string_view s, char* out);              // plain byte reversal

// Read (src/revcomp.hpp:41-55): a sequence and its reverse complement.  The
// pipeline computes the rc once per read per chunk and hands out views.
// GPU site checks of one read's NAM list (rsa_nam_site, include/rsa_gpu.h),
// indexed by nam_id; empty for the CPU engines (the host computes them)
struct SiteView {
    const rsa_nam_site* sites = nullptr;        // at each NAM's nam_id
    size_t n = 0;
    int64_t read_len = 0;
    const uint16_t* pool = nullptr;             // mismatch positions
    // the check of the NAM the host holds: its id, and its query span as found or reversed
    const rsa_nam_site* find(const rsa_nam& nam) const {
        if (!sites || nam.nam_id < 0 || (size_t)nam.nam_id >= n) return nullptr;
        const rsa_nam_site& s = sites[nam.nam_id];
        const bool as_found = nam.query_start == s.orig_query_start && nam.query_end == s.orig_query_end;
        const bool reversed = nam.query_start == read_len - s.orig_query_end &&
                              nam.query_end == read_len - s.orig_query_start;
        return (as_found || reversed) ? &s : nullptr;
    }
};

// A read's NAM list as part() works on it: the engine's download sorted in place
// (RSA_NAMS_BY_SCORE) or a vector; shuffled and reversed in place.
struct NamSpan {
    Nam* p = nullptr;
    size_t n = 0;
    NamSpan() = default;
    NamSpan(Nam* p_, size_t n_) : p(p_), n(n_) {}
    NamSpan(std::vector<Nam>& v) : p(v.data()), n(v.size()) {}
    Nam* begin() const { return p; }
    Nam* end() const { return p + n; }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
    Nam& operator[](size_t i) const { return p[i]; }
};

struct Read {
private:
    std::string own_;                           // rc when computed by this object
public:
    std::string_view seq;
    std::string_view rc;
    SiteView site;
    explicit Read(const std::string& s) : own_(reverse_complement(s)), seq(s), rc(own_) {}
    Read(std::string_view s, std::string_view rc_) : seq(s), rc(rc_) {}
    Read(const Read&) = delete;
    Read& operator=(const Read&) = delete;
    size_t size() const { return seq.size(); }
};
void to_uppercase(std::string& s);             // refs.cpp:10-16 (c & ~32)

struct References {                             // src/refs.hpp
    std::vector<std::string> names;
    std::vector<std::string> seqs;
    std::vector<uint64_t> offsets;              // concatenation offsets [n+1]
    std::string concat;                         // all contigs back to back (device upload)
    size_t size() const { return seqs.size(); }
    static References from_fasta(const std::string& path);
    // The host pipeline reads reference windows at random (NAM checks, Hamming
    // windows, SW job windows); make_hot() copies the contigs into one mapping
    // advised for transparent huge pages, so those reads stop missing the TLB.
    std::shared_ptr<char> hot;
    std::vector<std::string_view> views;        // contig i inside `hot`
    void make_hot();
    std::string_view seq(size_t i) const { return views.empty() ? std::string_view(seqs[i]) : views[i]; }
};

struct IndexParameters {                        // src/indexparameters.hpp
    int canonical_read_length = 150, k = 20, s = 16, t = 3, l = 1, u = 7, q = 255, max_dist = 80;
    unsigned w_min = 0, w_max = 0;
    static IndexParameters from_read_length(int read_length, int k = INT32_MIN, int s = INT32_MIN,
                                            int l = INT32_MIN, int u = INT32_MIN, int c = INT32_MIN,
                                            int max_seed_len = INT32_MIN);
    void finalize();
    bool operator==(const IndexParameters& o) const;
    std::string filename_extension() const;
};

struct StiIndex {                               // .sti contents (src/index.cpp:73-132)
    IndexParameters params;
    int filter_cutoff = 0;
    int bits = 0;
    std::vector<rsa_ref_randstrobe> randstrobes;
    std::vector<uint64_t> bucket_starts;
    void read(const std::string& path);
    void write(const std::string& path) const;
    void build(const References& refs, const IndexParameters& p, int bits_override, float f, int threads);
    // how the index was made: on the GPU (rsa_index_build_run) with its phase times
    // (upload, syncmers, randstrobes, sort, buckets, total; ms), or on the host
    bool built_on_device = false;
    double device_build_ms[6] = {0, 0, 0, 0, 0, 0};
    uint64_t replayed_segments = 0;
    // entries equal in (hash, position) to their predecessor: their order is pdqsort's
    // (sti_order.hpp), replayed by both builds when this is not 0
    uint64_t position_ties = 0;
    double ms_tie_replay = 0;                   // GPU build: host replay of the tie order, incl. transfers
    // a GPU build kept in HBM (no host copy): the GPU engine adopts it; a host
    // copy is downloaded only when something needs one (.sti write, a CPU engine)
    struct DeviceBuild {
        void* handle = nullptr;                 // rsa_index_build*, until an engine adopts it
        void (*release)(void*) = nullptr;
        ~DeviceBuild() { if (handle && release) release(handle); }
    };
    std::shared_ptr<DeviceBuild> device_build;
    uint64_t n_device = 0;                      // entries of the device-only index
    uint64_t size() const { return randstrobes.empty() ? n_device : randstrobes.size(); }
    bool host_copy() const { return !randstrobes.empty() || n_device == 0; }
};

// StrobemerIndex::populate as used by the CLI and the C API.  The host build
// (StiIndex::build) by default; the GPU engine's translation unit
// (engine_gpu.cpp) replaces it with the HIP build, so the product makes its
// index on the device it maps on.
// host_copy = false lets a GPU build stay in HBM for the engine to adopt.
void build_default_index(StiIndex& idx, const References& refs, const IndexParameters& p, int bits_override, float f,
                         int threads, int device, bool host_copy = true);

// --------------------------------------------------------------- engine ---
// Storage of engine outputs that an engine may fill by DMA: an allocator that is
// malloc by default and the engine's page-locked host memory when the engine
// installs it (the GPU engine copies its NAM / site output straight into it
// instead of through a staging buffer).  New elements are left uninitialised.
struct HostAllocFns {
    void* (*alloc)(size_t);
    void (*free)(void*);
};
template <class T> struct HostAlloc {
    using value_type = T;
    const HostAllocFns* fns = nullptr;          // nullptr: malloc / free
    HostAlloc() = default;
    explicit HostAlloc(const HostAllocFns* f) : fns(f) {}
    template <class U> HostAlloc(const HostAlloc<U>& o) noexcept : fns(o.fns) {}
    template <class U> struct rebind { using other = HostAlloc<U>; };
    T* allocate(size_t n) {
        void* p = fns ? fns->alloc(n * sizeof(T)) : std::malloc(n * sizeof(T));
        if (!p) throw std::bad_alloc();
        return (T*)p;
    }
    void deallocate(T* p, size_t) noexcept { if (fns) fns->free(p); else std::free(p); }
    template <class U> void construct(U* p) noexcept { ::new ((void*)p) U; }
    template <class U, class... A> void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
    using propagate_on_container_move_assignment = std::true_type;
    using propagate_on_container_copy_assignment = std::true_type;
    using propagate_on_container_swap = std::true_type;
    template <class U> bool operator==(const HostAlloc<U>& o) const { return fns == o.fns; }
    template <class U> bool operator!=(const HostAlloc<U>& o) const { return fns != o.fns; }
};

struct SeedBatchOut {
    std::vector<Nam, HostAlloc<Nam>> nams;
    std::vector<uint64_t> offsets;              // [n+1]
    std::vector<float> nonrep;
    std::vector<uint8_t> rescued;
    std::vector<rsa_nam_site, HostAlloc<rsa_nam_site>> sites;   // one per NAM when the engine computes the site checks
    std::vector<uint16_t, HostAlloc<uint16_t>> mm_pool;         // their mismatch positions
    // empty, keeping the storage (page-locked storage is expensive to allocate)
    void clear() {
        nams.clear(); offsets.clear(); nonrep.clear(); rescued.clear(); sites.clear(); mm_pool.clear();
    }
    // site view of read r's NAM list (empty without site checks)
    SiteView site_view(size_t r, size_t read_len) const {
        SiteView v;
        if (sites.empty()) return v;
        v.sites = sites.data() + offsets[r];
        v.n = offsets[r + 1] - offsets[r];
        v.read_len = (int64_t)read_len;
        v.pool = mm_pool.data();
        return v;
    }
    // the engine returned lists of <= 16 NAMs already in std::sort(by_score) order
    bool by_score = false;
};

struct SwJob {                                  // query host bytes vs reference window
    std::string_view query;                     // into the chunk's read / reverse complement, valid until store
    int ref_id;
    uint32_t ref_start, ref_len;
    // > 0: a mate rescue whose has_shared_substring(query, window, shared_k) test
    // (aln.cpp:1058) the engine makes (AlignmentInfo::no_shared); 0: none
    int shared_k = 0;
};
// has_shared_substring (aln.cpp:1000-1013)
bool has_shared_substring(std::string_view read_seq, std::string_view ref_seq, int k);
// the engine side of SwJob::shared_k for engines that align on the host: the test, and
// the SW skipped when it fails
inline bool shared_check_fails(const SwJob& j, std::string_view window) {
    return j.shared_k > 0 && !has_shared_substring(j.query, window, j.shared_k);
}

class Engine {
public:
    virtual ~Engine() = default;
    virtual const char* name() const = 0;
    // NAMs (pre-sort order) for every read, as align_*_read_part computes them (aln.cpp:1946-1962)
    virtual void seed(const std::vector<std::string_view>& reads, int rescue_level, unsigned rescue_cutoff,
                      SeedBatchOut& out) = 0;
    // The same for reads already packed back to back (read i at blob[offs[i] ..
    // offs[i] + lens[i])), in memory from io_alloc() -- engines that offer it
    // (io_alloc() != nullptr) take the batch without a packing copy.
    virtual void seed_packed(const char* blob, const uint64_t* offs, const uint32_t* lens, size_t n,
                             int rescue_level, unsigned rescue_cutoff, SeedBatchOut& out) {
        (void)blob; (void)offs; (void)lens; (void)n; (void)rescue_level; (void)rescue_cutoff; (void)out;
        throw std::runtime_error("seed_packed: not supported by this engine");
    }
    // allocator of host buffers this engine can DMA from / to (nullptr: none)
    virtual const HostAllocFns* io_alloc() const { return nullptr; }
    // Aligner::align for every job (aligner.cpp:114-210)
    virtual void extend(const std::vector<SwJob>& jobs, const AlignmentParameters& p,
                        std::vector<AlignmentInfo>& out) = 0;
    // device kernel timings/counters (GPU engine only)
    virtual bool kernel_stats(rsa_kernel_stats*) { return false; }
    // true when seed/extend run on a device and the calling thread only waits
    virtual bool offloads() const { return false; }
    virtual void reset_kernel_stats() {}
    // the host copy of an index the engine holds on its device (GPU engine only)
    virtual bool download_index(StiIndex&) { return false; }
    // the scores hamming_align runs with, for an engine that computes it with the site
    // checks (GPU engine: RSA_SITE_ALIGNED); set before the first seeding call
    virtual void set_alignment_params(const AlignmentParameters&) {}
};

// GPU engine over the C-ABI (engine_gpu.cpp)
std::unique_ptr<Engine> make_gpu_engine(const References& refs, const StiIndex& index, int device);

class Sam;

// ------------------------------------------------------------- mapping ---
struct MapContext {
    const References& refs;
    const IndexParameters& iparams;
    const AlignmentParameters& aparams;
    const MappingParameters& mparams;
};

// part / last split of src/aln.cpp:1927-2306 (PE) and 2372-2467 (SE).  `nams`
// are the pre-sort NAM lists of both mates (already through find_nams/rescue).
// sorted: nams[m] are already in std::sort(by_score) order (load_sorted_nams)
void align_PE_read_part(AlignTmpRes& res, const RecView& r1, const RecView& r2, const Read& read1, const Read& read2,
                        NamSpan nams[2],
                        const bool rescued[2], AlignmentStatistics& stats, InsertSizeDistribution& isize,
                        const MapContext& mc, std::minstd_rand& rng, bool sorted = false);
// dst = src[0 .. n) in the order std::sort(by_score) gives (aln.cpp:1962-1964), in one gather
void load_sorted_nams(std::vector<Nam>& dst, const Nam* src, size_t n);
// the same order in place: <= 16 NAMs by the insertion sort's rule, longer lists by std::sort
void sort_nams_by_score(NamSpan v);
void align_PE_read_last(AlignTmpRes& res, const RecView& r1, const RecView& r2, const Read& read1, const Read& read2,
                        Sam& sam,
                        AlignmentStatistics& stats, const InsertSizeDistribution& isize, const MapContext& mc,
                        std::minstd_rand& rng);
void align_SE_read_part(AlignTmpRes& res, const RecView& r, const Read& read, std::vector<Nam>& nams, bool rescued,
                        AlignmentStatistics& stats, const MapContext& mc, std::minstd_rand& rng);
void align_SE_read_last(AlignTmpRes& res, const RecView& r, const Read& read, Sam& sam, AlignmentStatistics& stats,
                        const MapContext& mc, std::minstd_rand& rng);

// SW jobs of a finished part() (pc.cpp:1604-1669 get_str) and storing their results (pc.cpp:1789-1844)
void collect_jobs_pe(AlignTmpRes& res, const RecView& r1, const RecView& r2, const Read& read1, const Read& read2,
                     const MapContext& mc, float mu, float sigma, std::vector<SwJob>& jobs);
size_t store_results_pe(AlignTmpRes& res, const Read& read1, const Read& read2, const MapContext& mc, float mu,
                        float sigma, std::vector<AlignmentInfo>& infos, size_t pos);
void collect_jobs_se(AlignTmpRes& res, const Read& read, const MapContext& mc, std::vector<SwJob>& jobs);
size_t store_results_se(AlignTmpRes& res, const Read& read, const MapContext& mc,
                        std::vector<AlignmentInfo>& infos, size_t pos);

// The pieces of those two that are pure arithmetic on one job, also used by the
// hand-derived host cases (tests/host_cases.py through bin/rsa_host_cases):
// extension_window: the reference window [start, start + len) of an extension job
// (pc.cpp:214-242); rescue_mate_window: of a mate rescue job (pc.cpp:333-368, with
// its int / size_t / float arithmetic); extension_alignment / rescue_alignment:
// the Alignment stored from the aligner's result (pc.cpp:177-212, 291-331).
void extension_window(const Nam& nam, size_t read_len, size_t contig_len, uint32_t& start, uint32_t& len);
void rescue_mate_window(const Nam& nam, size_t read_len, float mu, float sigma, size_t contig_len, uint32_t& start,
                        uint32_t& len);
void extension_alignment(const Nam& nam, size_t read_len, AlignmentInfo& info, Alignment& a);
void rescue_alignment(const Nam& nam, size_t read_len, float mu, float sigma, size_t contig_len, AlignmentInfo& info,
                      Alignment& a);

// Order-sensitive digest of a SAM body, independent of how it is chunked:
// D = sum_k line_hash(line_k) * P^(N-1-k) mod 2^64 over the N lines (without '\n').
// line_hash runs four independent 64-bit multiply-rotate lanes over 32-byte
// blocks (about 0.3 cycles/byte) so digesting stays off the critical path.
struct SamDigest {
    static constexpr uint64_t P = 0x100000001b3ULL;
    uint64_t h = 0, lines = 0;
    static uint64_t pow(uint64_t b, uint64_t e) {
        uint64_t r = 1;
        for (; e; e >>= 1, b *= b) if (e & 1) r *= b;
        return r;
    }
    static inline uint64_t rd64(const char* p) { uint64_t w; std::memcpy(&w, p, 8); return w; }
    static inline uint64_t mix(uint64_t a, uint64_t w) {
        a ^= w * 0xC2B2AE3D27D4EB4FULL;
        return ((a << 31) | (a >> 33)) * 0x9E3779B185EBCA87ULL;
    }
    static uint64_t line_hash(const char* p, size_t n) {
        uint64_t a = 0x9E3779B97F4A7C15ULL ^ n, b = 0x165667B19E3779F9ULL, c = 0x85EBCA77C2B2AE63ULL,
                 d = 0x27D4EB2F165667C5ULL;
        size_t i = 0;
        for (; i + 32 <= n; i += 32) {
            a = mix(a, rd64(p + i)); b = mix(b, rd64(p + i + 8));
            c = mix(c, rd64(p + i + 16)); d = mix(d, rd64(p + i + 24));
        }
        for (; i + 8 <= n; i += 8) a = mix(a, rd64(p + i));
        uint64_t t = 0;
        std::memcpy(&t, p + i, n - i);
        uint64_t h = mix(a, t) ^ ((b << 17) | (b >> 47)) ^ ((c << 29) | (c >> 35)) ^ ((d << 43) | (d >> 21));
        h ^= h >> 33; h *= 0xff51afd7ed558ccdULL; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ULL; h ^= h >> 33;
        return h;
    }
    static SamDigest of(const std::string& s) { return of(s.data(), s.size()); }
    static SamDigest of(const char* p, size_t n) {
        SamDigest d;
        const char* e = p + n;
        while (p < e) {
            const char* nl = (const char*)std::memchr(p, '\n', (size_t)(e - p));
            if (!nl) break;                      // an unterminated tail is not a line
            d.h = d.h * P + line_hash(p, (size_t)(nl - p));
            d.lines++;
            p = nl + 1;
        }
        return d;
    }
    void append(const SamDigest& o) { h = h * pow(P, o.lines) + o.h; lines += o.lines; }
};

// --------------------------------------------------------------- SAM -----
std::string sam_header(const References& refs, const std::string& rg_id, const std::vector<std::string>& rg,
                       const std::string& cmd_line);

// SAM text of a chunk.  A vector whose allocator leaves new elements
// uninitialised: a record is written into room reserved with resize() (an upper
// bound of its length) and the unused tail is cut off again, without the
// zero fill a std::string::resize would spend on every record.
// Buffers of 2 MB and more (a chunk's SAM text, its reverse complements) are their own
// anonymous mappings advised for transparent huge pages (RSA_HUGE_BUFFERS=0: the heap):
// the formatting stores and the writer's copy into the page cache then walk one TLB
// entry per 2 MB instead of 512.  The chunk buffers are pooled, so the mappings persist.
bool huge_buffers_on();                          // once per process (RSA_HUGE_BUFFERS, default on)
void* huge_buffer_alloc(size_t bytes);          // throws std::bad_alloc
void huge_buffer_free(void* p, size_t bytes);
constexpr size_t kHugeBufferMin = size_t(2) << 20;
template <class T> struct NoInitAlloc : std::allocator<T> {
    template <class U> struct rebind { using other = NoInitAlloc<U>; };
    NoInitAlloc() = default;
    template <class U> NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    template <class U> void construct(U* p) noexcept { ::new ((void*)p) U; }
    template <class U, class... A> void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
    T* allocate(size_t n) {
        if (n * sizeof(T) >= kHugeBufferMin && huge_buffers_on()) return (T*)huge_buffer_alloc(n * sizeof(T));
        return std::allocator<T>::allocate(n);
    }
    void deallocate(T* p, size_t n) {
        if (n * sizeof(T) >= kHugeBufferMin && huge_buffers_on()) huge_buffer_free(p, n * sizeof(T));
        else std::allocator<T>::deallocate(p, n);
    }
};
using SamText = std::vector<char, NoInitAlloc<char>>;

class Sam {                                     // src/sam.hpp:69-120
public:
    Sam(SamText& out, const References& refs, bool eqx, const std::string& rg_id, bool output_unmapped,
        bool details);
    void add(const Alignment& a, const RecView& r, std::string_view rc, uint8_t mapq, bool primary,
             const Details& d);
    void add_pair(const Alignment& a1, const Alignment& a2, const RecView& r1, const RecView& r2,
                  std::string_view rc1, std::string_view rc2, uint8_t mapq1, uint8_t mapq2, bool proper,
                  bool primary, const Details d[2]);
    void add_unmapped(const RecView& r, uint16_t flags = 4);
    void add_unmapped_pair(const RecView& r1, const RecView& r2);
    void add_unmapped_mate(const RecView& r, uint16_t flags, std::string_view mate_ref, uint32_t mate_pos);
    // fold every line into *d as it is written (while it is in cache) instead of a
    // second pass over the chunk's text; same value as SamDigest::of on the text
    void digest_into(SamDigest* d) { digest_ = d; }

private:
    void line_done(const char* p0, const char* p) {
        if (digest_) {
            digest_->h = digest_->h * SamDigest::P + SamDigest::line_hash(p0, (size_t)(p - p0) - 1);
            digest_->lines++;
        }
    }
    void add_record(std::string_view qname, uint16_t flags, std::string_view rname, uint32_t pos, uint8_t mapq,
                    const Cigar& cigar, std::string_view mate_rname, uint32_t mate_pos, int32_t tlen,
                    std::string_view seq, std::string_view seq_rc, std::string_view qual, int ed, int score,
                    const Details& d);
    SamText& out_;
    const References& refs_;
    bool eqx_, output_unmapped_, details_;
    std::string tail_;
    SamDigest* digest_ = nullptr;
};

bool is_proper_pair(const Alignment& a1, const Alignment& a2, float mu, float sigma);

// ------------------------------------------------------------- input -----
class FastxReader {                             // kseq++ record semantics (src/fastq.cpp)
public:
    explicit FastxReader(const std::string& path);
    ~FastxReader();
    bool next(Record& r);
    // every record of a file; read_pair() parses the two mate files on two threads
    static std::vector<Record> read_all(const std::string& path);
    static void read_pair(const std::string& p1, const std::string& p2, std::vector<Record>& r1,
                          std::vector<Record>& r2);
    // the same parser over bytes in memory (the rest of a mapped file after its
    // last record in the plain layout); `mem` must outlive the reader
    FastxReader(const char* mem, size_t len);
private:
    struct Impl;
    std::unique_ptr<Impl> impl_;
};

// ---------------------------------------------------------- read source ---
// One chunk of input as the reference's InputBuffer::read_records hands it out
// (src/pc.cpp:74-107): chunk `index`, up to chunk_size pairs (PE), reads (SE) or
// the pairs of a block of 2 x chunk_size interleaved records.  The views point
// into storage the chunk (`owned`) or the source keeps alive until release().
struct InputChunk {
    size_t index = 0;
    std::vector<RecView> r1, r2;                // pairs (r2 empty for single-end)
    uint64_t singletons = 0;                    // interleaved: unpaired records, read and dropped
    std::vector<Record> owned1, owned2;         // records parsed by the sequential reader
    void clear() {
        r1.clear(); r2.clear(); singletons = 0; owned1.clear(); owned2.clear();
    }
};

// Chunks are asked for in increasing index order (the pipeline claims them in
// order), possibly from different threads; get() blocks until chunk idx is read
// and returns false past the end of the input.  release() hands a chunk's
// storage back once its SAM is written (a mapped file's pages are dropped, so
// resident memory does not grow with the input).
class ReadSource {
public:
    virtual ~ReadSource() = default;
    virtual bool paired() const = 0;
    virtual bool get(size_t idx, InputChunk& out) = 0;
    virtual void release(InputChunk& c) { c.clear(); }
    // the CLI's read-length estimate (main.cpp:254-258, readlen.cpp:16-29) from the
    // source's own first records, before any chunk is taken; sources that are not
    // files have none and give the default profile's 150
    virtual int estimate_read_length() { return 150; }
    // the run failed: get() calls waiting on input return with an error instead of
    // waiting for a producer that may never write again
    virtual void cancel() {}
};

// Records already in memory (rsam_reads, tests): chunks are views into the
// caller's vectors (r2 null: single-end).
std::unique_ptr<ReadSource> make_vector_source(const std::vector<Record>* r1, const std::vector<Record>* r2,
                                               size_t chunk_size);
// Interleaved records in memory: chunk i pairs records [2ci, 2c(i+1)) by same_name.
std::unique_ptr<ReadSource> make_interleaved_vector_source(const std::vector<Record>* recs, size_t chunk_size);
// FASTQ/FASTA files, streamed: one reader thread per file parses blocks of
// records ahead of the pipeline (a bounded number of chunks ahead of the last
// one asked for).  Uncompressed files in the plain 4-line layout are mapped and
// split without copying (records are views into the mapping); gzip, pipes and
// any other layout go through FastxReader (kseq semantics).  path2 empty:
// single-end, or interleaved pairs when `interleaved`.
std::unique_ptr<ReadSource> open_fastq_source(const std::string& path1, const std::string& path2, bool interleaved,
                                              size_t chunk_size);

// ------------------------------------------------------- a rank's part ---
// rank/world mode: one input pair of FASTQ files (plain or gzip),
// mapped by `world` processes (one per GPU).  The records are cut into the same
// chunks of chunk_size pairs a single process maps, so every chunk keeps its
// chunk_index (the minstd_rand seed, pc.cpp:1583); rank r maps chunks
// [r*C/W, (r+1)*C/W) of the C chunks.  Each rank replays the single-worker
// timeline from chunk 0 until the insert-size estimate freezes (its output
// discarded), so it reaches the same frozen estimate; if the estimate is still
// open at the part's end, the next chunk's part() is replayed as well (the last
// chunk is stored with the estimate after it).  Rank r's SAM part holds
// exactly its chunks' records (rank 0's part starts with the header): the parts
// concatenated in rank order are the one-process SAM.
//
// Finding a part's first record needs the record count before it.  Each file is
// cut into world * kPartBlocks equal byte blocks; a rank counts the newlines of its
// own kPartBlocks blocks, the counts of all ranks are exchanged (an all-gather of
// world * kPartBlocks integers per file, done by the caller), and the plan follows:
// record i starts after newline 4i.  With no exchange a rank counts every block.
//
// A file that is not in that layout -- gzip (the reference's usual input, read with
// kseq++: src/fastq.cpp:1-65), wrapped lines, FASTA -- is planned by records instead
// (`by_record`): each rank counts the file's records with the kseq parser and skips
// the records before its part while it streams the file from its start.  The
// block counts of such a file are not used (rsam_part_count returns zeros for gzip).
constexpr int kPartBlocks = 64;
struct PartPlan {
    int rank = 0, world = 1;
    uint64_t chunk_size = 10000;
    uint64_t total_records = 0, n_chunks = 0;    // records (pairs) of the input, chunks of the input
    uint64_t first_chunk = 0, end_chunk = 0;     // this rank's chunks
    uint64_t first_record = 0, n_records = 0;    // this rank's records
    uint64_t offset1 = 0, offset2 = 0;           // byte offset of first_record in each file (record index when by_record)
    bool by_record1 = false, by_record2 = false; // the file is planned by records (see above)
};
// newline counts of rank `rank`'s kPartBlocks blocks of a file cut into world * kPartBlocks
std::vector<uint64_t> count_part_lines(const std::string& path, int rank, int world, int threads);
// the plan from all world * kPartBlocks counts of each file (an empty vector: counted here);
// p2 empty: single-end
PartPlan plan_part(const std::string& p1, const std::string& p2, int rank, int world, size_t chunk_size,
                   std::vector<uint64_t> lines1, std::vector<uint64_t> lines2, int threads);
// throws unless `plan` is a consistent part of these files (chunk and record bounds,
// a record starting at each byte offset)
void validate_part(const std::string& p1, const std::string& p2, const PartPlan& plan);
// the chunks of the plan, streamed (plus chunks 0.. from the file start when the
// paired pipeline replays the insert-size phase)
std::unique_ptr<ReadSource> open_fastq_part_source(const std::string& p1, const std::string& p2, const PartPlan& plan);

// ------------------------------------------------------------ pipeline ---
// called at the start of every pipeline worker thread (profiling hooks; null by default)
extern void (*g_worker_start_hook)();

struct PipelineOptions {
    int threads = 3;
    int chunk_size = 10000;
    std::string rg_id;
    bool digest = false;   // compute PipelineResult::sam_digest (in the workers, in parallel)
    // a rank's part (PartPlan): chunks [first_chunk, end_chunk) are this rank's.  The
    // paired pipeline still runs the chunks before them through part() until the
    // insert-size estimate freezes, and -- when it has not frozen by then -- chunk
    // end_chunk too, whose part() moves the estimate chunk end_chunk - 1 is stored
    // with (pc.cpp:1739-1798); it writes nothing of those
    size_t first_chunk = 0, end_chunk = SIZE_MAX;
};

// --interleaved input (InputBuffer::read_records + distribute_interleaved,
// src/pc.cpp:23-107): the file is read in blocks of 2 * chunk_size records, one
// block per chunk; within a block two consecutive records whose names are the
// same (ignoring /1 on the first and /2 on the second, same_name) form a pair,
// every other record is a singleton.  The reference's paired-end task
// (perform_task_async_pe, pc.cpp:1522-1887) maps only the pairs -- singletons
// are read and dropped -- and a pair split across two blocks is two singletons
// (the lookahead of distribute_interleaved is never set).  Appends the pairs
// of `block` to r1/r2 and returns the number of singletons.
size_t distribute_interleaved(const RecView* block, size_t n, std::vector<RecView>& r1, std::vector<RecView>& r2);
bool same_name(std::string_view n1, std::string_view n2);

// glibc malloc settings for the mapping process (once; library entry points and
// the CLI call it): free memory stays in the heap instead of being trimmed and
// re-faulted, and buffers up to 256 MB come from the heap instead of a fresh
// mmap each time.  The per-chunk work allocates and frees steadily; with glibc's
// defaults that cost 0.93-1.00 core-us a read on the box, with these 0.77-0.87
// (A/B, profiles/r02/ab_malloc.jsonl).  Only memory retention changes.
void tune_malloc();
// ends the pipeline's pooled worker threads and frees its pooled buffers (no mapping
// call may run; the engine that allocated page-locked buffers must still be open)
void release_pipeline_resources();

// thread-summed seconds per phase (instrumentation of the host pipeline)
struct PhaseTimes {
    double seed = 0, extend = 0, part = 0, collect = 0, last = 0, sequential = 0, load = 0, output = 0;
    // since the call started: chunk 0 loaded and seeded; the last chunk's finish began
    // ... its SAM text went to the sink; every worker was done (the sink may still be writing)
    double first_seeded = 0, last_start = 0, last_put = 0, workers_done = 0;
    // the first SAM text reached the writer; the first chunk's extension call began / returned
    double first_out = 0, first_ext_begin = 0, first_ext_end = 0;
    uint64_t replayed = 0;                      // chunks parted only for the insert-size estimate
    void add(const PhaseTimes& o) {
        first_out = std::max(first_out, o.first_out);
        first_ext_begin = std::max(first_ext_begin, o.first_ext_begin);
        first_ext_end = std::max(first_ext_end, o.first_ext_end);
        replayed += o.replayed;
        seed += o.seed; extend += o.extend; part += o.part; collect += o.collect; last += o.last;
        sequential += o.sequential; load += o.load; output += o.output;
        first_seeded = std::max(first_seeded, o.first_seeded);
        last_start = std::max(last_start, o.last_start);
        last_put = std::max(last_put, o.last_put);
        workers_done = std::max(workers_done, o.workers_done);
    }
};

struct PipelineResult {
    AlignmentStatistics stats;
    uint64_t singletons = 0;                    // interleaved input: unpaired records (not mapped)
    double map_seconds = 0;
    uint64_t sam_bytes = 0;
    SamDigest sam_digest;
    PhaseTimes phases;
};

// perform_task_async_{pe,se} (src/pc.cpp:814-1096, 1522-1887) with -t 1 semantics:
// chunks are processed strictly in the single-worker timeline until the insert
// size estimate freezes, then chunk-parallel over `threads` host workers.
using SamSink = void (*)(void* user, const char* chunk, size_t bytes);
// the pipeline over a read source (ReadSource: streamed files or records in memory)
PipelineResult run_pipeline_pe(ReadSource& src, Engine& eng, const MapContext& mc, const PipelineOptions& opt,
                               SamSink sink, void* user);
PipelineResult run_pipeline_se(ReadSource& src, Engine& eng, const MapContext& mc, const PipelineOptions& opt,
                               SamSink sink, void* user);
// the same over records in memory
PipelineResult run_pipeline_pe(const std::vector<Record>& r1, const std::vector<Record>& r2, Engine& eng,
                               const MapContext& mc, const PipelineOptions& opt, SamSink sink, void* user);
PipelineResult run_pipeline_se(const std::vector<Record>& r, Engine& eng, const MapContext& mc,
                               const PipelineOptions& opt, SamSink sink, void* user);

// CLI entry (main.cpp); the oracle CPU binary reuses it with its own engine factory
using EngineFactory = std::unique_ptr<Engine> (*)(const References&, const StiIndex&, int device);

// Several engines behind one (multi.cpp): every seed/extend call goes to the engine
// with the fewest calls in flight; the pipeline's chunk queue, chunk_index seeding,
// insert-size freeze and ordered writer are shared, so the SAM does not depend on
// the number of devices.  open_engines: one engine per device, each with a full
// index replica (a device-only index is copied to the host once and uploaded).
std::unique_ptr<Engine> make_multi_engine(std::vector<std::unique_ptr<Engine>> engines);
std::unique_ptr<Engine> open_engines(EngineFactory factory, const References& refs, StiIndex& idx,
                                     const std::vector<int>& devices);
std::vector<int> parse_devices(const std::string& s);   // comma-separated ordinals
int cli_main(int argc, char** argv, EngineFactory factory, const char* prog);

}  // namespace rsa
