// rsa_ctx.hip -- the C-ABI (include/rsa_gpu.h) on top of the gfx950 kernels.
//
// One context per GPU holds the index (RefRandstrobe AoS + bucket table) and
// the reference bytes resident in HBM.  Calls are served by "lanes": each lane
// owns a HIP stream and its growable device/pinned buffers, so concurrent host
// threads (the worker pool of the host pipeline) overlap H2D, kernels and D2H.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <mutex>
#include <string>
#include <vector>

#include "rsa_ext.h"
#include "rsa_seed.h"
#include "rsa_timer.h"

void launch_ext_scan(int rmax, dim3 grid, dim3 block, hipStream_t st, const ExtJobDev* jobs, int n, const int* idx,
                     const char* q, const char* ref, ScanRes* out, int match, int mismatch, int gO, int gE, const int* n_dev = nullptr);
int scan_g_rows(uint32_t qlen);
void scan_g_classes(int* rows5);
int scan_g_max_ref();
void launch_ext_scan_g(int rows, int n, hipStream_t st, const ExtJobDev* jobs, const int* order, const char* q,
                       const char* ref, ScanRes* out, int match, int mismatch, int gO, int gE);
bool scan_g_params_ok(int match, int mismatch, int gO, int gE);
__global__ void k_ext_band_panel(const ExtJobDev* jobs, const ScanRes* scan, int n_jobs, const int* idx_list,
                                 const char* qbuf, const char* ref, uint32_t* cig_pool, rsa_aln* out,
                                 uint8_t* scratch, int64_t scr_stride, int64_t dir_cap, int match, int mismatch,
                                 int gO, int gE, int bonus, int* overflow, int over_code, int* redo,
                                 int* redo_count);
void launch_ext_band16(int dircap, dim3 grid, hipStream_t st, const ExtJobDev* jobs, const ScanRes* scan, int n, const int* idx,
                       const char* q, const char* ref, uint32_t* cig, uint32_t* raw, rsa_aln* out, int match,
                       int mismatch, int gO, int gE, int bonus, int* queue, int* qcount, int* overflow, int* redo,
                       int* redo_count, int prio, const int* n_dev = nullptr);
void launch_shared_check(int nl, hipStream_t st, const ExtJobDev* jobs, const uint32_t* list, const char* q,
                         const char* ref, uint8_t* res);
void launch_ext_band64(dim3 grid, hipStream_t st, const ExtJobDev* jobs, const ScanRes* scan, const char* q,
                       const char* ref, uint32_t* cig, uint32_t* raw, rsa_aln* out, int match, int mismatch, int gO,
                       int gE, int bonus, const int* queue, const int* qcount, int* overflow, int* ocount, int* redo,
                       int* redo_count);
int scan_v_rows(uint32_t qlen);
int scan_v_wcap(uint32_t rlen);
void launch_ext_scan_v(int rv, int wcap, int n, hipStream_t st, const ExtJobDev* jobs, const int* order, const char* q,
                       const char* ref, ScanRes* out, int match, int mismatch, int gO, int gE, int* err, int prio);
void launch_cigar_compact(hipStream_t st, const rsa_aln* alns, rsa_aln* alns_out, int n_jobs, const uint32_t* slots,
                          uint32_t* dense, uint64_t* bsum, uint64_t* total);

void index_build_peek(const rsa_index_build* b, int* device, int* bits);
void index_build_release(rsa_index_build* b, int* device, char** ref, rsa_ref_randstrobe** rs, uint64_t** starts,
                         uint64_t* n, int* bits);

hipError_t bucket_lines_build(const uint64_t* starts, const rsa_ref_randstrobe* rs, int bits, BucketLine* lines,
                              hipStream_t st);
int seed_run(SeedBufs& b, hipStream_t st, KTimer& kt, const SeedIndexParams& p, const rsa_read_batch* rb,
             int32_t rescue_level, uint32_t rescue_cutoff, rsa_nam_batch* out, std::string& err, SeedCounters& c);
int seed_randstrobes_run(SeedBufs& b, hipStream_t st, const SeedIndexParams& p, const rsa_read_batch* rb,
                         rsa_randstrobe_batch* out, std::string& err);

// RSA_SYNC_DEBUG=1 (debugging): wait for every extension launch and name the one that failed
static bool sync_debug() {
    static const bool on = getenv("RSA_SYNC_DEBUG") && getenv("RSA_SYNC_DEBUG")[0] == '1';
    return on;
}
#define LAUNCHCHK(name, stream)                                                               \
    do {                                                                                      \
        HIPCHK(hipGetLastError());                                                            \
        if (sync_debug()) {                                                                   \
            const hipError_t s_ = hipStreamSynchronize(stream);                               \
            if (s_ != hipSuccess) {                                                           \
                set_err(ctx, std::string("after ") + (name) + ": " + hipGetErrorString(s_));  \
                return RSA_ERR_HIP;                                                           \
            }                                                                                 \
        }                                                                                     \
    } while (0)
#define HIPCHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            set_err(ctx, std::string(#x) + ": " + hipGetErrorString(e_));           \
            return RSA_ERR_HIP;                                                     \
        }                                                                           \
    } while (0)

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        size_t n = std::max(bytes, cap + cap / 2);
        hipError_t e = hipMalloc(&p, n);
        if (e != hipSuccess) { p = nullptr; cap = 0; return e; }
        cap = n;
        return rsa_poison(p, n);
    }
    template <class T> T* as() const { return (T*)p; }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
};

struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        size_t n = std::max(bytes, cap + cap / 2);
        hipError_t e = hipHostMalloc(&p, n, hipHostMallocDefault);
        if (e != hipSuccess) { p = nullptr; cap = 0; return e; }
        cap = n;
        return hipSuccess;
    }
    template <class T> T* as() const { return (T*)p; }
    void release() { if (p) (void)hipHostFree(p); p = nullptr; cap = 0; }
};

struct Lane {
    hipStream_t stream = nullptr;
    KTimer kt;
    bool busy = false;
    int kind = 0;                      // LANE_SEED or LANE_EXT (the pool it belongs to)
    // extension
    // d_jobs / h_jobs: one staged upload per call, [ExtJobDev x n | scan order x n | ExtStatus (zeroed)];
    // d_alns holds results with CIGAR slot offsets, d_alns_out the copy with packed offsets
    // d_redo: jobs whose certified word result the band path could not confirm (k_ext_scan_v)
    DevBuf d_q, d_jobs, d_scan, d_alns, d_alns_out, d_cig, d_dense, d_raw, d_scratch, d_over, d_queue, d_idx, d_bsum,
        d_redo, d_shl, d_shres;
    HostBuf h_jobs, h_over, h_status, h_shl, h_shres;   // h_shl / d_shl: (job, k) pairs of RSA_JOB_SHARED_CHECK
    // seeding
    SeedBufs sb;
};

}  // namespace

// k_ext_scan_v (one layout per pass, certified) unless RSA_SCAN_V=0 (k_ext_scan_g,
// both layouts in every pass); read when a context opens
static bool scan_v_env() {
    const char* v = getenv("RSA_SCAN_V");
    return !(v && v[0] == '0');
}

static const int BAND64_GRID_MAX = 1024;

struct rsa_ctx {
    int device = 0;
    bool scan_v = scan_v_env();
    std::string err;
    std::mutex err_m;
    // resident data
    char* d_ref = nullptr;
    uint64_t ref_bytes = 0;
    std::vector<uint64_t> contig_off;  // host copy [n+1]
    rsa_ref_randstrobe* d_rs = nullptr;
    uint64_t* d_coff = nullptr;        // contig offsets (device copy)
    uint64_t n_rs = 0;
    uint64_t* d_starts = nullptr;
    BucketLine* d_lines = nullptr;     // k_lookup's copy of the bucket table (rsa_seed.h)
    SeedIndexParams ip{};
    uint64_t resident = 0;
    // lanes
    std::vector<Lane*> lanes;
    std::mutex lane_m;
    std::condition_variable lane_cv;
    int n_pending = 0;                 // rsa_extend_async calls not yet waited for
    std::atomic<int> band64_recent{BAND64_GRID_MAX};   // decaying max of recent calls' band16 deferrals
    // stats
    std::mutex stat_m;
    rsa_kernel_stats stats{};
};

// the message of the calling thread's last failed call: concurrent calls on one
// context (the host pipeline's workers) never see each other's messages
static thread_local std::string t_err;
static thread_local std::vector<uint32_t> t_shl;    // a call's (job, k) shared-check pairs while it is staged

static void set_err(rsa_ctx* ctx, const std::string& s) {
    t_err = s;
    if (!ctx) return;
    std::lock_guard<std::mutex> g(ctx->err_m);
    ctx->err = s;
}

static const int RSA_MAX_LANES = 16;   // per pool
enum { LANE_SEED = 0, LANE_EXT = 1 };

// Extension calls have lanes of their own, on high-priority streams: an extension
// call finishes chunks whose SAM the ordered output waits for, while the seeding
// calls mostly run chunks ahead of it, so the command processor dispatches the
// extension kernels' workgroups first when both wait for compute units
// (RSA_EXT_PRIORITY=0: one pool at normal priority for both kinds).
// the extension kernels' waves raise their issue priority on the SIMDs they share with
// the seeding kernels (RSA_EXT_SETPRIO, read per call; default on)
static int ext_setprio() {
    const char* e = getenv("RSA_EXT_SETPRIO");
    return e && e[0] == '0' ? 0 : 1;
}

static bool ext_priority() {
    static const bool on = !(getenv("RSA_EXT_PRIORITY") && getenv("RSA_EXT_PRIORITY")[0] == '0');
    return on;
}

// RSA_SEED_CU_EIGHTHS=k (0..6): the seeding lanes' streams leave k eighths of the CUs to the
// extension kernels (hipExtStreamCreateWithCUMask).  CU i stays in the mask unless
// (i % 8 - i / 32) mod 8 < k: that removes k CUs of every 32-CU XCD whether the mask
// enumerates CUs XCD by XCD or interleaved across the XCDs.  Default 0: no mask.
static int seed_cu_eighths() {
    static const int k = [] {
        const char* v = getenv("RSA_SEED_CU_EIGHTHS");
        const int x = v ? atoi(v) : 0;
        return x < 0 ? 0 : (x > 6 ? 6 : x);
    }();
    return k;
}

static hipError_t create_seed_stream(hipStream_t* st) {
    const int k = seed_cu_eighths();
    int dev = 0, ncu = 0;
    if (k > 0 && hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0) {
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
        for (int i = 0; i < ncu; ++i)
            if ((((i % 8) - (i / 32)) % 8 + 8) % 8 >= k) mask[(size_t)i / 32] |= 1u << (i % 32);
        return hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size() * 32, mask.data());
    }
    return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
}

static Lane* acquire_lane(rsa_ctx* ctx, int kind) {
    if (!ext_priority()) kind = LANE_SEED;
    std::unique_lock<std::mutex> g(ctx->lane_m);
    for (;;) {
        int mine = 0;
        for (Lane* l : ctx->lanes) {
            if (l->kind != kind) continue;
            mine++;
            if (!l->busy) { l->busy = true; return l; }
        }
        if (mine < RSA_MAX_LANES) {
            Lane* l = new Lane();
            l->kind = kind;
            hipError_t e;
            if (kind == LANE_EXT) {
                int least = 0, greatest = 0;
                (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
                e = hipStreamCreateWithPriority(&l->stream, hipStreamNonBlocking, greatest);
            } else {
                e = create_seed_stream(&l->stream);
            }
            if (e != hipSuccess) { delete l; return nullptr; }
            l->busy = true;
            ctx->lanes.push_back(l);
            return l;
        }
        ctx->lane_cv.wait(g);
    }
}

static void release_lane(rsa_ctx* ctx, Lane* l) {
    {
        std::lock_guard<std::mutex> g(ctx->lane_m);
        l->busy = false;
    }
    ctx->lane_cv.notify_all();
}

// wall-time breakdown of one entry-point call into ctx->stats (call_ms / lane_wait_ms / device_wait_ms)
struct CallTimer {
    rsa_ctx* ctx;
    int which;
    std::chrono::steady_clock::time_point t0;
    double lane_ms = 0;
    CallTimer(rsa_ctx* c, int w) : ctx(c), which(w), t0(std::chrono::steady_clock::now()) { device_wait_ms() = 0; }
    Lane* lane(int kind) {
        const auto t = std::chrono::steady_clock::now();
        Lane* l = acquire_lane(ctx, kind);
        lane_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
        return l;
    }
    ~CallTimer() {
        const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::lock_guard<std::mutex> g(ctx->stat_m);
        ctx->stats.call_ms[which] += wall;
        ctx->stats.lane_wait_ms[which] += lane_ms;
        ctx->stats.device_wait_ms[which] += device_wait_ms();
    }
};

struct LaneGuard {
    rsa_ctx* ctx; Lane* l;
    ~LaneGuard() { if (l) release_lane(ctx, l); }
};

// The BucketLine table (one 128-byte line a bucket, 32 GiB at bits = 28) unless
// RSA_BUCKET_LINES=0 or it would take more than half of the free HBM; without it
// k_lookup reads the .sti bucket table and entries (two random lines a lookup).
static void open_bucket_lines(rsa_ctx* ctx) {
    const char* v = getenv("RSA_BUCKET_LINES");
    if ((v && v[0] == '0') || !ctx->d_starts || !ctx->d_rs) return;
    const size_t bytes = sizeof(BucketLine) << ctx->ip.bits;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || bytes > free_b / 2) return;
    if (hipMalloc(&ctx->d_lines, bytes) != hipSuccess) { ctx->d_lines = nullptr; (void)hipGetLastError(); return; }
    if (bucket_lines_build(ctx->d_starts, ctx->d_rs, ctx->ip.bits, ctx->d_lines, nullptr) != hipSuccess) {
        (void)hipFree(ctx->d_lines);
        ctx->d_lines = nullptr;
        (void)hipGetLastError();
        return;
    }
    ctx->ip.lines = ctx->d_lines;
    ctx->resident += bytes;
}

extern "C" {

rsa_ctx* rsa_open(int device, const rsa_index_view* v, char* errbuf, size_t err_len) {
    auto fail = [&](const std::string& s) -> rsa_ctx* {
        if (errbuf && err_len) { snprintf(errbuf, err_len, "%s", s.c_str()); }
        return nullptr;
    };
    if (!v) return fail("rsa_open: null index view");
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess || n_dev == 0) return fail("rsa_open: no HIP device visible");
    if (device < 0 || device >= n_dev) return fail("rsa_open: bad device ordinal");
    if (hipSetDevice(device) != hipSuccess) return fail("rsa_open: hipSetDevice failed");
    rsa_ctx* ctx = new rsa_ctx();
    ctx->device = device;
    ctx->contig_off.assign(v->contig_offsets, v->contig_offsets + v->n_contigs + 1);
    ctx->ref_bytes = ctx->contig_off.back();
    ctx->n_rs = v->n_randstrobes;
    const size_t n_starts = ((size_t)1 << v->bits) + 1;
    hipError_t e = hipMalloc(&ctx->d_ref, ctx->ref_bytes + 64);
    if (e == hipSuccess) e = hipMemcpy(ctx->d_ref, v->ref_seq, ctx->ref_bytes, hipMemcpyHostToDevice);
    // the tail padding the kernels' wide loads may touch (masked) holds zeros, not whatever
    // the allocation held: no context differs from another in any byte a kernel reads
    if (e == hipSuccess) e = hipMemset(ctx->d_ref + ctx->ref_bytes, 0, 64);
    if (e == hipSuccess && v->randstrobes && ctx->n_rs) {
        e = hipMalloc(&ctx->d_rs, sizeof(rsa_ref_randstrobe) * (ctx->n_rs + 1));
        if (e == hipSuccess) e = hipMemcpy(ctx->d_rs, v->randstrobes, sizeof(rsa_ref_randstrobe) * ctx->n_rs, hipMemcpyHostToDevice);
        // the entry past the last: all ones (a hash above every key), not whatever the allocation held
        if (e == hipSuccess) e = hipMemset(ctx->d_rs + ctx->n_rs, 0xFF, sizeof(rsa_ref_randstrobe));
    }
    if (e == hipSuccess) e = hipMalloc(&ctx->d_coff, sizeof(uint64_t) * ctx->contig_off.size());
    if (e == hipSuccess)
        e = hipMemcpy(ctx->d_coff, ctx->contig_off.data(), sizeof(uint64_t) * ctx->contig_off.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess && v->bucket_starts) {
        e = hipMalloc(&ctx->d_starts, sizeof(uint64_t) * n_starts);
        if (e == hipSuccess) e = hipMemcpy(ctx->d_starts, v->bucket_starts, sizeof(uint64_t) * n_starts, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();    // the fills above ran on the null stream
    if (e != hipSuccess) {
        std::string s = std::string("rsa_open upload: ") + hipGetErrorString(e);
        rsa_close(ctx);
        return fail(s);
    }
    ctx->ip.rs = ctx->d_rs;
    ctx->ip.starts = ctx->d_starts;
    ctx->ip.n = ctx->n_rs;
    ctx->ip.bits = v->bits;
    ctx->ip.filter_cutoff = (uint32_t)v->filter_cutoff;
    ctx->ip.k = v->k; ctx->ip.s = v->s; ctx->ip.t = v->t_syncmer;
    ctx->ip.w_min = v->w_min; ctx->ip.w_max = v->w_max; ctx->ip.max_dist = v->max_dist;
    ctx->ip.q = v->q;
    ctx->ip.ref = ctx->d_ref;
    ctx->ip.coff = ctx->d_coff;
    ctx->resident = ctx->ref_bytes + sizeof(rsa_ref_randstrobe) * ctx->n_rs + sizeof(uint64_t) * n_starts;
    open_bucket_lines(ctx);
    return ctx;
}

rsa_ctx* rsa_open_built(rsa_index_build* b, const rsa_index_view* v, char* errbuf, size_t err_len) {
    auto fail = [&](const std::string& s) -> rsa_ctx* {
        if (errbuf && err_len) { snprintf(errbuf, err_len, "%s", s.c_str()); }
        return nullptr;
    };
    if (!b || !v || !v->contig_offsets) return fail("rsa_open_built: null build or view");
    // everything that can fail happens before the build's buffers change hands:
    // on error `b` stays valid and owned by the caller (rsa_gpu.h)
    int dev = 0, bits = 0;
    index_build_peek(b, &dev, &bits);
    if (bits != v->bits) return fail("rsa_open_built: view bits differ from the build's");
    std::vector<uint64_t> coff(v->contig_offsets, v->contig_offsets + v->n_contigs + 1);
    uint64_t* d_coff = nullptr;
    hipError_t e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipMalloc(&d_coff, sizeof(uint64_t) * coff.size());
    if (e == hipSuccess) e = hipMemcpy(d_coff, coff.data(), sizeof(uint64_t) * coff.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (d_coff) (void)hipFree(d_coff);
        return fail(std::string("rsa_open_built: ") + hipGetErrorString(e));
    }
    rsa_ctx* ctx = new rsa_ctx();
    ctx->contig_off.swap(coff);
    ctx->ref_bytes = ctx->contig_off.back();
    ctx->d_coff = d_coff;
    index_build_release(b, &ctx->device, &ctx->d_ref, &ctx->d_rs, &ctx->d_starts, &ctx->n_rs, &bits);
    ctx->ip.rs = ctx->d_rs;
    ctx->ip.starts = ctx->d_starts;
    ctx->ip.n = ctx->n_rs;
    ctx->ip.bits = v->bits;
    ctx->ip.filter_cutoff = (uint32_t)v->filter_cutoff;
    ctx->ip.k = v->k; ctx->ip.s = v->s; ctx->ip.t = v->t_syncmer;
    ctx->ip.w_min = v->w_min; ctx->ip.w_max = v->w_max; ctx->ip.max_dist = v->max_dist;
    ctx->ip.q = v->q;
    ctx->ip.ref = ctx->d_ref;
    ctx->ip.coff = ctx->d_coff;
    ctx->resident = ctx->ref_bytes + sizeof(rsa_ref_randstrobe) * ctx->n_rs + sizeof(uint64_t) * (((size_t)1 << v->bits) + 1);
    open_bucket_lines(ctx);
    return ctx;
}

int rsa_index_download(rsa_ctx* ctx, rsa_ref_randstrobe* randstrobes, uint64_t* bucket_starts) {
    if (!ctx) return RSA_ERR_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    if (randstrobes && ctx->n_rs)
        HIPCHK(hipMemcpy(randstrobes, ctx->d_rs, sizeof(rsa_ref_randstrobe) * ctx->n_rs, hipMemcpyDeviceToHost));
    if (bucket_starts && ctx->d_starts)
        HIPCHK(hipMemcpy(bucket_starts, ctx->d_starts, sizeof(uint64_t) * (((size_t)1 << ctx->ip.bits) + 1),
                         hipMemcpyDeviceToHost));
    return RSA_OK;
}

void rsa_close(rsa_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    for (Lane* l : ctx->lanes) {
        if (l->stream) (void)hipStreamSynchronize(l->stream);
        for (DevBuf* b : {&l->d_q, &l->d_jobs, &l->d_scan, &l->d_alns, &l->d_alns_out, &l->d_cig, &l->d_dense, &l->d_raw,
                          &l->d_scratch, &l->d_over, &l->d_queue, &l->d_idx, &l->d_bsum})
            b->release();
        l->h_jobs.release(); l->h_over.release(); l->h_status.release();
        seed_bufs_release(l->sb);
        l->kt.destroy();
        if (l->stream) (void)hipStreamDestroy(l->stream);
        delete l;
    }
    if (ctx->d_ref) (void)hipFree(ctx->d_ref);
    if (ctx->d_rs) (void)hipFree(ctx->d_rs);
    if (ctx->d_starts) (void)hipFree(ctx->d_starts);
    if (ctx->d_lines) (void)hipFree(ctx->d_lines);
    if (ctx->d_coff) (void)hipFree(ctx->d_coff);
    delete ctx;
}

const char* rsa_last_error(rsa_ctx* ctx) { return ctx ? t_err.c_str() : "null context"; }

uint64_t rsa_resident_bytes(const rsa_ctx* ctx) { return ctx ? ctx->resident : 0; }

uint64_t rsa_extend_cigar_bound(const rsa_job_batch* jb) {
    uint64_t t = 0;
    for (uint32_t i = 0; i < jb->n_jobs; ++i)
        t += (uint64_t)(jb->jobs[i].query_len & RSA_JOB_LEN_MASK) + jb->jobs[i].ref_len + 8;
    return t;
}

// band scratch of k_ext_band_panel (per in-flight job): the direction matrix of the
// widest band a job can need (2 x 2000 + 1 cells x 1024 rows x 3 bytes < 16 MB) and
// the raw traceback ops
static const int64_t BIG_DIR_CAP = 16ll << 20;
static const int BIG_CHUNK = 32;
// k_ext_band16's direction capacity for a call whose longest query (windows <= 2 kb) is
// qmax: 8192 above 200 bp (see k_ext_band16); RSA_BAND16_DIRCAP=4096/8192/16384 fixes it
static int band16_dircap(uint32_t qmax) {
    const char* v = getenv("RSA_BAND16_DIRCAP");   // per call: the tests switch it
    const int forced = v ? atoi(v) : 0;
    if (forced > 0) return forced;
    return qmax > 200 ? 8192 : 4096;
}

// waves draining the band16 deferral queue: k_ext_band64 holds 35 KB of LDS, so a CU
// keeps 4 of them (one a SIMD) and 1024 cover the chip; a wave past the queue's end exits
// at once (PE 2x250 defers ~15 % of its jobs: 512 waves left half the SIMDs idle)
// The grid follows the deferrals of the context's recent calls (twice the decaying
// maximum, 64..1024 waves): with k_ext_band16's 8 KB class almost nothing is deferred,
// and 1024 idle waves of 35 KB each cost ~0.15 ms a call while they found CUs.  Extra
// deferrals only lengthen the grid-stride loop.  RSA_BAND64_GRID fixes the grid (A/B).
static int band64_grid(const rsa_ctx* ctx) {
    static const int g = getenv("RSA_BAND64_GRID") ? std::max(1, atoi(getenv("RSA_BAND64_GRID"))) : 0;
    if (g) return g;
    return std::min(BAND64_GRID_MAX, std::max(64, 2 * ctx->band64_recent.load(std::memory_order_relaxed)));
}
static const uint64_t DENSE_GUESS = 24;    // CIGAR ops per job copied before the total is known

static int64_t band_stride(int64_t dir_cap) {
    int64_t s = dir_cap + (int64_t)RSA_RAW_CAP * 4;
    return (s + 255) & ~(int64_t)255;
}

struct ExtStatus {            // device-side counters of one rsa_extend call
    int qcount;               // jobs deferred by k_ext_band16 (of the last band pass)
    int ocount;               // jobs k_ext_band64 could not hold (every pass)
    uint64_t total;           // dense CIGAR ops (k_cigar_compact)
    int rcount;               // jobs listed in d_redo (certificate not met)
    int err;                  // k_ext_scan_v found an alignment end outside its job (a defect)
    int qcount1;              // jobs deferred by the first band pass (the in-stream redo pass runs after it)
    int pad_;
};

// The jobs whose word result the band kernels could not certify (d_redo) are re-run in the
// same stream, before the results are compacted and copied (RSA_REDO_DEV, default on): the
// exact two-layout scan and the band kernels over the device's own list, on a grid for up to
// REDO_DEV_CAP jobs (an empty list costs three near-empty launches).  About two calls in
// three list a job (444 of 7.3 M jobs at 2 x 150 bp); without this every such call waited for
// the first results, launched the pass from the host and copied everything again.  A list
// longer than the cap takes the host path (ext_finish).  RSA_REDO_DEV=<cap> (tests: 0 = the
// host path only, 1 = a cap the redo tests exceed).
static const int REDO_DEV_CAP = 128;
static int redo_dev_cap() {
    const char* e = getenv("RSA_REDO_DEV");
    return e ? std::max(0, atoi(e)) : REDO_DEV_CAP;
}

// byte offsets of the scan order and the status in the staged job upload of n jobs
// one staged upload per call: [ExtJobDev x n | scan order x n | ExtJobDev x n in scan order | ExtStatus]
static size_t stage_order_off(uint32_t n) { return sizeof(ExtJobDev) * (size_t)n; }
static size_t stage_sorted_off(uint32_t n) { return (stage_order_off(n) + sizeof(int) * (size_t)n + 15) & ~(size_t)15; }
static size_t stage_status_off(uint32_t n) { return stage_sorted_off(n) + sizeof(ExtJobDev) * (size_t)n; }
static size_t stage_bytes(uint32_t n) { return stage_status_off(n) + sizeof(ExtStatus); }

}  // extern "C"

// One extension call between its enqueue and its completion: rsa_extend runs
// both halves back to back, rsa_extend_async returns between them.
struct rsa_pending {
    rsa_ctx* ctx = nullptr;
    Lane* L = nullptr;
    rsa_aln_batch* out = nullptr;
    uint32_t n = 0;
    int32_t match = 0, mismatch = 0, gap_open = 0, gap_extend = 0, end_bonus = 0;
    uint64_t guess = 0, cells = 0, qr_bytes = 0;
    int rmax = 1;                      // k_ext_scan's rows-per-lane bound for this call's jobs
    int band16_dircap = 4096;          // k_ext_band16's direction capacity for this call's queries
    int redo_dev = 0;                  // jobs the in-stream redo pass covers (0: none enqueued)
    uint32_t n_shared = 0;             // jobs with RSA_JOB_SHARED_CHECK (k_shared_check's list)
    ExtStatus* d_status = nullptr;     // in the lane's staged upload
};

// k_cigar_compact, then the status, results and the first `guess` CIGAR entries
// to the host; nothing waits here
static int ext_compact_copy(rsa_pending& P) {
    rsa_ctx* ctx = P.ctx;
    Lane* L = P.L;
    hipStream_t st = L->stream;
    launch_cigar_compact(st, L->d_alns.as<rsa_aln>(), L->d_alns_out.as<rsa_aln>(), (int)P.n, L->d_cig.as<uint32_t>(),
                         L->d_dense.as<uint32_t>(), L->d_bsum.as<uint64_t>(), &P.d_status->total);
    LAUNCHCHK("compaction", st);
    HIPCHK(hipMemcpyAsync(L->h_status.p, P.d_status, sizeof(ExtStatus), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(P.out->alns, L->d_alns_out.p, sizeof(rsa_aln) * P.n, hipMemcpyDeviceToHost, st));
    if (P.guess)
        HIPCHK(hipMemcpyAsync(P.out->cigar_pool, L->d_dense.p, sizeof(uint32_t) * P.guess, hipMemcpyDeviceToHost, st));
    return RSA_OK;
}

// first half: validate, stage, launch every kernel and the result copies on lane L
static int ext_enqueue(rsa_ctx* ctx, const rsa_job_batch* jb, rsa_aln_batch* out, rsa_pending& P) {
    Lane* L = P.L;
    const uint32_t n = jb->n_jobs;
    const uint64_t bound = rsa_extend_cigar_bound(jb);
    P.out = out;
    P.n = n;
    P.match = jb->match; P.mismatch = jb->mismatch; P.gap_open = jb->gap_open; P.gap_extend = jb->gap_extend;
    P.end_bonus = jb->end_bonus;
    if (rsa_poison_every())                        // tests: nothing an earlier call wrote survives
        for (DevBuf* b : {&L->d_q, &L->d_jobs, &L->d_scan, &L->d_alns, &L->d_alns_out, &L->d_cig, &L->d_dense, &L->d_raw,
                          &L->d_scratch, &L->d_over, &L->d_queue, &L->d_idx, &L->d_bsum, &L->d_redo, &L->d_shl,
                          &L->d_shres})
            if (b->p) HIPCHK(hipMemsetAsync(b->p, 0xA5, b->cap, L->stream));
    // host job descriptors
    HIPCHK(L->h_jobs.ensure(stage_bytes(n)));
    ExtJobDev* hj = L->h_jobs.as<ExtJobDev>();
    uint64_t cig_off = 0;
    uint64_t cells = 0, qr_bytes = 0;
    int rmax = 1;
    uint32_t qmax = 0;
    std::vector<uint32_t>& shl = t_shl;
    shl.clear();
    for (uint32_t i = 0; i < n; ++i) {
        rsa_job s = jb->jobs[i];
        if (s.query_len & RSA_JOB_SHARED_CHECK) {
            const uint32_t k = (s.query_len >> 24) & 0x7Fu;
            s.query_len &= RSA_JOB_LEN_MASK;
            if (s.query_len > RSA_SHARED_QMAX || s.ref_len > RSA_SHARED_WMAX || k < 3 || 2 * k / 3 > 24) {
                set_err(ctx, "rsa_extend: job " + std::to_string(i) + " asks for a shared-substring check outside "
                             "its limits (query <= 1024, window <= 4096, 3 <= k <= 37)");
                return RSA_ERR_ARG;
            }
            shl.push_back(i);
            shl.push_back(k);
        }
        s.query_len &= RSA_JOB_LEN_MASK;
        if (s.ref_id < 0 || s.ref_id >= (int)ctx->contig_off.size() - 1 || s.query_offset + s.query_len > jb->queries_len) {
            set_err(ctx, "rsa_extend: job " + std::to_string(i) + " out of range");
            return RSA_ERR_ARG;
        }
        const uint64_t clen = ctx->contig_off[s.ref_id + 1] - ctx->contig_off[s.ref_id];
        if ((uint64_t)s.ref_start + s.ref_len > clen) {
            set_err(ctx, "rsa_extend: job " + std::to_string(i) + " window exceeds contig");
            return RSA_ERR_ARG;
        }
        if (s.query_len > 1024 && s.ref_len <= 2000) {
            set_err(ctx, "rsa_extend: query longer than 1024 bp is not supported");
            return RSA_ERR_ARG;
        }
        hj[i].q_off = s.query_offset;
        hj[i].r_off = ctx->contig_off[s.ref_id] + s.ref_start;
        hj[i].qlen = s.query_len;
        hj[i].rlen = s.ref_len;
        hj[i].cig_off = cig_off;
        cig_off += (uint64_t)s.query_len + s.ref_len + 8;
        qr_bytes += (uint64_t)s.query_len + s.ref_len;
        if (s.ref_len <= 2000) {
            cells += (uint64_t)s.query_len * s.ref_len;
            rmax = std::max(rmax, (int)((s.query_len + 63) / 64));
            qmax = std::max(qmax, s.query_len);
        }
    }
    P.cells = cells;
    P.qr_bytes = qr_bytes;
    HIPCHK(L->d_q.ensure(jb->queries_len + 16));
    HIPCHK(L->d_jobs.ensure(stage_bytes(n)));
    HIPCHK(L->d_scan.ensure(sizeof(ScanRes) * n));
    HIPCHK(L->d_alns.ensure(sizeof(rsa_aln) * n));
    HIPCHK(L->d_alns_out.ensure(sizeof(rsa_aln) * n));
    HIPCHK(L->d_cig.ensure(sizeof(uint32_t) * (bound + 16)));
    HIPCHK(L->d_dense.ensure(sizeof(uint32_t) * (bound + 16)));
    HIPCHK(L->d_raw.ensure(sizeof(uint32_t) * (bound + 16)));
    HIPCHK(L->d_over.ensure(sizeof(int) * n));
    HIPCHK(L->d_queue.ensure(sizeof(int) * n));
    HIPCHK(L->d_redo.ensure(sizeof(int) * n));
    HIPCHK(L->d_bsum.ensure(sizeof(uint64_t) * ((n + 255) / 256 + 1)));
    HIPCHK(L->h_status.ensure(sizeof(ExtStatus)));
    hipStream_t st = L->stream;
    ExtStatus* dst = reinterpret_cast<ExtStatus*>(L->d_jobs.as<char>() + stage_status_off(n));
    P.d_status = dst;
    memset(L->h_jobs.as<char>() + stage_status_off(n), 0, sizeof(ExtStatus));
    HIPCHK(hipMemcpyAsync(L->d_q.p, jb->queries, jb->queries_len, hipMemcpyHostToDevice, st));
    // Scan routing: jobs a grouped kernel takes (query <= 256 bp, window <= 1 KB,
    // parameters it computes exactly) go to it per class, sorted by window length
    // (longest first) so the jobs of a wave run about as long; the rest -- and
    // sentinels -- to the one-job-per-wave kernel via an index list.  Classes:
    // k_ext_scan_v (default): rows per virtual lane 2..8 x window capacity 512 / 1024;
    // k_ext_scan_g (RSA_SCAN_V=0): rows per lane 4/7/10/13/16.
    const bool grouped = scan_g_params_ok(jb->match, jb->mismatch, jb->gap_open, jb->gap_extend);
    const bool use_v = ctx->scan_v;
    constexpr int NCLS_MAX = 14;
    const int ncls = use_v ? 14 : 5;
    int cls_rows[NCLS_MAX], cls_wcap[NCLS_MAX];
    if (use_v) {
        for (int c = 0; c < 14; ++c) { cls_rows[c] = 2 + c / 2; cls_wcap[c] = (c & 1) ? 1024 : 512; }
    } else {
        scan_g_classes(cls_rows);
        for (int c = 0; c < 5; ++c) cls_wcap[c] = scan_g_max_ref();
    }
    uint32_t cls_n[NCLS_MAX] = {0}, rest_n = 0;
    int* ord = reinterpret_cast<int*>(L->h_jobs.as<char>() + stage_order_off(n));
    // the descriptors again in scan order: a scan wave reads its jobs' descriptors and
    // result indices side by side (no dependent load through the order)
    ExtJobDev* sj = reinterpret_cast<ExtJobDev*>(L->h_jobs.as<char>() + stage_sorted_off(n));
    if (grouped) {
        const uint32_t maxr = 1024;
        std::vector<uint32_t> cnt((size_t)ncls * (maxr + 1), 0);
        auto cls_of = [&](const ExtJobDev& j) -> int {
            if (j.rlen > 2000 || j.qlen == 0 || j.qlen > 1024) return -1;
            if (use_v) {
                const int r = scan_v_rows(j.qlen), w = scan_v_wcap(j.rlen);
                if (r == 0 || w == 0) return -1;
                return (r - 2) * 2 + (w == 1024 ? 1 : 0);
            }
            if (j.rlen > (uint32_t)scan_g_max_ref()) return -1;
            const int r = scan_g_rows(j.qlen);
            for (int c = 0; c < 5; ++c) if (cls_rows[c] == r) return c;
            return -1;
        };
        std::vector<int8_t> cls(n);
        for (uint32_t i = 0; i < n; ++i) {
            cls[i] = (int8_t)cls_of(hj[i]);
            if (cls[i] < 0) rest_n++;
            else { cls_n[cls[i]]++; cnt[(size_t)cls[i] * (maxr + 1) + (maxr - hj[i].rlen)]++; }
        }
        // counting sort: class-major, then window length descending; the rest after
        uint64_t at = 0;
        for (int c = 0; c < ncls; ++c)
            for (uint32_t b = 0; b <= maxr; ++b) {
                uint32_t& x = cnt[(size_t)c * (maxr + 1) + b];
                const uint32_t k = x;
                x = (uint32_t)at;
                at += k;
            }
        uint64_t rest_at = at;
        for (uint32_t i = 0; i < n; ++i) {
            const uint64_t k = cls[i] < 0 ? rest_at++ : cnt[(size_t)cls[i] * (maxr + 1) + (maxr - hj[i].rlen)]++;
            ord[k] = (int)i;
            sj[k] = hj[i];
        }
    } else {
        rest_n = n;
        for (uint32_t i = 0; i < n; ++i) { ord[i] = (int)i; sj[i] = hj[i]; }
    }
    P.rmax = rmax;
    P.band16_dircap = band16_dircap(qmax);
    P.n_shared = (uint32_t)(shl.size() / 2);
    // jobs, scan order and the zeroed status in one copy
    HIPCHK(hipMemcpyAsync(L->d_jobs.p, L->h_jobs.p, stage_bytes(n), hipMemcpyHostToDevice, st));
    L->kt.arm();
    L->kt.begin(st, RSA_K_EXT_SCAN);
    {
        const int* d_ord = reinterpret_cast<const int*>(L->d_jobs.as<char>() + stage_order_off(n));
        const ExtJobDev* d_sj = reinterpret_cast<const ExtJobDev*>(L->d_jobs.as<char>() + stage_sorted_off(n));
        uint32_t off = 0;
        for (int c = 0; c < ncls; ++c) {
            if (!cls_n[c]) continue;
            if (use_v)
                launch_ext_scan_v(cls_rows[c], cls_wcap[c], (int)cls_n[c], st, d_sj + off, d_ord + off,
                                  L->d_q.as<char>(), ctx->d_ref, L->d_scan.as<ScanRes>(), jb->match, jb->mismatch,
                                  jb->gap_open, jb->gap_extend, &dst->err, ext_setprio());
            else
                launch_ext_scan_g(cls_rows[c], (int)cls_n[c], st, L->d_jobs.as<ExtJobDev>(), d_ord + off,
                                  L->d_q.as<char>(), ctx->d_ref, L->d_scan.as<ScanRes>(), jb->match, jb->mismatch,
                                  jb->gap_open, jb->gap_extend);
            LAUNCHCHK("scan class", st);
            off += cls_n[c];
        }
        if (rest_n) {
            launch_ext_scan(rmax, dim3((rest_n + 3) / 4), dim3(256), st, L->d_jobs.as<ExtJobDev>(),
                            (int)rest_n, d_ord + off, L->d_q.as<char>(), ctx->d_ref, L->d_scan.as<ScanRes>(),
                            jb->match, jb->mismatch, jb->gap_open, jb->gap_extend);
            LAUNCHCHK("scan rest", st);
        }
    }
    L->kt.end(st);
    // 16 lanes per job for the common narrow bands; the rest queue for 64-lane waves.
    // k_ext_band16 writes every job's result (an empty one for the jobs it queues, so
    // the compaction below never reads an unwritten result) and clears every job's
    // overflow flag, which k_ext_band64 sets for the bands it cannot hold
    L->kt.begin(st, RSA_K_EXT_BAND);
    launch_ext_band16(P.band16_dircap, dim3((n + 3) / 4), st, L->d_jobs.as<ExtJobDev>(), L->d_scan.as<ScanRes>(), (int)n, nullptr,
                      L->d_q.as<char>(), ctx->d_ref, L->d_cig.as<uint32_t>(), L->d_raw.as<uint32_t>(),
                      L->d_alns.as<rsa_aln>(), jb->match, jb->mismatch, jb->gap_open, jb->gap_extend, jb->end_bonus,
                      L->d_queue.as<int>(), &dst->qcount, L->d_over.as<int>(), L->d_redo.as<int>(), &dst->rcount,
                      ext_setprio());
    LAUNCHCHK("band16", st);
    L->kt.end(st);
    L->kt.begin(st, RSA_K_EXT_BAND_WIDE);
    launch_ext_band64(dim3(std::min<uint32_t>(n, (uint32_t)band64_grid(ctx))), st, L->d_jobs.as<ExtJobDev>(),
                      L->d_scan.as<ScanRes>(), L->d_q.as<char>(), ctx->d_ref, L->d_cig.as<uint32_t>(),
                      L->d_raw.as<uint32_t>(), L->d_alns.as<rsa_aln>(), jb->match, jb->mismatch, jb->gap_open,
                      jb->gap_extend, jb->end_bonus, L->d_queue.as<int>(), &dst->qcount, L->d_over.as<int>(),
                      &dst->ocount, L->d_redo.as<int>(), &dst->rcount);
    LAUNCHCHK("band64", st);
    L->kt.end(st);
    P.redo_dev = (int)std::min<uint32_t>(n, (uint32_t)redo_dev_cap());
    if (P.redo_dev > 0) {
        const int cap = P.redo_dev;
        const int* d_redo = L->d_redo.as<int>();
        HIPCHK(hipMemcpyAsync(&dst->qcount1, &dst->qcount, sizeof(int), hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemsetAsync(&dst->qcount, 0, sizeof(int), st));          // k_ext_band64's queue restarts
        L->kt.begin(st, RSA_K_EXT_REDO);
        launch_ext_scan(P.rmax, dim3((cap + 3) / 4), dim3(256), st, L->d_jobs.as<ExtJobDev>(), cap, d_redo,
                        L->d_q.as<char>(), ctx->d_ref, L->d_scan.as<ScanRes>(), jb->match, jb->mismatch,
                        jb->gap_open, jb->gap_extend, &dst->rcount);
        LAUNCHCHK("redo scan", st);
        launch_ext_band16(P.band16_dircap, dim3((cap + 3) / 4), st, L->d_jobs.as<ExtJobDev>(), L->d_scan.as<ScanRes>(),
                          cap, d_redo, L->d_q.as<char>(), ctx->d_ref, L->d_cig.as<uint32_t>(), L->d_raw.as<uint32_t>(),
                          L->d_alns.as<rsa_aln>(), jb->match, jb->mismatch, jb->gap_open, jb->gap_extend,
                          jb->end_bonus, L->d_queue.as<int>(), &dst->qcount, L->d_over.as<int>(), nullptr, nullptr,
                          ext_setprio(), &dst->rcount);
        LAUNCHCHK("redo band16", st);
        launch_ext_band64(dim3(std::min(cap, band64_grid(ctx))), st, L->d_jobs.as<ExtJobDev>(), L->d_scan.as<ScanRes>(),
                          L->d_q.as<char>(), ctx->d_ref, L->d_cig.as<uint32_t>(), L->d_raw.as<uint32_t>(),
                          L->d_alns.as<rsa_aln>(), jb->match, jb->mismatch, jb->gap_open, jb->gap_extend,
                          jb->end_bonus, L->d_queue.as<int>(), &dst->qcount, L->d_over.as<int>(), &dst->ocount,
                          nullptr, nullptr);
        LAUNCHCHK("redo band64", st);
        L->kt.end(st);
    }
    if (P.n_shared) {   // rescue_mate_part's has_shared_substring for the jobs that asked (aln.cpp:1058)
        HIPCHK(L->h_shl.ensure(sizeof(uint32_t) * shl.size()));
        memcpy(L->h_shl.p, shl.data(), sizeof(uint32_t) * shl.size());
        HIPCHK(L->d_shl.ensure(sizeof(uint32_t) * shl.size()));
        HIPCHK(L->d_shres.ensure(P.n_shared));
        HIPCHK(L->h_shres.ensure(P.n_shared));
        HIPCHK(hipMemcpyAsync(L->d_shl.p, L->h_shl.p, sizeof(uint32_t) * shl.size(), hipMemcpyHostToDevice, st));
        launch_shared_check((int)P.n_shared, st, L->d_jobs.as<ExtJobDev>(), L->d_shl.as<uint32_t>(), L->d_q.as<char>(),
                            ctx->d_ref, L->d_shres.as<uint8_t>());
        LAUNCHCHK("shared check", st);
        HIPCHK(hipMemcpyAsync(L->h_shres.p, L->d_shres.p, P.n_shared, hipMemcpyDeviceToHost, st));
    }
    P.guess = std::min<uint64_t>(bound, DENSE_GUESS * n);
    return ext_compact_copy(P);
}

// second half: wait, the rare panel pass for bands the 64-lane kernel could not
// hold, the CIGAR entries past the first guess, statistics
// the rare panel pass: bands the 64-lane kernel could not hold (overflow flag 1) ->
// one wave per job sweeping each band row in 64-cell panels (direction matrix in
// global scratch); then the CIGAR compaction and copies again
static int ext_panel(rsa_pending& P, ExtStatus& hs) {
    rsa_ctx* ctx = P.ctx;
    Lane* L = P.L;
    const uint32_t n = P.n;
    hipStream_t st = L->stream;
    HIPCHK(L->h_over.ensure(sizeof(int) * n));
    HIPCHK(hipMemcpyAsync(L->h_over.p, L->d_over.p, sizeof(int) * n, hipMemcpyDeviceToHost, st));
    HIPCHK(stream_wait(st, L->sb.done));
    std::vector<int> big;
    for (uint32_t i = 0; i < n; ++i)
        if (L->h_over.as<int>()[i]) big.push_back((int)i);
    const int64_t bstride = band_stride(BIG_DIR_CAP);
    HIPCHK(L->d_scratch.ensure((size_t)bstride * BIG_CHUNK));
    HIPCHK(L->d_idx.ensure(sizeof(int) * big.size()));
    HIPCHK(hipMemcpyAsync(L->d_idx.p, big.data(), sizeof(int) * big.size(), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(L->d_over.p, 0, sizeof(int) * n, st));
    for (size_t b = 0; b < big.size(); b += BIG_CHUNK) {
        const int cnt = (int)std::min<size_t>(BIG_CHUNK, big.size() - b);
        L->kt.begin(st, RSA_K_EXT_BAND_PANEL);
        hipLaunchKernelGGL(k_ext_band_panel, dim3(cnt), dim3(64), 0, st, L->d_jobs.as<ExtJobDev>(),
                           L->d_scan.as<ScanRes>(), cnt, L->d_idx.as<int>() + b, L->d_q.as<char>(), ctx->d_ref,
                           L->d_cig.as<uint32_t>(), L->d_alns.as<rsa_aln>(), L->d_scratch.as<uint8_t>(), bstride,
                           BIG_DIR_CAP, P.match, P.mismatch, P.gap_open, P.gap_extend, P.end_bonus,
                           L->d_over.as<int>(), 2, L->d_redo.as<int>(), &P.d_status->rcount);
        LAUNCHCHK("panel", st);
        L->kt.end(st);
    }
    HIPCHK(hipMemcpyAsync(L->h_over.p, L->d_over.p, sizeof(int) * n, hipMemcpyDeviceToHost, st));
    HIPCHK(stream_wait(st, L->sb.done));
    for (int i : big)
        if (L->h_over.as<int>()[i] > 1) { set_err(ctx, "rsa_extend: band scratch exhausted"); return RSA_ERR_NOMEM; }
    if (int rc = ext_compact_copy(P)) return rc;
    HIPCHK(stream_wait(st, L->sb.done));
    hs = *L->h_status.as<ExtStatus>();
    return RSA_OK;
}

// second half: wait, the rare panel pass, the rare re-run of jobs whose word
// result k_ext_scan_v could not certify, the CIGAR entries past the first guess,
// statistics
static int ext_finish(rsa_pending& P) {
    rsa_ctx* ctx = P.ctx;
    Lane* L = P.L;
    const uint32_t n = P.n;
    rsa_aln_batch* out = P.out;
    hipStream_t st = L->stream;
    const uint64_t guess = P.guess;
    HIPCHK(stream_wait(st, L->sb.done));
    ExtStatus hs = *L->h_status.as<ExtStatus>();
    if (hs.err) { set_err(ctx, "rsa_extend: k_ext_scan_v produced an alignment end outside its job"); return RSA_ERR_INTERNAL; }
    // the jobs listed before the panel pass: the in-stream redo pass covered them when
    // there were at most P.redo_dev; the panel pass below may list more, which it did not
    const int listed_in_stream = hs.rcount;
    if (hs.ocount > 0)
        if (int rc = ext_panel(P, hs)) return rc;
    int redo = hs.rcount;
    // the first band pass's deferrals (before the in-stream redo pass reset the queue)
    const int q1 = P.redo_dev > 0 ? hs.qcount1 : hs.qcount;
    uint64_t deferred = (uint64_t)q1 + (P.redo_dev > 0 ? (uint64_t)hs.qcount : 0), overflowed = (uint64_t)hs.ocount;
    {   // the next calls' k_ext_band64 grid (band64_grid)
        const int prev = ctx->band64_recent.load(std::memory_order_relaxed);
        ctx->band64_recent.store(std::max(q1, prev - prev / 4), std::memory_order_relaxed);
    }
    const int redo_total = redo;
    if (redo > 0 && redo == listed_in_stream && redo <= P.redo_dev) redo = 0;     // done in the stream already
    if (redo > 0) {
        // the listed jobs' path had an insertion next to a deletion (or no path): the
        // byte layout may score them differently, so they take the exact two-layout
        // scan (k_ext_scan: SSW's byte-then-word decision) and the band kernels again
        if (redo > (int)n) { set_err(ctx, "rsa_extend: redo list overflow"); return RSA_ERR_INTERNAL; }
        const int* d_redo = L->d_redo.as<int>();
        L->kt.begin(st, RSA_K_EXT_REDO);
        launch_ext_scan(P.rmax, dim3((redo + 3) / 4), dim3(256), st, L->d_jobs.as<ExtJobDev>(), redo, d_redo,
                        L->d_q.as<char>(), ctx->d_ref, L->d_scan.as<ScanRes>(), P.match, P.mismatch, P.gap_open,
                        P.gap_extend);
        LAUNCHCHK("host redo scan", st);
        HIPCHK(hipMemsetAsync(&P.d_status->qcount, 0, 2 * sizeof(int), st));    // qcount, ocount
        launch_ext_band16(P.band16_dircap, dim3((redo + 3) / 4), st, L->d_jobs.as<ExtJobDev>(), L->d_scan.as<ScanRes>(), redo, d_redo,
                          L->d_q.as<char>(), ctx->d_ref, L->d_cig.as<uint32_t>(), L->d_raw.as<uint32_t>(),
                          L->d_alns.as<rsa_aln>(), P.match, P.mismatch, P.gap_open, P.gap_extend, P.end_bonus,
                          L->d_queue.as<int>(), &P.d_status->qcount, L->d_over.as<int>(), nullptr, nullptr,
                          ext_setprio());
        LAUNCHCHK("host redo band16", st);
        launch_ext_band64(dim3(std::min(redo, band64_grid(ctx))), st, L->d_jobs.as<ExtJobDev>(), L->d_scan.as<ScanRes>(),
                          L->d_q.as<char>(), ctx->d_ref, L->d_cig.as<uint32_t>(), L->d_raw.as<uint32_t>(),
                          L->d_alns.as<rsa_aln>(), P.match, P.mismatch, P.gap_open, P.gap_extend, P.end_bonus,
                          L->d_queue.as<int>(), &P.d_status->qcount, L->d_over.as<int>(), &P.d_status->ocount,
                          nullptr, nullptr);
        LAUNCHCHK("host redo band64", st);
        L->kt.end(st);
        if (int rc = ext_compact_copy(P)) return rc;
        HIPCHK(stream_wait(st, L->sb.done));
        hs = *L->h_status.as<ExtStatus>();
        deferred += (uint64_t)hs.qcount;
        overflowed += (uint64_t)hs.ocount;
        if (hs.ocount > 0)
            if (int rc = ext_panel(P, hs)) return rc;
    }
    if (hs.total > guess) {
        HIPCHK(hipMemcpyAsync(out->cigar_pool + guess, L->d_dense.as<uint32_t>() + guess,
                              sizeof(uint32_t) * (hs.total - guess), hipMemcpyDeviceToHost, st));
        HIPCHK(stream_wait(st, L->sb.done));
    }
    out->cigar_used = hs.total;
    // scan_certified: the jobs whose word result stood on the band-path certificate, as the
    // band kernels flagged them (not a prediction from the query lengths)
    uint64_t certified = 0;
    for (uint32_t i = 0; i < n; ++i) certified += (out->alns[i].flags & RSA_ALN_WORD_CERT) ? 1 : 0;
    uint64_t no_shared = 0;
    for (uint32_t f = 0; f < P.n_shared; ++f)          // the stream has drained: the flags are here
        if (L->h_shres.as<uint8_t>()[f]) {
            out->alns[L->h_shl.as<uint32_t>()[2 * f]].flags |= RSA_ALN_NO_SHARED;
            no_shared++;
        }
    {
        std::lock_guard<std::mutex> g(ctx->stat_m);
        if (L->kt.on) {
            L->kt.collect(ctx->stats.kernel_ms, ctx->stats.launches);
            // scan: query + window in, ScanRes out; band: the segment bytes again, ScanRes in, rsa_aln + CIGAR out
            ctx->stats.alg_bytes[RSA_K_EXT_SCAN] += (double)P.qr_bytes + (double)(sizeof(ExtJobDev) + sizeof(ScanRes)) * n;
            ctx->stats.alg_bytes[RSA_K_EXT_BAND] += (double)P.qr_bytes + (double)(sizeof(ExtJobDev) + sizeof(ScanRes) +
                                                                                sizeof(rsa_aln)) * n + 4.0 * hs.total;
            ctx->stats.dp_cells_timed += P.cells;
            ctx->stats.ext_calls_timed++;
        }
        ctx->stats.ext_calls++;
        ctx->stats.jobs += n;
        ctx->stats.dp_cells += P.cells;
        ctx->stats.band_deferred += deferred;
        ctx->stats.band_overflow += overflowed;
        ctx->stats.scan_certified += certified;
        ctx->stats.scan_redo += (uint64_t)redo_total;
        ctx->stats.shared_checks += P.n_shared;
        ctx->stats.no_shared += no_shared;
    }
    return RSA_OK;
}


extern "C" {

int rsa_extend(rsa_ctx* ctx, const rsa_job_batch* jb, rsa_aln_batch* out) {
    if (!ctx || !jb || !out) return RSA_ERR_ARG;
    out->cigar_used = 0;
    if (jb->n_jobs == 0) return RSA_OK;
    if (out->cigar_capacity < rsa_extend_cigar_bound(jb)) {
        set_err(ctx, "rsa_extend: cigar_pool too small");
        return RSA_ERR_CAPACITY;
    }
    HIPCHK(hipSetDevice(ctx->device));
    CallTimer ct(ctx, 1);
    rsa_pending P;
    P.ctx = ctx;
    P.L = ct.lane(LANE_EXT);
    if (!P.L) { set_err(ctx, "rsa_extend: cannot create HIP stream"); return RSA_ERR_HIP; }
    LaneGuard guard{ctx, P.L};
    if (int rc = ext_enqueue(ctx, jb, out, P)) return rc;
    return ext_finish(P);
}

int rsa_extend_async(rsa_ctx* ctx, const rsa_job_batch* jb, rsa_aln_batch* out, rsa_pending** pending) {
    if (!ctx || !jb || !out || !pending) return RSA_ERR_ARG;
    *pending = nullptr;
    out->cigar_used = 0;
    if (out->cigar_capacity < rsa_extend_cigar_bound(jb)) {
        set_err(ctx, "rsa_extend_async: cigar_pool too small");
        return RSA_ERR_CAPACITY;
    }
    HIPCHK(hipSetDevice(ctx->device));
    {
        // every lane held by a pending call would make the acquire below wait forever
        std::lock_guard<std::mutex> g(ctx->lane_m);
        if (ctx->n_pending >= RSA_MAX_PENDING) {
            set_err(ctx, "rsa_extend_async: too many pending calls (rsa_wait some first)");
            return RSA_ERR_BUSY;
        }
        ctx->n_pending++;
    }
    auto unpend = [&]() {
        std::lock_guard<std::mutex> g(ctx->lane_m);
        ctx->n_pending--;
    };
    rsa_pending* P = new rsa_pending();
    P->ctx = ctx;
    P->out = out;
    if (jb->n_jobs == 0) { *pending = P; return RSA_OK; }   // nothing enqueued: rsa_wait returns at once
    P->L = acquire_lane(ctx, LANE_EXT);
    if (!P->L) {
        delete P;
        unpend();
        set_err(ctx, "rsa_extend_async: cannot create HIP stream");
        return RSA_ERR_HIP;
    }
    if (int rc = ext_enqueue(ctx, jb, out, *P)) {
        (void)hipStreamSynchronize(P->L->stream);   // the lane is reused: let what was enqueued drain
        release_lane(ctx, P->L);
        delete P;
        unpend();
        return rc;
    }
    *pending = P;
    return RSA_OK;
}

int rsa_ready(const rsa_pending* p) {
    if (!p || !p->L) return 1;
    return hipStreamQuery(p->L->stream) == hipErrorNotReady ? 0 : 1;
}

int rsa_wait(rsa_pending* p) {
    if (!p) return RSA_ERR_ARG;
    rsa_ctx* ctx = p->ctx;
    int rc = RSA_OK;
    if (p->L) {
        if (hipSetDevice(ctx->device) != hipSuccess) rc = RSA_ERR_HIP;
        if (rc == RSA_OK) rc = ext_finish(*p);
        if (rc != RSA_OK) (void)hipStreamSynchronize(p->L->stream);
        release_lane(ctx, p->L);
    }
    {
        std::lock_guard<std::mutex> g(ctx->lane_m);
        ctx->n_pending--;
    }
    delete p;
    return rc;
}

void* rsa_host_alloc(size_t bytes) {
    // portable: the product's multi-device engine (csrc/host/multi.cpp) hands one page-locked
    // buffer to whichever device's context serves the call
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable) != hipSuccess) return nullptr;
    return p;
}

void rsa_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

static int check_reads(rsa_ctx* ctx, const rsa_read_batch* rb) {
    if (!rb) return RSA_ERR_ARG;
    if (rb->n_reads && (!rb->seq || !rb->offsets || !rb->lengths)) { set_err(ctx, "null read buffers"); return RSA_ERR_ARG; }
    if (!ctx->d_rs && ctx->n_rs) { set_err(ctx, "context has no index"); return RSA_ERR_ARG; }
    return RSA_OK;
}

int rsa_randstrobes(rsa_ctx* ctx, const rsa_read_batch* rb, rsa_randstrobe_batch* out) {
    if (!ctx || !out) return RSA_ERR_ARG;
    int rc = check_reads(ctx, rb);
    if (rc) return rc;
    if (rb->n_reads == 0) { out->needed = 0; if (out->offsets) out->offsets[0] = 0; return RSA_OK; }
    HIPCHK(hipSetDevice(ctx->device));
    Lane* L = acquire_lane(ctx, LANE_SEED);
    if (!L) { set_err(ctx, "cannot create HIP stream"); return RSA_ERR_HIP; }
    LaneGuard guard{ctx, L};
    std::string err;
    rc = seed_randstrobes_run(L->sb, L->stream, ctx->ip, rb, out, err);
    if (rc) set_err(ctx, err);
    return rc;
}

int rsa_seed(rsa_ctx* ctx, const rsa_read_batch* rb, int32_t rescue_level, uint32_t rescue_cutoff, rsa_nam_batch* out) {
    if (!ctx || !out) return RSA_ERR_ARG;
    int rc = check_reads(ctx, rb);
    if (rc) return rc;
    if (rb->n_reads == 0) { out->needed = 0; if (out->offsets) out->offsets[0] = 0; return RSA_OK; }
    if (!ctx->d_rs || !ctx->d_starts) { set_err(ctx, "rsa_seed: context opened without an index"); return RSA_ERR_ARG; }
    HIPCHK(hipSetDevice(ctx->device));
    CallTimer ct(ctx, 0);
    Lane* L = ct.lane(LANE_SEED);
    if (!L) { set_err(ctx, "cannot create HIP stream"); return RSA_ERR_HIP; }
    LaneGuard guard{ctx, L};
    std::string err;
    SeedCounters c;
    L->kt.arm();
    rc = seed_run(L->sb, L->stream, L->kt, ctx->ip, rb, rescue_level, rescue_cutoff, out, err, c);
    if (rc) { set_err(ctx, err); return rc; }
    std::lock_guard<std::mutex> g(ctx->stat_m);
    if (L->kt.on) {
        L->kt.collect(ctx->stats.kernel_ms, ctx->stats.launches);
        for (int k = 0; k < RSA_K_COUNT; ++k) ctx->stats.alg_bytes[k] += c.alg_bytes[k];
        ctx->stats.seed_calls_timed++;
    }
    ctx->stats.seed_calls++;
    ctx->stats.reads += c.reads;
    ctx->stats.read_bases += c.read_bases;
    ctx->stats.query_randstrobes += c.qrs;
    ctx->stats.lookups_found += c.found;
    ctx->stats.filtered += c.filtered;
    ctx->stats.hits += c.hits;
    ctx->stats.nams += c.nams;
    ctx->stats.rescued_reads += c.rescued;
    ctx->stats.query_written += c.qw;
    ctx->stats.query_fixed_reads += c.qfix;
    ctx->stats.seed_second_trips += c.second_trip;
    return RSA_OK;
}

int rsa_get_stats(rsa_ctx* ctx, rsa_kernel_stats* out) {
    if (!ctx || !out) return RSA_ERR_ARG;
    std::lock_guard<std::mutex> g(ctx->stat_m);
    *out = ctx->stats;
    return RSA_OK;
}

void rsa_reset_stats(rsa_ctx* ctx) {
    if (!ctx) return;
    std::lock_guard<std::mutex> g(ctx->stat_m);
    ctx->stats = rsa_kernel_stats{};
}

}  // extern "C"
