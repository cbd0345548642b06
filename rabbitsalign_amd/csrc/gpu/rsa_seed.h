// rsa_seed.h -- host/device shared declarations of the seeding kernels.
#pragma once
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <hip/hip_runtime.h>
#include <mutex>
#include <stdint.h>
#include <stdlib.h>
#include "../../../include/rsa_gpu.h"

// Bucket lines: a device-side copy of the bucket table with each bucket's first
// entries beside its bounds, one 128-byte line per bucket -- 16 bytes {start,
// end} then up to BL_CAP RefRandstrobes (zero past the bucket's end; none when
// the bucket holds more).  A lookup in a bucket of at most BL_CAP entries reads
// one random line instead of two (bounds, then entries).  Built at rsa_open from
// the .sti arrays, which stay the index of record.
#define BL_CAP 7
struct __attribute__((aligned(128))) BucketLine {
    uint64_t start, end;
    rsa_ref_randstrobe e[BL_CAP];
};
static_assert(sizeof(BucketLine) == 128, "one bucket, one 128-byte line");

struct SeedIndexParams {
    const rsa_ref_randstrobe* rs;
    const uint64_t* starts;
    const BucketLine* lines;    // null: k_lookup reads starts + rs
    uint64_t n;
    int bits;
    uint32_t filter_cutoff;
    int k, s, t, w_min, w_max, max_dist;
    uint64_t q;
    const char* ref;            // resident reference (contigs back to back), for the site checks
    const uint64_t* coff;       // [n_contigs + 1] contig offsets in ref (device)
};

#define SEED_NBUF 40
#define SEED_NHBUF 8
struct SeedBufs {
    void* p[SEED_NBUF] = {nullptr};
    size_t cap[SEED_NBUF] = {0};
    void* h[SEED_NHBUF] = {nullptr};
    size_t hcap[SEED_NHBUF] = {0};
    uint64_t pool_n = 0;         // entries of the global-map / rescue pool (grows when a call runs out)
    // NAMs a read and pool words a NAM of the lane's last call: the first download's size
    // (a guess too small costs a second round trip, e.g. 9.4 NAMs a read on PE 2x250)
    double nam_rate = 0, mm_rate = 0;
    double resc_rate = -1;          // rescued reads a read in the lane's last call (-1: none yet)
    hipEvent_t done = nullptr;   // blocking-sync event (RSA_WAIT=event)
};

// Wait for everything queued on `s` so far without burning a host core; the
// host pipeline runs more workers than cores and a waiting worker hands its
// core to one that computes.
// time this thread spent blocked in stream_wait (the entry points read and reset it)
inline double& device_wait_ms() {
    static thread_local double ms = 0;
    return ms;
}

// The stream calls back (hipLaunchHostFunc) into a condition variable the
// thread sleeps on.  A blocking-sync event is not enough: the runtime spins on
// the HSA signal (with sched_yield) for a while before it sleeps, and with
// several waits a chunk that spinning took ~20 % of the workers' CPU time
// (RSA_PC_SAMPLE profile on the box).  Heap-held, so a wait abandoned on a
// stream error never leaves the callback a dangling pointer.
struct HostWaiter {
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
};
inline void host_waiter_wake(void* p) {
    HostWaiter* w = (HostWaiter*)p;
    {
        std::lock_guard<std::mutex> g(w->m);
        w->done = true;
    }
    w->cv.notify_one();
}

// RSA_WAIT: "callback" (default), "event" (blocking-sync event), "spin" (hipStreamSynchronize)
inline hipError_t stream_wait(hipStream_t s, hipEvent_t& e) {
    static const int mode = [] {
        const char* v = getenv("RSA_WAIT");
        if (v && strcmp(v, "event") == 0) return 1;
        if (v && strcmp(v, "spin") == 0) return 2;
        return 0;
    }();
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t err = hipSuccess;
    if (mode == 2) {
        err = hipStreamSynchronize(s);
    } else if (mode == 1) {
        if (!e) err = hipEventCreateWithFlags(&e, hipEventBlockingSync | hipEventDisableTiming);
        if (err == hipSuccess) err = hipEventRecord(e, s);
        if (err == hipSuccess) err = hipEventSynchronize(e);
    } else {
        HostWaiter* w = new HostWaiter();
        err = hipLaunchHostFunc(s, host_waiter_wake, w);
        if (err != hipSuccess) {
            delete w;
        } else {
            std::unique_lock<std::mutex> l(w->m);
            while (!w->cv.wait_for(l, std::chrono::seconds(1), [&] { return w->done; })) {
                // a failed stream never calls back: look at it every second -- without
                // holding w->m, which the runtime's callback thread needs to wake us
                l.unlock();
                const hipError_t q = hipStreamQuery(s);
                l.lock();
                if (q != hipErrorNotReady && q != hipSuccess && !w->done) { err = q; break; }
            }
            const bool done = w->done;
            l.unlock();
            if (done) delete w;                             // else left to a callback that may still come
        }
    }
    device_wait_ms() += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return err;
}

void seed_bufs_release(SeedBufs& b);

// RSA_POISON=1 (tests): fill every new device buffer with 0xA5 bytes, so a kernel
// that reads memory nothing wrote sees the same garbage in every run instead of
// whatever a freed allocation left (fresh pages happen to be zero).  Results never
// depend on it; an uninitialised read then fails every time, not now and then.
// RSA_POISON=2 (tests): also refill every buffer of a lane at the start of each call, in the
// call's stream, so a kernel that reads what an earlier call left behind fails too.
inline bool rsa_poison_every() {
    static const bool on = getenv("RSA_POISON") && getenv("RSA_POISON")[0] == '2';
    return on;
}
inline hipError_t rsa_poison(void* p, size_t n) {
    static const bool on = getenv("RSA_POISON") && (getenv("RSA_POISON")[0] == '1' || getenv("RSA_POISON")[0] == '2');
    if (!on) return hipSuccess;
    // hipMemset runs on the null stream, which the lanes' non-blocking streams do not wait
    // for: finish it before the caller queues the buffer's first upload
    const hipError_t e = hipMemset(p, 0xA5, n);
    return e == hipSuccess ? hipDeviceSynchronize() : e;
}
