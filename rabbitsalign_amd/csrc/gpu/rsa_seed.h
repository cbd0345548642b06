// rsa_seed.h -- host/device shared declarations of the seeding kernels.
#pragma once
#include <chrono>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "../../../include/rsa_gpu.h"

struct SeedIndexParams {
    const rsa_ref_randstrobe* rs;
    const uint64_t* starts;
    uint64_t n;
    int bits;
    uint32_t filter_cutoff;
    int k, s, t, w_min, w_max, max_dist;
    uint64_t q;
    const char* ref;            // resident reference (contigs back to back), for the site checks
    const uint64_t* coff;       // [n_contigs + 1] contig offsets in ref (device)
};

struct SeedBufs {
    void* p[32] = {nullptr};
    size_t cap[32] = {0};
    void* h[12] = {nullptr};
    size_t hcap[12] = {0};
    hipEvent_t done = nullptr;   // blocking-sync event: the calling thread sleeps instead of spinning
};

// Wait for everything queued on `s` so far without burning a host core
// (hipEventBlockingSync); the host pipeline runs more workers than cores.
// time this thread spent blocked in stream_wait (the entry points read and reset it)
inline double& device_wait_ms() {
    static thread_local double ms = 0;
    return ms;
}

inline hipError_t stream_wait(hipStream_t s, hipEvent_t& e) {
    static const bool spin = [] { const char* v = getenv("RSA_SPIN_WAIT"); return v && v[0] == '1'; }();
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t err;
    if (spin) {
        err = hipStreamSynchronize(s);
    } else {
        err = hipSuccess;
        if (!e) err = hipEventCreateWithFlags(&e, hipEventBlockingSync | hipEventDisableTiming);
        if (err == hipSuccess) err = hipEventRecord(e, s);
        if (err == hipSuccess) err = hipEventSynchronize(e);
    }
    device_wait_ms() += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return err;
}

void seed_bufs_release(SeedBufs& b);
