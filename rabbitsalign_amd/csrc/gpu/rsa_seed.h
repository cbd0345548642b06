// rsa_seed.h -- host/device shared declarations of the seeding kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../../include/rsa_gpu.h"

struct SeedIndexParams {
    const rsa_ref_randstrobe* rs;
    const uint64_t* starts;
    uint64_t n;
    int bits;
    uint32_t filter_cutoff;
    int k, s, t, w_min, w_max, max_dist;
    uint64_t q;
};

struct SeedBufs {
    void* p[24] = {nullptr};
    size_t cap[24] = {0};
    void* h[8] = {nullptr};
    size_t hcap[8] = {0};
};

void seed_bufs_release(SeedBufs& b);
