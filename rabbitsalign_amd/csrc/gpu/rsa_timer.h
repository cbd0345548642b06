// rsa_timer.h -- per-launch HIP-event timing of the path's kernels.  Each lane
// owns one KTimer; events are recorded on the lane's stream around the launches
// of a timed call and read back after the lane's final synchronisation.
// RSA_KTIMER_EVERY=N times one call in N per lane (default 4; 1 = every call,
// 0 = none): event records go through the runtime's launch path, so timing every
// call costs the host pipeline CPU.  The kernel statistics (rsa_kernel_stats
// kernel_ms / launches / alg_bytes / dp_cells_timed) cover the timed calls.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <vector>

#include "../../../include/rsa_gpu.h"

inline int ktimer_every() {
    static const int n = [] {
        const char* v = getenv("RSA_KTIMER_EVERY");
        return v ? atoi(v) : 4;
    }();
    return n;
}

struct KTimer {
    std::vector<hipEvent_t> ev;
    std::vector<int> kind;
    size_t used = 0;
    bool on = true;              // this call is timed
    uint64_t calls = 0;

    void reset() { used = 0; kind.clear(); }
    // start of a call: decide whether it is timed
    void arm() {
        reset();
        const int every = ktimer_every();
        on = every > 0 && (calls++ % (uint64_t)every) == 0;
    }
    hipEvent_t take() {
        if (used == ev.size()) {
            hipEvent_t e = nullptr;
            (void)hipEventCreate(&e);
            ev.push_back(e);
        }
        return ev[used++];
    }
    void begin(hipStream_t s, int k) {
        if (!on) return;
        (void)hipEventRecord(take(), s);
        kind.push_back(k);
    }
    void end(hipStream_t s) { if (on) (void)hipEventRecord(take(), s); }
    // call after the stream has been synchronised
    void collect(double* ms, uint64_t* launches) const {
        for (size_t i = 0; i < kind.size(); ++i) {
            float t = 0;
            (void)hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]);
            ms[kind[i]] += t;
            launches[kind[i]] += 1;
        }
    }
    void destroy() {
        for (auto e : ev) (void)hipEventDestroy(e);
        ev.clear();
        reset();
    }
};

// per-call counters and algorithmic bytes of the seeding kernels
struct SeedCounters {
    uint64_t reads = 0, read_bases = 0, qrs = 0, found = 0, filtered = 0, hits = 0, nams = 0, rescued = 0;
    uint64_t qw = 0, qfix = 0;      // query randstrobes written out; reads query_lane made them for
    uint64_t second_trip = 0;       // the first download was short
    double alg_bytes[RSA_K_COUNT] = {0};
};
