// Random 128-byte line fetches from a large table (the seeding lookup's access
// pattern): lines/s for table sizes and fetch shapes.
//   mode 0: each lane fetches its own line as 8 x 16-byte loads (the lookup today)
//   mode 1: 8 lanes fetch one line together (16 B each), 8 lines per instruction
//   mode 2: each lane one 16-byte load of its line (request-rate ceiling)
//   mode 3: each lane fetches its own line as 2 x 64-byte (4 x dwordx4 issued back to back from 2 halves)
//   mode 4: mode 1 with indices through LDS and ~200 dependent hashes between rounds
// hipcc --offload-arch=gfx950 -O3 line_probe.hip -o line_probe; ./line_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}

template <int MODE>
__global__ void __launch_bounds__(256) k_probe(const uint4* __restrict__ t, uint64_t n_lines, int reps, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (int r = 0; r < reps; ++r) {
        if (MODE == 0) {
            const uint64_t L = mix(gid * 1315423911ULL + r) % n_lines;
            const uint4* p = t + L * 8;
            uint4 w[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = p[i];
#pragma unroll
            for (int i = 0; i < 8; ++i) acc += w[i].x ^ w[i].w;
        } else if (MODE == 1) {
            // lane's own line index, fetched cooperatively: instruction j loads the lines
            // of lanes 8j .. 8j+7, lane l taking 16 bytes (l % 8) of line (8j + l / 8)
            const uint64_t L = mix(gid * 1315423911ULL + r) % n_lines;
            uint4 w[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int src = 8 * j + (lane >> 3);
                const uint64_t Lj = __shfl(L, src, 64);
                w[j] = t[Lj * 8 + (lane & 7)];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) acc += w[j].x ^ w[j].w;
        } else if (MODE == 4) {
            // mode 1 with the seeding kernel's rhythm: line indices through LDS, the fetch
            // consumed, then ~4k cycles of dependent integer work before the next round
            __shared__ uint64_t s_l[4][64];
            const int w = threadIdx.x >> 6;
            const uint64_t L = mix(gid * 1315423911ULL + r) % n_lines;
            s_l[w][lane] = L;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            uint4 w8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) w8[j] = t[s_l[w][8 * j + (lane >> 3)] * 8 + (lane & 7)];
            uint64_t x = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) x += __ballot(w8[j].x > w8[j].y);
            uint64_t h = x + acc;
            for (int i = 0; i < 200; ++i) h = mix(h);
            acc += (uint32_t)h;
        } else if (MODE == 2) {
            const uint64_t L = mix(gid * 1315423911ULL + r) % n_lines;
            const uint4 w = t[L * 8];
            acc += w.x ^ w.w;
        } else {
            const uint64_t L = mix(gid * 1315423911ULL + r) % n_lines;
            const uint4* p = t + L * 8;
            uint4 w[2];
            w[0] = p[0]; w[1] = p[4];
            acc += w[0].x ^ w[1].w;
        }
    }
    if (acc == 0x12345678u) out[gid] = acc;
}

int main(int argc, char** argv) {
    const double gb_max = argc > 1 ? atof(argv[1]) : 32;
    // argv[2] = "frag": allocate 40 x 1 GB and free every other one first, as an index build's
    // temporaries would, so the table's physical pages may no longer be contiguous
    std::vector<void*> keep;
    if (argc > 2 && std::string(argv[2]) == "frag") {
        std::vector<void*> tmp(40, nullptr);
        for (auto& q : tmp) if (hipMalloc(&q, 1ull << 30) != hipSuccess) q = nullptr;
        for (size_t i = 0; i < tmp.size(); ++i) {
            if (!tmp[i]) continue;
            if (i % 2) (void)hipFree(tmp[i]); else keep.push_back(tmp[i]);
        }
        printf("fragmented: kept %zu GB\n", keep.size());
    }
    // argv[2] = "holes": fill the device with 256 MB blocks, then free every other one, so a
    // 32 GB table can only be made of 256 MB pieces
    if (argc > 2 && std::string(argv[2]) == "holes") {
        std::vector<void*> tmp;
        for (int i = 0; i < 1200; ++i) {
            void* q = nullptr;
            if (hipMalloc(&q, 256ull << 20) != hipSuccess) { (void)hipGetLastError(); break; }
            tmp.push_back(q);
        }
        for (size_t i = 0; i < tmp.size(); ++i) {
            if (i % 2) (void)hipFree(tmp[i]); else keep.push_back(tmp[i]);
        }
        printf("holes: %zu blocks of 256 MB allocated, every other freed\n", tmp.size());
    }
    uint4* t = nullptr;
    const size_t bytes_max = (size_t)(gb_max * (1ull << 30));
    if (hipMalloc(&t, bytes_max) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(t, 1, bytes_max);
    uint32_t* out = nullptr;
    hipMalloc(&out, 64u << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int threads = 1 << 20;          // 1M lanes, 16k waves
    for (double gb : {1.0, 32.0}) {
        if (gb > gb_max) continue;
        const uint64_t n_lines = (uint64_t)(gb * (1ull << 30)) / 128;
        for (int mode = 0; mode < 5; ++mode) {
            for (int reps : {1, 4}) {
                float best = 1e30f;
                for (int it = 0; it < 5; ++it) {
                    hipEventRecord(e0);
                    if (mode == 0) hipLaunchKernelGGL(k_probe<0>, dim3(threads / 256), dim3(256), 0, 0, t, n_lines, reps, out);
                    if (mode == 1) hipLaunchKernelGGL(k_probe<1>, dim3(threads / 256), dim3(256), 0, 0, t, n_lines, reps, out);
                    if (mode == 2) hipLaunchKernelGGL(k_probe<2>, dim3(threads / 256), dim3(256), 0, 0, t, n_lines, reps, out);
                    if (mode == 3) hipLaunchKernelGGL(k_probe<3>, dim3(threads / 256), dim3(256), 0, 0, t, n_lines, reps, out);
                    if (mode == 4) hipLaunchKernelGGL(k_probe<4>, dim3(threads / 256), dim3(256), 0, 0, t, n_lines, reps, out);
                    hipEventRecord(e1);
                    hipEventSynchronize(e1);
                    float ms;
                    hipEventElapsedTime(&ms, e0, e1);
                    if (it && ms < best) best = ms;
                }
                const double lines = (double)threads * reps;
                printf("table %5.1f GB mode %d reps %d: %8.3f ms  %7.2f Glines/s  (%6.2f TB/s of 128 B lines)\n", gb, mode,
                       reps, best, lines / best / 1e6, lines * 128 / best / 1e9);
            }
        }
    }
    return 0;
}
