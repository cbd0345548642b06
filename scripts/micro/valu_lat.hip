// VALU latency microbenchmark (measurement tool, not product code): cycles per
// instruction of packed-f16 / int32 chains on gfx950, dependent vs independent,
// one wave per SIMD.  Build: hipcc --offload-arch=gfx950 -O3 valu_lat.hip -o valu_lat
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 hh2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ hh2 hmax(hh2 a, hh2 b) { return __builtin_elementwise_maximum(a, b); }

template <int MODE>
__global__ void k(float* out, long long* cyc, int iters, float seed) {
    hh2 a = {(_Float16)seed, (_Float16)(seed + 1)}, b = a, c = a, d = a, e = a, f = a, g = a, h = a;
    const hh2 k1 = {(_Float16)1, (_Float16)1};
    int x0 = (int)seed, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {            // dependent chain: add -> max3 -> add -> max3 ...
#pragma unroll
            for (int j = 0; j < 16; ++j) { a = a - k1; a = hmax(hmax(a, b), c); }
        } else if (MODE == 1) {     // 8 independent chains interleaved
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                a = a - k1; b = b - k1; c = c - k1; d = d - k1; e = e - k1; f = f - k1; g = g - k1; h = h - k1;
                a = hmax(hmax(a, k1), a); b = hmax(hmax(b, k1), b); c = hmax(hmax(c, k1), c); d = hmax(hmax(d, k1), d);
                e = hmax(hmax(e, k1), e); f = hmax(hmax(f, k1), f); g = hmax(hmax(g, k1), g); h = hmax(hmax(h, k1), h);
            }
        } else if (MODE == 2) {     // int32 dependent chain sub -> max3
#pragma unroll
            for (int j = 0; j < 16; ++j) { x0 = x0 - 1; x0 = max(max(x0, x1), x2); }
        } else {                    // DPP dependent chain (row_shr:1 then add)
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                x0 = __builtin_amdgcn_update_dpp(0, x0, 0x111, 0xf, 0xf, false);
                x0 = x0 + 1;
            }
        }
    }
    long long t1 = clock64();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)a.x + (float)b.y + (float)c.x + (float)d.y + (float)e.x +
        (float)f.y + (float)g.x + (float)h.y + x0 + x1 + x2 + x3;
}

template <int MODE>
void run(const char* name, int waves_per_simd) {
    const int iters = 20000, blocks = 256 * waves_per_simd;   // 4 waves a block: waves_per_simd per SIMD
    float* out; long long* cyc;
    hipMalloc(&out, sizeof(float) * blocks * 256);
    hipMalloc(&cyc, sizeof(long long) * blocks);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 1.0f);   // warm
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 1.0f);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long c; hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
    const double instr = (double)iters * 32;   // VALU ops per wave in the timed loop
    printf("%-28s waves/SIMD %d: %.2f clock64 cycles per instr (wave 0), %.3f ms, %.1f G wave-instr/s chip-wide\n", name,
           waves_per_simd, c / instr, ms, blocks * 4.0 * instr / (ms * 1e-3) / 1e9);
    hipFree(out); hipFree(cyc);
}

int main() {
    for (int w : {1, 2, 4, 8}) {
        run<0>("f16 dependent sub/max3", w);
        run<1>("f16 8 independent chains", w);
        run<2>("i32 dependent sub/max3", w);
        run<3>("dpp+add dependent", w);
    }
    return 0;
}
