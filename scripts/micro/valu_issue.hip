// VALU issue-rate microbenchmark (measurement tool, not product code).
// Question it answers: at how many cycles per wave64 instruction does a gfx950
// SIMD issue each VALU form the DP kernels use, with 1..8 waves per SIMD?
// Every mode is one inline-asm block of 8 independent chains over fixed VGPRs
// (v[40:71], chosen so the three sources of an instruction sit in different
// banks), 128 instructions a loop iteration, so the compiler cannot change the
// instruction count.  Build: hipcc --offload-arch=gfx950 -O3 valu_issue.hip -o valu_issue
#include <hip/hip_runtime.h>
#include <cstdio>

// 8 chains: destination/first source v40..v47, second source v48..v55, third v56..v63
#define CH8(OP)                                                   \
    OP " v40, v40, v49, v58\n" OP " v41, v41, v50, v59\n"          \
    OP " v42, v42, v51, v60\n" OP " v43, v43, v52, v61\n"          \
    OP " v44, v44, v53, v62\n" OP " v45, v45, v54, v63\n"          \
    OP " v46, v46, v55, v56\n" OP " v47, v47, v48, v57\n"
#define CH8_2(OP)                                                 \
    OP " v40, v40, v49\n" OP " v41, v41, v50\n"                    \
    OP " v42, v42, v51\n" OP " v43, v43, v52\n"                    \
    OP " v44, v44, v53\n" OP " v45, v45, v54\n"                    \
    OP " v46, v46, v55\n" OP " v47, v47, v48\n"
#define X16(S) S S S S S S S S S S S S S S S S

#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", \
             "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"

template <int MODE>
__global__ void __launch_bounds__(256) k(float* out, long long* cyc, int iters) {
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) asm volatile(X16(CH8("v_pk_maximum3_f16")) ::: CLOB);
        else if (MODE == 1) asm volatile(X16(CH8_2("v_pk_add_f16")) ::: CLOB);
        else if (MODE == 2) asm volatile(X16(CH8("v_max3_i32")) ::: CLOB);
        else if (MODE == 3) asm volatile(X16(CH8_2("v_add_u32")) ::: CLOB);
        else if (MODE == 4) asm volatile(X16(CH8("v_max3_f32")) ::: CLOB);
        else if (MODE == 5) asm volatile(X16(CH8_2("v_add_f32")) ::: CLOB);
        else if (MODE == 6) asm volatile(X16(CH8("v_fma_f32")) ::: CLOB);
        else if (MODE == 7) asm volatile(X16(CH8_2("v_pk_max_i16")) ::: CLOB);
        else if (MODE == 8) asm volatile(X16(CH8("v_pk_fma_f16")) ::: CLOB);
        else if (MODE == 10) asm volatile(X16(CH8("v_max3_i16")) ::: CLOB);
        else if (MODE == 11) asm volatile(X16(CH8_2("v_and_b32")) ::: CLOB);
    }
    long long t1 = clock64();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)(t1 - t0);
}

template <int MODE>
void run(const char* name, int waves_per_simd) {
    const int iters = 4000, blocks = 256 * waves_per_simd;   // 4 waves a block: waves_per_simd per SIMD
    float* out; long long* cyc;
    hipMalloc(&out, sizeof(float) * blocks * 256);
    hipMalloc(&cyc, sizeof(long long) * blocks);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);   // warm
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long c; hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
    const double instr = (double)iters * 128;   // VALU instructions per wave in the timed loop
    const double rate = blocks * 4.0 * instr / (ms * 1e-3);
    printf("%-20s waves/SIMD %d: wave0 %.2f clk/instr, %.3f ms, %.1f G wave-instr/s = %.2f cyc/instr/SIMD at 2.4 GHz\n",
           name, waves_per_simd, c / instr, ms, rate / 1e9, 1024.0 * 2.4e9 / rate);
    hipFree(out); hipFree(cyc);
    hipEventDestroy(e0); hipEventDestroy(e1);
}

int main() {
    for (int w : {1, 2, 4}) {
        run<0>("v_pk_maximum3_f16", w);
        run<1>("v_pk_add_f16", w);
        run<2>("v_max3_i32", w);
        run<3>("v_add_u32", w);
        run<4>("v_max3_f32", w);
        run<5>("v_add_f32", w);
        run<6>("v_fma_f32", w);
        run<7>("v_pk_max_i16", w);
        run<8>("v_pk_fma_f16", w);
        run<10>("v_max3_i16", w);
        run<11>("v_and_b32", w);
    }
    return 0;
}
