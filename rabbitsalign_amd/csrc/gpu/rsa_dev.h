// rsa_dev.h -- device-side helpers shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RSA_WAVE 64

// Base codes as selects on the case-folded byte, no branches: a switch compiles to
// a tree of divergent branches, and every kernel that translates bases (staging
// loops over a window, per-row lookups) paid its exec-mask bookkeeping per byte.
// c | 0x20 equals 'a'/'c'/'g'/'t'/'u' only for that letter in either case.

// SSW base translation (ext/ssw/ssw_cpp.cpp:12-25, kBaseTranslation):
// A/a/U/u -> 0, C/c -> 1, G/g -> 2, T/t -> 3, everything else -> 4.
__device__ __forceinline__ int ssw_code(unsigned char c) {
    const uint32_t u = (uint32_t)c | 0x20u;
    int r = 4;
    r = u == 't' ? 3 : r;
    r = u == 'g' ? 2 : r;
    r = u == 'c' ? 1 : r;
    r = (u == 'a' || u == 'u') ? 0 : r;
    return r;
}

// seq_nt4_table (src/randstrobes.cpp:14-31): U/u -> 3 (unlike SSW)
__device__ __forceinline__ int nt4_code(unsigned char c) {
    const uint32_t u = (uint32_t)c | 0x20u;
    int r = 4;
    r = (u == 't' || u == 'u') ? 3 : r;
    r = u == 'g' ? 2 : r;
    r = u == 'c' ? 1 : r;
    r = u == 'a' ? 0 : r;
    return r;
}

// lane l receives lane l-1's value; lane 0 receives 0 (DPP wave_shr:1)
__device__ __forceinline__ int wave_shr1(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false);
}

__device__ __forceinline__ int wave_min_i32(int v) {
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ int wave_max_i32(int v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

// xxh64 of a single u64 (src/hash.hpp:105-118)
__device__ __forceinline__ uint64_t xxh64_u64(uint64_t input) {
    const uint64_t P1 = 0x9E3779B185EBCA87ULL, P2 = 0xC2B2AE3D27D4EB4FULL, P3 = 0x165667B19E3779F9ULL,
                   P4 = 0x85EBCA77C2B2AE63ULL, P5 = 0x27D4EB2F165667C5ULL;
    uint64_t acc = P5 + 8;
    uint64_t k1 = input * P2;
    k1 = (k1 << 31) | (k1 >> 33);
    acc ^= k1 * P1;
    acc = ((acc << 27) | (acc >> 37)) * P1 + P4;
    acc ^= acc >> 33;
    acc *= P2;
    acc ^= acc >> 29;
    acc *= P3;
    acc ^= acc >> 32;
    return acc;
}
