// Device helpers shared by the k-means kernels (kmeans.hip: n_colors <= 5 on the cube
// table; kmeans_big.hip: any K up to LLFE_MAX_COLORS on the key list).
#pragma once
#include "llfe_internal.h"

namespace llfe {
namespace km {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// cv::RNG (multiply-with-carry): next() and uniform(0., 1.) as generateCentersPP uses them
__device__ __forceinline__ uint32_t cvrng_next(uint64_t &s) {
    s = (uint64_t)(uint32_t)s * 4164903690ull + (uint32_t)(s >> 32);
    return (uint32_t)s;
}
__device__ __forceinline__ double cvrng_double(uint64_t &s) {
    uint32_t t = cvrng_next(s);
    uint64_t v = ((uint64_t)t << 32) | cvrng_next(s);
    return (double)v * 5.4210108624275221700372640043497e-20;
}

// per-image cv::RNG state: splitmix64(seed + global index), 0 -> cv::RNG's default state,
// advanced to attempt `att`: each attempt's generateCentersPP consumes 1 + 6 (K - 1) draws
__device__ __forceinline__ uint64_t attempt_rng(unsigned long long seed, long long index, int att, int K) {
    uint64_t rng = splitmix64(seed + (unsigned long long)index);
    if (rng == 0) rng = 0xFFFFFFFFull;
    for (int q = 0, skip = att * (1 + 6 * (K - 1)); q < skip; q++) cvrng_next(rng);
    return rng;
}

// OpenCV normL2Sqr<float>(dims = 3) of the AVX2/FMA3 dispatch: t0*t0, fma(t1), fma(t2)
__device__ __forceinline__ float d2f(float x, float y, float z, float cx, float cy, float cz) {
    const float t0 = x - cx, t1 = y - cy, t2 = z - cz;
    float d = t0 * t0;
    d = __builtin_fmaf(t1, t1, d);
    d = __builtin_fmaf(t2, t2, d);
    return d;
}

// exact squared distance between integer colours (|a| <= 255: 24-bit multiplies)
__device__ __forceinline__ int d2i(int x, int y, int z, int cx, int cy, int cz) {
    const int a = x - cx, b = y - cy, c = z - cz;
    return __mul24(a, a) + __mul24(b, b) + __mul24(c, c);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__device__ __forceinline__ int key_r(uint32_t k) { return (int)((k >> 16) & 255u); }
__device__ __forceinline__ int key_g(uint32_t k) { return (int)((k >> 8) & 255u); }
__device__ __forceinline__ int key_b(uint32_t k) { return (int)(k & 255u); }

}  // namespace km
}  // namespace llfe
