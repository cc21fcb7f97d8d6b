// Dominant-colour path of ColorExtractor.extract_colors on gfx950
// (app/services/analyze/color_extractor.py:217-236).
//
//  k_color_bitmap   BGR->RGB (:150-151), + int8(N(0,0.5)) noise and clip (:223-225),
//                   packed key R<<16|G<<8|B into a 2^24-bit presence bitmap per image
//                   (+ a 32768-bit occupancy map of 512-bit blocks).  Replaces the
//                   sort inside np.unique(pixels, axis=0) (:177).
//  k_color_compact  bitmap -> ascending key list (= np.unique row order), clearing the
//                   bitmap behind itself so it never needs a separate memset.
// The k-means over the key list lives in kmeans.hip.
#include "llfe_internal.h"

namespace llfe {
namespace {

// ------------------------------------------------------------------ Philox4x32-10
struct U4 {
    uint32_t x, y, z, w;
};
__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}
// trunc(0.5 * Z) for Z ~ N(0,1) from one uniform u32 via exact tail thresholds:
// P(Z <= -2) = 0.0227501319, P(Z <= -4) = 3.16712e-5, P(Z <= -6) = 9.8659e-10.
__device__ __forceinline__ int noise_from_u32(uint32_t u) {
    const uint32_t T1 = 97711073u, T2 = 136027u, T3 = 4u;
    uint32_t v = u < 0x80000000u ? u : ~u;
    int mag = (v < T1) + (v < T2) + (v < T3);
    return u < 0x80000000u ? -mag : mag;
}

constexpr int CB = 256;   // threads per block in the bitmap kernel
constexpr int PPT = 16;   // consecutive pixels per thread per step (48 B of BGR)
constexpr int HSLOTS = CB * PPT;  // LDS hash slots = pixels per block step (load factor <= 1)
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

// Insert (word, bits) into the block's LDS open-addressing table; returns false when
// the probe budget is exhausted (the caller then ORs straight into global memory).
__device__ __forceinline__ bool hash_or(uint32_t *tags, uint32_t *vals, uint32_t word, uint32_t bits) {
    uint32_t slot = (word * 2654435761u) >> (32 - 12);
#pragma unroll 1
    for (int probe = 0; probe < 32; probe++, slot = (slot + 1) & (HSLOTS - 1)) {
        uint32_t t = tags[slot];
        if (t == kEmpty) t = atomicCAS(tags + slot, kEmpty, word);
        if (t == kEmpty || t == word) {
            atomicOr(vals + slot, bits);
            return true;
        }
    }
    return false;
}

// grid: (blocks_per_image, n).  A block step covers 4096 pixels (16 consecutive per
// thread, read as three 16-byte loads).  Keys are merged per 32-key bitmap word in an
// LDS hash table and the occupancy map is mirrored in LDS, so global memory sees one
// fire-and-forget atomicOr per distinct word per step (and per occupancy word per
// block) instead of one per pixel: flat UI regions and the hot occupancy words never
// become same-address atomic storms in L2.
__global__ __launch_bounds__(CB) void k_color_bitmap(const uint8_t *__restrict__ bgr, const int8_t *__restrict__ noise,
                                                     long long P, uint32_t seed_lo, uint32_t seed_hi,
                                                     long long index_base, uint32_t *__restrict__ bitmap,
                                                     uint32_t *__restrict__ occ) {
    __shared__ uint32_t tags[HSLOTS];
    __shared__ uint32_t vals[HSLOTS];
    __shared__ uint32_t locc[kOccWords];
    const int img = blockIdx.y;
    const uint8_t *src = bgr + (size_t)img * P * 3;
    const int8_t *nz = noise ? noise + (size_t)img * P * 3 : nullptr;
    uint32_t *bm = bitmap + (size_t)img * kBitmapWords;
    uint32_t *oc = occ + (size_t)img * kOccWords;
    const uint32_t g_lo = (uint32_t)(index_base + img), g_hi = (uint32_t)((index_base + img) >> 32);
    for (int i = threadIdx.x; i < HSLOTS; i += CB) {
        tags[i] = kEmpty;
        vals[i] = 0;
    }
    for (int i = threadIdx.x; i < kOccWords; i += CB) locc[i] = 0;
    const long long nchunks = (P + PPT - 1) / PPT;
    const long long nsteps = (nchunks + CB - 1) / CB;
    __syncthreads();
    for (long long st = blockIdx.x; st < nsteps; st += gridDim.x) {
        const long long c = st * CB + threadIdx.x;
        const long long p0 = c * PPT;
        const int cnt = (int)max(0LL, min((long long)PPT, P - p0));
        uint8_t px[3 * PPT];
        int8_t nv[3 * PPT];
        const uint8_t *sp = src + p0 * 3;
        if (cnt == PPT && (((uintptr_t)sp) & 15) == 0) {
            const uint4 *s16 = (const uint4 *)sp;
            *(uint4 *)&px[0] = s16[0];
            *(uint4 *)&px[16] = s16[1];
            *(uint4 *)&px[32] = s16[2];
        } else {
            for (int i = 0; i < 3 * PPT; i++) px[i] = i < cnt * 3 ? sp[i] : 0;
        }
        if (nz) {
            const int8_t *np_ = nz + p0 * 3;
            if (cnt == PPT && (((uintptr_t)np_) & 15) == 0) {
                const uint4 *n16 = (const uint4 *)np_;
                *(uint4 *)&nv[0] = n16[0];
                *(uint4 *)&nv[16] = n16[1];
                *(uint4 *)&nv[32] = n16[2];
            } else {
                for (int i = 0; i < 3 * PPT; i++) nv[i] = i < cnt * 3 ? np_[i] : 0;
            }
        }
        uint32_t prev = kEmpty;
#pragma unroll
        for (int i = 0; i < PPT; i++) {
            int b = px[3 * i], g = px[3 * i + 1], r = px[3 * i + 2];
            int nr, ng, nb;
            if (nz) {  // RGB-order stream: noise[p*3 + {R,G,B}]
                nr = nv[3 * i];
                ng = nv[3 * i + 1];
                nb = nv[3 * i + 2];
            } else {
                U4 u = philox(U4{(uint32_t)(p0 + i), g_lo, g_hi, 0x4C4C4645u}, seed_lo, seed_hi);
                nr = noise_from_u32(u.x);
                ng = noise_from_u32(u.y);
                nb = noise_from_u32(u.z);
            }
            r = min(max(r + nr, 0), 255);
            g = min(max(g + ng, 0), 255);
            b = min(max(b + nb, 0), 255);
            const uint32_t key = ((uint32_t)r << 16) | ((uint32_t)g << 8) | (uint32_t)b;
            if (i < cnt && key != prev) {
                if (!hash_or(tags, vals, key >> 5, 1u << (key & 31))) {
                    atomicOr(bm + (key >> 5), 1u << (key & 31));
                    atomicOr(locc + (key >> 14), 1u << ((key >> 9) & 31));
                }
                prev = key;
            }
        }
        __syncthreads();
        // flush the step's words (one global atomic per distinct word) and reset
        for (int i = threadIdx.x; i < HSLOTS; i += CB) {
            const uint32_t word = tags[i];
            if (word != kEmpty) {
                atomicOr(bm + word, vals[i]);
                atomicOr(locc + (word >> 9), 1u << ((word >> 4) & 31));
                tags[i] = kEmpty;
                vals[i] = 0;
            }
        }
        __syncthreads();
    }
    for (int i = threadIdx.x; i < kOccWords; i += CB)
        if (locc[i]) atomicOr(oc + i, locc[i]);
}

// ------------------------------------------------------------------ compaction
constexpr int PT = 1024;  // threads: thread t owns occupancy word t (32 blocks of 512 keys)

__device__ __forceinline__ long long block_excl_scan_1024(long long v, long long *tmp, long long *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    long long x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        long long y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) tmp[wid] = x;
    __syncthreads();
    if (wid == 0) {
        long long w = lane < (PT / 64) ? tmp[lane] : 0;
        long long s = w;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            long long y = __shfl_up(s, off);
            if (lane >= off) s += y;
        }
        if (lane < PT / 64) tmp[lane] = s - w;
        if (lane == PT / 64 - 1) tmp[PT / 64] = s;
    }
    __syncthreads();
    long long r = tmp[wid] + x - v;
    *total = tmp[PT / 64];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(PT) void k_color_compact(uint32_t *__restrict__ bitmap, uint32_t *__restrict__ occ,
                                                      uint32_t *__restrict__ keys, long long key_stride,
                                                      long long *__restrict__ n_unique) {
    __shared__ long long tmp[PT / 64 + 1];
    const int img = blockIdx.x;
    const int t = threadIdx.x;
    uint32_t *bm = bitmap + (size_t)img * kBitmapWords;
    uint32_t ow = occ[(size_t)img * kOccWords + t];
    long long cnt = 0;
    for (uint32_t w = ow; w; w &= w - 1) {
        int b = __builtin_ctz(w);
        const uint4 *blk = (const uint4 *)(bm + ((size_t)(t * 32 + b) << 4));
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint4 v = blk[q];
            cnt += __builtin_popcount(v.x) + __builtin_popcount(v.y) + __builtin_popcount(v.z) + __builtin_popcount(v.w);
        }
    }
    long long total;
    long long pos = block_excl_scan_1024(cnt, tmp, &total);
    uint32_t *out = keys + (size_t)img * key_stride;
    for (uint32_t w = ow; w; w &= w - 1) {
        int b = __builtin_ctz(w);
        uint32_t blk_id = (uint32_t)(t * 32 + b);
        uint32_t *blk = bm + ((size_t)blk_id << 4);
        for (int q = 0; q < 16; q++) {
            uint32_t word = blk[q];
            uint32_t kbase = (blk_id << 9) | ((uint32_t)q << 5);
            while (word) {
                int bit = __builtin_ctz(word);
                out[pos++] = kbase | (uint32_t)bit;
                word &= word - 1;
            }
            blk[q] = 0;
        }
    }
    occ[(size_t)img * kOccWords + t] = 0;
    if (t == 0) n_unique[img] = total;
}

}  // namespace

hipError_t launch_color_bitmap(const uint8_t *bgr, const int8_t *noise, int n, int h, int w, uint64_t seed,
                               int64_t index_base, uint32_t *bitmap, uint32_t *occ, hipStream_t s) {
    long long P = (long long)h * w;
    long long per_block = (long long)CB * PPT * 4;  // 4 block steps (16384 px) per block
    int bx = (int)min((P + per_block - 1) / per_block, 4096LL);
    if (bx < 1) bx = 1;
    hipLaunchKernelGGL(k_color_bitmap, dim3(bx, n), dim3(CB), 0, s, bgr, noise, P, (uint32_t)seed,
                       (uint32_t)(seed >> 32), (long long)index_base, bitmap, occ);
    return hipGetLastError();
}

hipError_t launch_color_compact(uint32_t *bitmap, uint32_t *occ, int n, uint32_t *keys, int64_t key_stride,
                                int64_t *n_unique, hipStream_t s) {
    hipLaunchKernelGGL(k_color_compact, dim3(n), dim3(PT), 0, s, bitmap, occ, keys, (long long)key_stride,
                       (long long *)n_unique);
    return hipGetLastError();
}


}  // namespace llfe
