// Dominant-colour path of ColorExtractor.extract_colors on gfx950
// (app/services/analyze/color_extractor.py:217-236).
//
//  k_color_bitmap   BGR->RGB (:150-151), + int8(N(0,0.5)) noise and clip (:223-225),
//                   packed key R<<16|G<<8|B into a 2^24-bit presence bitmap per image
//                   (+ a 32768-bit occupancy map of 512-bit blocks).  Replaces the
//                   sort inside np.unique(pixels, axis=0) (:177).
//  k_color_compact  bitmap -> ascending key list (= np.unique row order), clearing the
//                   bitmap behind itself so it never needs a separate memset.
//  k_kmeans         cv2.kmeans(float32(unique), K, None, (EPS+MAX_ITER, 200, 0.2), 10,
//                   KMEANS_PP_CENTERS) (:189-196): one 256-thread workgroup per
//                   (image, attempt), k-means++ with 3 trials per centre and Lloyd
//                   iterations, restating OpenCV's kmeans.cpp arithmetic (cv::RNG MWC
//                   stream, float32 normL2Sqr, empty-cluster repair, compactness).
//  k_kmeans_finalize best attempt -> centers.astype(uint8) (:197) + bincount (:232).
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

constexpr int CB = 256;  // threads per block in the bitmap kernel

__device__ __forceinline__ void set_key(uint32_t key, uint32_t *bm, uint32_t *occ) {
    uint32_t word = key >> 5, bit = 1u << (key & 31);
    uint32_t cur = __hip_atomic_load(bm + word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!(cur & bit)) {
        atomicOr(bm + word, bit);
        uint32_t ow = key >> 14, ob = 1u << ((key >> 9) & 31);
        uint32_t oc = __hip_atomic_load(occ + ow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!(oc & ob)) atomicOr(occ + ow, ob);
    }
}

// grid: (blocks_per_image, n). Each thread handles 4 consecutive pixels per step.
__global__ __launch_bounds__(CB) void k_color_bitmap(const uint8_t *__restrict__ bgr, const int8_t *__restrict__ noise,
                                                     long long P, uint32_t seed_lo, uint32_t seed_hi,
                                                     long long index_base, uint32_t *__restrict__ bitmap,
                                                     uint32_t *__restrict__ occ) {
    const int img = blockIdx.y;
    const uint8_t *src = bgr + (size_t)img * P * 3;
    const int8_t *nz = noise ? noise + (size_t)img * P * 3 : nullptr;
    uint32_t *bm = bitmap + (size_t)img * kBitmapWords;
    uint32_t *oc = occ + (size_t)img * kOccWords;
    const long long gimg = index_base + img;
    const long long stride = (long long)gridDim.x * CB * 4;
    uint32_t prev_lane_key = 0xFFFFFFFFu;
    for (long long p0 = ((long long)blockIdx.x * CB + threadIdx.x) * 4; p0 < P + 0; p0 += stride) {
        uint32_t keys[4];
        int cnt = (int)min(4LL, P - p0);
        uint8_t px[12];
        int8_t nv[12];
        if (cnt == 4 && (((uintptr_t)(src + p0 * 3)) & 3) == 0) {
            const uint32_t *s32 = (const uint32_t *)(src + p0 * 3);
            uint32_t a = s32[0], b = s32[1], c = s32[2];
            *(uint32_t *)&px[0] = a;
            *(uint32_t *)&px[4] = b;
            *(uint32_t *)&px[8] = c;
        } else {
            for (int i = 0; i < 12; i++) px[i] = i < cnt * 3 ? src[p0 * 3 + i] : 0;
        }
        if (nz) {
            if (cnt == 4 && (((uintptr_t)(nz + p0 * 3)) & 3) == 0) {
                const uint32_t *n32 = (const uint32_t *)(nz + p0 * 3);
                *(uint32_t *)&nv[0] = n32[0];
                *(uint32_t *)&nv[4] = n32[1];
                *(uint32_t *)&nv[8] = n32[2];
            } else {
                for (int i = 0; i < 12; i++) nv[i] = i < cnt * 3 ? nz[p0 * 3 + i] : 0;
            }
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            int b = px[3 * i], g = px[3 * i + 1], r = px[3 * i + 2];
            int nr, ng, nb;
            if (nz) {  // RGB-order stream: noise[p*3 + {R,G,B}]
                nr = nv[3 * i];
                ng = nv[3 * i + 1];
                nb = nv[3 * i + 2];
            } else {
                U4 u = philox(U4{(uint32_t)(p0 + i), (uint32_t)gimg, (uint32_t)(gimg >> 32), 0x4C4C4645u}, seed_lo,
                              seed_hi);
                nr = noise_from_u32(u.x);
                ng = noise_from_u32(u.y);
                nb = noise_from_u32(u.z);
            }
            r = min(max(r + nr, 0), 255);
            g = min(max(g + ng, 0), 255);
            b = min(max(b + nb, 0), 255);
            keys[i] = i < cnt ? (((uint32_t)r << 16) | ((uint32_t)g << 8) | (uint32_t)b) : 0xFFFFFFFFu;
        }
        // skip keys equal to the previous pixel (this lane or the lane before)
        uint32_t left = __shfl_up(keys[3], 1);
        if ((threadIdx.x & 63) == 0) left = prev_lane_key;
        prev_lane_key = __shfl(keys[3], 63);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint32_t k = keys[i];
            uint32_t before = i == 0 ? left : keys[i - 1];
            if (k != 0xFFFFFFFFu && k != before) set_key(k, bm, oc);
        }
    }
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

// ------------------------------------------------------------------ k-means
constexpr int KT = 256;     // threads per (image, attempt) workgroup
constexpr int KWAVES = KT / 64;
constexpr int STEP = 256;   // points per wave step (64 lanes x 4)

__device__ __forceinline__ uint32_t cvrng_next(uint64_t &s) {
    s = (uint64_t)(uint32_t)s * 4164903690ull + (uint32_t)(s >> 32);
    return (uint32_t)s;
}
__device__ __forceinline__ double cvrng_double(uint64_t &s) {
    uint32_t t = cvrng_next(s);
    uint64_t v = ((uint64_t)t << 32) | cvrng_next(s);
    return (double)v * 5.4210108624275221700372640043497e-20;
}

// OpenCV normL2Sqr<float>(dims=3), AVX2/FMA3 dispatch: t0*t0, fma(t1), fma(t2)
__device__ __forceinline__ float d2(float x, float y, float z, float cx, float cy, float cz) {
    float t0 = x - cx, t1 = y - cy, t2 = z - cz;
    float d = t0 * t0;
    d = __builtin_fmaf(t1, t1, d);
    d = __builtin_fmaf(t2, t2, d);
    return d;
}

__device__ __forceinline__ void key_xyz(uint32_t k, float &x, float &y, float &z) {
    x = (float)(k >> 16);
    y = (float)((k >> 8) & 255u);
    z = (float)(k & 255u);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

struct KmSmem {
    // lane-private Lloyd accumulators: A = x | y<<32, B = z | 1<<32 (per cluster)
    unsigned long long accA[kMaxK][KT];
    unsigned long long accB[kMaxK][KT];
    unsigned long long red[20][8];
    unsigned long long wtot[KWAVES][4];
    double dred[KWAVES];
    float c[kMaxK][3];     // current centres
    float cprev[kMaxK][3]; // centres of the last assignment
    float cc[kMaxK][3];    // k-means++ chosen centres
    long long sums[kMaxK][3];
    int counts[kMaxK];
    int moved_idx[kMaxK];
    int moved_lbl[kMaxK];
    int n_moved;
    long long scan_tmp[KT / 64 + 1];
    int found_step[3];
    unsigned long long found_excl[3];
    int ci[3];
    int flag;
    double maxd[KWAVES];
    int maxi[KWAVES];
};

// load the 4 keys of lane at step s (points s*256 + lane*4 .. +3); invalid -> mask
__device__ __forceinline__ int load4(const uint32_t *__restrict__ pts, long long N, long long s, int lane, uint32_t k[4]) {
    long long i0 = s * STEP + lane * 4;
    if (i0 + 3 < N) {
        uint4 v = *(const uint4 *)(pts + i0);
        k[0] = v.x; k[1] = v.y; k[2] = v.z; k[3] = v.w;
        return 4;
    }
    int c = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if (i0 + j < N) { k[j] = pts[i0 + j]; c++; } else k[j] = 0;
    }
    return c;
}

// label of point (x,y,z) against K centres (first minimum wins, as in
// KMeansDistanceComputer: `if (min_dist > dist)`)
__device__ __forceinline__ int argmin_label(float x, float y, float z, const float (*c)[3], int K, float *bestd) {
    float best = d2(x, y, z, c[0][0], c[0][1], c[0][2]);
    int lbl = 0;
#pragma unroll
    for (int k = 1; k < kMaxK; k++) {
        if (k < K) {
            float d = d2(x, y, z, c[k][0], c[k][1], c[k][2]);
            bool lt = d < best;
            best = lt ? d : best;
            lbl = lt ? k : lbl;
        }
    }
    *bestd = best;
    return lbl;
}

__device__ __forceinline__ int moved_label(const KmSmem &sm, long long i, int lbl) {
    for (int m = 0; m < sm.n_moved; m++)
        if (sm.moved_idx[m] == i) lbl = sm.moved_lbl[m];
    return lbl;
}

__global__ __launch_bounds__(KT) void k_kmeans(const uint32_t *__restrict__ keys, long long key_stride,
                                               const long long *__restrict__ n_unique, int n_colors,
                                               const uint64_t *__restrict__ rng_states,
                                               const int *__restrict__ order, uint32_t *__restrict__ scratch,
                                               long long scratch_stride, KmeansAttemptOut *__restrict__ out) {
    __shared__ KmSmem sm;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int img = order[blockIdx.x / kAttempts];
    const int att = blockIdx.x % kAttempts;
    const long long N = n_unique[img];
    const int K = (int)min((long long)n_colors, N);
    KmeansAttemptOut *o = out + (size_t)img * kAttempts + att;
    if (K <= 1) {
        if (tid == 0) {
            o->compactness = 0.0;
            o->iters = 0;
        }
        return;
    }
    const uint32_t *pts = keys + (size_t)img * key_stride;
    const long long M = (N + STEP - 1) / STEP;            // steps
    const long long Mw = (M + KWAVES - 1) / KWAVES;       // steps per wave
    const long long s_begin = wid * Mw, s_end = min(M, s_begin + Mw);
    uint32_t *ss = scratch + ((size_t)img * kAttempts + att) * (size_t)scratch_stride;  // 4 arrays of M
    uint32_t *SS[4] = {ss, ss + M, ss + 2 * M, ss + 3 * M};

    // cv::RNG state for this attempt: draws per attempt = 1 + 6*(K-1)
    uint64_t rng = rng_states[img];
    {
        long long skip = (long long)att * (1 + 6 * (K - 1));
        for (long long q = 0; q < skip; q++) cvrng_next(rng);
    }

    // ------------------------------------------------ k-means++ (generateCentersPP)
    int cur = 0;  // index of the step-sum array holding D (current min distances)
    {
        uint32_t c0 = cvrng_next(rng) % (uint32_t)N;
        if (tid == 0) {
            float x, y, z;
            key_xyz(pts[c0], x, y, z);
            sm.cc[0][0] = x; sm.cc[0][1] = y; sm.cc[0][2] = z;
        }
        __syncthreads();
        float cx = sm.cc[0][0], cy = sm.cc[0][1], cz = sm.cc[0][2];
        unsigned long long wt = 0;
        for (long long s = s_begin; s < s_end; s++) {
            uint32_t k[4];
            int c = load4(pts, N, s, lane, k);
            uint32_t ls = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                float x, y, z;
                key_xyz(k[j], x, y, z);
                float d = d2(x, y, z, cx, cy, cz);
                ls += j < c ? (uint32_t)d : 0u;
            }
            uint32_t st = wave_sum(ls);
            if (lane == 0) SS[0][s] = st;
            wt += st;
        }
        if (lane == 0) sm.wtot[wid][0] = wt;
    }
    __syncthreads();
    unsigned long long sum0 = 0;
    for (int w = 0; w < KWAVES; w++) sum0 += sm.wtot[w][0];
    __syncthreads();

    for (int kk = 1; kk < K; kk++) {
        double p[3];
        for (int j = 0; j < 3; j++) p[j] = cvrng_double(rng) * (double)sum0;
        // ---- locate ci_j = first i with prefix_incl(D, i) >= p_j (capped at N-1)
        const long long q = (M + KT - 1) / KT;
        const long long t0 = tid * q, t1 = min(M, t0 + q);
        unsigned long long R = 0;
        for (long long s = t0; s < t1; s++) R += SS[cur][s];
        long long total;
        {
            // block exclusive scan of R over KT threads
            unsigned long long x = R;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                unsigned long long y = __shfl_up(x, off);
                if (lane >= off) x += y;
            }
            if (lane == 63) sm.scan_tmp[wid] = (long long)x;
            if (tid < 3) { sm.found_step[tid] = -1; sm.ci[tid] = -1; }
            __syncthreads();
            long long pre = 0;
            for (int w = 0; w < wid; w++) pre += sm.scan_tmp[w];
            total = 0;
            for (int w = 0; w < KWAVES; w++) total += sm.scan_tmp[w];
            unsigned long long excl = (unsigned long long)pre + x - R;
            for (int j = 0; j < 3; j++) {
                if (p[j] > 0 && (double)excl < p[j] && p[j] <= (double)(excl + R)) {
                    unsigned long long e = excl;
                    for (long long s = t0; s < t1; s++) {
                        unsigned long long v = SS[cur][s];
                        if ((double)(e + v) >= p[j]) {
                            sm.found_step[j] = (int)s;
                            sm.found_excl[j] = e;
                            break;
                        }
                        e += v;
                    }
                }
            }
            __syncthreads();
        }
        (void)total;
        // waves 0..2 resolve the point inside the found step
        if (wid < 3) {
            int j = wid;
            if (!(p[j] > 0)) {
                if (lane == 0) sm.ci[j] = 0;
            } else if (sm.found_step[j] < 0) {
                if (lane == 0) sm.ci[j] = (int)(N - 1);
            } else {
                long long s = sm.found_step[j];
                uint32_t k[4];
                int c = load4(pts, N, s, lane, k);
                uint32_t dv[4];
                uint32_t lsum = 0;
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    float x, y, z;
                    key_xyz(k[jj], x, y, z);
                    float d = d2(x, y, z, sm.cc[0][0], sm.cc[0][1], sm.cc[0][2]);
                    for (int m = 1; m < kk; m++) d = fminf(d, d2(x, y, z, sm.cc[m][0], sm.cc[m][1], sm.cc[m][2]));
                    dv[jj] = jj < c ? (uint32_t)d : 0u;
                    lsum += dv[jj];
                }
                unsigned long long x = lsum;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    unsigned long long y = __shfl_up(x, off);
                    if (lane >= off) x += y;
                }
                unsigned long long e = sm.found_excl[j] + x - lsum;
                int hit = -1;
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    e += dv[jj];
                    if (hit < 0 && (double)e >= p[j]) hit = jj;
                }
                unsigned long long bal = __ballot(hit >= 0);
                int first = __builtin_ctzll(bal);
                int hitj = __shfl(hit, first);
                if (lane == 0) {
                    long long idx = s * STEP + first * 4 + hitj;
                    sm.ci[j] = (int)min(idx, N - 1);
                }
            }
        }
        __syncthreads();
        float tc[3][3];
        for (int j = 0; j < 3; j++) {
            uint32_t kk2 = pts[sm.ci[j]];
            key_xyz(kk2, tc[j][0], tc[j][1], tc[j][2]);
        }
        // ---- trial pass: T_j(i) = min(D(i), d(i, ci_j)); step sums into SS[slots]
        int slots[3], sl = 0;
        for (int a = 0; a < 4 && sl < 3; a++)
            if (a != cur) slots[sl++] = a;
        unsigned long long wt[3] = {0, 0, 0};
        for (long long s = s_begin; s < s_end; s++) {
            uint32_t k[4];
            int c = load4(pts, N, s, lane, k);
            uint32_t ls[3] = {0, 0, 0};
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                float x, y, z;
                key_xyz(k[jj], x, y, z);
                float d = d2(x, y, z, sm.cc[0][0], sm.cc[0][1], sm.cc[0][2]);
                for (int m = 1; m < kk; m++) d = fminf(d, d2(x, y, z, sm.cc[m][0], sm.cc[m][1], sm.cc[m][2]));
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    float t = fminf(d, d2(x, y, z, tc[j][0], tc[j][1], tc[j][2]));
                    ls[j] += jj < c ? (uint32_t)t : 0u;
                }
            }
#pragma unroll
            for (int j = 0; j < 3; j++) {
                uint32_t st = wave_sum(ls[j]);
                if (lane == 0) SS[slots[j]][s] = st;
                wt[j] += st;
            }
        }
        if (lane == 0) {
            sm.wtot[wid][0] = wt[0];
            sm.wtot[wid][1] = wt[1];
            sm.wtot[wid][2] = wt[2];
        }
        __syncthreads();
        unsigned long long S[3] = {0, 0, 0};
        for (int w = 0; w < KWAVES; w++)
            for (int j = 0; j < 3; j++) S[j] += sm.wtot[w][j];
        int best = 0;
        double bs = 1.7976931348623157e308;
        for (int j = 0; j < 3; j++)
            if ((double)S[j] < bs) { bs = (double)S[j]; best = j; }
        sum0 = S[best];
        cur = slots[best];
        __syncthreads();
        if (tid == 0) {
            sm.cc[kk][0] = tc[best][0];
            sm.cc[kk][1] = tc[best][1];
            sm.cc[kk][2] = tc[best][2];
        }
        __syncthreads();
    }

    // ------------------------------------------------ Lloyd iterations
    if (tid < kMaxK * 3) {
        int k = tid / 3, j = tid % 3;
        sm.c[k][j] = k < K ? sm.cc[k][j] : 0.f;
    }
    if (tid == 0) sm.n_moved = 0;
    __syncthreads();

    int iter = 1;
    double compactness = 0.0;
    const double eps2 = 0.2 * 0.2;
    for (;;) {
        // ---- assignment with centres c -> per-cluster sums / counts
        float c[kMaxK][3];
#pragma unroll
        for (int k = 0; k < kMaxK; k++)
#pragma unroll
            for (int j = 0; j < 3; j++) c[k][j] = sm.c[k][j];
#pragma unroll
        for (int k = 0; k < kMaxK; k++) {
            sm.accA[k][tid] = 0;
            sm.accB[k][tid] = 0;
        }
        for (long long s = s_begin; s < s_end; s++) {
            uint32_t kq[4];
            int cn = load4(pts, N, s, lane, kq);
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                if (jj < cn) {
                    float x, y, z, bd;
                    key_xyz(kq[jj], x, y, z);
                    int l = argmin_label(x, y, z, c, K, &bd);
                    unsigned long long a = (unsigned long long)(kq[jj] >> 16) |
                                           ((unsigned long long)((kq[jj] >> 8) & 255u) << 32);
                    unsigned long long b = (unsigned long long)(kq[jj] & 255u) | (1ull << 32);
                    atomicAdd(&sm.accA[l][tid], a);
                    atomicAdd(&sm.accB[l][tid], b);
                }
            }
        }
        __syncthreads();
        // reduce 20 values (5 clusters x {x,y,z,count}) over 256 lanes
        if (tid < 160) {
            int v = tid >> 3, part = tid & 7;
            int k = v >> 2, comp = v & 3;
            unsigned long long acc = 0;
            for (int l = part * 32; l < part * 32 + 32; l++) {
                unsigned long long w = comp < 2 ? sm.accA[k][l] : sm.accB[k][l];
                acc += (comp & 1) ? (w >> 32) : (w & 0xFFFFFFFFull);
            }
            sm.red[v][part] = acc;
        }
        __syncthreads();
        if (tid < 20) {
            unsigned long long acc = 0;
            for (int part = 0; part < 8; part++) acc += sm.red[tid][part];
            int k = tid >> 2, comp = tid & 3;
            if (comp < 3) sm.sums[k][comp] = (long long)acc;
            else sm.counts[k] = (int)acc;
        }
        __syncthreads();

        // ---- centres from sums (+ empty-cluster repair), shift, termination
        if (tid < kMaxK * 3) {
            int k = tid / 3, j = tid % 3;
            sm.cprev[k][j] = sm.c[k][j];
        }
        if (tid == 0) sm.n_moved = 0;
        __syncthreads();
        for (int ek = 0; ek < K; ek++) {
            if (sm.counts[ek] != 0) continue;  // uniform
            // biggest cluster
            int max_k = 0;
            for (int k1 = 1; k1 < K; k1++)
                if (sm.counts[max_k] < sm.counts[k1]) max_k = k1;
            float scale = 1.f / (float)sm.counts[max_k];
            float bx = (float)sm.sums[max_k][0] * scale, by = (float)sm.sums[max_k][1] * scale,
                  bz = (float)sm.sums[max_k][2] * scale;
            double md = -1.0;
            long long mi = -1;
            for (long long s = s_begin; s < s_end; s++) {
                uint32_t kq[4];
                int cn = load4(pts, N, s, lane, kq);
                for (int jj = 0; jj < cn; jj++) {
                    float x, y, z, bd;
                    key_xyz(kq[jj], x, y, z);
                    long long i = s * STEP + lane * 4 + jj;
                    int l = argmin_label(x, y, z, sm.cprev, K, &bd);
                    l = moved_label(sm, i, l);
                    if (l != max_k) continue;
                    double d = (double)d2(x, y, z, bx, by, bz);
                    if (md <= d) { md = d; mi = i; }
                }
            }
            // reduce (max d, then max index)
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                double od = __shfl_xor(md, off);
                long long oi = __shfl_xor(mi, off);
                if (od > md || (od == md && oi > mi)) { md = od; mi = oi; }
            }
            if (lane == 0) { sm.maxd[wid] = md; sm.maxi[wid] = (int)mi; }
            __syncthreads();
            if (tid == 0) {
                double bd = -1.0;
                long long bi = -1;
                for (int w = 0; w < KWAVES; w++)
                    if (sm.maxd[w] > bd || (sm.maxd[w] == bd && sm.maxi[w] > bi)) { bd = sm.maxd[w]; bi = sm.maxi[w]; }
                if (bi >= 0) {
                    float x, y, z;
                    key_xyz(pts[bi], x, y, z);
                    sm.counts[max_k]--;
                    sm.counts[ek]++;
                    sm.sums[max_k][0] -= (long long)x; sm.sums[max_k][1] -= (long long)y; sm.sums[max_k][2] -= (long long)z;
                    sm.sums[ek][0] += (long long)x; sm.sums[ek][1] += (long long)y; sm.sums[ek][2] += (long long)z;
                    sm.moved_idx[sm.n_moved] = (int)bi;
                    sm.moved_lbl[sm.n_moved] = ek;
                    sm.n_moved++;
                }
            }
            __syncthreads();
        }
        if (tid == 0) {
            double max_shift = 0.0;
            for (int k = 0; k < K; k++) {
                float scale = 1.f / (float)sm.counts[k];
                double dist = 0.0;
                for (int j = 0; j < 3; j++) {
                    float v = (float)sm.sums[k][j] * scale;
                    sm.c[k][j] = v;
                    double t = (double)(v - sm.cprev[k][j]);
                    dist += t * t;
                }
                max_shift = fmax(max_shift, dist);
            }
            iter++;
            sm.flag = (iter == 100 || max_shift <= eps2) ? 1 : 0;
        } else {
            iter++;
        }
        __syncthreads();
        if (sm.flag) break;
    }

    // ------------------------------------------------ final labels -> compactness
    {
        double acc = 0.0;
        for (long long s = s_begin; s < s_end; s++) {
            uint32_t kq[4];
            int cn = load4(pts, N, s, lane, kq);
            for (int jj = 0; jj < cn; jj++) {
                float x, y, z, bd;
                key_xyz(kq[jj], x, y, z);
                int l = argmin_label(x, y, z, sm.cprev, K, &bd);
                if (sm.n_moved) l = moved_label(sm, s * STEP + lane * 4 + jj, l);
                acc += (double)d2(x, y, z, sm.c[l][0], sm.c[l][1], sm.c[l][2]);
            }
        }
        acc = wave_sum(acc);
        if (lane == 0) sm.dred[wid] = acc;
        __syncthreads();
        if (tid == 0) {
            for (int w = 0; w < KWAVES; w++) compactness += sm.dred[w];
            o->compactness = compactness;
            o->iters = iter;
            for (int k = 0; k < kMaxK; k++) {
                for (int j = 0; j < 3; j++) o->centers[k][j] = k < K ? sm.c[k][j] : 0.f;
                o->counts[k] = k < K ? sm.counts[k] : 0;
            }
        }
    }
}

// LPT order: images sorted by U descending (bitonic sort in LDS, n <= 4096)
constexpr int OT = 1024;
constexpr int OMAX = 4096;
__global__ __launch_bounds__(OT) void k_kmeans_order(const long long *__restrict__ n_unique, int n, int *__restrict__ order) {
    __shared__ long long key[OMAX];
    __shared__ int idx[OMAX];
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    for (int i = threadIdx.x; i < np2; i += OT) {
        key[i] = i < n ? n_unique[i] : -1;
        idx[i] = i;
    }
    __syncthreads();
    for (int k = 2; k <= np2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < np2; i += OT) {
                int l = i ^ j;
                if (l > i) {
                    bool desc = (i & k) == 0;
                    // descending by key, ascending by index on ties
                    bool swap_ = desc ? (key[i] < key[l] || (key[i] == key[l] && idx[i] > idx[l]))
                                      : (key[i] > key[l] || (key[i] == key[l] && idx[i] < idx[l]));
                    if (swap_) {
                        long long tk = key[i]; key[i] = key[l]; key[l] = tk;
                        int ti = idx[i]; idx[i] = idx[l]; idx[l] = ti;
                    }
                }
            }
            __syncthreads();
        }
    for (int i = threadIdx.x; i < n; i += OT) order[i] = idx[i];
}

__global__ void k_kmeans_finalize(const uint32_t *__restrict__ keys, long long key_stride,
                                  const long long *__restrict__ n_unique, int n, int n_colors,
                                  const KmeansAttemptOut *__restrict__ att, KmeansImageOut *__restrict__ out) {
    int img = blockIdx.x * blockDim.x + threadIdx.x;
    if (img >= n) return;
    long long N = n_unique[img];
    int K = (int)min((long long)n_colors, N);
    KmeansImageOut r;
    memset(&r, 0, sizeof r);
    r.n_unique = N;
    if (K <= 1) {
        r.k = (int)N;
        if (N == 1) {
            uint32_t k = keys[(size_t)img * key_stride];
            r.centers_rgb[0][0] = (uint8_t)(k >> 16);
            r.centers_rgb[0][1] = (uint8_t)(k >> 8);
            r.centers_rgb[0][2] = (uint8_t)k;
            r.counts[0] = 1;
        }
        r.compactness = 0.0;
    } else {
        int best = 0;
        double bc = 1.7976931348623157e308;
        for (int a = 0; a < kAttempts; a++) {
            double c = att[(size_t)img * kAttempts + a].compactness;
            if (c < bc) { bc = c; best = a; }
        }
        const KmeansAttemptOut &b = att[(size_t)img * kAttempts + best];
        r.k = K;
        r.compactness = bc;
        for (int k = 0; k < K; k++) {
            for (int j = 0; j < 3; j++) r.centers_rgb[k][j] = (uint8_t)(int)b.centers[k][j];
            r.counts[k] = b.counts[k];
        }
    }
    out[img] = r;
}

}  // namespace

hipError_t launch_color_bitmap(const uint8_t *bgr, const int8_t *noise, int n, int h, int w, uint64_t seed,
                               int64_t index_base, uint32_t *bitmap, uint32_t *occ, hipStream_t s) {
    long long P = (long long)h * w;
    long long per_block = (long long)CB * 4 * 8;  // 8 steps per thread
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

hipError_t launch_kmeans(const uint32_t *keys, int64_t key_stride, const int64_t *n_unique, int n, int n_colors,
                         const uint64_t *rng_states, int32_t *order, uint32_t *scratch, int64_t scratch_stride,
                         KmeansAttemptOut *attempts, KmeansImageOut *out, hipStream_t s) {
    if (n > OMAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_kmeans_order, dim3(1), dim3(OT), 0, s, (const long long *)n_unique, n, order);
    hipLaunchKernelGGL(k_kmeans, dim3(n * kAttempts), dim3(KT), 0, s, keys, (long long)key_stride,
                       (const long long *)n_unique, n_colors, rng_states, order, scratch, (long long)scratch_stride,
                       attempts);
    hipLaunchKernelGGL(k_kmeans_finalize, dim3((n + 255) / 256), dim3(256), 0, s, keys, (long long)key_stride,
                       (const long long *)n_unique, n, n_colors, attempts, out);
    return hipGetLastError();
}

int64_t kmeans_scratch_stride(int64_t key_stride) { return 4 * ((key_stride + STEP - 1) / STEP) + 4; }

}  // namespace llfe
