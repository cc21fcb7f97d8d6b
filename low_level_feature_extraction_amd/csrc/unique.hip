// Dominant-colour front half of ColorExtractor.extract_colors on gfx950
// (app/services/analyze/color_extractor.py:217-236): BGR->RGB (:150-151), + int8(N(0,0.5))
// noise and clip (:223-225), then the set of distinct colours in ascending packed-key
// order = np.unique(pixels, axis=0) (:177), plus the 4x4x4 colour cubes the k-means
// Lloyd sweeps prune with (kmeans.hip).
//
// No global atomics on colours: keys are partitioned by their red quarter R = r >> 2
// (64 partitions; a partition is a contiguous range of the sorted key space), and each
// partition is deduplicated in a 32 KB LDS bitmap by one workgroup.
//
//   k_uq_noise    the launch's noise field (no caller noise): one image's worth, hashed
//   k_uq_scatter  pixel -> key r<<16|g<<8|b, each 4096-pixel step counting-sorted by R
//                 in LDS into its own segment + run table + per-image partition totals
//   k_uq_part     one 512-thread workgroup per (image, R): the partition's runs over the
//                 steps -> LDS bitmap of its 4 x 256 x 256 colours -> its sorted unique keys
//                 (at the partition's place in key order) and its 4x4x4 cubes (occupancy
//                 mask + exact sums, CubeEnt)
//   k_uq_gather   per image: prefix over the partitions, contiguous sorted keys + cube
//                 table
#include <algorithm>

#include "llfe_internal.h"

namespace llfe {
namespace {

// ------------------------------------------------------------------ noise
// trunc(0.5 * Z), Z ~ N(0, 1), from a 21-bit uniform u via tail thresholds:
// P(Z <= -2) * 2^21 = 47710.9 -> 47711, P(Z <= -4) * 2^21 = 66.4 -> 66 (|n| = 3 has
// probability 1e-9 per channel and is not produced).
// Written in plain VOP2 integer ops (shifts, xor, and, add / sub: 2 cycles per wave64
// instruction on gfx950, against 4 for the compares and selects they replace).
__device__ __forceinline__ int noise21(uint32_t u) {
    const uint32_t T1 = 47711u, T2 = 66u;
    const uint32_t hi = u >> 20;                      // 0: negative side, 1: positive
    const uint32_t v = (u ^ (0u - hi)) & 0xFFFFFu;    // u, or 2^21 - 1 - u
    const uint32_t mag = ((v - T1) >> 31) + ((v - T2) >> 31);  // (v < T1) + (v < T2), v < 2^20
    const uint32_t m = hi - 1u;                       // ~0 on the negative side, else 0
    return (int)((mag ^ m) - m);                      // -mag or mag
}

// 32-bit avalanche hash (lowbias32: two multiplies, three xor-shifts)
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

#ifndef LLFE_UQ_VSTORE
#define LLFE_UQ_VSTORE 0  // (experiment) the scatter's segment in 16-byte stores (2: non-temporal)
#endif
constexpr int KB = 256;  // threads per scatter block: a step is 4096 pixels (512 / 1024: the
                         // scatter 1.67 -> 2.19 / 2.55 ms for part 2.41 -> 2.13 / 2.04)
constexpr int PPT = 16;   // pixels per thread per block step
constexpr int NPART = 64;

__device__ __forceinline__ int med3i(int x, int lo, int hi) { return min(max(x, lo), hi); }  // (one v_med3_i32)
// field code c = (nr + 2) 25 + (ng + 2) 5 + (nb + 2) -> (nb + 2) | (ng + 2) << 8 | (nr + 2) << 16
__device__ __forceinline__ uint32_t noise_lut_entry(uint32_t c) {
    return (c % 5u) | ((c / 5u % 5u) << 8) | ((c / 25u) << 16);
}
__device__ __forceinline__ uint32_t key_of(int b, int g, int r, int nb, int ng, int nr) {
    r = min(max(r + nr, 0), 255);
    g = min(max(g + ng, 0), 255);
    b = min(max(b + nb, 0), 255);
    return ((uint32_t)r << 16) | ((uint32_t)g << 8) | (uint32_t)b;
}

// Noise source of a launch.  Parity mode: the caller's int8 arrays (RGB order p*3 + c,
// image stride P*3).  Field mode (no caller noise): ONE counter-hashed field of L pixels
// (L = P rounded up to 16) per launch, k_uq_noise, read by image i rotated by its own
// offset o_i (a multiple of 16 pixels from a hash of (stream, global index)):
// noise_i(p) = field[(p + o_i) mod L].  Within an image every pixel draws a distinct field
// entry, so its noise is i.i.d. int8(N(0, 0.5)) as before; hashing one image's worth per
// launch instead of every pixel of every image takes the two 32-bit hashes (four
// quarter-rate multiplies) off the per-pixel path.  A field pixel is one byte, the three
// channel values n in [-2, 2] in base 5: (nr + 2) * 25 + (ng + 2) * 5 + (nb + 2) -- one
// coalesced 16-B load per 16 pixels (|n| = 3 has probability 1e-9 and is not drawn).  The
// scatter reads the three digits from a 125-entry LDS table (conflict-free: distinct codes
// sit in distinct banks) instead of dividing by 25 and 5: 1.68 -> 1.61 ms per 512 x 1080p.
// Across the images of one launch the noise is NOT independent: each reads a rotation of
// the same field, and a small image has few distinct rotations (L / 16: 256 for 64 x 64),
// so images of a large batch can share identical noise.  Every per-image statistic (and
// the reference's own per-call draw) only needs the within-image i.i.d. property.
struct NoiseSrc {
    const int8_t *p;
    long long L;                // 0: parity mode
    unsigned long long stream;  // field mode
};

__device__ __forceinline__ long long field_offset(const NoiseSrc &ns, long long gidx) {
    if (!ns.L) return 0;
    const uint64_t h = mix64(ns.stream ^ mix64((uint64_t)gidx + 0x4C4C46454C4C4645ull));
    return (long long)(h % (uint64_t)(ns.L / PPT)) * PPT;
}

// the noise of pixels p0 .. p0 + 15 of image `img` (p0 a multiple of 16)
template <bool kField>
__device__ __forceinline__ const int8_t *noise_at(const NoiseSrc &ns, int img, long long P, long long off,
                                                   long long p0) {
    if (!kField) return ns.p + ((size_t)img * P + p0) * 3;
    long long q = p0 + off;
    if (q >= ns.L) q -= ns.L;
    return ns.p + q;
}

// true when the 64 lanes of the wave hold the 64 consecutive full 16-pixel chunks of one
// 16-B aligned 3 KB span (lane l at sp = base + 48 l): wave-uniform
__device__ __forceinline__ bool wave_span(const uint8_t *sp, long long p0, long long P) {
    const int lane = __lane_id();
    return __ballot(1) == ~0ull && p0 - 16LL * lane + 1024 <= P && ((((uintptr_t)sp) - 48u * lane) & 15) == 0;
}

// keys r<<16|g<<8|b of pixels p0 .. p0 + cnt - 1 (cnt <= 16; entries past cnt undefined).
// span (wave_span): the wave reads its 3 KB of BGR with coalesced 16-B loads (lane l
// bytes 16 l + 1024 k) and hands each lane its 48 B through the wave's 3 KB of LDS `wst`
// (reads at a 48-B stride touch all 64 banks once per 16 lanes), instead of 16-B loads at
// a 48-B lane stride
template <bool kField>
__device__ __forceinline__ void chunk_keys(const uint8_t *__restrict__ sp, const int8_t *__restrict__ np_, int cnt,
                                           bool span, uint4 *wst, const uint32_t *nlut, uint32_t kv[PPT]) {
    uint8_t px[3 * PPT];
    if (span) {
        const int lane = __lane_id();
        const uint4 *g = (const uint4 *)(sp - 48 * lane);
        const uint4 a = g[lane], b = g[64 + lane], c = g[128 + lane];
        wst[lane] = a;
        wst[64 + lane] = b;
        wst[128 + lane] = c;
        __builtin_amdgcn_wave_barrier();
        *(uint4 *)&px[0] = wst[3 * lane];
        *(uint4 *)&px[16] = wst[3 * lane + 1];
        *(uint4 *)&px[32] = wst[3 * lane + 2];
        __builtin_amdgcn_wave_barrier();
    } else if (cnt == PPT && (((uintptr_t)sp) & 15) == 0) {
        *(uint4 *)&px[0] = ((const uint4 *)sp)[0];
        *(uint4 *)&px[16] = ((const uint4 *)sp)[1];
        *(uint4 *)&px[32] = ((const uint4 *)sp)[2];
    } else {
        for (int i = 0; i < 3 * PPT; i++) px[i] = i < cnt * 3 ? sp[i] : 0;
    }
    if (kField) {
        uint8_t code[PPT];
        if (cnt == PPT) {  // (the field is 16-B aligned and offsets are multiples of 16)
            *(uint4 *)&code[0] = *(const uint4 *)np_;
        } else {
            for (int i = 0; i < PPT; i++) code[i] = i < cnt ? (uint8_t)np_[i] : 62;  // 62: no noise
        }
#pragma unroll
        for (int i = 0; i < PPT; i++) {
            // the code's three biased digits from the launch's LDS table (nlut), added per
            // channel and clipped as med3(x + n + 2, 2, 257) - 2 = clip(x + n, 0, 255)
            const uint32_t e = nlut[code[i]];
            const int b = med3i((int)px[3 * i] + (int)(e & 255u), 2, 257);
            const int g = med3i((int)px[3 * i + 1] + (int)((e >> 8) & 255u), 2, 257);
            const int r = med3i((int)px[3 * i + 2] + (int)(e >> 16), 2, 257);
            kv[i] = (uint32_t)((r << 16) + (g << 8) + b) - 0x020202u;
        }
    } else {
        int8_t nv[3 * PPT];
        if (cnt == PPT && (((uintptr_t)np_) & 15) == 0) {
            *(uint4 *)&nv[0] = ((const uint4 *)np_)[0];
            *(uint4 *)&nv[16] = ((const uint4 *)np_)[1];
            *(uint4 *)&nv[32] = ((const uint4 *)np_)[2];
        } else {
            for (int i = 0; i < 3 * PPT; i++) nv[i] = i < cnt * 3 ? np_[i] : 0;
        }
#pragma unroll
        for (int i = 0; i < PPT; i++)
            kv[i] = key_of(px[3 * i], px[3 * i + 1], px[3 * i + 2], nv[3 * i + 2], nv[3 * i + 1], nv[3 * i]);
    }
}

// grid (ceil(L / 256)): the noise field, pixel q from the counter lo(stream) + golden32 *
// (q + 1); two hash32 of it (the second keyed by hi(stream)) give three 21-bit uniforms
__global__ __launch_bounds__(256) void k_uq_noise(int8_t *__restrict__ field, long long L, unsigned long long stream) {
    const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
    if (q >= L) return;
    const uint32_t ctr = (uint32_t)stream + 0x9E3779B9u * (uint32_t)(q + 1);
    const uint32_t key2 = (uint32_t)(stream >> 32) | 1u;
    const uint32_t h1 = hash32(ctr), h2 = hash32(ctr ^ key2);
    const int nr = noise21(h1 & 0x1FFFFFu), ng = noise21((h1 >> 21) | ((h2 & 0x3FFu) << 11)), nb = noise21(h2 >> 11);
    field[q] = (int8_t)((nr + 2) * 25 + (ng + 2) * 5 + (nb + 2));
}

// exclusive prefix of the image's 64 partition sizes (one wave)
__device__ __forceinline__ uint32_t part_base(const uint32_t *h, int lane, uint32_t *total) {
    uint32_t v = lane < NPART ? h[lane] : 0u, x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    *total = __shfl(x, 63);
    return x - v;
}

constexpr int SK = KB * PPT;  // keys per scatter block step

// Step segments: each 4096-pixel step's keys, counting-sorted by partition in LDS, go to the
// step's own 4096-key segment (coalesced, no global cursors), with the step's 64 (offset,
// count) run entries in `tab` and the per-image partition totals in `hist`; k_uq_part reads
// a partition as its runs over the steps.  (No separate histogram pass over the pixels.)
template <bool kField>
__global__ __launch_bounds__(KB) void k_uq_scatter(const uint8_t *__restrict__ bgr, const uint64_t *__restrict__ img_tab,
                                                   NoiseSrc ns, long long P,
                                                   long long key_stride, ImgIndex index, uint32_t *__restrict__ hist,
                                                   uint32_t *__restrict__ tab, uint32_t *__restrict__ seg) {
    __shared__ uint32_t cnt[NPART], lbase[NPART], nlut[128];
    __shared__ __attribute__((aligned(16))) uint32_t stage[SK];
    const int img = blockIdx.y, t = threadIdx.x;
    if (kField && t < 128) nlut[t] = noise_lut_entry((uint32_t)t);  // (visible after the first barrier below)
    const uint8_t *src = img_tab ? (const uint8_t *)img_tab[img] : bgr + (size_t)img * P * 3;
    const long long off = field_offset(ns, index.at(img));
    uint32_t *out = seg + (size_t)img * key_stride;
    const long long nsteps = (P + SK - 1) / SK;
    for (long long st = blockIdx.x; st < nsteps; st += gridDim.x) {
        const long long p0 = st * SK + (long long)t * PPT;
        const int n = (int)max(0LL, min((long long)PPT, P - p0));
        if (t < NPART) cnt[t] = 0;
        __syncthreads();
        uint32_t kv[PPT], pos[PPT];
        // (the staging uses this wave's 3 KB of `stage`, free until the keys are sorted into it)
        const bool span = wave_span(src + p0 * 3, p0, P);
        if (n > 0)
            chunk_keys<kField>(src + p0 * 3, noise_at<kField>(ns, img, P, off, p0), n, span,
                               (uint4 *)stage + 192 * (t >> 6), nlut, kv);
        // rank within the block's bin: one LDS atomic per run of equal bins.  Static
        // register indexing only: the atomic sits on each run's last key and returns the
        // run's base, which a backward pass hands to the run's other keys.
        uint32_t bins[PPT], endm = 0;
#pragma unroll
        for (int i = 0; i < PPT; i++) bins[i] = kv[i] >> 18;
        {
            int run_start = 0;
#pragma unroll
            for (int i = 0; i < PPT; i++) {
                if (i > 0 && bins[i] != bins[i - 1]) run_start = i;
                const bool end = (i == PPT - 1) || (i + 1 >= n) || (bins[i + 1] != bins[i]);
                pos[i] = 0;
                if (i < n && end) {
                    pos[i] = atomicAdd(&cnt[bins[i]], (uint32_t)(i - run_start + 1)) - (uint32_t)run_start;
                    endm |= 1u << i;
                }
            }
            uint32_t cur = 0;
#pragma unroll
            for (int i = PPT - 1; i >= 0; i--) {
                if (endm & (1u << i)) cur = pos[i];
                pos[i] = cur + (uint32_t)i;
            }
        }
        __syncthreads();
        if (t < 64) {
            const uint32_t c = cnt[t];
            uint32_t x = c;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                uint32_t y = __shfl_up(x, off);
                if (t >= off) x += y;
            }
            lbase[t] = x - c;
            tab[((size_t)img * nsteps + st) * NPART + t] = (x - c) | (c << 16);
            if (c) atomicAdd(hist + (size_t)img * NPART + t, c);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PPT; i++)
            if (i < n) stage[lbase[bins[i]] + pos[i]] = kv[i];
        __syncthreads();
        const int tot = (int)min((long long)SK, P - st * SK);
        uint32_t *o = out + st * SK;
#if LLFE_UQ_VSTORE
        {  // (experiment) 16-byte stores of the step's segment (2: non-temporal)
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            const int t4 = tot >> 2;
            for (int i = t; i < t4; i += KB) {
                const u32x4 v = ((const u32x4 *)stage)[i];
                if (LLFE_UQ_VSTORE == 2) __builtin_nontemporal_store(v, (u32x4 *)o + i);
                else ((u32x4 *)o)[i] = v;
            }
            for (int i = (t4 << 2) + t; i < tot; i += KB) o[i] = stage[i];
        }
#else
        for (int i = t; i < tot; i += KB) o[i] = stage[i];
#endif
        __syncthreads();
    }
}

// ------------------------------------------------------------------ partitions
#ifndef LLFE_UQ_DMA
#define LLFE_UQ_DMA 0  // > 0: runs' first keys through an LDS double buffer, this many runs a group
#endif
// k_uq_part threads per (image, partition): 512 (four workgroups per CU by LDS) measured
// 2.34 ms per 512 x 1080p against 2.41 for 1024 and 3.04 for 256
#ifndef LLFE_UQ_UT
#define LLFE_UQ_UT 512
#endif
constexpr int UT = LLFE_UQ_UT;

__device__ __forceinline__ unsigned long long scan_u64_wg(unsigned long long v, unsigned long long *tmp,
                                                            unsigned long long *total) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    unsigned long long x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        unsigned long long y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) tmp[wid] = x;
    __syncthreads();
    if (wid == 0) {
        unsigned long long s = lane < UT / 64 ? tmp[lane] : 0ull;
#pragma unroll
        for (int off = 1; off < UT / 64; off <<= 1) {
            unsigned long long y = __shfl_up(s, off);
            if (lane >= off) s += y;
        }
        if (lane < UT / 64) tmp[lane] = s;
    }
    __syncthreads();
    const unsigned long long r = (wid ? tmp[wid - 1] : 0ull) + x - v;
    *total = tmp[UT / 64 - 1];
    __syncthreads();
    return r;
}

// grid (64, n).  amdgpu_waves_per_eu(8): the super-cell count (round 6) took the kernel from 62
// to 66 VGPRs (three workgroups per CU instead of four); held at 64 it needs no spill.
// Reads the partition's keys as its runs in the step segments (`tab`), writes
// the sorted unique keys to `skeys` at the partition's place in key order (capacity: its
// hist count), and up to 4096 cube entries to `seg_cubes`.
__global__ __launch_bounds__(UT) __attribute__((amdgpu_waves_per_eu(8))) void k_uq_part(const uint32_t *__restrict__ seg, long long key_stride, long long P,
                                                const uint32_t *__restrict__ hist, const uint32_t *__restrict__ tab,
                                                uint32_t *__restrict__ skeys,
                                                CubeEnt *__restrict__ seg_cubes, CellEnt *__restrict__ seg_cells,
                                                uint32_t *__restrict__ uq, uint32_t *__restrict__ cc,
                                                uint32_t *__restrict__ cl, uint32_t *__restrict__ cs) {
    __shared__ __attribute__((aligned(16))) uint32_t W[4 * 2048];  // rows r = 4R + i, word g << 3 | b >> 5
    __shared__ unsigned long long tmp[UT / 64];
    __shared__ uint32_t sbase, scount;
    const int R = blockIdx.x, img = blockIdx.y, t = threadIdx.x;
    if (t < 64) {
        uint32_t tot;
        const uint32_t b = part_base(hist + (size_t)img * NPART, t, &tot);
        if (t == R) {
            sbase = b;
            scount = hist[(size_t)img * NPART + R];
        }
    }
    __syncthreads();
    const uint32_t start = sbase, count = scount;
    if (count == 0) {  // (most partitions of a flat "ui" image): before zeroing the bitmap
        if (t == 0) {
            uq[(size_t)img * NPART + R] = 0;
            cc[(size_t)img * NPART + R] = 0;
            cl[(size_t)img * NPART + R] = 0;
            cs[(size_t)img * NPART + R] = 0;
        }
        return;
    }
    for (int i = t; i < 4 * 2048 / 4; i += UT) ((uint4 *)W)[i] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    // the partition's runs: wave w takes steps w + (UT / 64) j; lane j holds run j's (offset, count)
    // (one table load per lane for up to 64 runs), then the runs' first keys (one per lane,
    // photo runs average ~64 keys) are loaded RG runs at a time, and the rest of the long runs
    // (flat "ui" partitions: ~4096 keys per run) with RG loads in flight
    const uint32_t *sg = seg + (size_t)img * key_stride;
    const long long nsteps = (P + SK - 1) / SK;
    const uint32_t *tb = tab + (size_t)img * nsteps * NPART + R;
    const int lane = t & 63, wid = t >> 6;
    constexpr int RG = 8;  // runs (and tail loads) in flight per lane (16: 97 VGPRs, one workgroup per CU)
    auto mark = [&](uint32_t k) {
        // flat regions put one colour in every lane: test the bit with a (broadcast) read
        // first, so a wave does not serialise 64 atomics on one LDS word
        const uint32_t wi = ((k >> 16) & 3u) * 2048 + ((k >> 5) & 2047u), bit = 1u << (k & 31u);
        if (k != 0xFFFFFFFFu && !(W[wi] & bit)) atomicOr(&W[wi], bit);
    };
#if LLFE_UQ_DMA
    // (round 6 experiment) the runs' first 64 keys go straight to a per-wave LDS double buffer by
    // direct-to-LDS loads, one group of RGD runs ahead of the group being marked; a counted
    // vmcnt wait (the group issued after it) before a group's keys are read back
    constexpr int RGD = LLFE_UQ_DMA;
    __shared__ __attribute__((aligned(16))) uint32_t rstage[UT / 64][2][RGD][64];
    uint32_t(*const rs)[RGD][64] = rstage[__builtin_amdgcn_readfirstlane(wid)];
    auto wait_vm = [&](int n) __attribute__((always_inline)) {
        switch (n) {  // (s_waitcnt takes an immediate)
#define UQ_W(N) case N: __builtin_amdgcn_s_waitcnt((N) | (7 << 4) | (15 << 8)); break;
            UQ_W(0) UQ_W(1) UQ_W(2) UQ_W(3) UQ_W(4) UQ_W(5) UQ_W(6) UQ_W(7) UQ_W(8)
#undef UQ_W
            default: __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8)); break;
        }
    };
    for (long long base = 0; base < nsteps; base += (UT / 64) * 64) {
        const long long sl = base + wid + (UT / 64) * lane;  // this lane's run
        const uint32_t e = sl < nsteps ? tb[(size_t)sl * NPART] : 0u;
        const unsigned long long live = __ballot(e != 0u);
        auto next_group = [&](int j) {  // the first group from run j with a live run (64: none)
            while (j < 64 && !((live >> j) & ((1ull << RGD) - 1))) j += RGD;
            return j;
        };
        auto issue = [&](int j0, int buf) __attribute__((always_inline)) {
            int nd = 0;
#pragma unroll
            for (int j = 0; j < RGD; j++) {
                const uint32_t ej = __builtin_amdgcn_readlane(e, j0 + j);
                if (ej >> 16) {  // (uniform)
                    const size_t st = (size_t)(base + wid + (UT / 64) * (j0 + j));
                    if ((uint32_t)lane < (ej >> 16))
                        __builtin_amdgcn_global_load_lds((const void *)(sg + st * SK + (ej & 0xFFFFu) + lane),
                                                         (void *)&rs[buf][j][0], 4, 0, 0);
                    nd++;
                }
            }
            return nd;
        };
        int j0 = next_group(0), buf = 0;
        if (j0 < 64) issue(j0, 0);
        while (j0 < 64) {
            const int j1 = next_group(j0 + RGD);
            const int n1 = j1 < 64 ? issue(j1, buf ^ 1) : 0;
            wait_vm(n1);  // group j0's loads have landed (at most the n1 of group j1 outstanding)
#pragma unroll
            for (int j = 0; j < RGD; j++) {
                const uint32_t ej = __builtin_amdgcn_readlane(e, j0 + j);
                mark((uint32_t)lane < (ej >> 16) ? rs[buf][j][lane] : 0xFFFFFFFFu);
            }
#pragma unroll
            for (int j = 0; j < RGD; j++) {
                const uint32_t ej = __builtin_amdgcn_readlane(e, j0 + j), c = ej >> 16;
                if (c <= 64) continue;  // (uniform)
                const uint32_t *rp = sg + (size_t)(base + wid + (UT / 64) * (j0 + j)) * SK + (ej & 0xFFFFu);
                for (uint32_t i0 = 64; i0 < c; i0 += 64 * RG) {
                    uint32_t q[RG];
#pragma unroll
                    for (int i = 0; i < RG; i++) {
                        const uint32_t ix = i0 + 64 * i + lane;
                        q[i] = ix < c ? rp[ix] : 0xFFFFFFFFu;
                    }
#pragma unroll
                    for (int i = 0; i < RG; i++) mark(q[i]);
                }
            }
            j0 = j1;
            buf ^= 1;
        }
    }
#else
    for (long long base = 0; base < nsteps; base += (UT / 64) * 64) {
        const long long sl = base + wid + (UT / 64) * lane;  // this lane's run
        const uint32_t e = sl < nsteps ? tb[(size_t)sl * NPART] : 0u;
        const unsigned long long live = __ballot(e != 0u);
        for (int j0 = 0; j0 < 64; j0 += RG) {
            if (!((live >> j0) & ((1ull << RG) - 1))) continue;  // (uniform)
            uint32_t kk[RG];
#pragma unroll
            for (int j = 0; j < RG; j++) {
                const uint32_t ej = __builtin_amdgcn_readlane(e, j0 + j);
                const size_t st = (size_t)(base + wid + (UT / 64) * (j0 + j));
                kk[j] = (uint32_t)lane < (ej >> 16) ? sg[st * SK + (ej & 0xFFFFu) + lane] : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int j = 0; j < RG; j++) mark(kk[j]);
#pragma unroll
            for (int j = 0; j < RG; j++) {
                const uint32_t ej = __builtin_amdgcn_readlane(e, j0 + j), c = ej >> 16;
                if (c <= 64) continue;  // (uniform)
                const uint32_t *rp = sg + (size_t)(base + wid + (UT / 64) * (j0 + j)) * SK + (ej & 0xFFFFu);
                for (uint32_t i0 = 64; i0 < c; i0 += 64 * RG) {
                    uint32_t q[RG];
#pragma unroll
                    for (int i = 0; i < RG; i++) {
                        const uint32_t ix = i0 + 64 * i + lane;
                        q[i] = ix < c ? rp[ix] : 0xFFFFFFFFu;
                    }
#pragma unroll
                    for (int i = 0; i < RG; i++) mark(q[i]);
                }
            }
        }
    }
#endif
    __syncthreads();
    // (a) unique keys in ascending order: thread t owns words q * UT + t (q < NQ), so a
    // store instruction's lanes write neighbouring runs of the output (a few cache lines)
    // rather than UT runs spread over the partition.  The per-slice prefixes of the NQ
    // popcounts (<= 32 UT each) go through NQ / 4 scans of four packed 16-bit fields.
    {
        constexpr int NQ = 8192 / UT, NS = NQ / 4;
        uint32_t wq[NQ];
        unsigned long long cp[NS];
#pragma unroll
        for (int k = 0; k < NS; k++) cp[k] = 0;
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            wq[q] = W[q * UT + t];
            cp[q >> 2] |= (unsigned long long)__popc(wq[q]) << (16 * (q & 3));
        }
        unsigned long long pk[NS], tk[NS];
#pragma unroll
        for (int k = 0; k < NS; k++) pk[k] = scan_u64_wg(cp[k], tmp, &tk[k]);
        uint32_t *o = skeys + (size_t)img * key_stride + start;
        uint32_t sbase_q = 0;
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const int sh = 16 * (q & 3);
            uint32_t pos = sbase_q + (uint32_t)((pk[q >> 2] >> sh) & 0xFFFFu);
            sbase_q += (uint32_t)((tk[q >> 2] >> sh) & 0xFFFFu);
            const int word = q * UT + t;  // = i * 2048 + (g << 3 | b >> 5)
            const uint32_t kb = ((uint32_t)(4 * R + (word >> 11)) << 16) | ((uint32_t)(word & 2047) << 5);
            for (uint32_t m = wq[q]; m; m &= m - 1) o[pos++] = kb | (uint32_t)__builtin_ctz(m);
        }
        if (t == 0) uq[(size_t)img * NPART + R] = sbase_q;
    }
    // (b) the partition's 4x4x4 cubes and 4x8x8 cells, and its count of occupied 4x16x16
    // super-cells (their entries are built by k_uq_gather from the cells).  In pass h thread
    // t owns cell (G2, B2) = (c >> 5, c & 31), c = h UT + t, and its four cubes (G, B) =
    // (2 G2 + j, 2 B2 + cc), written in cell order and within a cell in (j, cc) order, so a
    // cell's cubes are consecutive; bit i*16 + jj*4 + bb of a cube = colour (4R + i, 4G + jj,
    // 4B + bb).  The cell's colours are the bytes (B2 & 3) of the 32 words W[i][8 G2 + g][B2 >> 2].
    // A wave holds the cell rows G2 = 2 G4, 2 G4 + 1: super-cell (G4, B4) is lanes {2 B4,
    // 2 B4 + 1} of both rows (lane quads {l, l ^ 1, l ^ 32, l ^ 33}, l = 2 B4).
    uint32_t cbase = 0, lbase = 0, sbase_s = 0;
    CubeEnt *ce = seg_cubes + ((size_t)img * NPART + R) * 4096;
    CellEnt *le = seg_cells + ((size_t)img * NPART + R) * kCellsPerPart;
#pragma unroll 1
    for (int h = 0; h < kCellsPerPart / UT; h++) {
        const int cell = h * UT + t, G2 = cell >> 5, B2 = cell & 31;
        const bool lead = (t & 33) == 0;  // the quad's (row 0, even B2) lane
        const int wsel = (G2 << 6) | (B2 >> 2), sh0 = (B2 & 3) * 8;
        unsigned long long mask[4];  // cube (j, c) = mask[2 j + c]
#pragma unroll
        for (int q = 0; q < 4; q++) mask[q] = 0;
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int g = 0; g < 8; g++) {
                const uint32_t byte = (W[i * 2048 + wsel + (g << 3)] >> sh0) & 255u;
                const int j = g >> 2, jj = g & 3;
                mask[2 * j] |= (unsigned long long)(byte & 15u) << (i * 16 + jj * 4);
                mask[2 * j + 1] |= (unsigned long long)(byte >> 4) << (i * 16 + jj * 4);
            }
        unsigned long long mine = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) mine += mask[q] ? 1ull : 0ull;
        // one cell; one super-cell on the quad's first thread when any of its cells is occupied
        // (fields: cubes bits 0..31, cells 32..47, super-cells 48..63 -- per pass <= 2048 /
        // 512 / 128, no carries)
        const bool any_cell = mine != 0;
        uint32_t mq = any_cell ? 1u : 0u;
        mq |= __shfl_xor(mq, 1);
        mq |= __shfl_xor(mq, 32);
        if (any_cell) mine |= 1ull << 32;
        if (lead && mq) mine |= 1ull << 48;
        unsigned long long tot;
        const unsigned long long pos = scan_u64_wg(mine, tmp, &tot);
        uint32_t ci = cbase + (uint32_t)pos;
        const uint32_t li = lbase + (uint32_t)((pos >> 32) & 0xFFFFu), first = ci;
        cbase += (uint32_t)tot;
        lbase += (uint32_t)((tot >> 32) & 0xFFFFu);
        sbase_s += (uint32_t)(tot >> 48);
        uint32_t ln = 0, lr = 0, lg = 0, lb = 0, l2 = 0;  // the cell's sums
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const unsigned long long m = mask[q];
            if (!m) continue;
            const int j = q >> 1, c4 = (q & 1) * 4, j4 = j * 4;
            const int G = 2 * G2 + j, B = 2 * B2 + (q & 1);
            const uint32_t n = (uint32_t)__popcll(m);
            uint32_t sr = 0, sg = 0, sb = 0, su2 = 0;  // over u = colour - cube origin
#pragma unroll
            for (int i = 1; i < 4; i++) {
                const uint32_t c = (uint32_t)__popcll(m & (0xFFFFull << (16 * i)));
                sr += i * c;
                su2 += i * i * c;
            }
#pragma unroll
            for (int jj = 1; jj < 4; jj++) {
                const uint32_t c = (uint32_t)__popcll(m & (0x000F000F000F000Full << (4 * jj)));
                sg += jj * c;
                su2 += jj * jj * c;
            }
#pragma unroll
            for (int bb = 1; bb < 4; bb++) {
                const uint32_t c = (uint32_t)__popcll(m & (0x1111111111111111ull << bb));
                sb += bb * c;
                su2 += bb * bb * c;
            }
            CubeEnt e;
            e.mask = m;
            e.id = ((uint32_t)R << 12) | ((uint32_t)G << 6) | (uint32_t)B | (su2 << 18);
            e.sums = n | (sr << 7) | (sg << 15) | (sb << 23);
            ce[ci++] = e;
            // relative to the cell origin the cube sits at (0, 4 j, 4 c)
            ln += n;
            lr += sr;
            lg += sg + j4 * n;
            lb += sb + c4 * n;
            l2 += su2 + 2u * (j4 * sg + c4 * sb) + n * (uint32_t)(j4 * j4 + c4 * c4);
        }
        if (ln) {
            CellEnt e;
            e.id = ((uint32_t)R << 10) | ((uint32_t)G2 << 5) | (uint32_t)B2 | ((ci - first - 1u) << 16) | (ln << 18);
            e.first = first;
            e.sums = lr | (lg << 10) | (lb << 21);
            e.s2 = l2;
            le[li] = e;
        }
    }
    if (t == 0) {
        cc[(size_t)img * NPART + R] = cbase;
        cl[(size_t)img * NPART + R] = lbase;
        cs[(size_t)img * NPART + R] = sbase_s;
    }
}

// grid (64, n): one workgroup per (partition, image) copies the partition's cube entries
// and cells -- and, with copy_keys, its sorted unique keys -- to their place in the
// contiguous per-image arrays (a cell's first cube index becomes image-global).  The batch
// path's k-means reads the keys where k_uq_part wrote them (KmeansCubes::part_hist), so
// only the small cube / cell tables move: 16 (C + L) instead of 8U + 16 (C + L) bytes.
constexpr int GT = 256;
__global__ __launch_bounds__(GT) void k_uq_gather(const uint32_t *__restrict__ skeys, long long key_stride,
                                                  const uint32_t *__restrict__ hist, const uint32_t *__restrict__ uq,
                                                  const uint32_t *__restrict__ cc, const uint32_t *__restrict__ cl,
                                                  const uint32_t *__restrict__ cs,
                                                  const CubeEnt *__restrict__ seg_cubes,
                                                  const CellEnt *__restrict__ seg_cells, uint32_t *__restrict__ keys,
                                                  CubeEnt *__restrict__ cubes, CellEnt *__restrict__ cells,
                                                  SupEnt *__restrict__ sups,
                                                  long long cube_stride, long long cell_stride, long long sup_stride,
                                                  long long *__restrict__ n_unique,
                                                  int *__restrict__ n_cubes, int *__restrict__ n_cells,
                                                  int *__restrict__ n_sups, int copy_keys) {
    __shared__ uint32_t sp, su, sc, sl, ss, nu, nc, nl, ns;
    const int R = blockIdx.x, img = blockIdx.y, t = threadIdx.x;
    if (t < 64) {
        uint32_t tot, ut, ct, lt, st;
        const uint32_t ps = part_base(hist + (size_t)img * NPART, t, &tot);
        const uint32_t ub = part_base(uq + (size_t)img * NPART, t, &ut);
        const uint32_t cb = part_base(cc + (size_t)img * NPART, t, &ct);
        const uint32_t lb = part_base(cl + (size_t)img * NPART, t, &lt);
        const uint32_t sb = part_base(cs + (size_t)img * NPART, t, &st);
        if (t == R) {
            sp = ps;
            su = ub;
            sc = cb;
            sl = lb;
            ss = sb;
            nu = uq[(size_t)img * NPART + R];
            nc = cc[(size_t)img * NPART + R];
            nl = cl[(size_t)img * NPART + R];
            ns = cs[(size_t)img * NPART + R];
        }
        if (t == 0 && R == 0) {
            n_unique[img] = ut;
            n_cubes[img] = (int)ct;
            n_cells[img] = (int)lt;
            n_sups[img] = (int)st;
        }
    }
    __syncthreads();
    const uint32_t U = nu, C = nc, L = nl, S = ns, cbase = sc, lbase = sl;
    const uint32_t *sk = skeys + (size_t)img * key_stride + sp;
    uint32_t *ok = keys + (size_t)img * key_stride + su;
    if (copy_keys)
        for (uint32_t i = t; i < U; i += GT) ok[i] = sk[i];
    const CubeEnt *scp = seg_cubes + ((size_t)img * NPART + R) * 4096;
    CubeEnt *oc = cubes + (size_t)img * cube_stride + sc;
    for (uint32_t i = t; i < C; i += GT) oc[i] = scp[i];
    const CellEnt *slp = seg_cells + ((size_t)img * NPART + R) * kCellsPerPart;
    CellEnt *ol = cells + (size_t)img * cell_stride + sl;
    for (uint32_t i = t; i < L; i += GT) {
        CellEnt e = slp[i];
        e.first += cbase;
        ol[i] = e;
    }
    // the partition's super-cells (round 6), thread t = super-cell (G4, B4) = (t >> 4, t & 15):
    // its cells (2 G4 + j, 2 B4 + c) from a map of the partition's cells by (G2, B2), its count
    // and sums over u = colour - (4R, 16 G4, 16 B4) from the cells' (cell offsets (0, 8j, 8c)),
    // its slot from a workgroup scan in (G4, B4) order (k_uq_part counted them: S)
    static_assert(GT == kSupsPerPart, "one thread per super-cell of a partition");
    __shared__ short cmap[kCellsPerPart];
    __shared__ uint32_t wsum[GT / 64];
    for (int i = t; i < kCellsPerPart; i += GT) cmap[i] = -1;
    __syncthreads();
    for (uint32_t i = t; i < L; i += GT) cmap[slp[i].id & (kCellsPerPart - 1)] = (short)i;
    __syncthreads();
    const int G4 = t >> 4, B4 = t & 15;
    int cix[4];
#pragma unroll
    for (int q = 0; q < 4; q++) cix[q] = cmap[((2 * G4 + (q >> 1)) << 5) | (2 * B4 + (q & 1))];
    const bool occ = (cix[0] & cix[1] & cix[2] & cix[3]) >= 0;  // some cell present (the AND is -1 only when all are)
    const unsigned long long bal = __ballot(occ);
    const int lane = t & 63, wv = t >> 6;
    if (lane == 0) wsum[wv] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    for (int w = 0; w < wv; w++) rank += wsum[w];
    if (occ && rank < S) {
        uint32_t n = 0, sr = 0, sg = 0, sb = 0, s2 = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (cix[q] < 0) continue;
            const CellEnt e = slp[cix[q]];
            const uint32_t j8 = 8u * (uint32_t)(q >> 1), c8 = 8u * (uint32_t)(q & 1);
            const uint32_t ln = (e.id >> 18) & 511u, lr = e.sums & 1023u, lg = (e.sums >> 10) & 2047u, lb = e.sums >> 21;
            n += ln;
            sr += lr;
            sg += lg + j8 * ln;
            sb += lb + c8 * ln;
            s2 += e.s2 + 2u * (j8 * lg + c8 * lb) + ln * (j8 * j8 + c8 * c8);
        }
        const uint32_t c0 = (cix[0] >= 0) + (cix[1] >= 0), c1 = (cix[2] >= 0) + (cix[3] >= 0);
        const uint32_t f0 = cix[0] >= 0 ? cix[0] : (cix[1] >= 0 ? cix[1] : 0);
        const uint32_t f1 = cix[2] >= 0 ? cix[2] : (cix[3] >= 0 ? cix[3] : 0);
        SupEnt e;
        e.id = ((uint32_t)R << 8) | ((uint32_t)G4 << 4) | (uint32_t)B4 | (c0 << 14) | (c1 << 16) | (n << 18) |
               ((s2 >> 18) << 29);
        e.first = (lbase + f0) | ((lbase + f1) << 16);  // (an image's cells are < 65536)
        e.srg = sr | (sg << 12);
        e.sb = sb | ((s2 & 0x3FFFFu) << 14);
        sups[(size_t)img * sup_stride + ss + rank] = e;
    }
}

}  // namespace

namespace {
NoiseSrc noise_src(const int8_t *noise, int8_t *field, int64_t P, uint64_t seed) {
    if (noise) return NoiseSrc{noise, 0, 0};
    return NoiseSrc{field, noise_field_pixels(P), (unsigned long long)mix64(seed ^ 0x4C4C46454C4C4645ull)};
}
}  // namespace

int64_t noise_field_pixels(int64_t P) { return (std::max<int64_t>(P, 1) + PPT - 1) / PPT * PPT; }

hipError_t launch_uq_noise(const int8_t *noise, int8_t *field, int64_t P, uint64_t seed, hipStream_t s) {
    if (noise) return hipSuccess;
    const NoiseSrc ns = noise_src(noise, field, P, seed);
    hipLaunchKernelGGL(k_uq_noise, dim3((unsigned)((ns.L + 255) / 256)), dim3(256), 0, s, field, ns.L, ns.stream);
    return hipGetLastError();
}

int64_t uq_steps(int64_t P) { return (P + SK - 1) / SK; }

hipError_t launch_uq_scatter(const uint8_t *bgr, const uint64_t *img_tab, const int8_t *noise, const int8_t *field,
                             int n, int h, int w,
                             uint64_t seed, ImgIndex index, int64_t key_stride, uint32_t *hist, uint32_t *tab,
                             uint32_t *seg, hipStream_t s) {
    const int64_t P = (int64_t)h * w;
    int bx = (int)std::min((P + SK * 2 - 1) / (SK * 2), (int64_t)2048);
    if (bx < 1) bx = 1;
    const NoiseSrc ns = noise_src(noise, (int8_t *)field, P, seed);
    if (ns.L)
        hipLaunchKernelGGL(k_uq_scatter<true>, dim3(bx, n), dim3(KB), 0, s, bgr, img_tab, ns, (long long)P, (long long)key_stride,
                           index, hist, tab, seg);
    else
        hipLaunchKernelGGL(k_uq_scatter<false>, dim3(bx, n), dim3(KB), 0, s, bgr, img_tab, ns, (long long)P,
                           (long long)key_stride, index, hist, tab, seg);
    return hipGetLastError();
}

hipError_t launch_uq_part(const uint32_t *seg, int n, int64_t key_stride, int64_t P, const uint32_t *hist,
                          const uint32_t *tab, uint32_t *skeys, CubeEnt *seg_cubes, CellEnt *seg_cells,
                          uint32_t *uq, uint32_t *cc, uint32_t *cl, uint32_t *cs, hipStream_t s) {
    hipLaunchKernelGGL(k_uq_part, dim3(NPART, n), dim3(UT), 0, s, seg, (long long)key_stride, (long long)P, hist, tab,
                       skeys, seg_cubes, seg_cells, uq, cc, cl, cs);
    return hipGetLastError();
}

hipError_t launch_uq_gather(const uint32_t *skeys, int n, int64_t key_stride, const uint32_t *hist, const uint32_t *uq,
                            const uint32_t *cc, const uint32_t *cl, const uint32_t *cs, const CubeEnt *seg_cubes,
                            const CellEnt *seg_cells, uint32_t *keys, CubeEnt *cubes,
                            CellEnt *cells, SupEnt *sups, int64_t cube_stride, int64_t cell_stride, int64_t sup_stride,
                            int64_t *n_unique, int32_t *n_cubes, int32_t *n_cells, int32_t *n_sups, bool copy_keys,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_uq_gather, dim3(NPART, n), dim3(GT), 0, s, skeys, (long long)key_stride, hist, uq, cc, cl, cs,
                       seg_cubes, seg_cells, keys, cubes, cells, sups, (long long)cube_stride,
                       (long long)cell_stride, (long long)sup_stride, (long long *)n_unique, (int *)n_cubes,
                       (int *)n_cells, (int *)n_sups, copy_keys ? 1 : 0);
    return hipGetLastError();
}

}  // namespace llfe
namespace llfe {
int64_t uq_tab_words(int64_t P) { return uq_steps(P) * 64; }  // u32 run entries (offset | count << 16)
}  // namespace llfe
