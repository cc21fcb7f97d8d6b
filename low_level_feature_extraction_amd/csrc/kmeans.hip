// cv2.kmeans(float32(unique_colors), K, None, (EPS+MAX_ITER, 200, 0.2), 10,
// KMEANS_PP_CENTERS) for a batch of images on gfx950
// (app/services/analyze/color_extractor.py:189-197).
//
// One 256-thread workgroup per (image, attempt), four per CU (round 6; 512 threads / two per CU
// before, LLFE_KM_THREADS); workgroups are issued largest-U
// first (LPT) so the many short "ui" attempts back-fill behind the long "photo" ones.
// The point set is the compacted unique-colour key list (4 B / point, ascending =
// np.unique row order); wave w owns a contiguous range of 256-point steps and reads
// it with 16-byte coalesced loads.
//
// OpenCV semantics restated (kmeans.cpp):
//  * attempt a starts from cv::RNG state advanced by a * (1 + 6 (K-1)) draws
//    (generateCentersPP consumes 1 + 3 trials x 2 draws per extra centre);
//  * k-means++: c0 = rng % N; for k >= 1, three trials p = rng.double * sum(D) ->
//    first i with prefix(D, i) >= p (exact: D are integers), keep the trial with the
//    smallest sum(min(D, d(., ci))) (first on ties);
//  * Lloyd: labels by the first minimum of the float32 normL2Sqr (t0*t0, fma, fma);
//    centres = float(sum) * (1.f / count); empty clusters take the farthest point of
//    the biggest cluster; stop when ++iter == 100 or max shift^2 <= 0.2^2;
//  * compactness = sum of double(normL2Sqr) to the final centres with the labels of
//    the last assignment.  Cluster sums are exact int64 (OpenCV accumulates float32
//    sequentially; the difference is far below the uint8 truncation of the output).
#include "kmeans_common.h"

#include <mutex>

namespace llfe {
namespace {

#ifndef LLFE_KM_CELL_MIN
#define LLFE_KM_CELL_MIN 8192
#endif
constexpr int kCellMinCubes = LLFE_KM_CELL_MIN;  // cube count from which the sweeps take cells / super-cells
#ifndef LLFE_KM_SPLIT
#define LLFE_KM_SPLIT 0  // the cube path in two launches (measured slower; kept as a build option)
#endif
#ifndef LLFE_KM_LLOYD_QUEUE
#define LLFE_KM_LLOYD_QUEUE 0  // (split) Lloyd as a work queue too (1) or one workgroup per attempt (0)
#endif
#ifndef LLFE_KM_PP_CALL
#define LLFE_KM_PP_CALL (!LLFE_KM_SPLIT)  // pp_cubes as a call in the one-launch kernel (its register budget)
#endif  // the sweeps test cells before cubes from this cube count on
#ifndef LLFE_KM_SUPS
#define LLFE_KM_SUPS 1  // Lloyd tests 4 x 16 x 16 super-cells before cells
#endif
#ifndef LLFE_KM_PP_SUPS
#define LLFE_KM_PP_SUPS 0  // k-means++ sweeps test 4 x 16 x 16 super-cells before cells (measured slower)
#endif
#ifndef LLFE_KM_PP_SUPS_KK
#define LLFE_KM_PP_SUPS_KK 0  // ... in the rounds with at most this many chosen centres (0: the first round)
#endif
#ifndef LLFE_KM_WIDE
#define LLFE_KM_WIDE 0  // 1: the second build of this file (_build.py: 512 threads, unroll 4) as
                        // launch_kmeans_wide, which launch_kmeans hands batches whose attempts all
                        // fit the GPU at once (small batches: an attempt on 8 waves finishes sooner)
#endif
#ifndef LLFE_KM_THREADS
#define LLFE_KM_THREADS 256  // (round 6) 256-thread workgroups, four per CU: the pipelined step 20.5 ->
                             // 18.8 ms although an isolated launch is slower
#endif
constexpr int KT = LLFE_KM_THREADS;  // threads per (image, attempt)
constexpr int KW = KT / 64;       // waves
constexpr int STEP = 256;         // points per wave step (64 lanes x 4)
constexpr float kFar = 1e30f;     // coordinate of an unused centre: its distance is +inf

using km::cvrng_double;
using km::cvrng_next;
using km::splitmix64;

__device__ __forceinline__ float uni(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// OpenCV normL2Sqr<float>(dims = 3) of the AVX2/FMA3 dispatch: t0*t0, fma(t1), fma(t2)
__device__ __forceinline__ float d2(float x, float y, float z, float cx, float cy, float cz) {
    float t0 = x - cx, t1 = y - cy, t2 = z - cz;
    float d = t0 * t0;
    d = __builtin_fmaf(t1, t1, d);
    d = __builtin_fmaf(t2, t2, d);
    return d;
}

struct P3 {
    float x, y, z;
};
__device__ __forceinline__ P3 unpack(uint32_t k) {
    return P3{(float)((k >> 16) & 255u), (float)((k >> 8) & 255u), (float)(k & 255u)};
}

struct Cent {
    float x[kMaxK], y[kMaxK], z[kMaxK];
};

// first minimum over 5 centres (unused centres sit at kFar -> +inf)
__device__ __forceinline__ int label5(const P3 &p, const Cent &c, float &best) {
    best = d2(p.x, p.y, p.z, c.x[0], c.y[0], c.z[0]);
    int l = 0;
#pragma unroll
    for (int k = 1; k < kMaxK; k++) {
        float d = d2(p.x, p.y, p.z, c.x[k], c.y[k], c.z[k]);
        bool lt = d < best;
        best = lt ? d : best;
        l = lt ? k : l;
    }
    return l;
}

// Same labels as label5, with the distances of centre pairs (0,1), (2,3), (4,far) in
// packed FP32 (v_pk_add/mul/fma_f32: two IEEE lanes, bit-identical to the scalar ops)
// and the arg-min as min-then-first-equal (= the first strict minimum of the scan).
typedef float f2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
struct CentP {
    f2 x[3], y[3], z[3];
};

__device__ __forceinline__ CentP pack_centres(const Cent &c) {
    CentP r;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const int a = 2 * j, b = 2 * j + 1;
        r.x[j] = f2{c.x[a], b < kMaxK ? c.x[b] : kFar};
        r.y[j] = f2{c.y[a], b < kMaxK ? c.y[b] : kFar};
        r.z[j] = f2{c.z[a], b < kMaxK ? c.z[b] : kFar};
    }
    return r;
}

__device__ __forceinline__ int label5p(uint32_t key, const CentP &c) {
    const float x = (float)((key >> 16) & 255u), y = (float)((key >> 8) & 255u), z = (float)(key & 255u);
    const f2 px = f2{x, x}, py = f2{y, y}, pz = f2{z, z};
    f2 d[3];
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const f2 t0 = px - c.x[j], t1 = py - c.y[j], t2 = pz - c.z[j];
        f2 dd = t0 * t0;
        dd = __builtin_elementwise_fma(t1, t1, dd);
        dd = __builtin_elementwise_fma(t2, t2, dd);
        d[j] = dd;
    }
    const float m = fminf(fminf(fminf(d[0].x, d[0].y), fminf(d[1].x, d[1].y)), d[2].x);
    int l = 4;
    l = d[1].y == m ? 3 : l;
    l = d[1].x == m ? 2 : l;
    l = d[0].y == m ? 1 : l;
    l = d[0].x == m ? 0 : l;
    return l;
}

constexpr int PF = 4;  // steps of 16-B key loads kept in flight per wave
// k-means++ selection: 256-key steps per wave chunk of a partition (<= 4 x 256 x 256 keys,
// + alignment) and steps whose loads are issued together
constexpr int kSelSteps = ((4 * 256 * 256 + 3 + STEP - 1) / STEP + KW - 1) / KW + 1;
constexpr int SEL_U = 4;
#ifndef LLFE_KM_UNROLL
#define LLFE_KM_UNROLL 2  // failing cubes per push trip (2: the 256-entry ring that fits four
                          // 256-thread workgroups per CU)
#endif
#ifndef LLFE_KM_PPRUN
#define LLFE_KM_PPRUN 4
#endif
constexpr int kPPRun = LLFE_KM_PPRUN;  // 64-cube chunks per k-means++ work grab
// per-wave LDS ring of boundary colours awaiting labelling: the Lloyd sweep drains it
// once 128 colours are pending, so it holds <= 127 pending + LLFE_KM_UNROLL x 64 pushed
// (k-means++ drains at 64); a power of two (ring indices are masked)
constexpr int ring_size(int need) { return need <= 256 ? 256 : (need <= 512 ? 512 : 1024); }
constexpr int kStage = ring_size(127 + 64 * LLFE_KM_UNROLL);
static_assert(kStage >= 127 + 64 * LLFE_KM_UNROLL && (kStage & (kStage - 1)) == 0, "boundary-colour ring too small");

// the 4 keys of lane `lane` in 256-point step `s` (zeros past the full steps)
__device__ __forceinline__ uint4 load_step(const uint32_t *pts, int s, int se_full, int lane) {
    if (s < se_full) return *(const uint4 *)(pts + (size_t)s * STEP + lane * 4);
    return make_uint4(0u, 0u, 0u, 0u);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

struct KmSmem {
    unsigned long long accA[kMaxK][KT];  // x | y << 32 per lane and cluster
    unsigned long long accB[kMaxK][KT];  // z | 1 << 32
    union {
        unsigned long long red[32][20];  // [part][cluster x component] (lanes read along v)
        int cs[KW][256];                 // (Lloyd sweep) per-wave list of the cells of a chunk's failing super-cells
    };
    unsigned long long wtot[KW][3];
    unsigned long long scan_w[KW];
    double dred[KW];
    double maxd[KW];
    int maxi[KW];
    float c[kMaxK][3];
    float cprev[kMaxK][3];
    float cc[kMaxK][3];
    long long sums[kMaxK][3];
    int counts[kMaxK];
    int moved_idx[kMaxK];
    int moved_lbl[kMaxK];
    int n_moved;
    int found_step[3];
    unsigned long long found_excl[3];
    int ci[3];
    int flag;
    int task;                            // work-queue item of the workgroup (persistent launches)
    int next_chunk;                      // next 64-cube chunk to hand out (cube sweeps)
    unsigned long long fail_pts;  // keys read point by point in this Lloyd sweep
    // cube-based k-means++ (pp_cubes)
    unsigned long long psum[3][kParts];  // per trial and red-quarter partition: sum of T_j
    unsigned long long pD[kParts];       // per partition: sum of D (the winning trial)
    unsigned long long pex[3];
    unsigned long long S[3];
    uint32_t pbase[kParts + 1];          // first sorted key of each partition (np.unique index)
    uint32_t kbeg[kParts];               // ... its address in the key array (= pbase, or the
                                         // segmented layout's hist prefix, KmeansCubes::part_hist)
    uint32_t kfirst, klast;              // addresses of the first / last key in np.unique order
    int pj[3];
    int icc[kMaxK][3];                   // chosen centres (integer colours)
    unsigned long long sel_pts;          // colours the selection scans read
    unsigned long long wchunk[3][KW];    // per trial: sum of D over each wave's chunk
    uint32_t stage[KW][kStage + 64];     // per-wave ring of boundary colours (+ a dummy row)
    float thrL[3][kMaxK * kMaxK];        // Lloyd margin thresholds [cube / cell / super-cell][owner k][j]
    int cq[KW][256];                     // per-wave list of the cubes of a chunk's failing cells
    unsigned long long qtot;             // sum of |p|^2 over all colours (exact)
    int marg[kMaxK * kMaxK + 6 * kMaxK]; // k-means++ corner margins: centre pairs, trial vs centre (+/-)
    int margc[kMaxK * kMaxK + 6 * kMaxK];  // the same for the 4 x 8 x 8 cells
    int margs[kMaxK * kMaxK + 6 * kMaxK];  // ... and the 4 x 16 x 16 super-cells
};

// 1024 / KT workgroups per CU (160 KB of LDS): two of 512 threads, four of 256
static_assert(sizeof(KmSmem) * (1024 / KT) <= 160 * 1024, "KmSmem must leave room for 1024 / KT workgroups per CU");
// the k-means++ selection's step sums alias the Lloyd accumulators (accA, then accB)
static_assert(offsetof(KmSmem, accB) == sizeof(((KmSmem *)nullptr)->accA) &&
                  3 * KW * kSelSteps * sizeof(uint32_t) <= 2 * sizeof(((KmSmem *)nullptr)->accA),
              "selection step sums overflow the Lloyd accumulators (KT too small)");

__device__ __forceinline__ Cent load_centres(const float (*c)[3]) {
    Cent r;
#pragma unroll
    for (int k = 0; k < kMaxK; k++) {
        r.x[k] = uni(c[k][0]);
        r.y[k] = uni(c[k][1]);
        r.z[k] = uni(c[k][2]);
    }
    return r;
}

__device__ __forceinline__ int moved_label(const KmSmem &sm, int i, int l) {
    for (int m = 0; m < sm.n_moved; m++)
        if (sm.moved_idx[m] == i) l = sm.moved_lbl[m];
    return l;
}

// ------------------------------------------------------------ cube-based k-means++
// k-means++ centres are data points, so every distance it sums is an exact integer and
// whole cubes can be summed in closed form: for a cube with origin o, n colours o + u
// (u in [0,3]^3), S_u = sum u and S_u2 = sum |u|^2,
//     sum |o + u - c|^2 = n |o - c|^2 + 2 (o - c) . S_u + S_u2.
// d(p, a) - d(p, b) is linear in p, so its extremes over the cube are at corners:
//     min = f(o) - 6 sum_d max(a_d - b_d, 0),  max = f(o) + 6 sum_d max(b_d - a_d, 0),
// f(o) = d(o, a) - d(o, b).  A cube is "owned" by chosen centre k when no other chosen
// centre is ever strictly closer (then D = d(., c_k) on it), and a trial t is decided on
// it when it is never strictly closer than c_k (T = D) or always at least as close
// (T = d(., t)).  Undecided cubes are summed colour by colour (enumerated from the
// occupancy mask); the totals and therefore every choice are bit-identical to the
// plain sweep.
//
// The selection prefix(D, i) >= p runs in np.unique order: the red-quarter partitions
// are contiguous ranges of the sorted keys and unions of whole cubes (cube id = R << 12
// | ...), so the partition holding p comes from per-partition cube totals and only that
// partition's sorted keys are scanned.
// |a|, |b|, |c| <= 255: 24-bit multiplies (v_mul_i32_i24 / v_mad_i32_i24, full rate) instead
// of the quarter-rate v_mul_lo_u32 a plain int product compiles to
__device__ __forceinline__ int d2i(int x, int y, int z, int cx, int cy, int cz) {
    const int a = x - cx, b = y - cy, c = z - cz;
    return __mul24(a, a) + __mul24(b, b) + __mul24(c, c);
}

struct ICent {
    int x[kMaxK], y[kMaxK], z[kMaxK];
};

// d(p, a) >= d(p, b) for every p of the cube at origin o
__device__ __forceinline__ bool never_closer(int ox, int oy, int oz, int ax, int ay, int az, int bx, int by, int bz) {
    const int f = d2i(ox, oy, oz, ax, ay, az) - d2i(ox, oy, oz, bx, by, bz);
    return f - 6 * (max(ax - bx, 0) + max(ay - by, 0) + max(az - bz, 0)) >= 0;
}
// d(p, a) <= d(p, b) for every p of the cube at origin o
__device__ __forceinline__ bool always_closer(int ox, int oy, int oz, int ax, int ay, int az, int bx, int by, int bz) {
    const int f = d2i(ox, oy, oz, ax, ay, az) - d2i(ox, oy, oz, bx, by, bz);
    return f + 6 * (max(bx - ax, 0) + max(by - ay, 0) + max(bz - az, 0)) <= 0;
}

struct CubeGeo {  // origin, count, sums of u = colour - origin and of |u|^2
    int ox, oy, oz, n, sx, sy, sz, s2;
};

// the colour of mask bit `bit` in the cube `id` (bit = i*16 + j*4 + b)
__device__ __forceinline__ uint32_t cube_key(uint32_t id, int bit) {
    return ((((id >> 12) & 63u) * 4u + (uint32_t)(bit >> 4)) << 16) |
           ((((id >> 6) & 63u) * 4u + (uint32_t)((bit >> 2) & 3)) << 8) | ((id & 63u) * 4u + (uint32_t)(bit & 3));
}
__device__ __forceinline__ CubeGeo cube_geo(const CubeEnt &e) {
    CubeGeo g;
    g.ox = (int)((e.id >> 12) & 63u) * 4;
    g.oy = (int)((e.id >> 6) & 63u) * 4;
    g.oz = (int)(e.id & 63u) * 4;
    g.n = (int)(e.sums & 127u);
    g.sx = (int)((e.sums >> 7) & 255u);
    g.sy = (int)((e.sums >> 15) & 255u);
    g.sz = (int)(e.sums >> 23);
    g.s2 = (int)(e.id >> 18);
    return g;
}
__device__ __forceinline__ uint32_t cube_sum(const CubeGeo &g, int cx, int cy, int cz) {
    // n <= 64, |a| <= 255, S_u <= 192: every factor fits 24 bits (n |o - c|^2 < 2^24 unsigned)
    const int ax = g.ox - cx, ay = g.oy - cy, az = g.oz - cz;
    const uint32_t q = (uint32_t)(__mul24(ax, ax) + __mul24(ay, ay) + __mul24(az, az));
    return __umul24((uint32_t)g.n, q) + 2u * (uint32_t)(__mul24(ax, g.sx) + __mul24(ay, g.sy) + __mul24(az, g.sz)) +
           (uint32_t)g.s2;
}

// per lane: bit `lane` of the wave-uniform 64-bit mask m ? a : b -- one v_cndmask_b32
// reading m as a lane mask from an SGPR pair
__device__ __forceinline__ uint32_t lane_sel(unsigned long long m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %2, %1, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}

// clear bit `b` of a wave-uniform 64-bit mask with one s_bitset0_b64 (fm &= fm - 1 is three
// scalar ops: the 64-bit subtract is two)
__device__ __forceinline__ unsigned long long clear_bit(unsigned long long m, int b) {
    asm("s_bitset0_b64 %0, %1" : "+s"(m) : "s"(b));
    return m;
}

// the colour of mask bit `lane` relative to its cube's origin (bit = i*16 + j*4 + b)
__device__ __forceinline__ uint32_t lane_offset(int lane) {
    return ((uint32_t)(lane >> 4) << 16) | ((uint32_t)((lane >> 2) & 3) << 8) | (uint32_t)(lane & 3);
}
__device__ __forceinline__ uint32_t cube_origin_key(uint32_t id) {
    return ((((id >> 12) & 63u) * 4u) << 16) | ((((id >> 6) & 63u) * 4u) << 8) | ((id & 63u) * 4u);
}

// Boundary colours are packed densely into the wave's lanes before they are labelled:
// the colours of cube (m, origin key) go to lanes [fill, fill + popc(m)) of pk (ds_permute
// push; lane b's rank among the set bits comes from mbcnt).  fill + popc(m) <= 64;
// m and id are wave-uniform (SGPRs).
__device__ __forceinline__ uint32_t lane_off_rel(int fill) { return (uint32_t)(__lane_id() - fill); }

// The cube table is streamed 64 entries per wave step with the next CPF steps' 16-B
// loads in flight (3 measured no faster: the sweeps are VALU-bound).
constexpr int CPF = 1;
struct CubeRing {
    CubeEnt r[CPF];
    __device__ __forceinline__ void init(const CubeEnt *t, int cb, int cend, int lane) {
#pragma unroll
        for (int q = 0; q < CPF; q++) {
            r[q].mask = 0;
            r[q].id = 0;
            r[q].sums = 0;
            if (cb + q * 64 + lane < cend) r[q] = t[cb + q * 64 + lane];
        }
    }
    // entry `ci` (this lane's cube of the current step); loads the step CPF ahead
    __device__ __forceinline__ CubeEnt next(const CubeEnt *t, int ci, int cend) {
        const CubeEnt e = r[0];
#pragma unroll
        for (int q = 0; q + 1 < CPF; q++) r[q] = r[q + 1];
        if (ci + CPF * 64 < cend) r[CPF - 1] = t[ci + CPF * 64];
        return e;
    }
};

// the uniform mask / id of the cube in lane `src`
__device__ __forceinline__ unsigned long long lane_mask(const CubeEnt &e, int src) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)e.mask, src);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(e.mask >> 32), src);
    return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ int unpack_r(uint32_t k) { return (int)((k >> 16) & 255u); }
__device__ __forceinline__ int unpack_g(uint32_t k) { return (int)((k >> 8) & 255u); }
__device__ __forceinline__ int unpack_b(uint32_t k) { return (int)(k & 255u); }

// D(p) for a packed key by the linear forms: d(p, c) = |p|^2 - H_c(p), H_c(p) = 2 p.c - |c|^2,
// 2 p.c = dot2((B, R), (2 c_B, 2 c_R)) + G 2 c_G (v_dot2_u32_u16 over one v_mad_u32_u24 whose
// addend is -|c|^2: the u32 arithmetic wraps to the exact int), so min over the chosen centres
// = |p|^2 - max H: three VALU ops per centre instead of d2i's six and a min
struct HCent {
    u16x2 rb2[kMaxK];      // (2 c_B, 2 c_R)
    uint32_t g2[kMaxK];    // 2 c_G
    uint32_t nc2[kMaxK];   // -|c|^2 (mod 2^32)
};
__device__ __forceinline__ HCent hcent(const ICent &ch) {
    HCent h;
#pragma unroll
    for (int m = 0; m < kMaxK; m++) {
        h.rb2[m] = u16x2{(uint16_t)(2 * ch.z[m]), (uint16_t)(2 * ch.x[m])};
        h.g2[m] = (uint32_t)(2 * ch.y[m]);
        h.nc2[m] = 0u - (uint32_t)(ch.x[m] * ch.x[m] + ch.y[m] * ch.y[m] + ch.z[m] * ch.z[m]);
    }
    return h;
}
template <int KK>
__device__ __forceinline__ uint32_t dmin_key(uint32_t kq, const HCent &h) {
    const u16x2 rb = __builtin_bit_cast(u16x2, kq & 0x00FF00FFu);  // (B, R)
    const uint32_t g = (kq >> 8) & 255u;
    const uint32_t p2 = __builtin_amdgcn_udot2(rb, rb, __umul24(g, g), false);
    int Hm = (int)__builtin_amdgcn_udot2(rb, h.rb2[0], __umul24(g, h.g2[0]) + h.nc2[0], false);
#pragma unroll
    for (int m = 1; m < KK; m++)
        Hm = max(Hm, (int)__builtin_amdgcn_udot2(rb, h.rb2[m], __umul24(g, h.g2[m]) + h.nc2[m], false));
    return p2 - (uint32_t)Hm;
}

// Partition p's keys in np.unique order, in the key array (wave 0): sm.pbase[p] (np.unique
// index of its first key, and the total at kParts), sm.kbeg[p] (its first key's address:
// = pbase when the keys are contiguous, the prefix of the partitions' pixel counts `hist`
// in k_uq_part's segmented layout), sm.kfirst / sm.klast (addresses of the first and the
// last key).  Returns, in every lane, the address of np.unique index `idx` (< total).
__device__ __forceinline__ uint32_t key_layout(KmSmem &sm, const uint32_t *__restrict__ part_uq,
                                               const uint32_t *__restrict__ hist, uint32_t idx) {
    const int lane = threadIdx.x & 63;
    const uint32_t v = part_uq[lane], hv = hist ? hist[lane] : v;
    uint32_t x = v, hx = hv;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off), hy = __shfl_up(hx, off);
        if (lane >= off) x += y, hx += hy;
    }
    const uint32_t pb = x - v, kb = hx - hv;
    sm.pbase[lane] = pb;
    sm.kbeg[lane] = kb;
    if (lane == 63) sm.pbase[kParts] = x;
    const unsigned long long ne = __ballot(v != 0);  // (total > 0: some partition is not empty)
    const int p0 = ne ? (int)__builtin_ctzll(ne) : 0, pl = ne ? 63 - (int)__builtin_clzll(ne) : 0;
    const uint32_t kf = __shfl(kb, p0), kl = __shfl(kb, pl) + __shfl(v, pl) - 1;
    if (lane == 0) {
        sm.kfirst = kf;
        sm.klast = kl;
    }
    // the partition of idx: the last one starting at or before it (empty ones share the
    // next one's start and precede it)
    const unsigned long long le = __ballot(pb <= idx);
    const int P = le ? 63 - (int)__builtin_clzll(le) : 0;
    return __shfl(kb, P) + (idx - __shfl(pb, P));
}

// A call in the one-launch kernel (inlined there it spilled 37 VGPRs); inlined into the
// split build's k-means++ kernel (105 VGPRs, no scratch; as a call that kernel needed 128
// VGPRs with 2 spilled).
#if LLFE_KM_PP_CALL
__device__
#else
__device__ __forceinline__
#endif
void pp_cubes(KmSmem &sm, const uint32_t *__restrict__ pts, int N, int K, uint64_t &rng,
                         const CubeEnt *__restrict__ ctab, int C, const CellEnt *__restrict__ ltab, int L,
                         const SupEnt *__restrict__ stab, int S, const uint32_t *__restrict__ part_uq, const uint32_t *__restrict__ hist,
                         unsigned long long &bytes, uint32_t &pp_pts, uint32_t &pp_sel, uint64_t &t_sel) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t c0 = cvrng_next(rng) % (uint32_t)N;  // (every thread advances its rng copy)
    if (wid == 0) {
        const uint32_t a0 = key_layout(sm, part_uq, hist, c0);
        if (lane == 0) {
            const uint32_t q0 = pts[a0];
            sm.icc[0][0] = unpack_r(q0);
            sm.icc[0][1] = unpack_g(q0);
            sm.icc[0][2] = unpack_b(q0);
        }
    }
    if (tid == 0) {
        sm.fail_pts = 0;
        sm.sel_pts = 0;
        sm.qtot = 0;
    }
    if (tid >= 64 && tid < 64 + (kMaxK - 1) * 3) (&sm.icc[1][0])[tid - 64] = 0;
    unsigned long long sum0 = 0, qacc = 0;  // qacc: sum |p|^2 over the lane's cubes
    for (int kk = 0; kk < K; kk++) {
        __syncthreads();
        ICent ch;  // chosen centres 0 .. kk-1 (uniform)
#pragma unroll
        for (int m = 0; m < kMaxK; m++) {
            ch.x[m] = __builtin_amdgcn_readfirstlane(sm.icc[m][0]);
            ch.y[m] = __builtin_amdgcn_readfirstlane(sm.icc[m][1]);
            ch.z[m] = __builtin_amdgcn_readfirstlane(sm.icc[m][2]);
        }
        int tx[3], ty[3], tz[3];
        if (kk == 0) {
#pragma unroll
            for (int j = 0; j < 3; j++) {
                tx[j] = ch.x[0];
                ty[j] = ch.y[0];
                tz[j] = ch.z[0];
            }
        } else {
            const uint64_t tsel0 = wall_clock64();
            double p[3];
#pragma unroll
            for (int j = 0; j < 3; j++) p[j] = cvrng_double(rng) * (double)sum0;
            // ---- partition holding prefix(D) >= p_j
            if (wid == 0) {
                const unsigned long long v = sm.pD[lane];
                unsigned long long x = v;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const unsigned long long y = __shfl_up(x, off);
                    if (lane >= off) x += y;
                }
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    const unsigned long long bal = __ballot((double)x >= p[j]);
                    const int P = bal ? (int)__builtin_ctzll(bal) : 0;
                    const unsigned long long ex = __shfl(x - v, P);
                    if (lane == 0) {
                        sm.pj[j] = !(p[j] > 0) ? -2 : (bal ? P : -1);
                        sm.pex[j] = ex;
                    }
                }
            }
            __syncthreads();
            // (the scans, instantiated per number of chosen centres as the round's sweep below)
            auto select = [&](auto KKc) __attribute__((always_inline)) {
                constexpr int KK = decltype(KKc)::value;
                // ---- the partition's sorted keys in KW wave chunks of whole 256-key steps
                // (aligned to the key list, so every lane reads its 4 keys with one 16-byte
                // load; keys outside the partition are masked): step sums of D into LDS and
                // chunk sums.  The three trials' chunks are walked together, SEL_U steps per
                // trip with their loads issued first -- these scans were chains of dependent
                // scalar loads (~75 us per k-means++ round on a photo).
                // Step sums alias the Lloyd accumulators (unused until Lloyd).
                uint32_t(*stp)[KW][kSelSteps] = reinterpret_cast<uint32_t(*)[KW][kSelSteps]>(&sm.accA[0][0]);
                const HCent hc = hcent(ch);
                uint32_t ca[3], cb2[3], cw0[3], cw1[3];  // partition [a, b), this wave's steps [w0, w1)
                // a partition two trials share is scanned once (the later trial reads the
                // earlier one's step and chunk sums: D is the same for all three)
                const int P0 = sm.pj[0], P1 = sm.pj[1], P2 = sm.pj[2];
                const bool dup[3] = {false, P1 >= 0 && P1 == P0, P2 >= 0 && (P2 == P0 || P2 == P1)};
    #pragma unroll
                for (int j = 0; j < 3; j++) {
                    const int P = dup[j] ? -1 : sm.pj[j];  // (its keys: addresses [kbeg, kbeg + count))
                    ca[j] = P >= 0 ? sm.kbeg[P] : 0u;
                    cb2[j] = P >= 0 ? sm.kbeg[P] + (sm.pbase[P + 1] - sm.pbase[P]) : 0u;
                    const uint32_t A = ca[j] & ~3u;
                    const uint32_t nst = (cb2[j] - A + STEP - 1) / STEP;   // steps over [A, b)
                    const uint32_t per = (nst + KW - 1) / KW;               // steps per wave (<= kSelSteps)
                    cw0[j] = A + min(nst, (uint32_t)wid * per) * STEP;
                    cw1[j] = A + min(nst, (uint32_t)(wid + 1) * per) * STEP;
                }
                {
                    uint32_t csum_lo[3] = {0u, 0u, 0u};  // per-lane partial chunk sums
                    unsigned long long cnt = 0;
    #pragma unroll
                    for (int j = 0; j < 3; j++) {
                        uint32_t ls = 0;
                        for (uint32_t s0 = cw0[j]; s0 < cw1[j]; s0 += SEL_U * STEP) {
                            uint4 kv[SEL_U];
    #pragma unroll
                            for (int u = 0; u < SEL_U; u++) {
                                const uint32_t i0 = s0 + (uint32_t)u * STEP + (uint32_t)lane * 4;
                                kv[u] = make_uint4(0u, 0u, 0u, 0u);
                                if (i0 < cw1[j] && i0 < cb2[j] && i0 + 4 > ca[j]) kv[u] = *(const uint4 *)(pts + i0);
                            }
    #pragma unroll
                            for (int u = 0; u < SEL_U; u++) {
                                const uint32_t st = s0 + (uint32_t)u * STEP;
                                if (st >= cw1[j]) break;  // (uniform)
                                const uint32_t i0 = st + (uint32_t)lane * 4;
                                const uint32_t kq[4] = {kv[u].x, kv[u].y, kv[u].z, kv[u].w};
                                uint32_t sd = 0;
    #pragma unroll
                                for (int jj = 0; jj < 4; jj++) {
                                    const uint32_t i = i0 + (uint32_t)jj;
                                    const bool in = i >= ca[j] && i < cb2[j];
                                    const uint32_t d = dmin_key<KK>(kq[jj], hc);
                                    sd += in ? d : 0u;
                                }
                                ls += sd;
                                const uint32_t ssum = wave_sum(sd);  // <= 256 x 195075 < 2^32
                                if (lane == 0) stp[j][wid][(st - cw0[j]) / STEP] = ssum;
                            }
                        }
                        csum_lo[j] = ls;
                        cnt += cw1[j] - cw0[j];
                    }
    #pragma unroll
                    for (int j = 0; j < 3; j++) {
                        const unsigned long long ws = wave_sum((unsigned long long)csum_lo[j]);
                        if (lane == 0) sm.wchunk[j][wid] = ws;
                    }
                    if (lane == 0) atomicAdd(&sm.sel_pts, cnt);
                }
                __syncthreads();
                // ... then wave j < 3 finds the chunk, the step (from the step sums) and the
                // first crossing in that one step
                if (wid < 3) {
                    const int j = wid;
                    const double pj = j == 0 ? p[0] : (j == 1 ? p[1] : p[2]);
                    const int P = j == 0 ? P0 : (j == 1 ? P1 : P2);  // (sm.pj[j] is being overwritten)
                    const int src = j == 1 ? (dup[1] ? 0 : 1) : (j == 2 ? (!dup[2] ? 2 : (P2 == P0 ? 0 : 1)) : 0);
                    // (key addresses; p <= 0: the first key, p beyond the total: the last)
                    int ci = (int)(P == -2 ? sm.kfirst : sm.klast);
                    if (P >= 0) {
                        const uint32_t a = sm.kbeg[P], b = a + (sm.pbase[P + 1] - sm.pbase[P]);  // (not ca[j]: no dynamic private indexing)
                        const uint32_t A = a & ~3u;
                        const uint32_t nst = (b - A + STEP - 1) / STEP, per = (nst + KW - 1) / KW;
                        unsigned long long e = sm.pex[j];
                        int w = 0;
                        for (; w < KW - 1; w++) {
                            if ((double)(e + sm.wchunk[src][w]) >= pj) break;
                            e += sm.wchunk[src][w];
                        }
                        const uint32_t w0 = A + min(nst, (uint32_t)w * per) * STEP, w1 = A + min(nst, (uint32_t)(w + 1) * per) * STEP;
                        const int ns = (int)((w1 - w0) / STEP);
                        // the step: inclusive prefix of the chunk's step sums, 64 at a time
                        int sidx = ns - 1;
                        for (int s_base = 0; s_base < ns; s_base += 64) {
                            const int si = s_base + lane;
                            const unsigned long long v = si < ns ? (unsigned long long)stp[src][w][si] : 0ull;
                            unsigned long long x = v;
    #pragma unroll
                            for (int off = 1; off < 64; off <<= 1) {
                                const unsigned long long y = __shfl_up(x, off);
                                if (lane >= off) x += y;
                            }
                            const unsigned long long bal = __ballot(si < ns && (double)(e + x) >= pj);
                            if (bal) {
                                const int f = (int)__builtin_ctzll(bal);
                                sidx = s_base + f;
                                e += __shfl(x - v, f);
                                break;
                            }
                            e += __shfl(x, 63);
                        }
                        int found = -1;
                        if (ns > 0) {
                            const uint32_t s0 = w0 + (uint32_t)sidx * STEP;
                            const uint32_t i0 = s0 + (uint32_t)lane * 4;
                            uint4 kv = make_uint4(0u, 0u, 0u, 0u);
                            if (i0 < b && i0 + 4 > a) kv = *(const uint4 *)(pts + i0);
                            const uint32_t kq[4] = {kv.x, kv.y, kv.z, kv.w};
                            uint32_t dv[4], ls = 0;
    #pragma unroll
                            for (int jj = 0; jj < 4; jj++) {
                                const uint32_t i = i0 + (uint32_t)jj;
                                const bool in = i >= a && i < b;
                                dv[jj] = in ? dmin_key<KK>(kq[jj], hc) : 0u;
                                ls += dv[jj];
                            }
                            unsigned long long x = ls;
    #pragma unroll
                            for (int off = 1; off < 64; off <<= 1) {
                                const unsigned long long y = __shfl_up(x, off);
                                if (lane >= off) x += y;
                            }
                            unsigned long long ee = e + x - ls;
                            int hit = -1;
    #pragma unroll
                            for (int jj = 0; jj < 4; jj++) {
                                const uint32_t i = i0 + (uint32_t)jj;
                                ee += dv[jj];
                                if (hit < 0 && i >= a && i < b && (double)ee >= pj) hit = jj;
                            }
                            const unsigned long long bal = __ballot(hit >= 0);
                            if (bal) {
                                const int first = (int)__builtin_ctzll(bal);
                                found = (int)(s0 + (uint32_t)first * 4) + __shfl(hit, first);
                            }
                            if (lane == 0) atomicAdd(&sm.sel_pts, (unsigned long long)STEP);
                        }
                        if (found >= 0) ci = found;  // (inside [a, b))
                    }
                    if (lane == 0) sm.pj[j] = ci;
                }
            };
            switch (kk) {
                case 1: select(std::integral_constant<int, 1>{}); break;
                case 2: select(std::integral_constant<int, 2>{}); break;
                case 3: select(std::integral_constant<int, 3>{}); break;
                default: select(std::integral_constant<int, kMaxK - 1>{}); break;
            }
            __syncthreads();
            t_sel += wall_clock64() - tsel0;
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const uint32_t k = pts[sm.pj[j]];
                tx[j] = __builtin_amdgcn_readfirstlane(unpack_r(k));
                ty[j] = __builtin_amdgcn_readfirstlane(unpack_g(k));
                tz[j] = __builtin_amdgcn_readfirstlane(unpack_b(k));
            }
        }
        // ---- trial sums T_j = sum min(D, d(., t_j)) per partition (kk == 0: sum d(., c0))
        // the round's sweep, instantiated per number of chosen centres (KK = kk <= kMaxK - 1):
        // the centre loops become straight-line code without per-centre guards
        auto sweep = [&](auto KKc) __attribute__((always_inline)) {
            constexpr int KK = decltype(KKc)::value;
            if (tid < 3 * kParts) (&sm.psum[0][0])[tid] = 0;
            if (tid == 0) sm.next_chunk = 0;
            __syncthreads();
            unsigned long long acc0 = 0, acc1 = 0, acc2 = 0, fails = 0;
            int Pcur = -1;
            // Round constants (wave-uniform).  Every test below is linear in the cube origin o:
            // with D_c(o) = |c|^2 - 2 o.c, d(o, c) = |o|^2 + D_c(o), so
            //   d(o, a) - d(o, b) = D_a(o) - D_b(o)          (never / always closer tests)
            //   sum over the cube |p - c|^2 = n (|o|^2 + D_c(o)) + 2 (o - c).S_u + S_u2
            // and the corner margins 6 sum max(+-(a - b), 0) depend on the centres only.
            // The pairwise corner margins live in LDS (per-lane reads indexed by the lane's
            // owner k); the per-centre constants stay in scalar registers.
            // (B, R) and G of the chosen centres and the trials, doubled: every use below is
            // 2 p.c (2 o.c, 2 S_u.c), so the doubling costs nothing and saves a shift per use
            int C2[kMaxK], T2[3], chg2[kMaxK], tg2[3];
            u16x2 chrb[kMaxK], trb[3];
    #pragma unroll
            for (int m = 0; m < kMaxK; m++) {
                chrb[m] = u16x2{(uint16_t)(2 * ch.z[m]), (uint16_t)(2 * ch.x[m])};
                chg2[m] = 2 * ch.y[m];
            }
    #pragma unroll
            for (int j = 0; j < 3; j++) {
                trb[j] = u16x2{(uint16_t)(2 * tz[j]), (uint16_t)(2 * tx[j])};
                tg2[j] = 2 * ty[j];
            }
    #pragma unroll
            for (int m = 0; m < kMaxK; m++) C2[m] = ch.x[m] * ch.x[m] + ch.y[m] * ch.y[m] + ch.z[m] * ch.z[m];
    #pragma unroll
            for (int j = 0; j < 3; j++) T2[j] = tx[j] * tx[j] + ty[j] * ty[j] + tz[j] * tz[j];
            // undecided cubes' colours go through the wave's LDS ring (as in the Lloyd
            // sweeps) and are summed 64 at a time
            const uint32_t loff = lane_offset(lane);
            uint32_t *stg = sm.stage[wid];
            int head = 0, tail = 0;  // wave-uniform ring counters
            auto sum_stage = [&](int count) {
                __builtin_amdgcn_wave_barrier();
                fails += (unsigned long long)count;
                if (lane < count) {
                    // d(p, c) = |p|^2 - H_c(p), H_c(p) = 2 p.c - |c|^2 (exact integers): the
                    // |p|^2 term is common to D and every trial, so min(D, d(p, t)) =
                    // |p|^2 - max(max_m H_m, H_t).  2 p.c - |c|^2 = dot2((B, R), 2 (c_B, c_R))
                    // over the 24-bit multiply-add G 2 c_G - |c|^2 (u32 arithmetic wraps to the
                    // exact int): two VALU ops per centre
                    const uint32_t kq = stg[(tail + lane) & (kStage - 1)];
                    const u16x2 rb = __builtin_bit_cast(u16x2, kq & 0x00FF00FFu);  // (B, R)
                    const uint32_t g = (kq >> 8) & 255u;
                    const uint32_t p2 = __builtin_amdgcn_udot2(rb, rb, __umul24(g, g), false);
                    auto H = [&](u16x2 crb2, int cg2, int c2) {
                        return (int)__builtin_amdgcn_udot2(rb, crb2, __umul24(g, (uint32_t)cg2) + (0u - (uint32_t)c2), false);
                    };
                    int Hm = H(chrb[0], chg2[0], C2[0]);
    #pragma unroll
                    for (int m = 1; m < kMaxK; m++)
                        if (m < KK) Hm = max(Hm, H(chrb[m], chg2[m], C2[m]));
                    acc0 += p2 - (uint32_t)max(Hm, H(trb[0], tg2[0], T2[0]));
                    acc1 += p2 - (uint32_t)max(Hm, H(trb[1], tg2[1], T2[1]));
                    acc2 += p2 - (uint32_t)max(Hm, H(trb[2], tg2[2], T2[2]));
                }
                tail += count;
            };
            auto flush_pk = [&]() {
                while (head - tail >= 64) sum_stage(64);
                if (head > tail) sum_stage(head - tail);
            };
            if (tid < kMaxK * kMaxK) {  // Mkk[m][k] = 6 sum max(c_m - c_k, 0)
                const int m = tid / kMaxK, k2 = tid % kMaxK;
                sm.marg[tid] = 6 * (max(sm.icc[m][0] - sm.icc[k2][0], 0) + max(sm.icc[m][1] - sm.icc[k2][1], 0) +
                                    max(sm.icc[m][2] - sm.icc[k2][2], 0));
            } else if (tid < kMaxK * kMaxK + 6 * kMaxK) {  // NA[j][k], NB[j][k]
                const int q = tid - kMaxK * kMaxK, j = (q / kMaxK) % 3, k2 = q % kMaxK;
                const int t[3] = {j == 0 ? tx[0] : (j == 1 ? tx[1] : tx[2]), j == 0 ? ty[0] : (j == 1 ? ty[1] : ty[2]),
                                  j == 0 ? tz[0] : (j == 1 ? tz[1] : tz[2])};
                const int sg = q < 3 * kMaxK ? 1 : -1;  // NA: t - c_k ; NB: c_k - t
                int acc = 0;
    #pragma unroll
                for (int d = 0; d < 3; d++) acc += max(sg * (t[d] - sm.icc[k2][d]), 0);
                sm.marg[tid] = 6 * acc;
            }
            // the same corner margins for a 4 x 8 x 8 cell: 2 (3, 7, 7) . max(+-(a - b), 0)
            if (tid >= 64 && tid < 64 + kMaxK * kMaxK) {
                const int q = tid - 64, m = q / kMaxK, k2 = q % kMaxK;
                sm.margc[q] = 6 * max(sm.icc[m][0] - sm.icc[k2][0], 0) + 14 * max(sm.icc[m][1] - sm.icc[k2][1], 0) +
                              14 * max(sm.icc[m][2] - sm.icc[k2][2], 0);
            } else if (tid >= 64 + kMaxK * kMaxK && tid < 64 + kMaxK * kMaxK + 6 * kMaxK) {
                const int q = tid - 64 - kMaxK * kMaxK, j = (q / kMaxK) % 3, k2 = q % kMaxK;
                const int t[3] = {j == 0 ? tx[0] : (j == 1 ? tx[1] : tx[2]), j == 0 ? ty[0] : (j == 1 ? ty[1] : ty[2]),
                                  j == 0 ? tz[0] : (j == 1 ? tz[1] : tz[2])};
                const int sg = q < 3 * kMaxK ? 1 : -1;
                sm.margc[kMaxK * kMaxK + q] = 6 * max(sg * (t[0] - sm.icc[k2][0]), 0) +
                                              14 * max(sg * (t[1] - sm.icc[k2][1]), 0) +
                                              14 * max(sg * (t[2] - sm.icc[k2][2]), 0);
            }
            // ... and for a 4 x 16 x 16 super-cell: 2 (3, 15, 15) . max(+-(a - b), 0)
            if (tid >= 128 && tid < 128 + kMaxK * kMaxK) {
                const int q = tid - 128, m = q / kMaxK, k2 = q % kMaxK;
                sm.margs[q] = 6 * max(sm.icc[m][0] - sm.icc[k2][0], 0) + 30 * max(sm.icc[m][1] - sm.icc[k2][1], 0) +
                              30 * max(sm.icc[m][2] - sm.icc[k2][2], 0);
            } else if (tid >= 128 + kMaxK * kMaxK && tid < 128 + kMaxK * kMaxK + 6 * kMaxK) {
                const int q = tid - 128 - kMaxK * kMaxK, j = (q / kMaxK) % 3, k2 = q % kMaxK;
                const int t[3] = {j == 0 ? tx[0] : (j == 1 ? tx[1] : tx[2]), j == 0 ? ty[0] : (j == 1 ? ty[1] : ty[2]),
                                  j == 0 ? tz[0] : (j == 1 ? tz[1] : tz[2])};
                const int sg = q < 3 * kMaxK ? 1 : -1;
                sm.margs[kMaxK * kMaxK + q] = 6 * max(sg * (t[0] - sm.icc[k2][0]), 0) +
                                              30 * max(sg * (t[1] - sm.icc[k2][1]), 0) +
                                              30 * max(sg * (t[2] - sm.icc[k2][2]), 0);
            }
            __syncthreads();
            const int *Mkk = sm.marg, *NA = sm.marg + kMaxK * kMaxK, *NB = sm.marg + kMaxK * kMaxK + 3 * kMaxK;
            // waves take 64-cube chunks from a shared LDS counter, read two chunks ahead
            // (ascending per wave, so the partition bookkeeping below still sees its
            // partitions in order)
            // Waves take runs of kPPRun 64-cube chunks: every partition change of a wave
            // costs a flush (the staged colours summed as a partial batch, three wave sums,
            // three LDS atomics), and single chunks handed out round-robin put nearly
            // every chunk of a wave in a new partition.
            constexpr int kRun = 64 * kPPRun;
            auto grab = [&]() {
                int b = 0;
                if (lane == 0) b = atomicAdd(&sm.next_chunk, kRun);
                return b;
            };
            // Closed forms of a box (a cube, or a cell of up to four cubes) with origin o,
            // count n, colour-offset sums S_u and S_u2: v_j = sum over its colours of
            // min(D, d(., t_j)) (kk == 0: d(., t_0)), `fail` when some chosen centre or trial
            // is not decided on the whole box.  ext: the box's offsets to its centre
            // doubled, (3, 3, 3) for a cube, (3, 7, 7) for a cell; MK / NAx / NBx: its corner
            // margins.
            auto box_vals = [&](int ox, int oy, int oz, int n, int sx, int sy, int sz, int s2, const int *MK,
                                const int *NAx, const int *NBx, int ex, int ey, int ez, uint32_t &v0, uint32_t &v1,
                                uint32_t &v2, bool &fail) __attribute__((always_inline)) {
                fail = false;
                if (KK == 0) {
                    auto bsum = [&](int cx, int cy, int cz) {
                        const int ax = ox - cx, ay = oy - cy, az = oz - cz;
                        const uint32_t q = (uint32_t)(__mul24(ax, ax) + __mul24(ay, ay) + __mul24(az, az));
                        return __umul24((uint32_t)n, q) + 2u * (uint32_t)(__mul24(ax, sx) + __mul24(ay, sy) + __mul24(az, sz)) +
                               (uint32_t)s2;
                    };
                    v0 = bsum(tx[0], ty[0], tz[0]);
                    qacc += bsum(0, 0, 0);
                    v1 = v2 = 0;
                    return;
                }
                // owner candidate: nearest chosen centre to the box centre q = o + ext / 2:
                // argmin_m |q - c_m|^2 = argmin_m (D_m(o) - ext . c_m), first minimum.
                // Dot products of (R, B) pairs by v_dot2_u32_u16 plus the G term by a
                // 24-bit multiply (operands <= 255 and sums <= 1792, results < 2^32: exact)
                const u16x2 orb = u16x2{(uint16_t)oz, (uint16_t)ox};
                const u16x2 srb = u16x2{(uint16_t)sz, (uint16_t)sx};
                auto odot = [&](u16x2 crb, int cg) {  // o . c (o . 2c with the doubled constants)
                    return (int)__builtin_amdgcn_udot2(orb, crb, __umul24((uint32_t)oy, (uint32_t)cg), false);
                };
                auto sdot = [&](u16x2 crb, int cg) {  // S_u . c (S_u . 2c with the doubled constants)
                    return (int)__builtin_amdgcn_udot2(srb, crb, __umul24((uint32_t)sy, (uint32_t)cg), false);
                };
                int Dc[kMaxK];
    #pragma unroll
                for (int m = 0; m < kMaxK; m++) {  // (only the KK chosen centres are read)
                    Dc[m] = 0;
                    if (m < KK) Dc[m] = C2[m] - odot(chrb[m], chg2[m]);
                }
                auto sq = [&](int m) { return ex * ch.x[m] + ey * ch.y[m] + ez * ch.z[m]; };
                int k = 0, bd = Dc[0] - sq(0);
    #pragma unroll
                for (int m = 1; m < kMaxK; m++) {
                    if (m >= KK) break;
                    const int d = Dc[m] - sq(m);
                    if (d < bd) {
                        bd = d;
                        k = m;
                    }
                }
                // owner k's values (per-lane selects from the uniform tables)
                int Dk = Dc[0], ky = chg2[0];
                u16x2 krb = chrb[0];
    #pragma unroll
                for (int m = 1; m < kMaxK; m++) {
                    if (m >= KK) break;
                    Dk = k == m ? Dc[m] : Dk;
                    ky = k == m ? chg2[m] : ky;
                    krb = k == m ? chrb[m] : krb;
                }
                // owned: no other chosen centre is ever strictly closer on the box
                bool owned = true;
    #pragma unroll
                for (int m = 0; m < kMaxK; m++) {
                    if (m >= KK) break;
                    if (m != k) owned = owned & (Dc[m] - Dk - MK[m * kMaxK + k] >= 0);
                }
                // box sums: P + n D_c(o) - 2 c.S_u, P = n |o|^2 + 2 o.S_u + S_u2
                const int Pc = __mul24(n, odot(orb, oy)) + 2 * sdot(orb, oy) + s2;
                const uint32_t ds = (uint32_t)(Pc + __mul24(n, Dk) - sdot(krb, ky));
                uint32_t vv[3];
                bool dec = owned;
    #pragma unroll
                for (int j = 0; j < 3; j++) {
                    const int Dt = T2[j] - odot(trb[j], tg2[j]);
                    const int f = Dt - Dk;
                    const bool A = f - NAx[j * kMaxK + k] >= 0;  // t_j never strictly closer than c_k
                    const bool B = f + NBx[j * kMaxK + k] <= 0;  // t_j always at least as close
                    dec = dec & (A | B);
                    vv[j] = A ? ds : (uint32_t)(Pc + __mul24(n, Dt) - sdot(trb[j], tg2[j]));
                }
                v0 = vv[0];
                v1 = vv[1];
                v2 = vv[2];
                fail = !dec;
            };
            auto cube_vals = [&](const CubeEnt &e, uint32_t &v0, uint32_t &v1, uint32_t &v2,
                                 bool &fail) __attribute__((always_inline)) {
                const CubeGeo g = cube_geo(e);
                box_vals(g.ox, g.oy, g.oz, g.n, g.sx, g.sy, g.sz, g.s2, Mkk, NA, NB, 3, 3, 3, v0, v1, v2, fail);
            };
            // undecided cubes among the lanes of `fm`: their colours (enumerated from the
            // occupancy mask) packed densely into the lanes, summed 64 at a time
            auto push_cubes = [&](unsigned long long fm, const CubeEnt &e) __attribute__((always_inline)) {
                const uint32_t okey = cube_origin_key(e.id);  // read back per cube below
                const uint32_t mlo = (uint32_t)e.mask, mhi = (uint32_t)(e.mask >> 32);
                while (fm) {
    #pragma unroll
                    for (int u = 0; u < LLFE_KM_UNROLL; u++) {
                        if (u > 0 && !fm) break;
                        const int src = __builtin_ctzll(fm);
                        fm = clear_bit(fm, src);
                        const unsigned long long m =
                            ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(mhi, src) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane(mlo, src);
                        const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        stg[lane_sel(m, ((uint32_t)head + r) & (kStage - 1), kStage + lane)] =
                            (uint32_t)__builtin_amdgcn_readlane(okey, src) | loff;
                        head += __popcll(m);
                    }
                    while (head - tail >= 64) sum_stage(64);
                }
            };
            auto next_part = [&](int Pseg) __attribute__((always_inline)) {
                if (Pseg != Pcur) {
                    if (Pcur >= 0) {
                        flush_pk();
                        const unsigned long long a0 = wave_sum(acc0), a1 = wave_sum(acc1), a2 = wave_sum(acc2);
                        if (lane == 0) {
                            atomicAdd(&sm.psum[0][Pcur], a0);
                            atomicAdd(&sm.psum[1][Pcur], a1);
                            atomicAdd(&sm.psum[2][Pcur], a2);
                        }
                    }
                    acc0 = acc1 = acc2 = 0;
                    Pcur = Pseg;
                }
            };
            // Cells pay off on large cube tables (photo-like images: k-means++ 0.99 -> 0.86 ms
            // per attempt, r4b); on small ones (ui: 3k cubes) the extra level cost more than it
            // saved (0.18 -> 0.24 ms), so the choice is per image (uniform).
            if (C >= kCellMinCubes) {
                // cells first: a decided cell adds its closed forms; the cubes of the undecided
                // cells of a chunk (per partition) are listed in the wave's LDS list and go through
                // the cube path above, 64 at a time
                const int *MKc = sm.margc, *NAc = sm.margc + kMaxK * kMaxK, *NBc = sm.margc + kMaxK * kMaxK + 3 * kMaxK;
                int *ql = sm.cq[wid];
                auto mrank = [&](unsigned long long m) {
                    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                };
                auto cell_vals = [&](const CellEnt &e, uint32_t &v0, uint32_t &v1, uint32_t &v2,
                                     bool &fail) __attribute__((always_inline)) {
                    box_vals((int)((e.id >> 10) & 63u) * 4, (int)((e.id >> 5) & 31u) * 8, (int)(e.id & 31u) * 8,
                             (int)((e.id >> 18) & 511u), (int)(e.sums & 1023u), (int)((e.sums >> 10) & 2047u),
                             (int)(e.sums >> 21), (int)e.s2, MKc, NAc, NBc, 3, 7, 7, v0, v1, v2, fail);
                };
                // the failing cells among the lanes of cf (one partition): their cubes, 64 at a time
                auto cell_cubes = [&](const CellEnt &e, const bool cf) __attribute__((always_inline)) {
                    const uint32_t nc1 = (e.id >> 16) & 3u;
                    const unsigned long long F = __ballot(cf), B0 = __ballot(cf && (nc1 & 1u)),
                                             B1 = __ballot(cf && (nc1 & 2u));
                    if (F) {
                        const uint32_t pre = mrank(F) + mrank(B0) + 2u * mrank(B1);
                        const int total = __popcll(F) + __popcll(B0) + 2 * __popcll(B1);
                        if (cf) {
    #pragma unroll
                            for (uint32_t jj = 0; jj < 4; jj++)
                                if (jj <= nc1) ql[pre + jj] = (int)(e.first + jj);
                        }
                        __builtin_amdgcn_wave_barrier();
                        for (int b = 0; b < total; b += 64) {
                            const bool cv = b + lane < total;
                            CubeEnt ce;
                            ce.mask = 0;
                            ce.id = 0;
                            ce.sums = 0;
                            if (cv) ce = ctab[ql[b + lane]];
                            uint32_t c0 = 0, c1 = 0, c2 = 0;
                            bool cfail = false;
                            if (cv) cube_vals(ce, c0, c1, c2, cfail);
                            if (cv && !cfail) {
                                acc0 += c0;
                                acc1 += c1;
                                acc2 += c2;
                            }
                            const unsigned long long fm = __ballot(cv && cfail);
                            if (fm) push_cubes(fm, ce);
                        }
                        __builtin_amdgcn_wave_barrier();  // (the list is rewritten next)
                    }
                };
                // (round 6) the first round (KK = 0: the sums of d(., c0), every box decided) walks
                // the super-cells; the later rounds only with LLFE_KM_PP_SUPS (measured slower)
                if (stab && (LLFE_KM_PP_SUPS || KK <= LLFE_KM_PP_SUPS_KK)) {
                    // super-cells first, the same closed forms with extents (3, 15, 15); the
                    // cells of the undecided ones (one partition at a time) are listed in the wave's
                    // cell list (sm.cs) and go through the cell path, 64 at a time
                    const int *MKs = sm.margs, *NAs = sm.margs + kMaxK * kMaxK, *NBs = sm.margs + kMaxK * kMaxK + 3 * kMaxK;
                    int *qs = sm.cs[wid];
                    int run = __builtin_amdgcn_readfirstlane(grab());  // the current run's first super-cell
                    int base = run;
                    int ahead = grab();
                    SupEnt en{0u, 0u, 0u, 0u};
                    if (base + lane < S) en = stab[base + lane];
                    while (base < S) {
                        const bool valid = base + lane < S;
                        const SupEnt e = en;
                        int nb = base + 64;
                        if (nb >= run + kRun || nb >= S) {  // (uniform) next run
                            run = __builtin_amdgcn_readfirstlane(ahead);
                            nb = run;
                            if (nb < S) ahead = grab();
                        }
                        if (nb + lane < S) en = stab[nb + lane];
                        const int P = valid ? (int)((e.id >> 8) & 63u) : kParts;
                        uint32_t v0 = 0, v1 = 0, v2 = 0;
                        bool fail = false;
                        if (valid)
                            box_vals((int)((e.id >> 8) & 63u) * 4, (int)((e.id >> 4) & 15u) * 16, (int)(e.id & 15u) * 16,
                                     (int)((e.id >> 18) & 2047u), (int)(e.srg & 4095u), (int)(e.srg >> 12),
                                     (int)(e.sb & 16383u), (int)((e.sb >> 14) | (((e.id >> 29) & 1u) << 18)), MKs, NAs,
                                     NBs, 3, 15, 15, v0, v1, v2, fail);
                        // lanes hold ascending super-cell ids: visit the batch's partitions in order
                        int Pseg = __shfl(P, 0);
                        for (;;) {
                            next_part(Pseg);
                            const bool mine = P == Pseg;
                            if (mine && !fail) {
                                acc0 += v0;
                                acc1 += v1;
                                acc2 += v2;
                            }
                            const bool sf = mine && fail;
                            const uint32_t c0 = (e.id >> 14) & 3u, ns1 = c0 + ((e.id >> 16) & 3u) - 1u;
                            const unsigned long long F = __ballot(sf), B0 = __ballot(sf && (ns1 & 1u)),
                                                     B1 = __ballot(sf && (ns1 & 2u));
                            if (F) {
                                const uint32_t pre = mrank(F) + mrank(B0) + 2u * mrank(B1);
                                const int total = __popcll(F) + __popcll(B0) + 2 * __popcll(B1);
                                if (sf) {
    #pragma unroll
                                    for (uint32_t jj = 0; jj < 4; jj++)
                                        if (jj <= ns1)
                                            qs[pre + jj] = (int)(jj < c0 ? (e.first & 0xFFFFu) + jj : (e.first >> 16) + jj - c0);
                                }
                                __builtin_amdgcn_wave_barrier();
                                for (int b = 0; b < total; b += 64) {
                                    const bool cv = b + lane < total;
                                    CellEnt ce{0u, 0u, 0u, 0u};
                                    if (cv) ce = ltab[qs[b + lane]];
                                    uint32_t c0v = 0, c1v = 0, c2v = 0;
                                    bool cfail = false;
                                    if (cv) cell_vals(ce, c0v, c1v, c2v, cfail);
                                    if (cv && !cfail) {
                                        acc0 += c0v;
                                        acc1 += c1v;
                                        acc2 += c2v;
                                    }
                                    cell_cubes(ce, cv && cfail);
                                }
                                __builtin_amdgcn_wave_barrier();  // (the list is rewritten next)
                            }
                            const unsigned long long rest = __ballot(P > Pseg && P < kParts);
                            if (!rest) break;
                            Pseg = __shfl(P, (int)__builtin_ctzll(rest));
                        }
                        base = nb;
                    }
                } else
                {
                int run = __builtin_amdgcn_readfirstlane(grab());  // the current run's first cell
                int base = run;
                int ahead = grab();
                CellEnt en{0u, 0u, 0u, 0u};
                if (base + lane < L) en = ltab[base + lane];
                while (base < L) {
                    const bool valid = base + lane < L;
                    const CellEnt e = en;
                    int nb = base + 64;
                    if (nb >= run + kRun || nb >= L) {  // (uniform) next run
                        run = __builtin_amdgcn_readfirstlane(ahead);
                        nb = run;
                        if (nb < L) ahead = grab();
                    }
                    if (nb + lane < L) en = ltab[nb + lane];
                    const int P = valid ? (int)((e.id >> 10) & 63u) : kParts;
                    uint32_t v0 = 0, v1 = 0, v2 = 0;
                    bool fail = false;
                    if (valid) cell_vals(e, v0, v1, v2, fail);
                    // lanes hold ascending cell ids: visit the batch's partitions in order
                    int Pseg = __shfl(P, 0);
                    for (;;) {
                        next_part(Pseg);
                        const bool mine = P == Pseg;
                        if (mine && !fail) {
                            acc0 += v0;
                            acc1 += v1;
                            acc2 += v2;
                        }
                        cell_cubes(e, mine && fail);
                        const unsigned long long rest = __ballot(P > Pseg && P < kParts);
                        if (!rest) break;
                        Pseg = __shfl(P, (int)__builtin_ctzll(rest));
                    }
                    base = nb;
                }
                }
            } else {
                int run = __builtin_amdgcn_readfirstlane(grab());  // the current run's first cube
                int base = run;
                int ahead = grab();
                CubeEnt en;
                en.mask = 0;
                en.id = 0;
                en.sums = 0;
                if (base + lane < C) en = ctab[base + lane];
                while (base < C) {
                    const bool valid = base + lane < C;
                    const CubeEnt e = en;
                    int nb = base + 64;
                    if (nb >= run + kRun || nb >= C) {  // (uniform) next run
                        run = __builtin_amdgcn_readfirstlane(ahead);
                        nb = run;
                        if (nb < C) ahead = grab();
                    }
                    if (nb + lane < C) en = ctab[nb + lane];
                    const int P = valid ? (int)((e.id >> 12) & 63u) : kParts;
                    uint32_t v0 = 0, v1 = 0, v2 = 0;
                    bool fail = false;
                    if (valid) cube_vals(e, v0, v1, v2, fail);
                    // lanes hold ascending cube ids: visit the batch's partitions in order
                    int Pseg = __shfl(P, 0);
                    for (;;) {
                        next_part(Pseg);
                        const bool mine = P == Pseg;
                        if (mine && !fail) {
                            acc0 += v0;
                            acc1 += v1;
                            acc2 += v2;
                        }
                        const unsigned long long fm = __ballot(mine && fail);
                        if (fm) push_cubes(fm, e);
                        const unsigned long long rest = __ballot(P > Pseg && P < kParts);
                        if (!rest) break;
                        Pseg = __shfl(P, (int)__builtin_ctzll(rest));
                    }
                    base = nb;
            }
            }
            if (Pcur >= 0) {
                flush_pk();
                const unsigned long long a0 = wave_sum(acc0), a1 = wave_sum(acc1), a2 = wave_sum(acc2);
                if (lane == 0) {
                    atomicAdd(&sm.psum[0][Pcur], a0);
                    atomicAdd(&sm.psum[1][Pcur], a1);
                    atomicAdd(&sm.psum[2][Pcur], a2);
                }
            }
            if (lane == 0 && fails) atomicAdd(&sm.fail_pts, fails);
        };
        switch (kk) {
            case 0: sweep(std::integral_constant<int, 0>{}); break;
            case 1: sweep(std::integral_constant<int, 1>{}); break;
            case 2: sweep(std::integral_constant<int, 2>{}); break;
            case 3: sweep(std::integral_constant<int, 3>{}); break;
            default: sweep(std::integral_constant<int, kMaxK - 1>{}); break;
        }
        __syncthreads();
        if (wid == 0) {
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const unsigned long long s = wave_sum(sm.psum[j][lane]);
                if (lane == 0) sm.S[j] = s;
            }
        }
        __syncthreads();
        int best = 0;
        if (kk > 0) {
            double bs = 1.7976931348623157e308;
            for (int j = 0; j < 3; j++)
                if ((double)sm.S[j] < bs) {
                    bs = (double)sm.S[j];
                    best = j;
                }
        }
        sum0 = sm.S[best];
        if (tid < kParts) sm.pD[tid] = sm.psum[best][tid];
        if (tid == 0 && kk > 0) {
            sm.icc[kk][0] = best == 0 ? tx[0] : (best == 1 ? tx[1] : tx[2]);
            sm.icc[kk][1] = best == 0 ? ty[0] : (best == 1 ? ty[1] : ty[2]);
            sm.icc[kk][2] = best == 0 ? tz[0] : (best == 1 ? tz[1] : tz[2]);
        }
    }
    qacc = wave_sum(qacc);
    if (lane == 0) atomicAdd(&sm.qtot, qacc);
    __syncthreads();
    if (tid < kMaxK * 3) {
        const int k = tid / 3, j = tid % 3;
        sm.cc[k][j] = k < K ? (float)sm.icc[k][j] : kFar;
    }
    if (tid == 0) {
        // K passes over the cube table + colours read one by one (undecided cubes and
        // the partition scans)
        bytes += 16ull * (unsigned long long)C * (unsigned long long)K + 4ull * sm.sel_pts;
        pp_pts = (uint32_t)sm.fail_pts;
        pp_sel = (uint32_t)sm.sel_pts;
        sm.fail_pts = 0;
    }
    __syncthreads();
}

#ifndef LLFE_KM_MINW
#define LLFE_KM_MINW 4
#endif
// k-means attempts, one workgroup per (image, attempt) task; tasks are numbered in LPT
// order (task t = attempt t % 10 of image order[t / 10]).  kPhase: 3 = k-means++ and Lloyd
// (the plain path, one launch); 1 = k-means++ only (the cube path's first launch: the
// chosen centres, Sum |p|^2 and the k-means++ counters go to the attempt record); 2 =
// Lloyd only (the cube path's second launch, starting from that record).  kQueue: one
// workgroup per resident slot takes tasks from the global counter `queue` until they run
// out (else task = blockIdx.x).  kCubes: the cube-table path (the batch pipeline);
// !kCubes: plain sweeps over caller-supplied keys (llfe_kmeans).  Separate instantiations
// keep the plain path's register-heavy prefetch out of the hot kernels.  (The body stays
// in the kernel: as an inlined device function the Lloyd sweep lost its register budget
// and spilled 20 VGPRs.)
#ifndef LLFE_KM_HIDE
#define LLFE_KM_HIDE 0  // Lloyd: label staged colours between a list gather's issue and its use
                        // (bit-identical, measured no faster: 14.54-14.59 vs 14.56-14.62 ms)
#endif
#ifndef LLFE_KM_XCD
#define LLFE_KM_XCD 0  // measured slower: 14.45-14.48 -> 14.61-14.63 ms pipelined
#endif
// XCD-aware task order (round 6 experiment): workgroup b runs on XCD b mod 8 (in-order dispatch), and
// the ten attempts of an image read the same cube / cell / super-cell tables and keys, so the
// attempts of image slot i (LPT order) all go to XCD i mod 8 -- its r-th workgroup takes
// attempt r mod 10 of its (r / 10)-th image -- and share that XCD's L2 instead of pulling the
// tables into all eight.  The tasks of the last n mod 8 images keep their places.
__device__ __forceinline__ int xcd_task(int b, int n_tasks) {
    constexpr int X = 8;
    const int t8 = n_tasks / (X * kAttempts) * (X * kAttempts);
    if (!LLFE_KM_XCD || b >= t8) return b;
    const int x = b % X, r = b / X;
    return (x + X * (r / kAttempts)) * kAttempts + r % kAttempts;
}

template <bool kCubes, int kPhase, bool kQueue>
__global__ __launch_bounds__(KT, LLFE_KM_MINW) void k_kmeans(const uint32_t *__restrict__ keys, long long key_stride,
                                                   const long long *__restrict__ n_unique, int n_colors,
                                                   unsigned long long seed, ImgIndex index,
                                                   const int *__restrict__ order, int n_tasks,
                                                   int *__restrict__ queue, uint32_t *__restrict__ scratch,
                                                   long long scratch_stride, KmeansAttemptOut *__restrict__ out,
                                                   const KmeansCubes cubes) {
    static_assert(kPhase == 3 || kCubes, "the plain path runs both phases in one workgroup");
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    KmSmem &sm = *reinterpret_cast<KmSmem *>(smem_raw);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int task = kQueue ? (int)blockIdx.x : xcd_task((int)blockIdx.x, n_tasks);
    if (kQueue) {
        if (tid == 0) sm.task = atomicAdd(queue, 1);
        __syncthreads();
        task = sm.task;
        __syncthreads();
    }
    while (task < n_tasks) {  // (every workgroup of a queue launch leaves once the counter passes n_tasks)
    {
    const int img = order[task / kAttempts];
    const int att = task % kAttempts;
    const int N = (int)n_unique[img];
    const int K = min(n_colors, N);
    KmeansAttemptOut *o = out + (size_t)img * kAttempts + att;
    if (kPhase == 1 && K <= 1) goto next_task;  // (no k-means: the Lloyd launch writes the record)
    if (tid == 0) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const uint64_t t = wall_clock64();
        if (kPhase & 1) {
            o->t_start = t;
            o->hw_id = hw;
            o->xcc_id = xcc;
        }
        if (kPhase & 2) {
            o->t_lstart = t;
            o->hw_id2 = hw;
            o->xcc_id2 = xcc;
        }
    }
    if (K <= 1) {
        if (tid == 0) {
            o->compactness = 0.0;
            o->iters = 0;
            o->bytes = 0;
            o->pp_pts = 0;
            o->n_cubes = 0;
            o->t_sel = 0;
            o->ll_pts = 0;
            o->t_sw = 0;
            o->drift_hist = 0;
            o->pad = 0;
            o->t_end = wall_clock64();
            if (kPhase == 2) {  // (the k-means++ launch skipped the attempt)
                o->t_start = o->t_pp = o->t_lstart;
                o->hw_id = o->hw_id2;
                o->xcc_id = o->xcc_id2;
            }
        }
        goto next_task;
    }
    const uint32_t *pts = keys + (size_t)img * key_stride;
    const int M = (N + STEP - 1) / STEP;         // steps
    const int Mw = (M + KW - 1) / KW;            // steps per wave
    const int sb = min(M, wid * Mw), se = min(M, sb + Mw);
    // steps whose 256 points are all valid end at se_full; [se_full, se) is at most the
    // one partial step, and empty for waves whose range lies past it (sb == se == M)
    const int se_full = max(sb, min(se, N / STEP));
    uint32_t *ss = scratch + ((size_t)img * kAttempts + att) * (size_t)scratch_stride;
    // cube-pruned Lloyd sweeps (when the cube table was built): waves own contiguous
    // ranges of cubes
    constexpr bool use_cubes = kCubes;
    const int C = use_cubes ? cubes.n_cubes[img] : 0;
    const CubeEnt *ctab = use_cubes ? cubes.cubes + (size_t)img * cubes.cube_stride : nullptr;
    uint32_t pp_pts = 0, pp_sel = 0;
    uint64_t t_sel = 0, ll_pts = 0;
    // plain path: k-means++ + compactness passes; the cube path adds what its passes read
    unsigned long long bytes = use_cubes ? 0ull : 4ull * (unsigned long long)N * (unsigned long long)(K + 1);
    if (tid == 0) sm.fail_pts = 0;
#define SSLOT(slot) (ss + (size_t)(slot) * (size_t)M)

    if (kPhase & 1) {
    uint64_t rng = splitmix64(seed + (unsigned long long)index.at(img));
    if (rng == 0) rng = 0xFFFFFFFFull;  // cv::RNG(0) takes the default state
    for (int q = 0, skip = att * (1 + 6 * (K - 1)); q < skip; q++) cvrng_next(rng);

    // ------------------------------------------------ k-means++ (generateCentersPP)
    if (use_cubes) {
        pp_cubes(sm, pts, N, K, rng, ctab, C, cubes.cells + (size_t)img * cubes.cell_stride, cubes.n_cells[img],
                 cubes.sups ? cubes.sups + (size_t)img * cubes.sup_stride : nullptr, cubes.sups ? cubes.n_sups[img] : 0,
                 cubes.part_uq + (size_t)img * kParts, cubes.part_hist ? cubes.part_hist + (size_t)img * kParts : nullptr,
                 bytes, pp_pts, pp_sel, t_sel);
    } else {
    int cur = 0;
    {
        const uint32_t c0 = cvrng_next(rng) % (uint32_t)N;
        const P3 q0 = unpack(pts[c0]);
        if (tid == 0) {
            sm.cc[0][0] = q0.x; sm.cc[0][1] = q0.y; sm.cc[0][2] = q0.z;
        }
        const float cx = uni(q0.x), cy = uni(q0.y), cz = uni(q0.z);
        unsigned long long wt = 0;
        for (int s = sb; s < se; s++) {
            const int i0 = s * STEP + lane * 4;
            uint32_t ls = 0;
            if (s < se_full) {
                uint4 v = *(const uint4 *)(pts + i0);
                uint32_t kq[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    P3 p = unpack(kq[j]);
                    ls += (uint32_t)d2(p.x, p.y, p.z, cx, cy, cz);
                }
            } else {
                for (int j = 0; j < 4; j++)
                    if (i0 + j < N) {
                        P3 p = unpack(pts[i0 + j]);
                        ls += (uint32_t)d2(p.x, p.y, p.z, cx, cy, cz);
                    }
            }
            uint32_t st = wave_sum(ls);
            if (lane == 0) SSLOT(0)[s] = st;
            wt += st;
        }
        if (lane == 0) sm.wtot[wid][0] = wt;
    }
    __syncthreads();
    unsigned long long sum0 = 0;
    for (int w = 0; w < KW; w++) sum0 += sm.wtot[w][0];
    __syncthreads();

    for (int kk = 1; kk < K; kk++) {
        double p[3];
#pragma unroll
        for (int j = 0; j < 3; j++) p[j] = cvrng_double(rng) * (double)sum0;
        // chosen centres so far (uniform)
        Cent ch;
#pragma unroll
        for (int m = 0; m < kMaxK; m++) {
            bool u = m < kk;
            ch.x[m] = u ? uni(sm.cc[m][0]) : kFar;
            ch.y[m] = u ? uni(sm.cc[m][1]) : kFar;
            ch.z[m] = u ? uni(sm.cc[m][2]) : kFar;
        }
        // ---- locate the step holding prefix(D) >= p_j: thread-contiguous step ranges
        {
            const int q = (M + KT - 1) / KT;
            const int t0 = min(M, tid * q), t1 = min(M, t0 + q);
            unsigned long long R = 0;
            const uint32_t *scur = SSLOT(cur);
            for (int s = t0; s < t1; s++) R += scur[s];
            unsigned long long x = R;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                unsigned long long y = __shfl_up(x, off);
                if (lane >= off) x += y;
            }
            if (lane == 63) sm.scan_w[wid] = x;
            if (tid < 3) {
                sm.found_step[tid] = -1;
                sm.ci[tid] = -1;
            }
            __syncthreads();
            unsigned long long pre = 0;
            for (int w = 0; w < wid; w++) pre += sm.scan_w[w];
            const unsigned long long excl = pre + x - R;
#pragma unroll
            for (int j = 0; j < 3; j++) {
                if (p[j] > 0 && (double)excl < p[j] && p[j] <= (double)(excl + R)) {
                    unsigned long long e = excl;
                    for (int s = t0; s < t1; s++) {
                        unsigned long long v = scur[s];
                        if ((double)(e + v) >= p[j]) {
                            sm.found_step[j] = s;
                            sm.found_excl[j] = e;
                            break;
                        }
                        e += v;
                    }
                }
            }
            __syncthreads();
        }
        // ---- waves 0..2 resolve the point inside the found step
        if (wid < 3) {
            const int j = wid;
            const double pj = j == 0 ? p[0] : (j == 1 ? p[1] : p[2]);
            if (!(pj > 0)) {
                if (lane == 0) sm.ci[j] = 0;
            } else if (sm.found_step[j] < 0) {
                if (lane == 0) sm.ci[j] = N - 1;
            } else {
                const int s = sm.found_step[j];
                const int i0 = s * STEP + lane * 4;
                uint32_t dv[4], lsum = 0;
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    dv[jj] = 0;
                    if (i0 + jj < N) {
                        P3 pp = unpack(pts[i0 + jj]);
                        float d = d2(pp.x, pp.y, pp.z, ch.x[0], ch.y[0], ch.z[0]);
#pragma unroll
                        for (int m = 1; m < kMaxK; m++)
                            if (m < kk) d = fminf(d, d2(pp.x, pp.y, pp.z, ch.x[m], ch.y[m], ch.z[m]));
                        dv[jj] = (uint32_t)d;
                    }
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
                    if (hit < 0 && (double)e >= pj) hit = jj;
                }
                unsigned long long bal = __ballot(hit >= 0);
                int first = (int)__builtin_ctzll(bal);
                int hitj = __shfl(hit, first);
                if (lane == 0) sm.ci[j] = min(s * STEP + first * 4 + hitj, N - 1);
            }
        }
        __syncthreads();
        Cent tc;  // trial centres in x[0..2]
#pragma unroll
        for (int j = 0; j < 3; j++) {
            P3 pp = unpack(pts[sm.ci[j]]);
            tc.x[j] = uni(pp.x);
            tc.y[j] = uni(pp.y);
            tc.z[j] = uni(pp.z);
        }
        // ---- trial pass: T_j(i) = min(D(i), d(i, ci_j)); step sums into three free slots
        // the three slots other than `cur`, in increasing order
        const int sl0 = cur == 0 ? 1 : 0, sl1 = cur <= 1 ? 2 : 1, sl2 = cur <= 2 ? 3 : 2;
        uint32_t *o0 = SSLOT(sl0), *o1 = SSLOT(sl1), *o2 = SSLOT(sl2);
        unsigned long long wt0 = 0, wt1 = 0, wt2 = 0;
        for (int s = sb; s < se; s++) {
            const int i0 = s * STEP + lane * 4;
            uint32_t kq[4];
            int cnt = 4;
            if (s < se_full) {
                uint4 v = *(const uint4 *)(pts + i0);
                kq[0] = v.x; kq[1] = v.y; kq[2] = v.z; kq[3] = v.w;
            } else {
                cnt = max(0, min(4, N - i0));
                for (int jj = 0; jj < 4; jj++) kq[jj] = jj < cnt ? pts[i0 + jj] : 0u;
            }
            uint32_t l0 = 0, l1 = 0, l2 = 0;
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                P3 pp = unpack(kq[jj]);
                float d = d2(pp.x, pp.y, pp.z, ch.x[0], ch.y[0], ch.z[0]);
#pragma unroll
                for (int m = 1; m < kMaxK; m++)
                    if (m < kk) d = fminf(d, d2(pp.x, pp.y, pp.z, ch.x[m], ch.y[m], ch.z[m]));
                uint32_t v0 = (uint32_t)fminf(d, d2(pp.x, pp.y, pp.z, tc.x[0], tc.y[0], tc.z[0]));
                uint32_t v1 = (uint32_t)fminf(d, d2(pp.x, pp.y, pp.z, tc.x[1], tc.y[1], tc.z[1]));
                uint32_t v2 = (uint32_t)fminf(d, d2(pp.x, pp.y, pp.z, tc.x[2], tc.y[2], tc.z[2]));
                bool ok = jj < cnt;
                l0 += ok ? v0 : 0u;
                l1 += ok ? v1 : 0u;
                l2 += ok ? v2 : 0u;
            }
            uint32_t a0 = wave_sum(l0), a1 = wave_sum(l1), a2 = wave_sum(l2);
            if (lane == 0) {
                o0[s] = a0;
                o1[s] = a1;
                o2[s] = a2;
            }
            wt0 += a0;
            wt1 += a1;
            wt2 += a2;
        }
        if (lane == 0) {
            sm.wtot[wid][0] = wt0;
            sm.wtot[wid][1] = wt1;
            sm.wtot[wid][2] = wt2;
        }
        __syncthreads();
        unsigned long long S[3] = {0, 0, 0};
        for (int w = 0; w < KW; w++)
            for (int j = 0; j < 3; j++) S[j] += sm.wtot[w][j];
        int best = 0;
        double bs = 1.7976931348623157e308;
        for (int j = 0; j < 3; j++)
            if ((double)S[j] < bs) {
                bs = (double)S[j];
                best = j;
            }
        sum0 = S[best];
        cur = best == 0 ? sl0 : (best == 1 ? sl1 : sl2);
        __syncthreads();
        if (tid == 0) {
            sm.cc[kk][0] = tc.x[best];
            sm.cc[kk][1] = tc.y[best];
            sm.cc[kk][2] = tc.z[best];
        }
        __syncthreads();
    }

    }  // k-means++
    if (tid == 0) o->t_pp = wall_clock64();
    // (diagnostics, llfe_kmeans_attempts: the k-means++ centres of the attempt)
    if (tid < kMaxK * 3) (&o->pp_centers[0][0])[tid] = sm.cc[tid / 3][tid % 3];
    }  // kPhase & 1
    if (kPhase == 1) {
        // hand the attempt to the Lloyd launch: chosen centres, Sum |p|^2, counters
        if (tid < kMaxK * 3) (&o->centers[0][0])[(tid / 3) * 3 + tid % 3] = sm.cc[tid / 3][tid % 3];
        if (tid == 0) {
            o->qtot = sm.qtot;
            o->bytes = bytes;
            o->pp_pts = pp_pts;
            o->pad = (int32_t)pp_sel;
            o->t_sel = t_sel;
        }
        goto next_task;
    }
    if (kPhase == 2) {
        if (tid < kMaxK * 3) {
            const int k = tid / 3, j = tid % 3;
            sm.cc[k][j] = k < K ? o->centers[k][j] : kFar;
        }
        if (tid == 0) sm.qtot = o->qtot;
        bytes = o->bytes;
        __syncthreads();
    }
    // ------------------------------------------------ Lloyd iterations
    if (tid < kMaxK * 3) {
        int k = tid / 3, j = tid % 3;
        sm.c[k][j] = k < K ? sm.cc[k][j] : kFar;
    }
    __syncthreads();

    if (tid == 0) sm.next_chunk = 0;
    __syncthreads();
    int iter = 1;
    const double eps2 = 0.2 * 0.2;
    uint64_t t_sw = 0;  // (trace) time in the labelling sweeps
    uint64_t drift_hist = 0;  // (trace)
    for (;;) {
        const uint64_t tsw0 = wall_clock64();
        const CentP c = pack_centres(load_centres(sm.c));
#pragma unroll
        for (int k = 0; k < kMaxK; k++) {
            sm.accA[k][tid] = 0;
            sm.accB[k][tid] = 0;
        }
        // (lane-private slots: no barrier needed between zeroing and accumulation)
        if (use_cubes) {
            // Margin test per 4x4x4 cube, q = its centre, k = argmin d(q, c_k):
            //   d_j(p) - d_k(p) is linear in p, so over the cube it is >= (d_j(q) - d_k(q))
            //   - 3 L1(c_j - c_k); when d_j(q) - d_k(q) > 3 L1(c_j - c_k) + 1 for every
            //   j != k, every colour of the cube is at least 1 closer to c_k than to any
            //   other centre in exact arithmetic, far above the float error of
            //   normL2Sqr (< 0.1 at these magnitudes): OpenCV labels it k.
            // pairwise thresholds T[k][j] = 3 L1(c_j - c_k) + 1 (uniform); -inf where the
            // pair needs no test (j == k, or an unused centre)
            const Cent cu = load_centres(sm.c);
            // cube-centre forms L_j(q) = |c_j|^2 - 2 q.c_j = d_j(q) - |q|^2 (pairs (0,1),
            // (2,3), (4,-)): three packed FMAs per pair instead of the six packed ops of the
            // distances; the tests below only use differences L_a - L_b = d_a - d_b, and the
            // margin's +1 absorbs the float rounding of either form (<= 0.1 at these
            // magnitudes).  Unused centres get L = +inf (never the minimum, always farther).
            f2 lw_x[3], lw_y[3], lw_z[3], lc2[3];
#pragma unroll
            for (int j = 0; j < 3; j++) {
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int m = 2 * j + h;
                    const bool used = m < K;
                    const float cx = m < kMaxK ? cu.x[m] : 0.f, cy = m < kMaxK ? cu.y[m] : 0.f,
                                cz = m < kMaxK ? cu.z[m] : 0.f;
                    const float wx = used ? -2.f * cx : 0.f, wy = used ? -2.f * cy : 0.f, wz = used ? -2.f * cz : 0.f;
                    const float c2 = used ? cx * cx + cy * cy + cz * cz : __builtin_inff();
                    if (h == 0) {
                        lw_x[j].x = wx, lw_y[j].x = wy, lw_z[j].x = wz, lc2[j].x = c2;
                    } else {
                        lw_x[j].y = wx, lw_y[j].y = wy, lw_z[j].y = wz, lc2[j].y = c2;
                    }
                }
            }
            // Pair thresholds T[k][j] in LDS, read per lane for the lane's owner k: a box
            // passes when d_j(q) - d_k(q) > T[k][j] for every j (T[k][k] = -inf), five
            // compares against the owner's row instead of the ten centre pairs' compares
            // combined by the owner masks.  Cube: 3 L1(c_j - c_k) + 1; 4 x 8 x 8 cell:
            // 3 |dx| + 7 (|dy| + |dz|) + 1; 4 x 16 x 16 super-cell: 3 |dx| + 15 (|dy| + |dz|) + 1
            // (twice the half extents).
            if (tid < 3 * kMaxK * kMaxK) {
                const int kind = tid / (kMaxK * kMaxK), k = (tid / kMaxK) % kMaxK, j = tid % kMaxK;
                const float dx = fabsf(sm.c[j][0] - sm.c[k][0]), dy = fabsf(sm.c[j][1] - sm.c[k][1]),
                            dz = fabsf(sm.c[j][2] - sm.c[k][2]);
                sm.thrL[kind][k * kMaxK + j] = (j == k || j >= K || k >= K) ? -__builtin_inff()
                                               : kind == 0 ? 3.f * (dx + dy + dz) + 1.f
                                               : kind == 1 ? 3.f * dx + 7.f * (dy + dz) + 1.f
                                                           : 3.f * dx + 15.f * (dy + dz) + 1.f;
            }
            __syncthreads();
            unsigned long long fails = 0;
            // boundary colours: each undecided cube's lanes (lane = mask bit) store their
            // colour into this wave's LDS ring at head + rank (a dummy slot per lane when
            // the bit is clear); 64 staged colours at a time are read back densely and
            // labelled.  Stores are fire-and-forget, so cubes do not serialise on LDS
            // latency the way a register permute would.
            uint32_t *stg = sm.stage[wid];
            const uint32_t loff = lane_offset(lane);
            int head = 0, tail = 0;  // wave-uniform ring counters
            auto label_stage = [&](int count) {
                __builtin_amdgcn_wave_barrier();
                if (lane < count) {
                    const uint32_t kq = stg[(tail + lane) & (kStage - 1)];
                    const int l = label5p(kq, c);
                    atomicAdd(&sm.accA[l][tid], (unsigned long long)((kq >> 16) & 255u) |
                                                    ((unsigned long long)((kq >> 8) & 255u) << 32));
                    atomicAdd(&sm.accB[l][tid], (unsigned long long)(kq & 255u) | (1ull << 32));
                }
                tail += count;
            };
            // two full batches at once: the two LDS reads and label chains interleave
            auto label_stage2 = [&]() {
                __builtin_amdgcn_wave_barrier();
                const uint32_t k0 = stg[(tail + lane) & (kStage - 1)], k1 = stg[(tail + 64 + lane) & (kStage - 1)];
                const int l0 = label5p(k0, c), l1 = label5p(k1, c);
                atomicAdd(&sm.accA[l0][tid], (unsigned long long)((k0 >> 16) & 255u) |
                                                 ((unsigned long long)((k0 >> 8) & 255u) << 32));
                atomicAdd(&sm.accB[l0][tid], (unsigned long long)(k0 & 255u) | (1ull << 32));
                atomicAdd(&sm.accA[l1][tid], (unsigned long long)((k1 >> 16) & 255u) |
                                                 ((unsigned long long)((k1 >> 8) & 255u) << 32));
                atomicAdd(&sm.accB[l1][tid], (unsigned long long)(k1 & 255u) | (1ull << 32));
                tail += 128;
            };
#define LABEL_FULL() while (head - tail >= 128) label_stage2()
            // Waves take 64-entry chunks from a shared LDS counter, not fixed ranges: the
            // boundary cubes cluster, and with fixed ranges the other waves idled at the
            // iteration barrier behind the wave that drew the boundary (measured: 94 ->
            // 74 us per photo iteration; round-robin chunks 79).  The counter is read two
            // chunks ahead and the entries one chunk ahead.
            auto grab = [&]() {
                int b = 0;
                if (lane == 0) b = atomicAdd(&sm.next_chunk, 64);
                return b;  // (lane 0's; read with readfirstlane one chunk later)
            };
            auto cube_body = [&](const CubeEnt &e, const bool valid) __attribute__((always_inline)) {
                bool pass = false;
                int k = 0;
                if (valid) {
                    const float qx = (float)((e.id >> 12) & 63u) * 4.f + 1.5f, qy = (float)((e.id >> 6) & 63u) * 4.f + 1.5f,
                                qz = (float)(e.id & 63u) * 4.f + 1.5f;
                    const f2 px = f2{qx, qx}, py = f2{qy, qy}, pz = f2{qz, qz};
                    f2 d[3];
#pragma unroll
                    for (int j = 0; j < 3; j++) {
                        f2 dd = __builtin_elementwise_fma(px, lw_x[j], lc2[j]);
                        dd = __builtin_elementwise_fma(py, lw_y[j], dd);
                        d[j] = __builtin_elementwise_fma(pz, lw_z[j], dd);
                    }
                    const float dv[5] = {d[0].x, d[0].y, d[1].x, d[1].y, d[2].x};
                    const float m1 = fminf(fminf(fminf(dv[0], dv[1]), fminf(dv[2], dv[3])), dv[4]);
                    // k = first minimum; every other centre j must be farther by more than
                    // T[k][j] at q (dv[k] = m1, so dv[j] - m1 = |dv[j] - dv[k]|)
                    k = dv[0] == m1 ? 0 : (dv[1] == m1 ? 1 : (dv[2] == m1 ? 2 : (dv[3] == m1 ? 3 : 4)));
                    const float *tk = &sm.thrL[0][k * kMaxK];
                    pass = (dv[0] - m1 > tk[0]) & (dv[1] - m1 > tk[1]) & (dv[2] - m1 > tk[2]) &
                           (dv[3] - m1 > tk[3]) & (dv[4] - m1 > tk[4]);
                }
                if (pass) {
                    const CubeGeo g = cube_geo(e);
                    atomicAdd(&sm.accA[k][tid], (unsigned long long)(g.n * g.ox + g.sx) |
                                                    ((unsigned long long)(g.n * g.oy + g.sy) << 32));
                    atomicAdd(&sm.accB[k][tid], (unsigned long long)(g.n * g.oz + g.sz) |
                                                    ((unsigned long long)g.n << 32));
                }
                // cubes straddling a boundary: their colours (enumerated from the
                // occupancy mask, no key loads) packed densely into the lanes and
                // labelled 64 at a time
                unsigned long long fm = __ballot(valid && !pass);
                // per lane: the origin key of its cube (read back per failing cube with one
                // readlane instead of rebuilding it in scalar code)
                const uint32_t okey = cube_origin_key(e.id);
                const uint32_t mlo = (uint32_t)e.mask, mhi = (uint32_t)(e.mask >> 32);
                // LLFE_KM_UNROLL failing cubes per trip: independent readlane / mbcnt chains
                // interleave; the ring (kStage) holds <= 127 pending + UNROLL x 64 new colours
                auto push = [&](int src) {
                    const unsigned long long m =
                        ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(mhi, src) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane(mlo, src);
                    const uint32_t k = __builtin_amdgcn_readlane(okey, src);
                    const uint32_t r =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    stg[lane_sel(m, ((uint32_t)head + r) & (kStage - 1), kStage + lane)] = k | loff;
                    head += __popcll(m);
                };
                while (fm) {
#pragma unroll
                    for (int u = 0; u < LLFE_KM_UNROLL; u++) {
                        if (u > 0 && !fm) break;
                        const int src = __builtin_ctzll(fm);
                        fm = clear_bit(fm, src);
                        push(src);
                    }
                    LABEL_FULL();
                }
            };
            // Cells first (CellEnt: the up to four cubes of a 4 x 8 x 8 box, consecutive in the
            // cube table): a cell whose box passes the margin test at its centre
            // q = origin + (1.5, 3.5, 3.5), with the thresholds weighted by the half extents,
            // thrC[k][j] = 2 (1.5 |dx| + 3.5 |dy| + 3.5 |dz|) + 1, is added from its sums (the
            // same argument as for a cube: every colour of the box is at least 1 closer to
            // c_k); the cubes of the failing cells of a chunk are listed in the wave's LDS
            // list and go through the cube test 64 at a time.
            // (per image, as in k-means++: cells pay off on large cube tables -- a photo's
            // Lloyd iteration 74.5 -> 69.8 us, r4b -- not on a ui image's ~3k cubes)
            if (C >= kCellMinCubes) {
                const int L = cubes.n_cells[img];
                const CellEnt *ltab = cubes.cells + (size_t)img * cubes.cell_stride;
                int *ql = sm.cq[wid];
                auto mrank = [&](unsigned long long m) {
                    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                };
                // the margin test of a box with origin-derived centre (qx, qy, qz) against the
                // thresholds of `kind`: the owner k (first minimum at q) and pass
                auto box_test = [&](float qx, float qy, float qz, int kind, int &k) __attribute__((always_inline)) {
                    const f2 px = f2{qx, qx}, py = f2{qy, qy}, pz = f2{qz, qz};
                    f2 d[3];
#pragma unroll
                    for (int j = 0; j < 3; j++) {
                        f2 dd = __builtin_elementwise_fma(px, lw_x[j], lc2[j]);
                        dd = __builtin_elementwise_fma(py, lw_y[j], dd);
                        d[j] = __builtin_elementwise_fma(pz, lw_z[j], dd);
                    }
                    const float dv[5] = {d[0].x, d[0].y, d[1].x, d[1].y, d[2].x};
                    const float m1 = fminf(fminf(fminf(dv[0], dv[1]), fminf(dv[2], dv[3])), dv[4]);
                    k = dv[0] == m1 ? 0 : (dv[1] == m1 ? 1 : (dv[2] == m1 ? 2 : (dv[3] == m1 ? 3 : 4)));
                    const float *tk = &sm.thrL[kind][k * kMaxK];
                    return (dv[0] - m1 > tk[0]) & (dv[1] - m1 > tk[1]) & (dv[2] - m1 > tk[2]) &
                           (dv[3] - m1 > tk[3]) & (dv[4] - m1 > tk[4]);
                };
                // one 64-lane batch of cells: passing cells add their sums, the failing cells'
                // cubes go to list slots [pre_c, pre_c + nc), pre_c = sum of nc over the failing
                // lanes below (three ballots: the count and its two low bits), 64 at a time
                // through the cube test
                auto cell_body = [&](const CellEnt &e, const bool lvalid) __attribute__((always_inline)) {
                    bool pass = false;
                    int k = 0;
                    if (lvalid)
                        pass = box_test((float)((e.id >> 10) & 63u) * 4.f + 1.5f, (float)((e.id >> 5) & 31u) * 8.f + 3.5f,
                                        (float)(e.id & 31u) * 8.f + 3.5f, 1, k);
                    if (pass) {
                        // colour sums = n origin + sum u (origin (4R, 8G2, 8B2))
                        const uint32_t n = (e.id >> 18) & 511u;
                        const uint32_t ox = ((e.id >> 10) & 63u) * 4u, oy = ((e.id >> 5) & 31u) * 8u, oz = (e.id & 31u) * 8u;
                        atomicAdd(&sm.accA[k][tid], (unsigned long long)(n * ox + (e.sums & 1023u)) |
                                                        ((unsigned long long)(n * oy + ((e.sums >> 10) & 2047u)) << 32));
                        atomicAdd(&sm.accB[k][tid], (unsigned long long)(n * oz + (e.sums >> 21)) |
                                                        ((unsigned long long)n << 32));
                    }
                    const bool cf = lvalid && !pass;
                    const uint32_t nc1 = (e.id >> 16) & 3u;
                    const unsigned long long F = __ballot(cf), B0 = __ballot(cf && (nc1 & 1u)),
                                             B1 = __ballot(cf && (nc1 & 2u));
                    if (F) {
                        const uint32_t pre = mrank(F) + mrank(B0) + 2u * mrank(B1);
                        const int total = __popcll(F) + __popcll(B0) + 2 * __popcll(B1);
                        if (cf) {
#pragma unroll
                            for (uint32_t jj = 0; jj < 4; jj++)
                                if (jj <= nc1) ql[pre + jj] = (int)(e.first + jj);
                        }
                        __builtin_amdgcn_wave_barrier();
                        for (int b = 0; b < total; b += 64) {
                            const bool v = b + lane < total;
                            CubeEnt ce;
                            ce.mask = 0;
                            ce.id = 0;
                            ce.sums = 0;
                            if (v) ce = ctab[ql[b + lane]];
#if LLFE_KM_HIDE
                            // staged boundary colours need no ce: label them while the gather is
                            // in flight (integer sums, any order gives the same totals)
                            while (head - tail >= 64) label_stage(64);
#endif
                            cube_body(ce, v);
                        }
                        __builtin_amdgcn_wave_barrier();  // (the next batch rewrites the list)
                    }
                };
#if LLFE_KM_SUPS
                if (cubes.sups) {
                    // Super-cells first (SupEnt: the up to four cells of a 4 x 16 x 16 box, two
                    // pairs in the cell table), the same test with centre
                    // q = origin + (1.5, 7.5, 7.5); the cells of the failing super-cells of a chunk
                    // are listed in the wave's cell list (sm.cs) and go through cell_body 64 at a time.
                    const int S = cubes.n_sups[img];
                    const SupEnt *stab = cubes.sups + (size_t)img * cubes.sup_stride;
                    int *qs = sm.cs[wid];
                    int base = __builtin_amdgcn_readfirstlane(grab());
                    int ahead = grab();
                    SupEnt sn{0u, 0u, 0u, 0u};
                    if (base + lane < S) sn = stab[base + lane];
                    while (base < S) {
                        const bool svalid = base + lane < S;
                        const SupEnt e = sn;
                        const int nb = __builtin_amdgcn_readfirstlane(ahead);
                        if (nb + lane < S) sn = stab[nb + lane];
                        if (nb < S) ahead = grab();
                        bool pass = false;
                        int k = 0;
                        if (svalid)
                            pass = box_test((float)((e.id >> 8) & 63u) * 4.f + 1.5f, (float)((e.id >> 4) & 15u) * 16.f + 7.5f,
                                            (float)(e.id & 15u) * 16.f + 7.5f, 2, k);
                        if (pass) {
                            const uint32_t n = (e.id >> 18) & 2047u;
                            const uint32_t ox = ((e.id >> 8) & 63u) * 4u, oy = ((e.id >> 4) & 15u) * 16u, oz = (e.id & 15u) * 16u;
                            atomicAdd(&sm.accA[k][tid], (unsigned long long)(n * ox + (e.srg & 4095u)) |
                                                            ((unsigned long long)(n * oy + (e.srg >> 12)) << 32));
                            atomicAdd(&sm.accB[k][tid], (unsigned long long)(n * oz + (e.sb & 16383u)) | ((unsigned long long)n << 32));
                        }
                        const bool sf = svalid && !pass;
                        const uint32_t c0 = (e.id >> 14) & 3u, ns1 = c0 + ((e.id >> 16) & 3u) - 1u;
                        const unsigned long long F = __ballot(sf), B0 = __ballot(sf && (ns1 & 1u)),
                                                 B1 = __ballot(sf && (ns1 & 2u));
                        if (F) {
                            const uint32_t pre = mrank(F) + mrank(B0) + 2u * mrank(B1);
                            const int total = __popcll(F) + __popcll(B0) + 2 * __popcll(B1);
                            if (sf) {
#pragma unroll
                                for (uint32_t jj = 0; jj < 4; jj++)
                                    if (jj <= ns1)
                                        qs[pre + jj] = (int)(jj < c0 ? (e.first & 0xFFFFu) + jj : (e.first >> 16) + jj - c0);
                            }
                            __builtin_amdgcn_wave_barrier();
                            for (int b = 0; b < total; b += 64) {
                                const bool v = b + lane < total;
                                CellEnt ce{0u, 0u, 0u, 0u};
                                if (v) ce = ltab[qs[b + lane]];
#if LLFE_KM_HIDE
                                while (head - tail >= 64) label_stage(64);  // (as above)
#endif
                                cell_body(ce, v);
                            }
                            __builtin_amdgcn_wave_barrier();
                        }
                        base = nb;
                    }
                } else
#endif
                {
                    int base = __builtin_amdgcn_readfirstlane(grab());
                    int ahead = grab();
                    CellEnt ln{0u, 0u, 0u, 0u};
                    if (base + lane < L) ln = ltab[base + lane];
                    while (base < L) {
                        const bool lvalid = base + lane < L;
                        const CellEnt e = ln;
                        const int nb = __builtin_amdgcn_readfirstlane(ahead);
                        if (nb + lane < L) ln = ltab[nb + lane];
                        if (nb < L) ahead = grab();
                        cell_body(e, lvalid);
                        base = nb;
                    }
                }
            } else {
                int base = __builtin_amdgcn_readfirstlane(grab());
                int ahead = grab();
                CubeEnt en;
                en.mask = 0;
                en.id = 0;
                en.sums = 0;
                if (base + lane < C) en = ctab[base + lane];
                while (base < C) {
                    const bool valid = base + lane < C;
                    const CubeEnt e = en;
                    const int nb = __builtin_amdgcn_readfirstlane(ahead);
                    if (nb + lane < C) en = ctab[nb + lane];
                    if (nb < C) ahead = grab();
                    cube_body(e, valid);
                    base = nb;
                }
            }
            while (head - tail >= 64) label_stage(64);
            if (head > tail) label_stage(head - tail);
#undef LABEL_FULL
            fails = (unsigned long long)head;
            if (lane == 0 && fails) atomicAdd(&sm.fail_pts, fails);
        } else {
        // The sweep is load-latency bound: keep the next PF steps' 16-B loads in flight
        // while the current PF steps are labelled.
        {
            uint4 cur[PF], nxt[PF];
#pragma unroll
            for (int d = 0; d < PF; d++) cur[d] = load_step(pts, sb + d, se_full, lane);
            for (int s = sb; s < se_full; s += PF) {
#pragma unroll
                for (int d = 0; d < PF; d++) nxt[d] = load_step(pts, s + PF + d, se_full, lane);
#pragma unroll
                for (int d = 0; d < PF; d++) {
                    if (s + d >= se_full) break;
                    const uint32_t kq[4] = {cur[d].x, cur[d].y, cur[d].z, cur[d].w};
#pragma unroll
                    for (int jj = 0; jj < 4; jj++) {
                        int l = label5p(kq[jj], c);
                        unsigned long long a = (unsigned long long)((kq[jj] >> 16) & 255u) |
                                               ((unsigned long long)((kq[jj] >> 8) & 255u) << 32);
                        unsigned long long b = (unsigned long long)(kq[jj] & 255u) | (1ull << 32);
                        atomicAdd(&sm.accA[l][tid], a);
                        atomicAdd(&sm.accB[l][tid], b);
                    }
                }
#pragma unroll
                for (int d = 0; d < PF; d++) cur[d] = nxt[d];
            }
        }
        for (int s = se_full; s < se; s++) {  // at most one partial step
            const int i0 = s * STEP + lane * 4;
            for (int jj = 0; jj < 4; jj++) {
                if (i0 + jj >= N) break;
                uint32_t kq = pts[i0 + jj];
                int l = label5p(kq, c);
                atomicAdd(&sm.accA[l][tid], (unsigned long long)((kq >> 16) & 255u) |
                                                ((unsigned long long)((kq >> 8) & 255u) << 32));
                atomicAdd(&sm.accB[l][tid], (unsigned long long)(kq & 255u) | (1ull << 32));
            }
        }
        }  // point sweep
        __syncthreads();
        t_sw += wall_clock64() - tsw0;
        if (tid == 0) {
            if (use_cubes) {
                bytes += 16ull * (unsigned long long)C;  // boundary colours come from the masks
                ll_pts += sm.fail_pts;
                sm.fail_pts = 0;
            } else {
                bytes += 4ull * (unsigned long long)N;
            }
        }
        // reduce 20 values (5 clusters x {x, y, z, count}) over the KT lanes: part p of
        // value v sums lanes p, p + 32, p + 64, ... so the 32 threads of a value read 32
        // consecutive 8-byte slots per step (lanes p * 16 .. p * 16 + 15 put 16 threads on
        // two LDS banks); integer sums, so any grouping gives the same totals
        for (int q = tid; q < 640; q += KT) {
            constexpr int LPP = KT / 32;  // lanes per part
            const int v = q >> 5, part = q & 31;
            const int k = v >> 2, comp = v & 3;
            unsigned long long acc = 0;
            const unsigned long long *src = comp < 2 ? sm.accA[k] : sm.accB[k];
#pragma unroll 4
            for (int j = 0; j < LPP; j++) {
                unsigned long long wv = src[part + 32 * j];
                acc += (comp & 1) ? (wv >> 32) : (wv & 0xFFFFFFFFull);
            }
            sm.red[part][v] = acc;
        }
        __syncthreads();
        if (tid < 20) {
            unsigned long long acc = 0;
            for (int part = 0; part < 32; part++) acc += sm.red[part][tid];
            const int k = tid >> 2, comp = tid & 3;
            if (comp < 3) sm.sums[k][comp] = (long long)acc;
            else sm.counts[k] = (int)acc;
        } else if (tid < 20 + kMaxK * 3) {
            const int q = tid - 20, k = q / 3, j = q % 3;
            sm.cprev[k][j] = sm.c[k][j];
        } else if (tid == 64) {
            sm.n_moved = 0;
        }
        __syncthreads();

        // ---- empty clusters: move the farthest point of the biggest cluster (rare)
        for (int ek = 0; ek < K; ek++) {
            if (sm.counts[ek] != 0) continue;  // uniform
            int max_k = 0;
            for (int k1 = 1; k1 < K; k1++)
                if (sm.counts[max_k] < sm.counts[k1]) max_k = k1;
            const float scale = 1.f / (float)sm.counts[max_k];
            const float bx = (float)sm.sums[max_k][0] * scale, by = (float)sm.sums[max_k][1] * scale,
                        bz = (float)sm.sums[max_k][2] * scale;
            const Cent cp = load_centres(sm.cprev);
            double md = -1.0;
            int mi = -1;
            auto visit = [&](int i) {  // key address i (increasing with the np.unique index)
                P3 pp = unpack(pts[i]);
                float bd;
                int l = moved_label(sm, i, label5(pp, cp, bd));
                if (l != max_k) return;
                double d = (double)d2(pp.x, pp.y, pp.z, bx, by, bz);
                if (md <= d) {
                    md = d;
                    mi = i;
                }
            };
            if (kCubes && cubes.part_hist) {
                // segmented keys: partition by partition, in np.unique order
                if (wid == 0) (void)key_layout(sm, cubes.part_uq + (size_t)img * kParts,
                                               cubes.part_hist + (size_t)img * kParts, 0u);
                __syncthreads();
                for (int P = 0; P < kParts; P++) {
                    const int a0 = (int)sm.kbeg[P], a1 = a0 + (int)(sm.pbase[P + 1] - sm.pbase[P]);
                    for (int i = a0 + tid; i < a1; i += KT) visit(i);
                }
            } else {
                for (int s = sb; s < se; s++) {
                    const int i0 = s * STEP + lane * 4;
                    for (int jj = 0; jj < 4; jj++) {
                        const int i = i0 + jj;
                        if (i >= N) break;
                        visit(i);
                    }
                }
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                double od = __shfl_xor(md, off);
                int oi = __shfl_xor(mi, off);
                if (od > md || (od == md && oi > mi)) {
                    md = od;
                    mi = oi;
                }
            }
            if (lane == 0) {
                sm.maxd[wid] = md;
                sm.maxi[wid] = mi;
            }
            __syncthreads();
            if (tid == 0) {
                double bd2 = -1.0;
                int bi = -1;
                for (int w = 0; w < KW; w++)
                    if (sm.maxd[w] > bd2 || (sm.maxd[w] == bd2 && sm.maxi[w] > bi)) {
                        bd2 = sm.maxd[w];
                        bi = sm.maxi[w];
                    }
                if (bi >= 0) {
                    P3 pp = unpack(pts[bi]);
                    sm.counts[max_k]--;
                    sm.counts[ek]++;
                    sm.sums[max_k][0] -= (long long)pp.x;
                    sm.sums[max_k][1] -= (long long)pp.y;
                    sm.sums[max_k][2] -= (long long)pp.z;
                    sm.sums[ek][0] += (long long)pp.x;
                    sm.sums[ek][1] += (long long)pp.y;
                    sm.sums[ek][2] += (long long)pp.z;
                    sm.moved_idx[sm.n_moved] = bi;
                    sm.moved_lbl[sm.n_moved] = ek;
                    sm.n_moved++;
                }
            }
            __syncthreads();
        }
        if (tid == 0) {
            double max_shift = 0.0;
            for (int k = 0; k < K; k++) {
                const float scale = 1.f / (float)sm.counts[k];
                double dist = 0.0;
                for (int j = 0; j < 3; j++) {
                    float v = (float)sm.sums[k][j] * scale;
                    sm.c[k][j] = v;
                    double t = (double)(v - sm.cprev[k][j]);
                    dist += t * t;
                }
                max_shift = fmax(max_shift, dist);
            }
            sm.flag = (iter + 1 == 100 || max_shift <= eps2) ? 1 : 0;
            sm.next_chunk = 0;
            // (trace) iterations by their largest centre move, 8 u8 bins
            // [0,.25) [.25,.5) [.5,1) [1,2) [2,4) [4,8) [8,16) [16,inf)
            const double mv = sqrt(max_shift);
            int bin = 0;
            for (double t = 0.25; bin < 7 && mv >= t; t *= 2.0) bin++;
            const unsigned long long sh = 8ull * (unsigned)bin;
            if (((drift_hist >> sh) & 255ull) < 255ull) drift_hist += 1ull << sh;
        }
        iter++;
        __syncthreads();
        if (sm.flag) break;
    }

    if (tid == 0) o->t_lloyd = wall_clock64();
    // ------------------------------------------------ compactness with the last labels
    if (use_cubes) {
        // sum_k sum_{p in k} |p - c_k|^2 = sum_p |p|^2 - sum_k (2 c_k . S_k - n_k |c_k|^2)
        // with the last assignment's exact sums S_k, n_k: no pass over the colours.  (OpenCV
        // sums float normL2Sqr per colour; the two differ by float rounding, ~1e-7
        // relative -- compactness only ranks the attempts.)
        if (tid == 0) {
            double acc = (double)sm.qtot;
            for (int k = 0; k < K; k++) {
                double cs = 0.0, c2 = 0.0;
                for (int j = 0; j < 3; j++) {
                    const double cj = (double)sm.c[k][j];
                    cs += cj * (double)sm.sums[k][j];
                    c2 += cj * cj;
                }
                acc -= 2.0 * cs - (double)sm.counts[k] * c2;
            }
            sm.dred[0] = acc;
            for (int w = 1; w < KW; w++) sm.dred[w] = 0.0;
        }
        __syncthreads();
    } else {
        const Cent cp = load_centres(sm.cprev);
        const Cent cn = load_centres(sm.c);
        const bool moved = sm.n_moved > 0;
        double acc = 0.0;
        for (int s = sb; s < se; s++) {
            const int i0 = s * STEP + lane * 4;
            for (int jj = 0; jj < 4; jj++) {
                const int i = i0 + jj;
                if (i >= N) break;
                P3 pp = unpack(pts[i]);
                float bd;
                int l = label5(pp, cp, bd);
                if (moved) l = moved_label(sm, i, l);
                float cx = cn.x[0], cy = cn.y[0], cz = cn.z[0];
#pragma unroll
                for (int k = 1; k < kMaxK; k++) {
                    cx = l == k ? cn.x[k] : cx;
                    cy = l == k ? cn.y[k] : cy;
                    cz = l == k ? cn.z[k] : cz;
                }
                acc += (double)d2(pp.x, pp.y, pp.z, cx, cy, cz);
            }
        }
        acc = wave_sum(acc);
        if (lane == 0) sm.dred[wid] = acc;
        __syncthreads();
    }
    {
        if (tid == 0) {
            double compactness = 0.0;
            for (int w = 0; w < KW; w++) compactness += sm.dred[w];
            o->compactness = compactness;
            o->iters = iter;
            o->bytes = bytes;
            if (kPhase & 1) {
                o->pp_pts = pp_pts;
                o->pad = (int32_t)pp_sel;
                o->t_sel = t_sel;
            }
            o->ll_pts = ll_pts;
            o->t_sw = t_sw;
            o->n_cubes = (uint32_t)C;
            o->drift_hist = drift_hist;
            o->t_end = wall_clock64();
            for (int k = 0; k < kMaxK; k++) {
                for (int j = 0; j < 3; j++) o->centers[k][j] = k < K ? sm.c[k][j] : 0.f;
                o->counts[k] = k < K ? sm.counts[k] : 0;
            }
        }
    }
    }  // (the task's scope)
    next_task:
    if (!kQueue) break;
    __syncthreads();  // (the task's last LDS reads before thread 0 rewrites sm.task)
    if (tid == 0) sm.task = atomicAdd(queue, 1);
    __syncthreads();
    task = sm.task;
    __syncthreads();
    }
}

// The cube path runs in two launches.  Attempt durations vary 1-8x (k-means++ on ~3k-cube
// ui tables vs ~35k-cube photos; Lloyd 12-97 iterations), and the dispatcher places
// workgroup i on XCD i mod 8 in order, so with one workgroup per attempt a slot freed on
// one XCD waits while the next workgroup's XCD is full: ~15 % of the slots idled between
// attempts (profiles/r4/dispatch_gap/).  A work queue removes that -- one
// workgroup per resident slot takes the next task from a global counter -- but the task
// loop around the whole attempt spilled registers (round 4).  Split, each phase is its own
// kernel with its own register allocation: k-means++ as a work queue (<true, 1, true>),
// then Lloyd from its centres (<true, 2, LLFE_KM_LLOYD_QUEUE>).  The counters sit after the
// LPT order (order[n], order[n + 1]), zeroed by k_kmeans_order.

// LPT order: images sorted by U descending, index ascending on ties (n <= 4096): each
// image's rank is the number of images before it in that order (LDS broadcast reads;
// one pass instead of the 45 barrier-separated stages of a bitonic sort)
constexpr int OT = 1024;
constexpr int OMAX = 4096;
__global__ __launch_bounds__(OT) void k_kmeans_order(const long long *__restrict__ n_unique, int n,
                                                     int *__restrict__ order) {
    __shared__ long long key[OMAX];
    for (int i = threadIdx.x; i < n; i += OT) key[i] = n_unique[i];
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += OT) {
        const long long ki = key[i];
        int r = 0;
        for (int j = 0; j < n; j++) {
            const long long kj = key[j];
            r += (kj > ki) | ((kj == ki) & (j < i));
        }
        order[r] = i;
    }
    if (threadIdx.x < 2) order[n + threadIdx.x] = 0;  // the work-queue counters
}

__global__ void k_kmeans_finalize(const uint32_t *__restrict__ keys, long long key_stride,
                                  const long long *__restrict__ n_unique, int n, int n_colors,
                                  const KmeansAttemptOut *__restrict__ att, KmeansImageOut *__restrict__ out,
                                  const uint32_t *__restrict__ part_uq, const uint32_t *__restrict__ part_hist) {
    int img = blockIdx.x * blockDim.x + threadIdx.x;
    if (img >= n) return;
    long long N = n_unique[img];
    int K = (int)min((long long)n_colors, N);
    KmeansImageOut r;
    memset(&r, 0, sizeof r);
    r.n_unique = N;
    if (K <= 1) {
        // _get_dominant_colors (color_extractor.py:185-186) skips k-means and returns
        // every unique colour with labels [0] * U, so bincount gives [U, 0, ...] (U > 1)
        // or no bincount at all (U == 1, count 1): keep the first min(U, kMaxK)
        // colours in np.unique order
        r.k = (int)min(N, (long long)kMaxK);
        // (segmented keys: the first keys of the first non-empty partitions)
        uint32_t P = 0, off = 0, seg = 0, left = part_hist ? part_uq[(size_t)img * kParts] : 0u;
        for (int k = 0; k < r.k; k++) {
            uint32_t a = (uint32_t)k;
            if (part_hist) {
                while (left == 0) {
                    seg += part_hist[(size_t)img * kParts + P];
                    P++;
                    off = 0;
                    left = part_uq[(size_t)img * kParts + P];
                }
                a = seg + off++;
                left--;
            }
            const uint32_t key = keys[(size_t)img * key_stride + a];
            r.centers_rgb[k][0] = (uint8_t)(key >> 16);
            r.centers_rgb[k][1] = (uint8_t)(key >> 8);
            r.centers_rgb[k][2] = (uint8_t)key;
            r.counts[k] = k == 0 ? (int)N : 0;
        }
        r.compactness = 0.0;
    } else {
        int best = 0;
        double bc = 1.7976931348623157e308;
        for (int a = 0; a < kAttempts; a++) {  // first attempt with the strictly smallest compactness
            double c = att[(size_t)img * kAttempts + a].compactness;
            if (c < bc) {
                bc = c;
                best = a;
            }
        }
        const KmeansAttemptOut &b = att[(size_t)img * kAttempts + best];
        // algorithmic bytes: 4 U per fused multi-attempt pass over the
        // keys x passes (K k-means++ passes + the Lloyd sweeps of the longest attempt)
        int sweeps = 0;
        for (int a = 0; a < kAttempts; a++) sweeps = max(sweeps, att[(size_t)img * kAttempts + a].iters - 1);
        r.bytes = 4ull * (unsigned long long)N * (unsigned long long)(K + sweeps);
        r.k = K;
        r.compactness = bc;
        for (int k = 0; k < K; k++) {
            for (int j = 0; j < 3; j++) r.centers_rgb[k][j] = (uint8_t)(int)b.centers[k][j];  // astype(uint8)
            r.counts[k] = b.counts[k];
        }
    }
    out[img] = r;
}

}  // namespace

#if LLFE_KM_WIDE
hipError_t launch_kmeans_wide(
#else
hipError_t launch_kmeans(
#endif
                         const uint32_t *keys, int64_t key_stride, const int64_t *n_unique, int n, int n_colors,
                         uint64_t seed, ImgIndex index, int32_t *order, uint32_t *scratch, int64_t scratch_stride,
                         KmeansAttemptOut *attempts, KmeansImageOut *out, const KmeansCubes &cubes,
                         hipStream_t s) {
    if (n > OMAX) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    // the dynamic-LDS attribute is per device: set once per device id, under a lock (one
    // context per GPU per host thread, so several threads / devices can get here at once);
    // with it the resident workgroup slots of the work-queue kernels (CUs x workgroups
    // per CU at this LDS / register use)
    static std::mutex attr_mu;
    static uint64_t attr_set = 0;  // bit d: set on device d
    static int slots_pp[64], slots_ll[64];
    const size_t smem = sizeof(KmSmem);
    constexpr bool kLloydQueue = LLFE_KM_LLOYD_QUEUE;
    const void *plain = (const void *)k_kmeans<false, 3, false>,
               *pp = LLFE_KM_SPLIT ? (const void *)k_kmeans<true, 1, true> : (const void *)k_kmeans<true, 3, false>,
               *lloyd = (const void *)k_kmeans<true, 2, kLloydQueue>;
    int dev = 0;
    {
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        if (dev >= 64) return hipErrorInvalidDevice;
        std::lock_guard<std::mutex> lk(attr_mu);
        const uint64_t bit = 1ull << dev;
        if (!(attr_set & bit)) {
            for (const void *f : {plain, pp, lloyd}) {
                e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
                if (e != hipSuccess) return e;
            }
            int cus = 0, per_pp = 0, per_ll = 0;
            e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            if (e != hipSuccess) return e;
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_pp, pp, KT, smem);
            if (e != hipSuccess) return e;
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_ll, lloyd, KT, smem);
            if (e != hipSuccess) return e;
            slots_pp[dev] = std::max(1, cus * per_pp);
            slots_ll[dev] = std::max(1, cus * per_ll);
            attr_set |= bit;
        }
    }
#if !LLFE_KM_WIDE
    // a batch whose attempts all fit at once gains nothing from the narrow workgroups' packing
    // beside other kernels and runs each attempt at half width: the 512-thread build (round 6,
    // 64 x 512^2 colours: 32.5k -> 41k images/s; 512 x 1080p: 27.2k narrow vs 24.9k wide)
    if (cubes.cubes && n_colors <= kMaxK && !LLFE_KM_SPLIT && (int64_t)n * kAttempts <= slots_pp[dev])
        return launch_kmeans_wide(keys, key_stride, n_unique, n, n_colors, seed, index, order, scratch,
                                  scratch_stride, attempts, out, cubes, s);
#endif
    hipLaunchKernelGGL(k_kmeans_order, dim3(1), dim3(OT), 0, s, (const long long *)n_unique, n, order);
    if (n_colors > kMaxK) {  // general K: plain sweeps over the keys (kmeans_big.hip)
        const hipError_t e = launch_kmeans_big(keys, key_stride, n_unique, n, n_colors, seed, index, order,
                                               scratch, scratch_stride, attempts, s);
        if (e != hipSuccess) return e;
    } else if (!cubes.cubes) {
        hipLaunchKernelGGL((k_kmeans<false, 3, false>), dim3(n * kAttempts), dim3(KT), smem, s, keys,
                           (long long)key_stride, (const long long *)n_unique, n_colors, (unsigned long long)seed,
                           index, order, n * kAttempts, nullptr, scratch, (long long)scratch_stride, attempts, cubes);
    } else if (!LLFE_KM_SPLIT) {
        // one workgroup per (image, attempt) in LPT order, k-means++ then Lloyd
        hipLaunchKernelGGL((k_kmeans<true, 3, false>), dim3(n * kAttempts), dim3(KT), smem, s, keys,
                           (long long)key_stride, (const long long *)n_unique, n_colors, (unsigned long long)seed,
                           index, order, n * kAttempts, nullptr, nullptr, 0LL, attempts, cubes);
    } else {
        const int tasks = n * kAttempts;
        hipLaunchKernelGGL((k_kmeans<true, 1, true>), dim3(std::min(tasks, slots_pp[dev])), dim3(KT), smem, s, keys,
                           (long long)key_stride, (const long long *)n_unique, n_colors, (unsigned long long)seed,
                           index, order, tasks, order + n, nullptr, 0LL, attempts, cubes);
        hipLaunchKernelGGL((k_kmeans<true, 2, kLloydQueue>), dim3(kLloydQueue ? std::min(tasks, slots_ll[dev]) : tasks),
                           dim3(KT), smem, s, keys, (long long)key_stride, (const long long *)n_unique, n_colors,
                           (unsigned long long)seed, index, order, tasks, order + n + 1, nullptr, 0LL, attempts,
                           cubes);
    }
    hipLaunchKernelGGL(k_kmeans_finalize, dim3((n + 255) / 256), dim3(256), 0, s, keys, (long long)key_stride,
                       (const long long *)n_unique, n, n_colors, attempts, out, cubes.part_uq,
                       cubes.cubes ? cubes.part_hist : nullptr);
    return hipGetLastError();
}

#if !LLFE_KM_WIDE
int64_t kmeans_scratch_stride(int64_t key_stride) { return 4 * ((key_stride + STEP - 1) / STEP) + 4; }
#endif

}  // namespace llfe
