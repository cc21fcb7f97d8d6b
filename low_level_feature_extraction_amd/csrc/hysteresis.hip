// Canny hysteresis + dilate for ShapeAnalyzer.preprocess_image (shape pyc @L24-28) as
// connected components on gfx950.
//
// Canny keeps a "maybe" pixel (class 0) iff it is 8-connected through maybe pixels to a
// strong pixel (class 2).  That is a connected-components question, answered here with
// union-find in a fixed number of launches instead of relaunching a flood fill until it
// stops moving (weak-pixel networks in noisy images percolate across the whole frame):
//
//   k_tile_list   the tiles the stencil flagged (a class != 1 pixel inside) as a list (every
//                 tile when the class map comes without flags)
//   k_ccl_runs    per listed 64x64 tile, one wave (lane = row, tiles from a work counter):
//                 union-find over the rows' candidate runs (class != 1; node = the run's
//                 first pixel) in LDS, local root per run (lab), strong flag per root, root
//                 list per tile, and the edge words the tile decides alone: the runs of a
//                 component with a strong pixel in the tile
//   k_ccl_border  atomicMin union of the global ids of 8-neighbour candidates that sit
//                 in different tiles (tile right column / bottom row)
//   k_ccl_flatten every local root -> its global root (one hop); strong flags OR-ed
//                 into the global root
//   k_ccl_strong  per tile: bit per local root promoted by the global unions (not strong
//                 in its tile, strong through another), and a flag for the tiles with one
//   k_ccl_edge    per listed tile (one wave): the runs with a promoted root OR-ed into the
//                 edge words
//   k_bits_dilate 3x3 dilate on the packed words (shifts and ORs)
#include <algorithm>

#include "llfe_internal.h"

namespace llfe {
namespace {

// 64 x 64 tiles (the GPU contour pass keeps 64 x 32: contours_gpu.hip): one 64-bit word per
// tile row (round 3: 64 x 64 instead of 64 x 32 tiles, hysteresis 1.61 -> 1.34 ms per 512 x
// 1080p, when every tile still cost a workgroup launch)
constexpr int TW = kTileW, TH = 64, TP = TW * TH;  // 4096 pixels per tile
inline int htiles_y(int h) { return (h + TH - 1) / TH; }
constexpr int NT = 256;
static_assert(TW == 64, "k_ccl_dilate packs one 64-pixel word per tile row");

#ifndef LLFE_HYST_WATCHDOG
#define LLFE_HYST_WATCHDOG 0  // (debug builds) bounded union-find loops, printf on overrun
#endif
__device__ __forceinline__ int lds_find(int *L, int a) {
#if LLFE_HYST_WATCHDOG
    for (int guard = 0;; guard++) {
        if (guard > 8192) {
            printf("llfe watchdog: lds_find a=%d L[a]=%d\n", a, L[a]);
            return a;
        }
#else
    for (;;) {
#endif
        int p = __hip_atomic_load(L + a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (p == a) return a;
        a = p;
    }
}

__device__ __forceinline__ void lds_union(int *L, int a, int b) {
#if LLFE_HYST_WATCHDOG
    for (int guard = 0;; guard++) {
        if (guard > 8192) {
            printf("llfe watchdog: lds_union a=%d b=%d\n", a, b);
            return;
        }
#else
    for (;;) {
#endif
        a = lds_find(L, a);
        b = lds_find(L, b);
        if (a == b) return;
        if (a > b) {
            int t = a;
            a = b;
            b = t;
        }
        int old = atomicMin(L + b, a);
        if (old == b) return;
        b = old;
    }
}

__device__ __forceinline__ int g_find(int *P, int a) {
#if LLFE_HYST_WATCHDOG
    for (int guard = 0;; guard++) {
        if (guard > (1 << 22)) {
            printf("llfe watchdog: g_find a=%d P[a]=%d\n", a, P[a]);
            return a;
        }
#else
    for (;;) {
#endif
        int p = __hip_atomic_load(P + a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p == a) return a;
        a = p;
    }
}

__device__ __forceinline__ void g_union(int *P, int a, int b) {
#if LLFE_HYST_WATCHDOG
    for (int guard = 0;; guard++) {
        if (guard > (1 << 20)) {
            printf("llfe watchdog: g_union a=%d b=%d\n", a, b);
            return;
        }
#else
    for (;;) {
#endif
        a = g_find(P, a);
        b = g_find(P, b);
        if (a == b) return;
        if (a > b) {
            int t = a;
            a = b;
            b = t;
        }
        int old = atomicMin(P + b, a);
        if (old == b) return;
        b = old;
    }
}

// ------------------------------------------------------------------ run-based local CCL
// One wave per listed tile, lane = tile row.  A row's candidates (class != 1) are a 64-bit
// mask and its runs (maximal 1-bit sequences) the union-find nodes -- node id = row * 32 +
// the run's rank in its row (< 2048: at most 32 runs in 64 pixels) -- united with the runs
// of the row above that touch them 8-connectedly (the run widened by one pixel each side,
// AND the row above).  A component's local id (lab, the roots list, parent / sroot at
// tile base + id) is its root node.
constexpr int RW = 4;  // waves (tiles in flight) per workgroup

__device__ __forceinline__ unsigned long long bits_upto(int b) {  // bits 0..b (b in -1..63)
    return b >= 63 ? ~0ull : ((1ull << (b + 1)) - 1ull);
}
// length of the 1-run of m starting at bit a (m bit a set)
__device__ __forceinline__ int run_len(unsigned long long m, int a) {
    const unsigned long long z = ~(m >> a);
    return z ? __builtin_ctzll(z) : 64 - a;
}

// the row's candidate (class != 1) and strong (class 2) masks; zero outside the image
__device__ __forceinline__ void row_masks(const uint8_t *__restrict__ cls, int img, int H, int W, int tx0, int y,
                                          unsigned long long &C, unsigned long long &S) {
    C = S = 0;
    if (y >= H) return;
    const uint8_t *row = cls + ((size_t)img * H + y) * W + tx0;
    const int nx = min(64, W - tx0);
    if (nx == 64 && (((uintptr_t)row) & 15) == 0) {
        uint32_t d[16];
#pragma unroll
        for (int q = 0; q < 4; q++) *(uint4 *)&d[4 * q] = ((const uint4 *)row)[q];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            // classes 0 / 1 / 2 per byte: candidate = byte != 1, strong = bit 1; the four
            // bytes' flag bits (0, 8, 16, 24) gathered to bits 0..3
            const uint32_t t1 = d[j] ^ 0x01010101u;
            uint32_t c = (t1 | (t1 >> 1)) & 0x01010101u, s = (d[j] >> 1) & 0x01010101u;
            c |= c >> 7;
            s |= s >> 7;
            c |= c >> 14;
            s |= s >> 14;
            C |= (unsigned long long)(c & 15u) << (4 * j);
            S |= (unsigned long long)(s & 15u) << (4 * j);
        }
    } else {
        for (int x = 0; x < nx; x++) {
            const uint8_t b = row[x];
            if (b != 1) C |= 1ull << x;
            if (b == 2) S |= 1ull << x;
        }
    }
}

// Outputs as the per-pixel union-find had them (with node ids for pixel ids), except lab:
// written at each run's first pixel, at x = 63 of the runs that end there, and over the
// whole of rows 0 and 63 -- every pixel k_ccl_border reads (its tile's right column and
// bottom row, the neighbours' left column and top row) and every run start k_ccl_edge
// reads.  Plus the edge words the tile decides alone (runs whose local root holds a strong
// pixel).
constexpr int kNodes = 64 * 32;
__device__ __forceinline__ void ccl_runs_tile(const uint8_t *__restrict__ cls, int H, int W, int ntx, int ntiles,
                                              int wpr, int tt, int lane, int nb, int *P, uint32_t *sflag, int *cnt,
                                              uint16_t *__restrict__ lab, int *__restrict__ parent,
                                              uint8_t *__restrict__ sroot, uint16_t *__restrict__ roots,
                                              int *__restrict__ nroots, uint64_t *__restrict__ ebits) {
    const int img = tt / ntiles, t = tt % ntiles;
    const int tx0 = (t % ntx) * TW, ty0 = (t / ntx) * TH, y = ty0 + lane;
    unsigned long long C, S;
    row_masks(cls, img, H, W, tx0, y, C, S);
    if (__ballot(C != 0) == 0) {  // (the tile list without the stencil's flags)
        if (lane == 0) nroots[(size_t)img * ntiles + t] = 0;
        return;
    }
    const unsigned long long starts = C & ~(C << 1);
    const int nr = __popcll(starts);
    for (int j = 0; j < nr; j++) P[nb + j] = nb + j;
    sflag[lane] = 0;  // (kNodes / 32 = 64 words)
    if (lane == 0) *cnt = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // unions with the runs of the row above (8-connected)
    unsigned long long Cu = __shfl_up(C, 1);
    if (lane == 0) Cu = 0;
    const unsigned long long startsU = Cu & ~(Cu << 1);
    int j = 0;
    for (unsigned long long m = starts; m; m &= m - 1, j++) {
        const int a = __builtin_ctzll(m), b = a + run_len(C, a) - 1;
        const unsigned long long M = bits_upto(b) & ~bits_upto(a - 1);
        unsigned long long ov = Cu & (M | (M << 1) | (M >> 1));
        while (ov) {
            const int x = __builtin_ctzll(ov);
            // the run of the row above holding x: its rank = starts above at or below x, - 1
            const int ju = __popcll(startsU & bits_upto(x)) - 1;
            lds_union(P, nb + j, nb - 32 + ju);
            ov &= ~bits_upto(x + run_len(Cu, x) - 1);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // strong flags on the roots
    j = 0;
    for (unsigned long long m = starts; m; m &= m - 1, j++) {
        const int a = __builtin_ctzll(m), b = a + run_len(C, a) - 1;
        if (S & bits_upto(b) & ~bits_upto(a - 1)) {
            const int r = lds_find(P, nb + j);
            atomicOr(&sflag[r >> 5], 1u << (r & 31));
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const size_t gbase = ((size_t)img * ntiles + t) * TP;
    uint16_t *const lrow = lab + ((size_t)img * H + y) * W + tx0;
    unsigned long long E = 0;
    j = 0;
    for (unsigned long long m = starts; m; m &= m - 1, j++) {
        const int a = __builtin_ctzll(m), len = run_len(C, a), b = a + len - 1, id = nb + j;
        const int r = lds_find(P, id);
        if ((sflag[r >> 5] >> (r & 31)) & 1u) E |= bits_upto(b) & ~bits_upto(a - 1);
        lrow[a] = (uint16_t)r;
        if (lane == 0 || lane == 63)
            for (int q = 1; q < len; q++) lrow[a + q] = (uint16_t)r;
        else if (b == 63 && a < 63)
            lrow[63] = (uint16_t)r;
        if (r == id) {
            parent[gbase + id] = (int)(gbase + id);
            sroot[gbase + id] = (sflag[id >> 5] >> (id & 31)) & 1;  // bit 0: strong in the tile
            roots[gbase + atomicAdd(cnt, 1)] = (uint16_t)id;
        }
    }
    if (E) ebits[((size_t)img * H + y) * wpr + (tx0 >> 6)] = E;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) nroots[(size_t)img * ntiles + t] = *cnt;
}

__global__ __launch_bounds__(64 * RW) void k_ccl_runs(const uint8_t *__restrict__ cls, int H, int W, int ntx, int nty,
                                                    uint16_t *__restrict__ lab, int *__restrict__ parent,
                                                    uint8_t *__restrict__ sroot, uint16_t *__restrict__ roots,
                                                    int *__restrict__ nroots, const int *__restrict__ ftlist,
                                                    int *__restrict__ ftcount, uint64_t *__restrict__ ebits) {
    __shared__ int Pall[RW][kNodes];
    __shared__ uint32_t sfl[RW][kNodes / 32];
    __shared__ int cntw[RW];
    __shared__ int s_base;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int *const P = Pall[wv];
    uint32_t *const sflag = sfl[wv];
    const int ntiles = ntx * nty, nft = ftcount[0], wpr = (W + 63) >> 6;
    const int nb = lane * 32;  // this row's first node id
    // kGrab tiles per workgroup per round from a work counter (ftcount[1]), its base read
    // from LDS between two workgroup barriers: the tile index never crosses lanes.  (Round
    // 5's first version broadcast a per-wave counter from lane 0 with __shfl; hipcc threaded
    // the latch's lane != 0 path back to that shuffle, so lanes 1-63 relabelled list entry
    // 0's tile without lane 0, whose root counter reset they skipped: roots[] ran past its
    // buffer -- DESIGN.md §3, profiles/r6/ccl_root_cause/, tests/test_ccl_isa.py pins this
    // loop's compiled shape.)  The later passes walk the same list (no per-tile append: one
    // global atomic per tile on one counter costs ~100 us per 512 x 1080p)
    constexpr int kGrab = 2 * RW;
    for (;;) {
        if (threadIdx.x == 0) s_base = atomicAdd(&ftcount[1], kGrab);
        __syncthreads();
        const int base = s_base;
        __syncthreads();
        if (base >= nft) break;
#pragma unroll 1
        for (int q = wv; q < kGrab; q += RW) {
            const int it = base + q;
            if (it < nft) ccl_runs_tile(cls, H, W, ntx, ntiles, wpr, ftlist[it], lane, nb, P, sflag, &cntw[wv], lab,
                                        parent, sroot, roots, nroots, ebits);
        }
    }
}

// The flagged tiles (a byte per tile, set by the stencil where a class != 1 pixel sits)
// as a list: one atomic per 1024-tile block.
constexpr int LT = 1024;
__global__ __launch_bounds__(LT) void k_tile_list(const uint8_t *__restrict__ tflag, int total,
                                                  int *__restrict__ ftlist, int *__restrict__ ftcount) {
    __shared__ int wbase[LT / 64];
    const int i = blockIdx.x * LT + threadIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const bool f = i < total && (!tflag || tflag[i]);  // (no flags: every tile)
    const unsigned long long m = __ballot(f);
    if (lane == 0) wbase[wid] = __popcll(m);
    __syncthreads();
    if (wid == 0) {
        const int c = lane < LT / 64 ? wbase[lane] : 0;
        int x = c;
#pragma unroll
        for (int off = 1; off < LT / 64; off <<= 1) {
            const int y = __shfl_up(x, off);
            if (lane >= off) x += y;
        }
        const int tot = __shfl(x, LT / 64 - 1);
        int base = 0;
        if (lane == 0 && tot) base = atomicAdd(ftcount, tot);
        base = __shfl(base, 0);
        if (lane < LT / 64) wbase[lane] = base + x - c;
    }
    __syncthreads();
    if (f) ftlist[wbase[wid] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = i;
}

__device__ __forceinline__ int gid_of(const uint16_t *lab, int img, int H, int W, int ntx, int ntiles, int y, int x) {
    int t = (y / TH) * ntx + x / TW;
    return (int)(((size_t)img * ntiles + t) * TP) + lab[((size_t)img * H + y) * W + x];
}

// The passes after k_ccl_runs visit only the listed tiles (those with a candidate; 15 % of
// the ui / photo mix): a fixed grid loops over the list instead of launching one workgroup
// per tile of the batch.  Edge words of unlisted tiles stay zero (memset).  16k workgroups
// (round 5; 4096 before): border + flatten + edge 210 -> 183 us on the mix, 64k no better.
constexpr int kListBlocks = 16384;

// threads 0..31 the tile's right column (look east), 32..95 its bottom row (look south)
__global__ __launch_bounds__(128) void k_ccl_border(const uint8_t *__restrict__ cls, const uint16_t *__restrict__ lab,
                                                    int H, int W, int ntx, int nty, const int *__restrict__ tlist,
                                                    const int *__restrict__ tcount, int *__restrict__ parent) {
    const int tid = threadIdx.x, ntiles = ntx * nty, ntl = *tcount;
    for (int it = blockIdx.x; it < ntl; it += gridDim.x) {
        const int tt = tlist[it], img = tt / ntiles, t = tt % ntiles;
        const int tx0 = (t % ntx) * TW, ty0 = (t / ntx) * TH;
        const uint8_t *c = cls + (size_t)img * H * W;
        int x, y;
        if (tid < TH) {
            x = tx0 + TW - 1;
            y = ty0 + tid;
        } else if (tid < TH + TW) {
            x = tx0 + tid - TH;
            y = ty0 + TH - 1;
        } else {
            continue;
        }
        if (x >= W || y >= H || c[(size_t)y * W + x] == 1) continue;
        const int a = gid_of(lab, img, H, W, ntx, ntiles, y, x);
        const int ty = y / TH, txi = x / TW;
        for (int dy = -1; dy <= 1; dy++)
            for (int dx = -1; dx <= 1; dx++) {
                if (!dx && !dy) continue;
                const int yy = y + dy, xx = x + dx;
                if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
                if (yy / TH == ty && xx / TW == txi) continue;  // same tile: already merged locally
                if (tid < TH ? dx != 1 : dy != 1) continue;     // right column looks east, bottom row south
                if (c[(size_t)yy * W + xx] == 1) continue;
                g_union(parent, a, gid_of(lab, img, H, W, ntx, ntiles, yy, xx));
            }
    }
}

__global__ __launch_bounds__(NT) void k_ccl_flatten(const int *__restrict__ tlist, const int *__restrict__ tcount,
                                                     const uint16_t *__restrict__ roots, const int *__restrict__ nroots,
                                                     int *__restrict__ parent, uint8_t *__restrict__ sroot) {
    const int ntl = *tcount;
    for (int it = blockIdx.x; it < ntl; it += gridDim.x) {
        const size_t tile = (size_t)tlist[it], gbase = tile * TP;
        const int n = nroots[tile];
        for (int k = threadIdx.x; k < n; k += NT) {
            const int g = (int)(gbase + roots[gbase + k]);
            const int r = g_find(parent, g);
            // bit 1 of the global root: some member component is strong (every writer sets
            // the same bit, bit 0 -- strong in its own tile -- is only read)
            if (sroot[g] & 1) sroot[r] |= 2;
            if (r != g) parent[g] = r;
        }
    }
}

// per listed tile (one wave): one bit per *promoted* local root -- not strong in its tile,
// but its global root's component is (sroot != 0) -- and pflag[it] = whether the tile has
// one (most have none: their edge words are final after k_ccl_runs).  A flag per list
// entry and one wave per tile: the list of promoted tiles built with a global atomic each
// and a 256-thread workgroup per tile took 117 us per 512 x 1080p mix, this 17.5 us.
__global__ __launch_bounds__(64 * RW) void k_ccl_strong(const int *__restrict__ tlist, const int *__restrict__ tcount,
                                                        const uint16_t *__restrict__ roots,
                                                        const int *__restrict__ nroots, const int *__restrict__ parent,
                                                        const uint8_t *__restrict__ sroot, uint32_t *__restrict__ tstrong,
                                                        int *__restrict__ pflag) {
    __shared__ uint32_t rsa[RW][kNodes / 32];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, ntl = *tcount;
    uint32_t *const rs = rsa[wv];
    for (int it = blockIdx.x * RW + wv; it < ntl; it += gridDim.x * RW) {
        const size_t tile = (size_t)tlist[it], gbase = tile * TP;
        const int n = nroots[tile];
        rs[lane] = 0;
        __builtin_amdgcn_wave_barrier();
        bool any = false;
        for (int k = lane; k < n; k += 64) {
            const int i = roots[gbase + k];
            const uint8_t own = sroot[gbase + i];
            const int p = parent[gbase + i];
            if (!(own & 1) && sroot[p]) {
                atomicOr(&rs[i >> 5], 1u << (i & 31));
                any = true;
            }
        }
        __builtin_amdgcn_wave_barrier();
        const bool prom = __ballot(any) != 0;
        if (prom) tstrong[tile * (TP / 32) + lane] = rs[lane];
        if (lane == 0) pflag[it] = prom ? 1 : 0;
        __builtin_amdgcn_wave_barrier();
    }
}

// per listed tile with a promoted root (one wave, lane = row): the runs whose local root
// (lab at the run's first pixel) is promoted OR-ed into the row words k_ccl_runs wrote
__global__ __launch_bounds__(64 * RW) void k_ccl_edge(const uint8_t *__restrict__ cls, const uint16_t *__restrict__ lab,
                                                      int H, int W, int ntx, int nty, const int *__restrict__ tlist,
                                                      const int *__restrict__ tcount, const int *__restrict__ pflag,
                                                      const uint32_t *__restrict__ tstrong, uint64_t *__restrict__ ebits) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ntiles = ntx * nty, ntl = *tcount, wpr = (W + 63) >> 6;
    for (int it = blockIdx.x * RW + wv; it < ntl; it += gridDim.x * RW) {
        if (!pflag[it]) continue;  // (uniform)
        const int tt = tlist[it], img = tt / ntiles, t = tt % ntiles;
        const int tx0 = (t % ntx) * TW, ty0 = (t / ntx) * TH, y = ty0 + lane;
        unsigned long long C, S;
        row_masks(cls, img, H, W, tx0, y, C, S);
        const uint32_t *rs = tstrong + (size_t)tt * (TP / 32);
        const uint16_t *lrow = lab + ((size_t)img * H + y) * W + tx0;
        unsigned long long E = 0;
        for (unsigned long long m = C & ~(C << 1); m; m &= m - 1) {
            const int a = __builtin_ctzll(m), b = a + run_len(C, a) - 1;
            const uint32_t r = lrow[a] & (TP - 1);
            if ((rs[r >> 5] >> (r & 31)) & 1u) E |= bits_upto(b) & ~bits_upto(a - 1);
        }
        if (E) ebits[((size_t)img * H + y) * wpr + (tx0 >> 6)] |= E;
    }
}

// 3x3 dilate on the packed edge words: one thread per 64-pixel word
__global__ __launch_bounds__(NT) void k_bits_dilate(const uint64_t *__restrict__ eb, int n, int H, int W,
                                                     uint64_t *__restrict__ bits, uint8_t *__restrict__ mask_u8) {
    const int wpr = (W + 63) / 64;
    const size_t total = (size_t)n * H * wpr;
    for (size_t i = (size_t)blockIdx.x * NT + threadIdx.x; i < total; i += (size_t)gridDim.x * NT) {
        const int k = (int)(i % wpr);
        const size_t row = i / wpr;  // img * H + y
        const int y = (int)(row % H);
        uint64_t d = 0;
#pragma unroll
        for (int dy = -1; dy <= 1; dy++) {
            if ((unsigned)(y + dy) >= (unsigned)H) continue;
            const uint64_t *r = eb + (row + dy) * wpr;
            const uint64_t w = r[k], wl = k > 0 ? r[k - 1] : 0ull, wr = k + 1 < wpr ? r[k + 1] : 0ull;
            d |= w | (w << 1) | (w >> 1) | (wl >> 63) | (wr << 63);
        }
        if (k == wpr - 1 && (W & 63)) d &= (1ull << (W & 63)) - 1ull;
        if (bits) bits[i] = d;
        if (mask_u8) {
            uint8_t *m = mask_u8 + row * W + (size_t)k * 64;
            const int nx = min(64, W - k * 64);
            for (int b = 0; b < nx; b++) m[b] = ((d >> b) & 1ull) ? 255 : 0;
        }
    }
}

// Canny edges without the dilation (llfe_canny): packed edge words -> 0 / 255 bytes
__global__ __launch_bounds__(NT) void k_bits_unpack(const uint64_t *__restrict__ eb, int n, int H, int W,
                                                    uint8_t *__restrict__ mask_u8) {
    const int wpr = (W + 63) / 64;
    const size_t total = (size_t)n * H * wpr;
    for (size_t i = (size_t)blockIdx.x * NT + threadIdx.x; i < total; i += (size_t)gridDim.x * NT) {
        const int k = (int)(i % wpr);
        const size_t row = i / wpr;
        const uint64_t d = eb[i];
        uint8_t *m = mask_u8 + row * W + (size_t)k * 64;
        const int nx = min(64, W - k * 64);
        for (int b = 0; b < nx; b++) m[b] = ((d >> b) & 1ull) ? 255 : 0;
    }
}

// dilate(src, ones(3, 3)) of n u8 images (any values): 3x3 max, the border never wins
// (llfe_dilate3; the shapes path dilates the packed edge bits in k_bits_dilate)
__global__ __launch_bounds__(NT) void k_dilate3_u8(const uint8_t *__restrict__ src, int n, int H, int W,
                                                   uint8_t *__restrict__ dst) {
    const size_t total = (size_t)n * H * W;
    for (size_t i = (size_t)blockIdx.x * NT + threadIdx.x; i < total; i += (size_t)gridDim.x * NT) {
        const int x = (int)(i % W);
        const size_t row = i / W;
        const int y = (int)(row % H);
        int m = 0;
#pragma unroll
        for (int dy = -1; dy <= 1; dy++) {
            if ((unsigned)(y + dy) >= (unsigned)H) continue;
            const uint8_t *r = src + (size_t)((long long)row + dy) * W;
#pragma unroll
            for (int dx = -1; dx <= 1; dx++)
                if ((unsigned)(x + dx) < (unsigned)W) m = max(m, (int)r[x + dx]);
        }
        dst[i] = (uint8_t)m;
    }
}

// the connected-component passes up to the packed edge words wk.ebits
hipError_t launch_ccl(const uint8_t *cls, int n, int h, int w, const HystWork &wk, hipStream_t s) {
    const int ntx = tiles_x(w), nty = htiles_y(h), ntiles = ntx * nty;
    const size_t words = (size_t)n * h * words_per_row(w);
    hipError_t e;
    if ((e = hipMemsetAsync(wk.ebits, 0, sizeof(uint64_t) * words, s)) != hipSuccess) return e;
    const dim3 lgrid((unsigned)std::min<int64_t>((int64_t)ntiles * n, kListBlocks));
    // the tiles to label: the stencil's flagged ones, or every tile of the batch
    if ((e = hipMemsetAsync(wk.ftcount, 0, 2 * sizeof(int), s)) != hipSuccess) return e;
    const int total = ntiles * n;
    hipLaunchKernelGGL(k_tile_list, dim3((unsigned)((total + LT - 1) / LT)), dim3(LT), 0, s, wk.tflag, total, wk.ftlist,
                       wk.ftcount);
    // (a work counter hands out the tiles, eight per workgroup; 1024 workgroups cover the
    // 4 x 256 resident ones)
    const dim3 rgrid((unsigned)std::min<int64_t>(((int64_t)total + RW - 1) / RW, 1024));
    hipLaunchKernelGGL(k_ccl_runs, rgrid, dim3(64 * RW), 0, s, cls, h, w, ntx, nty, wk.lab, wk.parent, wk.sroot,
                       wk.roots, wk.nroots, (const int *)wk.ftlist, wk.ftcount, wk.ebits);
    // the later passes visit the same listed tiles (with the stencil's flags exactly those
    // with a candidate; without them every tile, the empty ones with nroots = 0)
    const int *tl = wk.ftlist, *tc = wk.ftcount;
    hipLaunchKernelGGL(k_ccl_border, lgrid, dim3(128), 0, s, cls, wk.lab, h, w, ntx, nty, tl, tc,
                       wk.parent);
    hipLaunchKernelGGL(k_ccl_flatten, lgrid, dim3(NT), 0, s, tl, tc, wk.roots, wk.nroots, wk.parent,
                       wk.sroot);
    hipLaunchKernelGGL(k_ccl_strong, lgrid, dim3(64 * RW), 0, s, tl, tc, wk.roots, wk.nroots, wk.parent,
                       wk.sroot, wk.tstrong, wk.pflag);
    hipLaunchKernelGGL(k_ccl_edge, lgrid, dim3(64 * RW), 0, s, cls, wk.lab, h, w, ntx, nty, tl, tc, (const int *)wk.pflag, wk.tstrong, wk.ebits);
    return hipGetLastError();
}

}  // namespace

size_t hysteresis_ids(int n, int h, int w) { return (size_t)n * tiles_x(w) * htiles_y(h) * TP; }
size_t hysteresis_tiles(int n, int h, int w) { return (size_t)n * tiles_x(w) * htiles_y(h); }
size_t hysteresis_tile_words() { return TP / 32; }

hipError_t launch_canny_edges(const uint8_t *cls, int n, int h, int w, const HystWork &wk, uint8_t *edges_u8,
                              hipStream_t s) {
    hipError_t e = launch_ccl(cls, n, h, w, wk, s);
    if (e != hipSuccess) return e;
    const size_t words = (size_t)n * h * words_per_row(w);
    const int blocks = (int)std::min<size_t>((words + NT - 1) / NT, 65536);
    hipLaunchKernelGGL(k_bits_unpack, dim3(blocks), dim3(NT), 0, s, wk.ebits, n, h, w, edges_u8);
    return hipGetLastError();
}

hipError_t launch_dilate3_u8(const uint8_t *src, int n, int h, int w, uint8_t *dst, hipStream_t s) {
    const size_t total = (size_t)n * h * w;
    const int blocks = (int)std::min<size_t>((total + NT - 1) / NT, 65536);
    if (total) hipLaunchKernelGGL(k_dilate3_u8, dim3(blocks), dim3(NT), 0, s, src, n, h, w, dst);
    return hipGetLastError();
}

hipError_t launch_hysteresis_dilate(const uint8_t *cls, int n, int h, int w, const HystWork &wk, uint64_t *bits,
                                    uint8_t *mask_u8, hipStream_t s) {
    hipError_t e = launch_ccl(cls, n, h, w, wk, s);
    if (e != hipSuccess) return e;
    const size_t words = (size_t)n * h * words_per_row(w);
    const int blocks = (int)std::min<size_t>((words + NT - 1) / NT, 65536);
    hipLaunchKernelGGL(k_bits_dilate, dim3(blocks), dim3(NT), 0, s, wk.ebits, n, h, w, bits, mask_u8);
    return hipGetLastError();
}

}  // namespace llfe
