// Canny hysteresis + dilate for ShapeAnalyzer.preprocess_image (shape pyc @L24-28) as
// connected components on gfx950.
//
// Canny keeps a "maybe" pixel (class 0) iff it is 8-connected through maybe pixels to a
// strong pixel (class 2).  That is a connected-components question, answered here with
// union-find in a fixed number of launches instead of relaunching a flood fill until it
// stops moving (weak-pixel networks in noisy images percolate across the whole frame):
//
//   k_tile_list   the tiles the stencil flagged (a class != 1 pixel inside) as a list
//   k_ccl_local   per flagged 64x64 tile (a work counter hands them out): LDS union-find
//                 over candidate pixels (class != 1), local root per pixel (u16), strong
//                 flag per root, root list per tile.  Without the stencil's flags (a class
//                 map from elsewhere): one workgroup per tile of the batch
//   k_ccl_border  atomicMin union of the global ids of 8-neighbour candidates that sit
//                 in different tiles (tile right column / bottom row)
//   k_ccl_flatten every local root -> its global root (one hop); strong flags OR-ed
//                 into the global root
//   k_ccl_strong  per tile: bit per local root whose global root is strong
//   k_ccl_edge    edge = strong || (maybe && root strong), packed per 64-pixel row
//                 segment with __ballot (no halo)
//   k_bits_dilate 3x3 dilate on the packed words (shifts and ORs)
#include <algorithm>

#include "llfe_internal.h"

namespace llfe {
namespace {

// 64 x 64 tiles (the GPU contour pass keeps 64 x 32: contours_gpu.hip): the 85 % of tiles
// without a Canny candidate cost one workgroup launch each in k_ccl_local, so half as many
// tiles: hysteresis 1.61 -> 1.34 ms per 512 x 1080p
constexpr int TW = kTileW, TH = 64, TP = TW * TH;  // 4096 pixels per tile
inline int htiles_y(int h) { return (h + TH - 1) / TH; }
constexpr int NT = 256;
static_assert(TW == 64, "k_ccl_dilate packs one 64-pixel word per tile row");

__device__ __forceinline__ int lds_find(int *L, int a) {
    for (;;) {
        int p = __hip_atomic_load(L + a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (p == a) return a;
        a = p;
    }
}

__device__ __forceinline__ void lds_union(int *L, int a, int b) {
    for (;;) {
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
    for (;;) {
        int p = __hip_atomic_load(P + a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p == a) return a;
        a = p;
    }
}

__device__ __forceinline__ void g_union(int *P, int a, int b) {
    for (;;) {
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

// One tile's local components (below).  kList: the grid loops over the tiles the stencil
// flagged (llfe_internal.h HystWork::tflag) instead of one workgroup per tile of the batch.
template <bool kList>
__global__ __launch_bounds__(NT) void k_ccl_local(const uint8_t *__restrict__ cls, int H, int W, int ntx, int nty,
                                                  uint16_t *__restrict__ lab, int *__restrict__ parent,
                                                  uint8_t *__restrict__ sroot, uint16_t *__restrict__ roots,
                                                  int *__restrict__ nroots, int *__restrict__ tlist,
                                                  int *__restrict__ tcount, const int *__restrict__ ftlist,
                                                  int *__restrict__ ftcount) {
    __shared__ int L[TP];
    __shared__ uint32_t sflag[TP / 32];
    __shared__ __attribute__((aligned(16))) uint8_t cb[TP];
    __shared__ int cnt;
    __shared__ int s_it;
    const int ntiles = ntx * nty;
    const int nft = kList ? ftcount[0] : 1;
    for (int it0 = 0;; it0++) {
    // (tid opaque per tile: otherwise the compiler hoists the 16 per-k pixel offsets of
    // every address out of the tile loop -- 173 VGPRs instead of 40)
    int tid = threadIdx.x;
    if (kList) asm volatile("" : "+v"(tid));
    int img, t;
    if (kList) {
        // tiles handed out by a counter (ftcount[1]): the workgroups that start last do
        // not each bring a fixed share of tiles into the launch's tail
        if (tid == 0) s_it = atomicAdd(&ftcount[1], 1);
        __syncthreads();
        const int it = s_it;  // (read by every thread before the next barrier of this tile)
        if (it >= nft) break;
        const int tt = ftlist[it];
        img = tt / ntiles;
        t = tt % ntiles;
    } else {
        if (it0) break;
        img = blockIdx.y;
        t = blockIdx.x;
    }
    const int tx0 = (t % ntx) * TW, ty0 = (t / ntx) * TH;
    const uint8_t *c = cls + (size_t)img * H * W;
    bool any = false;
    static_assert(TP == 16 * NT, "one 16-byte load per thread");
    if ((W & 15) == 0 && tx0 + TW <= W) {  // one 16-byte load per thread, through LDS
        const int row = tid >> 2, col = (tid & 3) * 16, y = ty0 + row;
        const uint4 ones = make_uint4(0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u);
        const uint4 w = y < H ? *(const uint4 *)(c + (size_t)y * W + tx0 + col) : ones;
        any = (w.x ^ ones.x) | (w.y ^ ones.y) | (w.z ^ ones.z) | (w.w ^ ones.w);
        *(uint4 *)&cb[row * TW + col] = w;
    } else {
        for (int k = 0; k < TP / NT; k++) {
            const int i = tid + k * NT, y = ty0 + (i >> 6), x = tx0 + (i & 63);
            cb[i] = (y < H && x < W) ? c[(size_t)y * W + x] : 1;
            any |= cb[i] != 1;
        }
    }
    if (tid < TP / 32) sflag[tid] = 0;
    if (tid == 0) cnt = 0;
    // most tiles hold no Canny candidate (85 % over the ui / photo mix): no roots, and
    // the later kernels skip the tile on nroots == 0
    if (!__syncthreads_or(any)) {
        if (tid == 0) nroots[(size_t)img * ntiles + t] = 0;
        continue;  // (no thread touches cb / L / sflag / cnt after the barrier)
    }
    uint8_t v[TP / NT];
#pragma unroll
    for (int k = 0; k < TP / NT; k++) {
        const int i = tid + k * NT;
        v[k] = cb[i];
        L[i] = v[k] != 1 ? i : -1;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < TP / NT; k++) {
        if (v[k] == 1) continue;
        int i = tid + k * NT, ly = i >> 6, lx = i & 63;
        if (lx > 0 && L[i - 1] >= 0) lds_union(L, i, i - 1);
        if (ly > 0) {
            if (lx > 0 && L[i - 65] >= 0) lds_union(L, i, i - 65);
            if (L[i - 64] >= 0) lds_union(L, i, i - 64);
            if (lx < 63 && L[i - 63] >= 0) lds_union(L, i, i - 63);
        }
    }
    __syncthreads();
    int r[TP / NT];
#pragma unroll
    for (int k = 0; k < TP / NT; k++) {
        int i = tid + k * NT;
        r[k] = -1;
        if (v[k] == 1) continue;
        r[k] = lds_find(L, i);
        if (v[k] == 2) atomicOr(&sflag[r[k] >> 5], 1u << (r[k] & 31));
    }
    __syncthreads();
    const size_t gbase = ((size_t)img * ntiles + t) * TP;
#pragma unroll
    for (int k = 0; k < TP / NT; k++) {
        if (r[k] < 0) continue;
        int i = tid + k * NT, ly = i >> 6, lx = i & 63;
        lab[((size_t)img * H + ty0 + ly) * W + tx0 + lx] = (uint16_t)r[k];
        if (r[k] == i) {
            parent[gbase + i] = (int)(gbase + i);
            sroot[gbase + i] = (sflag[i >> 5] >> (i & 31)) & 1;
            int pos = atomicAdd(&cnt, 1);
            roots[gbase + pos] = (uint16_t)i;
        }
    }
    __syncthreads();  // (also orders this tile's LDS reads before the next tile's writes)
    if (tid == 0) {
        nroots[(size_t)img * ntiles + t] = cnt;
        tlist[atomicAdd(tcount, 1)] = img * ntiles + t;  // the later passes visit only these
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
    const bool f = i < total && tflag[i];
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

// The passes after k_ccl_local visit only the tiles it listed (those with a candidate;
// 15 % of the ui / photo mix): a fixed grid loops over tlist instead of launching one
// workgroup per tile.  Edge words of unlisted tiles stay zero (memset).
constexpr int kListBlocks = 4096;

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
            if (sroot[g]) sroot[r] = 1;
            if (r != g) parent[g] = r;
        }
    }
}

// per listed tile: one bit per local root, set when its global root is strong
__global__ __launch_bounds__(NT) void k_ccl_strong(const int *__restrict__ tlist, const int *__restrict__ tcount,
                                                    const uint16_t *__restrict__ roots, const int *__restrict__ nroots,
                                                    const int *__restrict__ parent, const uint8_t *__restrict__ sroot,
                                                    uint32_t *__restrict__ tstrong) {
    __shared__ uint32_t rs[TP / 32];
    const int tid = threadIdx.x, ntl = *tcount;
    for (int it = blockIdx.x; it < ntl; it += gridDim.x) {
        const size_t tile = (size_t)tlist[it], gbase = tile * TP;
        const int n = nroots[tile];
        if (tid < TP / 32) rs[tid] = 0;
        __syncthreads();
        for (int k = tid; k < n; k += NT) {
            const int i = roots[gbase + k];
            if (sroot[parent[gbase + i]]) atomicOr(&rs[i >> 5], 1u << (i & 31));
        }
        __syncthreads();
        if (tid < TP / 32) tstrong[tile * (TP / 32) + tid] = rs[tid];
        __syncthreads();
    }
}

// per listed tile, no halo: edge = strong || (maybe && strong local root); one wave
// per 64-pixel row segment packs the row's edge word with __ballot
__global__ __launch_bounds__(NT) void k_ccl_edge(const uint8_t *__restrict__ cls, const uint16_t *__restrict__ lab,
                                                  int H, int W, int ntx, int nty, const int *__restrict__ tlist,
                                                  const int *__restrict__ tcount, const uint32_t *__restrict__ tstrong,
                                                  uint64_t *__restrict__ ebits) {
    __shared__ uint32_t rs[TP / 32];
    constexpr int RPW = TH / (NT / 64);  // rows per wave
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ntiles = ntx * nty, ntl = *tcount, wpr = (W + 63) / 64;
    for (int it = blockIdx.x; it < ntl; it += gridDim.x) {
        const int tt = tlist[it], img = tt / ntiles, t = tt % ntiles;
        const int tx0 = (t % ntx) * TW, ty0 = (t / ntx) * TH, x = tx0 + lane;
        const size_t tile = (size_t)tt;
        const uint8_t *c = cls + (size_t)img * H * W;
        const uint16_t *lb = lab + (size_t)img * H * W;
        uint32_t v[RPW], l[RPW];
#pragma unroll
        for (int r = 0; r < RPW; r++) {
            const int y = ty0 + wid + r * (NT / 64);
            const bool in = y < H && x < W;
            v[r] = in ? c[(size_t)y * W + x] : 1u;
            l[r] = in ? lb[(size_t)y * W + x] : 0u;  // meaningful only where v == 0
        }
        if (tid < TP / 32) rs[tid] = tstrong[tile * (TP / 32) + tid];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RPW; r++) {
            const int y = ty0 + wid + r * (NT / 64);
            const uint32_t li = l[r] & (TP - 1);
            const bool on = v[r] == 2u || (v[r] == 0u && ((rs[li >> 5] >> (li & 31)) & 1u));
            const unsigned long long b = __ballot(on);
            if (lane == 0 && y < H) ebits[((size_t)img * H + y) * wpr + (tx0 >> 6)] = b;
        }
        __syncthreads();
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
    dim3 grid(ntiles, n);
    const size_t words = (size_t)n * h * words_per_row(w);
    hipError_t e;
    if ((e = hipMemsetAsync(wk.tcount, 0, sizeof(int), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(wk.ebits, 0, sizeof(uint64_t) * words, s)) != hipSuccess) return e;
    const dim3 lgrid((unsigned)std::min<int64_t>((int64_t)ntiles * n, kListBlocks));
    if (wk.tflag) {
        // only the tiles the stencil flagged: no workgroup per empty tile, no read of its
        // class bytes (85 % of the ui / photo mix)
        if ((e = hipMemsetAsync(wk.ftcount, 0, 2 * sizeof(int), s)) != hipSuccess) return e;
        const int total = ntiles * n;
        hipLaunchKernelGGL(k_tile_list, dim3((unsigned)((total + LT - 1) / LT)), dim3(LT), 0, s, wk.tflag, total,
                           wk.ftlist, wk.ftcount);
        // (a work counter hands out the tiles: 2048 workgroups cover the 7 x 256 resident slots)
        const dim3 qgrid((unsigned)std::min<int64_t>((int64_t)ntiles * n, 2048));
        hipLaunchKernelGGL(k_ccl_local<true>, qgrid, dim3(NT), 0, s, cls, h, w, ntx, nty, wk.lab, wk.parent, wk.sroot,
                           wk.roots, wk.nroots, wk.tlist, wk.tcount, (const int *)wk.ftlist, wk.ftcount);
    } else {
        hipLaunchKernelGGL(k_ccl_local<false>, grid, dim3(NT), 0, s, cls, h, w, ntx, nty, wk.lab, wk.parent, wk.sroot,
                           wk.roots, wk.nroots, wk.tlist, wk.tcount, (const int *)nullptr, (int *)nullptr);
    }
    hipLaunchKernelGGL(k_ccl_border, lgrid, dim3(128), 0, s, cls, wk.lab, h, w, ntx, nty, wk.tlist, wk.tcount,
                       wk.parent);
    hipLaunchKernelGGL(k_ccl_flatten, lgrid, dim3(NT), 0, s, wk.tlist, wk.tcount, wk.roots, wk.nroots, wk.parent,
                       wk.sroot);
    hipLaunchKernelGGL(k_ccl_strong, lgrid, dim3(NT), 0, s, wk.tlist, wk.tcount, wk.roots, wk.nroots, wk.parent,
                       wk.sroot, wk.tstrong);
    hipLaunchKernelGGL(k_ccl_edge, lgrid, dim3(NT), 0, s, cls, wk.lab, h, w, ntx, nty, wk.tlist, wk.tcount, wk.tstrong,
                       wk.ebits);
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
