// Canny hysteresis + dilate for ShapeAnalyzer.preprocess_image (shape pyc @L24-28) as
// connected components on gfx950.
//
// Canny keeps a "maybe" pixel (class 0) iff it is 8-connected through maybe pixels to a
// strong pixel (class 2).  That is a connected-components question, answered here with
// union-find in a fixed number of launches instead of relaunching a flood fill until it
// stops moving (weak-pixel networks in noisy images percolate across the whole frame):
//
//   k_ccl_local   per 64x32 tile: LDS union-find over candidate pixels (class != 1),
//                 local root per pixel (u16), strong flag per root, root list per tile
//   k_ccl_border  atomicMin union of the global ids of 8-neighbour candidates that sit
//                 in different tiles (tile right column / bottom row)
//   k_ccl_flatten every local root -> its global root (one hop); strong flags OR-ed
//                 into the global root
//   k_ccl_dilate  edge = strong || (maybe && root strong); 3x3 dilate in LDS; one wave
//                 per 64-pixel row segment packs the mask with __ballot
#include "llfe_internal.h"

namespace llfe {
namespace {

constexpr int TW = kTileW, TH = kTileH, TP = TW * TH;  // 2048 pixels per tile
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

__global__ __launch_bounds__(NT) void k_ccl_local(const uint8_t *__restrict__ cls, int H, int W, int ntx, int nty,
                                                  uint16_t *__restrict__ lab, int *__restrict__ parent,
                                                  uint8_t *__restrict__ sroot, uint16_t *__restrict__ roots,
                                                  int *__restrict__ nroots) {
    __shared__ int L[TP];
    __shared__ uint32_t sflag[TP / 32];
    __shared__ int cnt;
    const int tid = threadIdx.x, img = blockIdx.y, t = blockIdx.x;
    const int ntiles = ntx * nty;
    const int tx0 = (t % ntx) * TW, ty0 = (t / ntx) * TH;
    const uint8_t *c = cls + (size_t)img * H * W;
    uint8_t v[TP / NT];
#pragma unroll
    for (int k = 0; k < TP / NT; k++) {
        int i = tid + k * NT, ly = i >> 6, lx = i & 63, y = ty0 + ly, x = tx0 + lx;
        v[k] = (y < H && x < W) ? c[(size_t)y * W + x] : 1;
        L[i] = v[k] != 1 ? i : -1;
    }
    if (tid < TP / 32) sflag[tid] = 0;
    if (tid == 0) cnt = 0;
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
    __syncthreads();
    if (tid == 0) nroots[(size_t)img * ntiles + t] = cnt;
}

__device__ __forceinline__ int gid_of(const uint16_t *lab, int img, int H, int W, int ntx, int ntiles, int y, int x) {
    int t = (y / TH) * ntx + x / TW;
    return (int)(((size_t)img * ntiles + t) * TP) + lab[((size_t)img * H + y) * W + x];
}

// grid (ntiles, n): threads 0..31 right column, 32..95 bottom row of the tile
__global__ __launch_bounds__(128) void k_ccl_border(const uint8_t *__restrict__ cls, const uint16_t *__restrict__ lab,
                                                    int H, int W, int ntx, int nty, int *__restrict__ parent) {
    const int tid = threadIdx.x, img = blockIdx.y, t = blockIdx.x;
    const int ntiles = ntx * nty;
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
        return;
    }
    if (x >= W || y >= H || c[(size_t)y * W + x] == 1) return;
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

__global__ __launch_bounds__(NT) void k_ccl_flatten(int ntiles, const uint16_t *__restrict__ roots,
                                                     const int *__restrict__ nroots, int *__restrict__ parent,
                                                     uint8_t *__restrict__ sroot) {
    const size_t tile = (size_t)blockIdx.y * ntiles + blockIdx.x;
    const int n = nroots[tile];
    const size_t gbase = tile * TP;
    for (int k = threadIdx.x; k < n; k += NT) {
        const int g = (int)(gbase + roots[gbase + k]);
        const int r = g_find(parent, g);
        if (sroot[g]) sroot[r] = 1;
        if (r != g) parent[g] = r;
    }
}

constexpr int EH = TH + 2, EW = TW + 2, EWP = TW + 8;
__device__ __forceinline__ uint8_t edge_global(const uint8_t *c, const uint16_t *lab, int img, int H, int W, int ntx,
                                               int ntiles, int y, int x, const int *parent, const uint8_t *sroot) {
    if ((unsigned)y >= (unsigned)H || (unsigned)x >= (unsigned)W) return 0;
    const uint8_t v = c[(size_t)y * W + x];
    if (v == 2) return 1;
    if (v != 0) return 0;
    return sroot[parent[gid_of(lab, img, H, W, ntx, ntiles, y, x)]];
}

// The tile's own pixels resolve "maybe" through an LDS bit per local root (one global
// parent/sroot lookup per root instead of per pixel); only the 1-pixel ring of
// neighbouring tiles' pixels goes through the global tables.
__global__ __launch_bounds__(NT) void k_ccl_dilate(const uint8_t *__restrict__ cls, const uint16_t *__restrict__ lab,
                                                    int H, int W, int ntx, int nty, const uint16_t *__restrict__ roots,
                                                    const int *__restrict__ nroots, const int *__restrict__ parent,
                                                    const uint8_t *__restrict__ sroot, uint64_t *__restrict__ bits,
                                                    uint8_t *__restrict__ mask_u8) {
    __shared__ __attribute__((aligned(16))) uint8_t e[EH][EWP];  // local column lx at lx + 3
    __shared__ uint32_t rs[TP / 32];
    const int tid = threadIdx.x, img = blockIdx.y, t = blockIdx.x;
    const int ntiles = ntx * nty;
    const int tx0 = (t % ntx) * TW, ty0 = (t / ntx) * TH;
    const uint8_t *c = cls + (size_t)img * H * W;
    const size_t tile = (size_t)img * ntiles + t, gbase = tile * TP;
    if (tid < TP / 32) rs[tid] = 0;
    // the tile's classes and local labels first (independent of the root lookups below)
    constexpr int NQ = TH * (TW / 4) / NT;
    const bool full = tx0 + TW <= W && (W & 3) == 0;
    uint32_t v4[NQ];
    uint2 l4[NQ];
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const int u = tid + k * NT, ly = u / (TW / 4), q = u - ly * (TW / 4), y = ty0 + ly, x = tx0 + 4 * q;
        v4[k] = 0x01010101u;
        l4[k] = make_uint2(0u, 0u);
        if (y < H) {
            if (full) {
                v4[k] = *(const uint32_t *)(c + (size_t)y * W + x);
                l4[k] = *(const uint2 *)(lab + ((size_t)img * H + y) * W + x);
            } else {
                uint32_t v = 0, l0 = 0, l1 = 0;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t cv = x + j < W ? c[(size_t)y * W + x + j] : 1u;
                    const uint32_t lv = (x + j < W && cv == 0) ? lab[((size_t)img * H + y) * W + x + j] : 0u;
                    v |= cv << (8 * j);
                    if (j < 2) l0 |= lv << (16 * j);
                    else l1 |= lv << (16 * (j - 2));
                }
                v4[k] = v;
                l4[k] = make_uint2(l0, l1);
            }
        }
    }
    __syncthreads();
    const int nr = nroots[tile];
    for (int k = tid; k < nr; k += NT) {
        const int i = roots[gbase + k];
        if (sroot[parent[gbase + i]]) atomicOr(&rs[i >> 5], 1u << (i & 31));
    }
    // ring: top / bottom rows (EW each), left / right columns (TH each)
    if (tid < 2 * EW + 2 * TH) {
        int ly, lx;
        if (tid < EW) {
            ly = 0;
            lx = tid;
        } else if (tid < 2 * EW) {
            ly = EH - 1;
            lx = tid - EW;
        } else if (tid < 2 * EW + TH) {
            ly = 1 + tid - 2 * EW;
            lx = 0;
        } else {
            ly = 1 + tid - 2 * EW - TH;
            lx = EW - 1;
        }
        e[ly][lx + 3] = edge_global(c, lab, img, H, W, ntx, ntiles, ty0 - 1 + ly, tx0 - 1 + lx, parent, sroot);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const int u = tid + k * NT, ly = u / (TW / 4), q = u - ly * (TW / 4);
        const uint32_t lv[4] = {l4[k].x & 0xFFFFu, l4[k].x >> 16, l4[k].y & 0xFFFFu, l4[k].y >> 16};
        uint32_t o = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t v = (v4[k] >> (8 * j)) & 255u;
            const uint32_t on = v == 2u ? 1u : (v == 0u ? (rs[(lv[j] >> 5) & (TP / 32 - 1)] >> (lv[j] & 31)) & 1u : 0u);
            o |= on << (8 * j);
        }
        *(uint32_t *)&e[ly + 1][4 * q + 4] = o;
    }
    __syncthreads();
    const int lane = tid & 63, wid = tid >> 6;
    const int wpr = (W + 63) / 64;
    for (int ly = wid; ly < TH; ly += NT / 64) {
        const int y = ty0 + ly, x = tx0 + lane;
        if (y >= H) break;
        bool on = false;
        if (x < W)
            on = e[ly][lane + 3] | e[ly][lane + 4] | e[ly][lane + 5] | e[ly + 1][lane + 3] | e[ly + 1][lane + 4] |
                 e[ly + 1][lane + 5] | e[ly + 2][lane + 3] | e[ly + 2][lane + 4] | e[ly + 2][lane + 5];
        const unsigned long long b = __ballot(on);
        if (bits && lane == 0) bits[((size_t)img * H + y) * wpr + (tx0 >> 6)] = b;
        if (mask_u8 && x < W) mask_u8[((size_t)img * H + y) * W + x] = on ? 255 : 0;
    }
}

}  // namespace

size_t hysteresis_ids(int n, int h, int w) { return (size_t)n * tiles_x(w) * tiles_y(h) * TP; }

hipError_t launch_hysteresis_dilate(const uint8_t *cls, int n, int h, int w, const HystWork &wk, uint64_t *bits,
                                    uint8_t *mask_u8, hipStream_t s) {
    const int ntx = tiles_x(w), nty = tiles_y(h), ntiles = ntx * nty;
    dim3 grid(ntiles, n);
    hipLaunchKernelGGL(k_ccl_local, grid, dim3(NT), 0, s, cls, h, w, ntx, nty, wk.lab, wk.parent, wk.sroot, wk.roots,
                       wk.nroots);
    hipLaunchKernelGGL(k_ccl_border, grid, dim3(128), 0, s, cls, wk.lab, h, w, ntx, nty, wk.parent);
    hipLaunchKernelGGL(k_ccl_flatten, grid, dim3(NT), 0, s, ntiles, wk.roots, wk.nroots, wk.parent, wk.sroot);
    hipLaunchKernelGGL(k_ccl_dilate, grid, dim3(NT), 0, s, cls, wk.lab, h, w, ntx, nty, wk.roots, wk.nroots,
                       wk.parent, wk.sroot, bits, mask_u8);
    return hipGetLastError();
}

}  // namespace llfe
