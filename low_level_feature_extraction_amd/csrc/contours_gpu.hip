// ShapeAnalyzer.analyze_shapes (shape pyc @L125-189) on the GPU: findContours(
// RETR_EXTERNAL, CHAIN_APPROX_SIMPLE) of the dilated Canny mask (@L140) and the
// per-contour geometry of the loop @L144-181 (contourArea, boundingRect, arcLength,
// approxPolyDP at 0.02 / 0.04 x perimeter, convex-hull area of detect_border_radius
// @L32-61), with the same contour set, order and vertices as OpenCV's sequential
// Suzuki-Abe scan (restated on the host in contours.cpp and in oracle/llfe_oracle.c).
//
// OpenCV's scan is sequential: a border is followed when the raster scan meets an
// unmarked foreground pixel after a background pixel and the last border mark it
// passed on that row (lnbd) is a right-bound mark or the frame.  The marks a border
// following leaves depend only on the followed component (they are its own pixels,
// and the final mark of a pixel is "right bound" if any visit marked it so, else
// "visited"), so the work splits into:
//
//   k_ct_local / k_ct_border / k_ct_flatten   8-connected components of the mask,
//              union-find over raster keys: the root of a component is its first pixel
//              in raster order, which is where OpenCV would start its outer border
//   k_ct_collect   one record per component, first-pixel bitmap F
//   k_ct_trace     every component's outer border followed from its first pixel, one
//                  thread each (count pass, then vertices + marks + area + bbox)
//   k_ct_scan      one wave per image replays the raster scan row by row on bit planes:
//                  64 lanes evaluate a 4096-pixel window at once (events and lnbd as a
//                  wave scan), decide which first pixels start a border, and follow the
//                  rare borders OpenCV starts elsewhere (inside a component whose
//                  right-bound mark sits on the left wall of a hole) serially
//   k_ct_bases / k_ct_shapes   reversed start order, area >= 100 filter, one wave per
//                  kept contour: perimeter, Douglas-Peucker counts, hull area
//
// Every floating-point quantity is exact or computed in OpenCV's order: areas are
// integer shoelace sums, segment lengths are float sqrt of integers (double sqrt then
// float rounding is the correctly rounded float sqrt for integers < 2^26), their sum in
// double is exact in any order (all partial sums fit in 53 bits), and the
// Douglas-Peucker distances are exact integer products in double.
#include <algorithm>

#include "../../include/llfe.h"
#include "llfe_internal.h"

namespace llfe {
namespace {

constexpr int TW = kTileW, TH = kTileH, TP = TW * TH;
constexpr int NT = 256;
constexpr uint8_t kUndecided = 0, kAccepted = 1, kRejected = 2;
constexpr int kRejBoxes = 64;     // rejected-component boxes kept in LDS by k_ct_scan
constexpr int kDpStack = 512;     // Douglas-Peucker slice stack (pairs)
constexpr int kPtsLds = 1024;     // contours up to this many vertices are staged in LDS
constexpr int kHullCols = kCtMaxWidth;  // widest contour bbox the hull pass handles

__constant__ int kDX[8] = {1, 1, 0, -1, -1, -1, 0, 1};
__constant__ int kDY[8] = {0, -1, -1, -1, 0, 1, 1, 1};

struct Geo {
    int H, W, wpr, ntx, ntiles, n;
};

// raster key (y * W + x) <-> tile-major id of the same pixel
__device__ __forceinline__ int64_t gid_of_key(const Geo &g, int img, int key) {
    const int y = key / g.W, x = key - y * g.W;
    const int t = (y / TH) * g.ntx + (x >> 6);
    return ((int64_t)img * g.ntiles + t) * TP + (y % TH) * TW + (x & 63);
}

__device__ __forceinline__ int k_find(const Geo &g, int img, const int *P, int a) {
    for (;;) {
        const int p = __hip_atomic_load(P + gid_of_key(g, img, a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p == a) return a;
        a = p;
    }
}

__device__ __forceinline__ void k_union(const Geo &g, int img, int *P, int a, int b) {
    for (;;) {
        a = k_find(g, img, P, a);
        b = k_find(g, img, P, b);
        if (a == b) return;
        if (a > b) {
            const int t = a;
            a = b;
            b = t;
        }
        const int old = atomicMin(P + gid_of_key(g, img, b), a);
        if (old == b) return;
        b = old;
    }
}

__device__ __forceinline__ int lds_find(int *L, int a) {
    for (;;) {
        const int p = __hip_atomic_load(L + a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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
            const int t = a;
            a = b;
            b = t;
        }
        const int old = atomicMin(L + b, a);
        if (old == b) return;
        b = old;
    }
}

// ---------------------------------------------------------------- components
// per 64x32 tile: LDS union-find; the local root (smallest tile index) is the
// component's first pixel within the tile.  P[tile root] = its raster key.
__global__ __launch_bounds__(NT) void k_ct_local(const uint64_t *__restrict__ bits, Geo g, uint16_t *__restrict__ lab,
                                                 int *__restrict__ P, uint16_t *__restrict__ roots,
                                                 int *__restrict__ nroots) {
    __shared__ int L[TP];
    __shared__ uint64_t rows[TH];
    __shared__ int cnt, s_any;
    const int tid = threadIdx.x;
    for (int64_t tt = blockIdx.x; tt < (int64_t)g.ntiles * g.n; tt += gridDim.x) {
    const int img = (int)(tt / g.ntiles), t = (int)(tt % g.ntiles);
    const int tx = t % g.ntx, ty0 = (t / g.ntx) * TH, tx0 = tx * TW;
    if (tid < TH) rows[tid] = ty0 + tid < g.H ? bits[((size_t)img * g.H + ty0 + tid) * g.wpr + tx] : 0ull;
    if (tid == 0) cnt = 0;
    __syncthreads();
    if (tid < 64) {  // empty tile (most of an edge mask): no roots
        const bool any = __any(tid < TH && rows[tid] != 0ull);
        if (tid == 0) s_any = any;
    }
    __syncthreads();
    if (!s_any) {
        if (tid == 0) nroots[(size_t)img * g.ntiles + t] = 0;
        continue;
    }
    bool on[TP / NT];
#pragma unroll
    for (int k = 0; k < TP / NT; k++) {
        const int i = tid + k * NT;
        on[k] = (rows[i >> 6] >> (i & 63)) & 1ull;
        L[i] = on[k] ? i : -1;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < TP / NT; k++) {
        if (!on[k]) continue;
        const int i = tid + k * NT, ly = i >> 6, lx = i & 63;
        if (lx > 0 && L[i - 1] >= 0) lds_union(L, i, i - 1);
        if (ly > 0) {
            if (lx > 0 && L[i - 65] >= 0) lds_union(L, i, i - 65);
            if (L[i - 64] >= 0) lds_union(L, i, i - 64);
            if (lx < 63 && L[i - 63] >= 0) lds_union(L, i, i - 63);
        }
    }
    __syncthreads();
    const size_t gbase = ((size_t)img * g.ntiles + t) * TP;
#pragma unroll
    for (int k = 0; k < TP / NT; k++) {
        if (!on[k]) continue;
        const int i = tid + k * NT, y = ty0 + (i >> 6), x = tx0 + (i & 63);
        const int r = lds_find(L, i);
        lab[((size_t)img * g.H + y) * g.W + x] = (uint16_t)r;
        if (r == i) {
            P[gbase + i] = y * g.W + x;
            roots[gbase + atomicAdd(&cnt, 1)] = (uint16_t)i;
        }
    }
    __syncthreads();
    if (tid == 0) nroots[(size_t)img * g.ntiles + t] = cnt;
    __syncthreads();
    }
}

__device__ __forceinline__ int root_key_of_pixel(const Geo &g, const uint16_t *lab, int img, int y, int x) {
    const int l = lab[((size_t)img * g.H + y) * g.W + x];
    const int ty0 = (y / TH) * TH, tx0 = x & ~63;
    return (ty0 + (l >> 6)) * g.W + tx0 + (l & 63);
}

__device__ __forceinline__ bool bit_at(const uint64_t *b, const Geo &g, int img, int y, int x) {
    if ((unsigned)y >= (unsigned)g.H || (unsigned)x >= (unsigned)g.W) return false;
    return (b[((size_t)img * g.H + y) * g.wpr + (x >> 6)] >> (x & 63)) & 1ull;
}

// grid (ntiles, n): threads 0..31 the tile's right column (look east), 32..95 its
// bottom row (look south)
__global__ __launch_bounds__(128) void k_ct_border(const uint64_t *__restrict__ bits, Geo g,
                                                   const uint16_t *__restrict__ lab, const int *__restrict__ nroots,
                                                   int *__restrict__ P) {
    const int tid = threadIdx.x;
    for (int64_t tt = blockIdx.x; tt < (int64_t)g.ntiles * g.n; tt += gridDim.x) {
    const int img = (int)(tt / g.ntiles), t = (int)(tt % g.ntiles);
    if (!nroots[tt]) continue;  // no foreground in the tile
    const int tx0 = (t % g.ntx) * TW, ty0 = (t / g.ntx) * TH;
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
    if (!bit_at(bits, g, img, y, x)) continue;
    const int a = root_key_of_pixel(g, lab, img, y, x);
    for (int dy = -1; dy <= 1; dy++)
        for (int dx = -1; dx <= 1; dx++) {
            if (!dx && !dy) continue;
            const int yy = y + dy, xx = x + dx;
            if (tid < TH ? dx != 1 : dy != 1) continue;
            if (yy / TH == y / TH && (xx >> 6) == (x >> 6)) continue;
            if (!bit_at(bits, g, img, yy, xx)) continue;
            k_union(g, img, P, a, root_key_of_pixel(g, lab, img, yy, xx));
        }
    }
}

__global__ __launch_bounds__(NT) void k_ct_flatten(Geo g, const uint16_t *__restrict__ roots,
                                                    const int *__restrict__ nroots, int *__restrict__ P) {
    for (int64_t tt = blockIdx.x; tt < (int64_t)g.ntiles * g.n; tt += gridDim.x) {
        const int n = nroots[tt];
        if (!n) continue;
        const int img = (int)(tt / g.ntiles), t = (int)(tt % g.ntiles);
        const size_t gbase = (size_t)tt * TP;
        const int tx0 = (t % g.ntx) * TW, ty0 = (t / g.ntx) * TH;
        for (int k = threadIdx.x; k < n; k += NT) {
            const int l = roots[gbase + k];
            const int key = (ty0 + (l >> 6)) * g.W + tx0 + (l & 63);
            const int r = k_find(g, img, P, key);
            if (r != key) P[gbase + l] = r;
        }
    }
}

// every tile root -> -(slot + 1) of its component: a pixel's slot is two loads
__global__ __launch_bounds__(NT) void k_ct_finalize(Geo g, const uint16_t *__restrict__ roots,
                                                     const int *__restrict__ nroots, int *__restrict__ P) {
    for (int64_t tt = blockIdx.x; tt < (int64_t)g.ntiles * g.n; tt += gridDim.x) {
        const int n = nroots[tt];
        if (!n) continue;
        const int img = (int)(tt / g.ntiles);
        const size_t gbase = (size_t)tt * TP;
        for (int k = threadIdx.x; k < n; k += NT) {
            const int l = roots[gbase + k];
            const int v = P[gbase + l];
            if (v >= 0) P[gbase + l] = P[gid_of_key(g, img, v)];
        }
    }
}

// global roots -> component records; P[root] = -(slot + 1); F bit at the first pixel
__global__ __launch_bounds__(NT) void k_ct_collect(Geo g, const uint16_t *__restrict__ roots,
                                                    const int *__restrict__ nroots, int *__restrict__ P,
                                                    CtComp *__restrict__ comps, uint8_t *__restrict__ acc,
                                                    uint64_t *__restrict__ fplane, CtCounters *__restrict__ ctr,
                                                    int *__restrict__ img_info, int64_t comp_cap) {
    for (int64_t tt = blockIdx.x; tt < (int64_t)g.ntiles * g.n; tt += gridDim.x) {
    const int n = nroots[tt];
    if (!n) continue;
    const int img = (int)(tt / g.ntiles), t = (int)(tt % g.ntiles);
    const size_t gbase = (size_t)tt * TP;
    const int tx0 = (t % g.ntx) * TW, ty0 = (t / g.ntx) * TH;
    for (int k = threadIdx.x; k < n; k += NT) {
        const int l = roots[gbase + k];
        const int key = (ty0 + (l >> 6)) * g.W + tx0 + (l & 63);
        if (P[gbase + l] != key) continue;
        const unsigned slot = atomicAdd(&ctr->comps, 1u);
        atomicAdd(&img_info[img * kCtInfo + 0], 1);
        if (slot >= comp_cap) {
            atomicOr(&ctr->flags, kCtOverflowComps);
            continue;
        }
        P[gbase + l] = -(int)slot - 1;
        CtComp c;
        c.key = key;
        c.img = img;
        c.nv = 0;
        c.off = 0;
        c.area2 = 0;
        c.x0 = c.y0 = c.x1 = c.y1 = 0;
        comps[slot] = c;
        acc[slot] = kUndecided;
        const int y = ty0 + (l >> 6), x = tx0 + (l & 63);
        atomicOr((unsigned long long *)&fplane[((size_t)img * g.H + y) * g.wpr + (x >> 6)], 1ull << (x & 63));
    }
    }
}

__device__ __forceinline__ int slot_of_pixel(const Geo &g, const uint16_t *lab, const int *P, int img, int y, int x) {
    const int l = lab[((size_t)img * g.H + y) * g.W + x];
    const int t = (y / TH) * g.ntx + (x >> 6);
    return -P[((size_t)img * g.ntiles + t) * TP + l] - 1;  // k_ct_finalize: every tile root holds -(slot + 1)
}

// ---------------------------------------------------------------- border following
// Suzuki-Abe outer border from (x0, y0) as OpenCV's icvFetchContour (see
// contours.cpp trace_outer): 3x3 neighbourhood as an 8-bit mask per step.
__device__ __forceinline__ uint32_t row3(const uint64_t *b, const Geo &g, int img, int y, int x) {
    // bits (x-1, x, x+1) of row y as bits 0..2
    if ((unsigned)y >= (unsigned)g.H) return 0;
    const uint64_t *r = b + ((size_t)img * g.H + y) * g.wpr;
    const int q = x >> 6, s = x & 63;
    const uint64_t w = r[q];
    uint32_t v = (uint32_t)((w >> s) & 1ull) << 1;
    if (s > 0) v |= (uint32_t)((w >> (s - 1)) & 1ull);
    else if (q > 0) v |= (uint32_t)(r[q - 1] >> 63);
    if (s < 63) {
        if (x + 1 < g.W) v |= (uint32_t)((w >> (s + 1)) & 1ull) << 2;
    } else if (q + 1 < g.wpr) {
        v |= (uint32_t)(r[q + 1] & 1ull) << 2;
    }
    return v;
}

// neighbour mask: bit s = pixel in chain direction s is foreground
__device__ __forceinline__ uint32_t nbhd(const uint64_t *b, const Geo &g, int img, int x, int y) {
    const uint32_t up = row3(b, g, img, y - 1, x), mid = row3(b, g, img, y, x), dn = row3(b, g, img, y + 1, x);
    // directions: 0 E, 1 NE, 2 N, 3 NW, 4 W, 5 SW, 6 S, 7 SE
    return ((mid >> 2) & 1u) | (((up >> 2) & 1u) << 1) | (((up >> 1) & 1u) << 2) | ((up & 1u) << 3) |
           ((mid & 1u) << 4) | ((dn & 1u) << 5) | (((dn >> 1) & 1u) << 6) | (((dn >> 2) & 1u) << 7);
}

struct TraceCount {
    uint32_t nv = 0;
    __device__ void vertex(int, int) { nv++; }
    __device__ void mark(int, int, bool) {}
};

struct TraceWrite {
    int2 *pts;          // vertex destination (capacity cap)
    uint64_t *mv, *mn;  // mark planes of the image (row stride wpr), null: no marks
    int wpr;
    bool on;            // this lane stores (the wave traces redundantly, lane 0 writes)
    uint32_t cap;
    uint32_t nv = 0;
    int fx = 0, fy = 0, px = 0, py = 0;
    int64_t a2 = 0;
    int x0 = 1 << 30, y0 = 1 << 30, x1 = -1, y1 = -1;
    int my = -1, mq = -1;  // marks of one 64-pixel word are OR-ed once per visit of the word
    unsigned long long bv = 0, bn = 0;
    __device__ void vertex(int x, int y) {
        if (on && nv < cap) pts[nv] = make_int2(x, y);
        if (nv == 0) {
            fx = x;
            fy = y;
        } else {
            a2 += (int64_t)px * y - (int64_t)py * x;
        }
        px = x;
        py = y;
        x0 = min(x0, x);
        y0 = min(y0, y);
        x1 = max(x1, x);
        y1 = max(y1, y);
        nv++;
    }
    __device__ void flush() {
        if (on && mv && bv) {
            const size_t w = (size_t)my * wpr + mq;
            atomicOr((unsigned long long *)&mv[w], bv);
            if (bn) atomicOr((unsigned long long *)&mn[w], bn);
        }
        bv = bn = 0;
    }
    __device__ void mark(int x, int y, bool right) {
        if (y != my || (x >> 6) != mq) {
            flush();
            my = y;
            mq = x >> 6;
        }
        const unsigned long long b = 1ull << (x & 63);
        bv |= b;
        if (right) bn |= b;
    }
    __device__ void close() {
        a2 += (int64_t)px * fy - (int64_t)py * fx;
        flush();
    }
};

// neighbourhood providers: straight from the bit planes (one thread), or from a
// 64-row x 256-pixel window of them that the whole wave stages in LDS (all lanes run
// the trace in lockstep; a step that leaves the window -> one cooperative reload), with
// the 3 x 3 words around the current word cached in registers
struct NbGlobal {
    const uint64_t *b;
    const Geo &g;
    int img;
    __device__ uint32_t operator()(int x, int y) { return nbhd(b, g, img, x, y); }
};

constexpr int kWinRows = 64, kWinWords = 4;
// wave-uniform copies (the trace state then lives in SGPRs and runs on the scalar ALU)
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return ((uint64_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}
struct NbWindow {
    const uint64_t *b;
    const Geo &g;
    int img, lane;
    uint64_t *win;  // kWinRows x kWinWords
    int wy0 = -(1 << 30), wq0 = 0;
    int cy = -(1 << 30), cq = 0;
    uint64_t r0[3] = {0, 0, 0}, r1[3] = {0, 0, 0}, r2[3] = {0, 0, 0};  // rows cy-1..cy+1 x words cq-1..cq+1
    __device__ void reload(int q, int y) {
        wy0 = y - kWinRows / 2;
        wq0 = q - 1;
        __syncthreads();
        const int row = wy0 + lane;
        const bool rin = (unsigned)row < (unsigned)g.H;
        const uint64_t *r = b + ((size_t)img * g.H + (rin ? row : 0)) * g.wpr;
#pragma unroll
        for (int k = 0; k < kWinWords; k++) {
            const int qq = wq0 + k;
            win[lane * kWinWords + k] = (rin && (unsigned)qq < (unsigned)g.wpr) ? r[qq] : 0ull;
        }
        __syncthreads();
    }
    __device__ static uint32_t bits3(const uint64_t *r, int s) {  // (x-1, x, x+1) as bits 0..2
        uint32_t v = (uint32_t)((r[1] >> s) & 1ull) << 1;
        v |= s > 0 ? (uint32_t)((r[1] >> (s - 1)) & 1ull) : (uint32_t)(r[0] >> 63);
        v |= (s < 63 ? (uint32_t)((r[1] >> (s + 1)) & 1ull) : (uint32_t)(r[2] & 1ull)) << 2;
        return v;
    }
    __device__ uint32_t operator()(int x, int y) {
        const int q = x >> 6;
        if (y != cy || q != cq) {
            if (y - 1 < wy0 || y + 1 >= wy0 + kWinRows || q - 1 < wq0 || q + 1 >= wq0 + kWinWords) reload(q, y);
            const uint64_t *w = win + (y - 1 - wy0) * kWinWords + (q - 1 - wq0);
#pragma unroll
            for (int k = 0; k < 3; k++) {
                r0[k] = uni64(w[k]);
                r1[k] = uni64(w[kWinWords + k]);
                r2[k] = uni64(w[2 * kWinWords + k]);
            }
            cy = y;
            cq = q;
        }
        const int s = x & 63;
        const uint32_t up = bits3(r0, s), mid = bits3(r1, s), dn = bits3(r2, s);
        return ((mid >> 2) & 1u) | (((up >> 2) & 1u) << 1) | (((up >> 1) & 1u) << 2) | ((up & 1u) << 3) |
               ((mid & 1u) << 4) | ((dn & 1u) << 5) | (((dn >> 1) & 1u) << 6) | (((dn >> 2) & 1u) << 7);
    }
};

// returns false when the step bound is hit (malformed input; never for a real border)
template <class NB, class F>
__device__ bool trace_outer(NB &nbh, const Geo &g, int x0, int y0, F &f) {
    uint32_t nb = nbh(x0, y0);
    int s = 4;
    do {
        s = (s - 1) & 7;
    } while (!((nb >> s) & 1u) && s != 4);
    if (s == 4 && !((nb >> 4) & 1u)) {  // isolated pixel
        f.mark(x0, y0, true);
        f.vertex(x0, y0);
        return true;
    }
    const int x1 = x0 + kDX[s], y1 = y0 + kDY[s];
    int x3 = x0, y3 = y0, prev_s = s ^ 4;
    const int64_t limit = 8ll * g.H * g.W + 16;
    for (int64_t it = 0; it < limit; it++) {
        const int s_end = s;
        nb = nbh(x3, y3);
        // counter-clockwise search from s_end + 1 (OpenCV: while (s < 15) i4 = i3 + d[++s])
        const uint32_t nb2 = nb | (nb << 8);
        const uint32_t cand = (nb2 >> (s_end + 1)) & ((1u << (15 - s_end)) - 1u);
        s = (s_end + 1 + (cand ? __builtin_ctz(cand) : 14 - s_end)) & 7;
        const int x4 = x3 + kDX[s], y4 = y3 + kDY[s];
        f.mark(x3, y3, (unsigned)(s - 1) < (unsigned)s_end);
        if (s != prev_s) {
            f.vertex(x3, y3);
            prev_s = s;
        }
        if (x4 == x0 && y4 == y0 && x3 == x1 && y3 == y1) return true;
        x3 = x4;
        y3 = y4;
        s = (s + 4) & 7;
    }
    return false;
}

// one wave per component, one pass: vertices go to the block's staging area (exact
// length known afterwards -> allocate -> copy), marks to the planes; a border longer
// than the staging area is followed a second time straight into its allocation
constexpr uint32_t kStage = kCtStage;
__global__ __launch_bounds__(64) void k_ct_trace(const uint64_t *__restrict__ bits, Geo g, CtComp *__restrict__ comps,
                                                  int64_t comp_cap, int2 *__restrict__ pts, int64_t pts_cap,
                                                  int2 *__restrict__ stage, uint64_t *__restrict__ mv,
                                                  uint64_t *__restrict__ mn, CtCounters *__restrict__ ctr) {
    __shared__ uint64_t win[kWinRows * kWinWords];
    __shared__ unsigned long long s_off;
    const int lane = threadIdx.x;
    const int64_t ncomp = min((int64_t)ctr->comps, comp_cap);
    int2 *st = stage + (size_t)blockIdx.x * kStage;
    for (int64_t slot = blockIdx.x; slot < ncomp; slot += gridDim.x) {
        CtComp c = comps[slot];
        c.key = (uint32_t)__builtin_amdgcn_readfirstlane((int)c.key);
        c.img = __builtin_amdgcn_readfirstlane(c.img);
        const int y = c.key / g.W, x = c.key - y * g.W;
        const size_t pb = (size_t)c.img * g.H * g.wpr;
        NbWindow nbh{bits, g, c.img, lane, win};
        TraceWrite f{st, mv + pb, mn + pb, g.wpr, lane == 0, kStage};
        const bool ok = trace_outer(nbh, g, x, y, f);
        f.close();
        if (lane == 0) {
            if (!ok) atomicOr(&ctr->flags, kCtBadTrace);
            s_off = atomicAdd(&ctr->pts, (unsigned long long)f.nv);
        }
        __threadfence();  // lane 0's staged vertices, read back by every lane below
        __syncthreads();
        const unsigned long long off = s_off;
        const bool fits = off + f.nv <= (unsigned long long)pts_cap;
        if (fits) {
            if (f.nv <= kStage) {
                for (uint32_t i = lane; i < f.nv; i += 64) {
                    const unsigned long long v = __hip_atomic_load((const unsigned long long *)(st + i),
                                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    pts[off + i] = *(const int2 *)&v;
                }
            } else {
                NbWindow nb2{bits, g, c.img, lane, win};
                TraceWrite f2{pts + off, nullptr, nullptr, g.wpr, lane == 0, f.nv};
                trace_outer(nb2, g, x, y, f2);
            }
        }
        if (lane == 0) {
            if (!fits) atomicOr(&ctr->flags, kCtOverflowPts);
            c.nv = fits ? f.nv : 0;
            c.off = fits ? (uint32_t)off : 0;
            c.area2 = f.a2;
            c.x0 = (uint16_t)f.x0;
            c.y0 = (uint16_t)f.y0;
            c.x1 = (uint16_t)f.x1;
            c.y1 = (uint16_t)f.y1;
            comps[slot] = c;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- the raster scan
struct ScanPlanes {
    const uint64_t *nz, *mv, *mn, *f;  // image base pointers (row stride wpr)
    uint64_t *qv, *qn;                 // marks of borders started away from a first pixel
};

__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the current value of pixel (x, y) is "right-bound mark" (the lnbd test), from globals
__device__ bool pix_is_right_mark(const ScanPlanes &sp, const Geo &g, const uint16_t *lab, const int *P,
                                  const uint8_t *acc, int img, int y, int x) {
    const size_t w = (size_t)y * g.wpr + (x >> 6);
    const uint64_t b = 1ull << (x & 63);
    if (!(sp.nz[w] & b)) return false;
    if (ld_relaxed(sp.qn + w) & b) return true;
    if (!(sp.mn[w] & b)) return false;
    const int slot = slot_of_pixel(g, lab, P, img, y, x);
    return __hip_atomic_load(acc + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != kRejected;
}

struct QuirkWrite {  // a border followed from a non-first pixel: marks go to the Q planes
    int2 *pts;
    uint64_t *qv, *qn;
    int wpr;
    uint32_t nv = 0;
    int fx = 0, fy = 0, px = 0, py = 0;
    int64_t a2 = 0;
    int x0 = 1 << 30, y0 = 1 << 30, x1 = -1, y1 = -1;
    __device__ void vertex(int x, int y) {
        pts[nv] = make_int2(x, y);
        if (nv == 0) {
            fx = x;
            fy = y;
        } else {
            a2 += (int64_t)px * y - (int64_t)py * x;
        }
        px = x;
        py = y;
        x0 = min(x0, x);
        y0 = min(y0, y);
        x1 = max(x1, x);
        y1 = max(y1, y);
        nv++;
    }
    __device__ void mark(int x, int y, bool right) {
        const size_t w = (size_t)y * wpr + (x >> 6);
        const unsigned long long b = 1ull << (x & 63);
        atomicOr((unsigned long long *)&qv[w], b);
        if (right) atomicOr((unsigned long long *)&qn[w], b);
    }
    __device__ void close() { a2 += (int64_t)px * fy - (int64_t)py * fx; }
};

__device__ __forceinline__ int wave_min(int v) {
    for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_max(int v) {
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_excl_max(int v, int lane) {  // max over lanes < lane (-1 if none)
    int x = __shfl_up(v, 1);
    if (lane == 0) x = -1;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x = max(x, y);
    }
    return x;
}
__device__ __forceinline__ int wave_excl_sum(int v, int lane) {
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    return x - v;
}

// one 64-lane workgroup per image: replays OpenCV's RETR_EXTERNAL raster scan
// (contours.cpp scan_external) and writes the image's contours in start order
__global__ __launch_bounds__(64) void k_ct_scan(const uint64_t *__restrict__ bits, Geo g,
                                                 const uint16_t *__restrict__ lab, const int *__restrict__ P,
                                                 uint64_t *__restrict__ planes, size_t plane_stride,
                                                 CtComp *__restrict__ comps, int64_t comp_cap,
                                                 uint8_t *__restrict__ acc, int2 *__restrict__ pts, int64_t pts_cap,
                                                 int2 *__restrict__ refs, int64_t ref_cap,
                                                 CtCounters *__restrict__ ctr, int *__restrict__ img_info) {
    __shared__ uint64_t s_vn[64];
    __shared__ int s_rej_n;
    __shared__ ushort4 s_rej[kRejBoxes];
    __shared__ int s_bcast[4];
    const int img = blockIdx.x, lane = threadIdx.x;
    const size_t ib = (size_t)img * g.H * g.wpr;
    ScanPlanes sp{bits + ib, planes + 0 * plane_stride + ib, planes + 1 * plane_stride + ib,
                  planes + 4 * plane_stride + ib, planes + 2 * plane_stride + ib, planes + 3 * plane_stride + ib};
    if (ctr->flags & (kCtOverflowComps | kCtOverflowPts)) return;
    const int ncomp = img_info[img * kCtInfo + 0];
    const int cap_img = ncomp + kCtQuirkCap;
    int base = 0;
    if (lane == 0) {
        base = (int)atomicAdd(&ctr->refs, (unsigned)cap_img);
        s_rej_n = 0;
    }
    base = __shfl(base, 0);
    if ((int64_t)base + cap_img > ref_cap) {
        if (lane == 0) atomicOr(&ctr->flags, kCtOverflowRefs);
        return;
    }
    __syncthreads();
    int nref = 0;
    bool any_quirk = false;  // Q planes are all zero until a border starts off a first pixel
    // the first window of row y + 1 is loaded while row y is scanned
    const bool v0 = lane >= 1 && lane - 1 < g.wpr;
    const size_t o0 = v0 ? lane - 1 : 0;
    uint64_t n_nz = v0 ? sp.nz[o0] : 0ull, n_mv = v0 ? sp.mv[o0] : 0ull, n_mn = v0 ? sp.mn[o0] : 0ull,
             n_fb = v0 ? sp.f[o0] : 0ull;
    for (int y = 0; y < g.H; y++) {
        int lnbd = -1;  // pixel position (x) of lnbd on this row, -1 = frame
        int seg = 0;    // first pixel position not yet scanned
        const uint64_t c_nz = n_nz, c_mv = n_mv, c_mn = n_mn, c_fb = n_fb;
        if (y + 1 < g.H) {
            const size_t o = (size_t)(y + 1) * g.wpr + o0;
            n_nz = v0 ? sp.nz[o] : 0ull;
            n_mv = v0 ? sp.mv[o] : 0ull;
            n_mn = v0 ? sp.mn[o] : 0ull;
            n_fb = v0 ? sp.f[o] : 0ull;
        }
        for (int w0 = 0; w0 < g.wpr; w0 += 63) {
            const int wk = w0 - 1 + lane;  // lane 0 holds the word left of the window
            const bool valid = wk >= 0 && wk < g.wpr;
            const size_t wi = (size_t)y * g.wpr + (valid ? wk : 0);
            const uint64_t nz = w0 == 0 ? c_nz : (valid ? sp.nz[wi] : 0ull);
            if (!__any(nz != 0ull)) {
                seg = (w0 + 63) * 64;
                continue;
            }
            const uint64_t mv = w0 == 0 ? c_mv : (valid ? sp.mv[wi] : 0ull);
            const uint64_t mn = w0 == 0 ? c_mn : (valid ? sp.mn[wi] : 0ull);
            const uint64_t fb = w0 == 0 ? c_fb : (valid ? sp.f[wi] : 0ull);
            const int wpos = wk * 64;
            for (;;) {
                uint64_t qv = 0ull, qn = 0ull;
                if (any_quirk && valid) {
                    qv = ld_relaxed(sp.qv + wi);
                    qn = ld_relaxed(sp.qn + wi);
                }
                // marks of rejected components are not live
                uint64_t live = ~0ull;
                const int nrej = s_rej_n;
                if (nrej > 0 && ((mv | mn) & nz)) {
                    bool hit = nrej > kRejBoxes;
                    for (int r = 0; r < nrej && r < kRejBoxes && !hit; r++) {
                        const ushort4 bx = s_rej[r];
                        hit = y >= bx.y && y <= bx.w && wpos + 63 >= bx.x && wpos <= bx.z;
                    }
                    if (hit) {
                        uint64_t runs = nz & ~(nz << 1);  // run starts
                        while (runs) {
                            const int s0 = __builtin_ctzll(runs);
                            const uint64_t above = (s0 == 0) ? ~0ull : ~((1ull << s0) - 1ull);
                            const uint64_t holes = ~nz & above;
                            const uint64_t run = holes ? (above & ((holes & (~holes + 1)) - 1ull)) : above;
                            runs &= ~run;
                            if (!((mv | mn) & run)) continue;
                            const int slot = slot_of_pixel(g, lab, P, img, y, wpos + s0);
                            if (__hip_atomic_load(acc + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kRejected)
                                live &= ~run;
                        }
                    }
                }
                const uint64_t vn = nz & ((mn & live) | qn);
                const uint64_t v2 = nz & ~vn & ((mv & live) | qv);
                const uint64_t v1 = nz & ~vn & ~v2;
                s_vn[lane] = vn;
                const uint64_t unz = __shfl_up(nz, 1), uvn = __shfl_up(vn, 1), uv2 = __shfl_up(v2, 1);
                const uint64_t pnz = (nz << 1) | (lane ? unz >> 63 : 0ull);
                const uint64_t pvn = (vn << 1) | (lane ? uvn >> 63 : 0ull);
                const uint64_t pv2 = (v2 << 1) | (lane ? uv2 >> 63 : 0ull);
                uint64_t segm = 0ull;
                if (wpos + 64 <= seg) segm = 0ull;
                else if (wpos >= seg) segm = ~0ull;
                else segm = ~0ull << (seg - wpos);
                if (!valid) segm = 0ull;
                const uint64_t e1 = ((vn & ~pvn) | (v2 & ~pv2)) & ~fb & segm;
                const uint64_t e2 = ~nz & pv2 & segm;
                const uint64_t ev = e1 | e2;
                const uint64_t q = nz & ~pnz & (v1 | fb) & segm;
                int lastev = -1;
                if (ev) {
                    const int e = 63 - __builtin_clzll(ev);
                    lastev = wpos + e - (int)((e2 >> e) & 1ull);
                }
                int prior = wave_excl_max(lastev, lane);
                if (prior < 0) prior = lnbd;
                __syncthreads();
                // start test at every query pixel
                uint64_t start = 0ull, qq = q;
                while (qq) {
                    const int bq = __builtin_ctzll(qq);
                    qq &= qq - 1;
                    const uint64_t below = ev & ((1ull << bq) - 1ull);
                    int L = prior;
                    if (below) {
                        const int e = 63 - __builtin_clzll(below);
                        L = wpos + e - (int)((e2 >> e) & 1ull);
                    }
                    bool st;
                    if (L < 0) st = true;
                    else if (L >= (w0 - 1) * 64) st = (s_vn[(L >> 6) - (w0 - 1)] >> (L & 63)) & 1ull;
                    else st = pix_is_right_mark(sp, g, lab, P, acc, img, y, L);
                    if (st) start |= 1ull << bq;
                }
                const uint64_t rej = q & fb & ~start, quirk = q & ~fb & start;
                uint64_t accm = q & fb & start;
                const uint64_t brk = rej | quirk;
                const int bpos = wave_min(brk ? wpos + __builtin_ctzll(brk) : 0x7fffffff);
                if (bpos != 0x7fffffff) {
                    const int rel = bpos - wpos;
                    if (rel <= 0) accm = 0ull;
                    else if (rel < 64) accm &= (1ull << rel) - 1ull;
                }
                // accepted first pixels left of the break, in order
                const int cnt = __popcll(accm);
                const int pre = wave_excl_sum(cnt, lane);
                const int tot = __shfl(pre + cnt, 63);
                if (nref + tot > cap_img) {
                    if (lane == 0) atomicOr(&ctr->flags, kCtOverflowRefs);
                    return;
                }
                int j = 0;
                while (accm) {
                    const int bq = __builtin_ctzll(accm);
                    accm &= accm - 1;
                    const int slot = slot_of_pixel(g, lab, P, img, y, wpos + bq);
                    __hip_atomic_store(acc + slot, kAccepted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    refs[base + nref + pre + j] = make_int2(slot, -1);
                    j++;
                }
                nref += tot;
                if (bpos == 0x7fffffff) {  // window done
                    const int le = wave_max(lastev);
                    if (le >= 0) lnbd = le;
                    seg = (w0 + 63) * 64;
                    break;
                }
                // the break pixel's lane: lnbd before it, then reject or follow
                const int owner = (bpos >> 6) - (w0 - 1);
                if (lane == owner) {
                    const int bq = bpos & 63;
                    const uint64_t below = ev & ((1ull << bq) - 1ull);
                    int L = prior;
                    if (below) {
                        const int e = 63 - __builtin_clzll(below);
                        L = wpos + e - (int)((e2 >> e) & 1ull);
                    }
                    s_bcast[0] = L;
                    if ((rej >> bq) & 1ull) {
                        const int slot = slot_of_pixel(g, lab, P, img, y, bpos);
                        __hip_atomic_store(acc + slot, kRejected, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const CtComp c = comps[slot];
                        if (s_rej_n < kRejBoxes) s_rej[s_rej_n] = make_ushort4(c.x0, c.y0, c.x1, c.y1);
                        s_rej_n = s_rej_n + 1;
                        s_bcast[1] = 0;
                    } else {
                        s_bcast[1] = 1;
                        // a border started away from a component's first pixel
                        TraceCount fc;
                        NbGlobal nbg{bits, g, img};
                        bool ok = trace_outer(nbg, g, bpos, y, fc);
                        const unsigned slot = atomicAdd(&ctr->comps, 1u);
                        const unsigned long long off = atomicAdd(&ctr->pts, (unsigned long long)fc.nv);
                        if (!ok) atomicOr(&ctr->flags, kCtBadTrace);
                        if (slot >= comp_cap || off + fc.nv > (unsigned long long)pts_cap || nref >= cap_img) {
                            atomicOr(&ctr->flags, slot >= comp_cap ? kCtOverflowComps
                                                                   : (nref >= cap_img ? kCtOverflowRefs : kCtOverflowPts));
                            s_bcast[1] = -1;
                        } else {
                            QuirkWrite fw{pts + off, sp.qv, sp.qn, g.wpr};
                            trace_outer(nbg, g, bpos, y, fw);
                            fw.close();
                            CtComp c;
                            c.key = y * g.W + bpos;
                            c.img = img;
                            c.nv = fw.nv;
                            c.off = (uint32_t)off;
                            c.area2 = fw.a2;
                            c.x0 = (uint16_t)fw.x0;
                            c.y0 = (uint16_t)fw.y0;
                            c.x1 = (uint16_t)fw.x1;
                            c.y1 = (uint16_t)fw.y1;
                            comps[slot] = c;
                            acc[slot] = kAccepted;
                            refs[base + nref] = make_int2((int)slot, -1);
                            __threadfence();
                        }
                    }
                }
                __syncthreads();
                lnbd = s_bcast[0];
                const int kind = s_bcast[1];
                if (kind < 0) return;
                if (kind == 1) {
                    nref++;
                    any_quirk = true;
                    atomicAdd(&ctr->quirks, 1u);
                }
                seg = bpos + 1;
                __syncthreads();
            }
        }
    }
    // shapes are listed newest contour first, contourArea >= 100 (|2A| >= 200)
    __threadfence();
    __syncthreads();
    int kept = 0;
    for (int c0 = 0; c0 < nref; c0 += 64) {
        const int idx = nref - 1 - (c0 + lane);
        bool keep = false;
        int2 r = make_int2(0, -1);
        if (idx >= 0) {  // written by this wave: coherent loads
            r.x = __hip_atomic_load(&refs[base + idx].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int64_t a2 = __hip_atomic_load(&comps[r.x].area2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            keep = (a2 < 0 ? -a2 : a2) >= 200;
        }
        const uint64_t bal = __ballot(keep);
        const int before = __popcll(bal & ((1ull << lane) - 1ull));
        if (idx >= 0) refs[base + idx] = make_int2(r.x, keep ? kept + before : -1);
        kept += __popcll(bal);
    }
    if (lane == 0) {
        img_info[img * kCtInfo + 1] = base;
        img_info[img * kCtInfo + 2] = nref;
        img_info[img * kCtInfo + 3] = kept;
    }
}

// exclusive scan of the kept counts over images -> shape base per image
__global__ __launch_bounds__(1024) void k_ct_bases(int n, int *__restrict__ img_info, CtCounters *__restrict__ ctr,
                                                    int64_t shape_cap) {
    __shared__ int s[1024];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int c0 = 0; c0 < n; c0 += 1024) {
        const int i = c0 + threadIdx.x;
        const int v = i < n ? img_info[i * kCtInfo + 3] : 0;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const int add = (int)threadIdx.x >= o ? s[threadIdx.x - o] : 0;
            __syncthreads();
            s[threadIdx.x] += add;
            __syncthreads();
        }
        if (i < n) img_info[i * kCtInfo + 4] = carry + s[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += s[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        ctr->shapes = (unsigned)carry;
        if (carry > shape_cap) atomicOr(&ctr->flags, kCtOverflowShapes);
    }
}

// ---------------------------------------------------------------- geometry
constexpr int kDpOut = 1024;  // Douglas-Peucker output points kept in LDS
struct GeoLds {  // ~49 KB: three waves per CU
    int2 stack[kDpStack];
    uint32_t dpo[kDpOut];              // Douglas-Peucker output (x << 16 | y)
    uint32_t col[kHullCols];           // per-column y extreme, then the merged hull chain
    uint32_t ch[kHullCols + 64];       // per-lane chunk chains
    int nl[64];
    int2 pts[kPtsLds];
    int flags;
};

__device__ __forceinline__ double wave_sum_d(double v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
// max of (d << 28 | (2^28 - 1 - k)): the largest d, earliest k on ties (d < 2^36, k < 2^28)
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
    for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}
constexpr uint64_t kKMask = (1ull << 28) - 1;

__device__ __forceinline__ double perimeter_of(const int2 *p, int n, int lane) {
    if (n <= 1) return 0.0;
    double s = 0.0;
    for (int i = lane; i < n; i += 64) {
        const int2 a = p[i == 0 ? n - 1 : i - 1], b = p[i];
        const int dx = b.x - a.x, dy = b.y - a.y;
        s += (double)(float)__builtin_sqrt((double)(dx * dx + dy * dy));
    }
    return wave_sum_d(s);
}

// cv::approxPolyDP(closed) vertex count, OpenCV's iterative Douglas-Peucker
// (contours.cpp dp_vertex_count): the farthest-point scans run across the wave; the
// distances are exact integers (|coordinates| < 2^16, widths < 2^12)
__device__ int dp_count(const int2 *p, int count, double eps, GeoLds &sm, int lane) {
    if (count == 0) return 0;
    eps *= eps;
    int pos = 0, rs_start = 0, sx = 0, sy = 0;
    bool le_eps = false;
    for (int it = 0; it < 3; it++) {
        pos = (pos + rs_start) % count;
        const int2 s0 = p[pos];
        sx = s0.x;
        sy = s0.y;
        uint64_t best = 0;
        for (int j = 1 + lane; j < count; j += 64) {
            int idx = pos + j;
            if (idx >= count) idx -= count;
            const int2 q = p[idx];
            const int64_t dx = q.x - sx, dy = q.y - sy, d = dx * dx + dy * dy;
            const uint64_t key = ((uint64_t)d << 28) | (kKMask - (uint64_t)j);
            if (d > 0 && key > best) best = key;
        }
        best = wave_max_u64(best);
        const uint64_t dmax = best >> 28;
        if (dmax > 0) rs_start = (int)(kKMask - (best & kKMask));
        le_eps = (double)dmax <= eps;
    }
    int nout = 0, top = 0;
    if (!le_eps) {
        const int a = pos % count, b = (rs_start + a) % count;
        if (lane == 0) {
            sm.stack[0] = make_int2(b, a);  // (sstart, send) pairs: processed last
            sm.stack[1] = make_int2(a, b);  // processed first
        }
        top = 2;
    } else {
        if (lane == 0) sm.dpo[0] = ((uint32_t)sx << 16) | (uint32_t)sy;
        nout = 1;
    }
    __syncthreads();
    while (top > 0) {
        const int2 sl = sm.stack[--top];
        const int sstart = sl.x, send = sl.y;
        const int2 e = p[send], s0 = p[sstart];
        int m = send - sstart - 1;  // points strictly between (cyclic)
        if (m < 0) m += count;
        bool ok = true;
        int split = 0;
        if (m > 0) {
            const int dx = e.x - s0.x, dy = e.y - s0.y;
            uint64_t best = 0;
            for (int j = 1 + lane; j <= m; j += 64) {
                int idx = sstart + j;
                if (idx >= count) idx -= count;
                const int2 q = p[idx];
                int64_t d = (int64_t)(q.y - s0.y) * dx - (int64_t)(q.x - s0.x) * dy;
                d = d < 0 ? -d : d;
                const uint64_t key = ((uint64_t)d << 28) | (kKMask - (uint64_t)j);
                if (d > 0 && key > best) best = key;
            }
            best = wave_max_u64(best);
            const double dmax = (double)(best >> 28);
            if (best >> 28) {
                split = sstart + (int)(kKMask - (best & kKMask));
                if (split >= count) split -= count;
            }
            ok = dmax * dmax <= eps * ((double)dx * dx + (double)dy * dy);
        }
        __syncthreads();
        if (ok) {
            if (nout >= kDpOut) {
                if (lane == 0) sm.flags |= 1;
                return 0;
            }
            if (lane == 0) sm.dpo[nout] = ((uint32_t)s0.x << 16) | (uint32_t)s0.y;
            nout++;
        } else {
            if (top + 2 > kDpStack) {
                if (lane == 0) sm.flags |= 1;
                return 0;
            }
            if (lane == 0) {
                sm.stack[top] = make_int2(split, send);
                sm.stack[top + 1] = make_int2(sstart, split);
            }
            top += 2;
        }
        __syncthreads();
    }
    __syncthreads();
    // clean-up of [almost] collinear points (closed contour), serial
    int newc = nout;
    if (lane == 0) {
        const int cnt = nout;
        uint32_t *dst = sm.dpo;
        auto X = [](uint32_t v) { return (int)(v >> 16); };
        auto Y = [](uint32_t v) { return (int)(v & 0xffffu); };
        int rp = cnt - 1;
        auto rdd = [&](int &pp, int &xx, int &yy) {
            xx = X(dst[pp]);
            yy = Y(dst[pp]);
            if (++pp >= cnt) pp = 0;
        };
        int px, py, qx, qy;
        int sx2, sy2;
        rdd(rp, sx2, sy2);
        int wpos = rp;
        rdd(rp, px, py);
        for (int i = 0; i < cnt && newc > 2; i++) {
            rdd(rp, qx, qy);
            const double dx = qx - sx2, dy = qy - sy2;
            const double d = fabs((px - sx2) * dy - (py - sy2) * dx);
            const double sip = (double)(px - sx2) * (qx - px) + (double)(py - sy2) * (qy - py);
            if (d * d <= 0.5 * eps * (dx * dx + dy * dy) && dx != 0 && dy != 0 && sip >= 0) {
                newc--;
                sx2 = qx;
                sy2 = qy;
                dst[wpos] = ((uint32_t)qx << 16) | (uint32_t)qy;
                if (++wpos >= cnt) wpos = 0;
                rdd(rp, px, py);
                i++;
                continue;
            }
            sx2 = px;
            sy2 = py;
            dst[wpos] = ((uint32_t)px << 16) | (uint32_t)py;
            if (++wpos >= cnt) wpos = 0;
            px = qx;
            py = qy;
        }
    }
    newc = __shfl(newc, 0);
    __syncthreads();
    return newc;
}

// One convex chain of the hull: UPPER = false -> the chain over each column's minimum y
// (x ascending), UPPER = true -> over each column's maximum y (x descending), both with
// Andrew's "pop while cross <= 0" rule.  Each lane first reduces its own run of columns
// to its chain (points off it cannot be on the hull), lane 0 then merges the chunks.
// Returns the chain's shoelace sum over its edges; *first / *last are its end points.
template <bool UPPER>
__device__ int64_t hull_chain(const int2 *p, int n, int x0, int width, GeoLds &sm, int lane, uint32_t *first,
                              uint32_t *last) {
    auto X = [](uint32_t v) { return (int)(v >> 16); };
    auto Y = [](uint32_t v) { return (int)(v & 0xffffu); };
    auto cross = [&](uint32_t o, uint32_t a, uint32_t b) {  // 32 x 32 -> 64-bit products
        return (int64_t)(X(a) - X(o)) * (Y(b) - Y(o)) - (int64_t)(Y(a) - Y(o)) * (X(b) - X(o));
    };
    for (int i = lane; i < width; i += 64) sm.col[i] = UPPER ? 0u : 0xffffffffu;
    __syncthreads();
    for (int i = lane; i < n; i += 64) {
        const int2 q = p[i];
        if (UPPER) atomicMax(&sm.col[q.x - x0], (uint32_t)q.y + 1u);
        else atomicMin(&sm.col[q.x - x0], (uint32_t)q.y);
    }
    __syncthreads();
    {
        const int clo = (int)((int64_t)width * lane / 64), chi = (int)((int64_t)width * (lane + 1) / 64);
        uint32_t *C = sm.ch + clo + lane;  // room for chi - clo + 1 entries
        int k = 0;
        for (int t = 0; t < chi - clo; t++) {
            const int c = UPPER ? chi - 1 - t : clo + t;
            const uint32_t v = sm.col[c];
            if (UPPER ? v == 0u : v == 0xffffffffu) continue;
            const uint32_t q = ((uint32_t)(x0 + c) << 16) | (UPPER ? v - 1u : v);
            while (k >= 2 && cross(C[k - 2], C[k - 1], q) <= 0) k--;
            C[k++] = q;
        }
        sm.nl[lane] = k;
    }
    __syncthreads();
    int64_t sum = 0;
    if (lane == 0) {
        uint32_t *H = sm.col;  // the column extremes are dead now
        int k = 0;
        uint32_t t1 = 0, t2 = 0;  // H[k - 1], H[k - 2]
        for (int li = 0; li < 64; li++) {
            const int l = UPPER ? 63 - li : li;
            const int clo = (int)((int64_t)width * l / 64);
            const uint32_t *C = sm.ch + clo + l;
            for (int j = 0, nj = sm.nl[l]; j < nj; j++) {
                const uint32_t q = C[j];
                while (k >= 2 && cross(t2, t1, q) <= 0) {
                    k--;
                    t1 = t2;
                    t2 = k >= 2 ? H[k - 2] : 0u;
                }
                H[k++] = q;
                t2 = t1;
                t1 = q;
            }
        }
        for (int i = 1; i < k; i++)
            sum += (int64_t)X(H[i - 1]) * Y(H[i]) - (int64_t)Y(H[i - 1]) * X(H[i]);
        *first = H[0];
        *last = H[k - 1];
    }
    __syncthreads();
    return sum;
}

// convex-hull area of the contour: lower chain (column minima) + upper chain (column
// maxima) closed by the two vertical sides; exact integer shoelace
__device__ double hull_area_of(const int2 *p, int n, int x0, int width, GeoLds &sm, int lane) {
    if (n < 3) return 0.0;
    uint32_t lf = 0, ll = 0, uf = 0, ul = 0;
    const int64_t sl = hull_chain<false>(p, n, x0, width, sm, lane, &lf, &ll);
    const int64_t su = hull_chain<true>(p, n, x0, width, sm, lane, &uf, &ul);
    double area = 0.0;
    if (lane == 0) {
        auto X = [](uint32_t v) { return (int64_t)(v >> 16); };
        auto Y = [](uint32_t v) { return (int64_t)(v & 0xffffu); };
        const int64_t a2 = sl + su + (X(ll) * Y(uf) - Y(ll) * X(uf)) + (X(ul) * Y(lf) - Y(ul) * X(lf));
        area = fabs((double)a2 * 0.5);
    }
    return __shfl(area, 0);
}

// grid (G, n), one wave per block: the kept contours of image blockIdx.y
__global__ __launch_bounds__(64) void k_ct_shapes(const CtComp *__restrict__ comps, const int2 *__restrict__ pts,
                                                   const int2 *__restrict__ refs, const int *__restrict__ img_info,
                                                   CtCounters *__restrict__ ctr, llfe_shape *__restrict__ shapes) {
    __shared__ GeoLds sm;
    const int img = blockIdx.y, lane = threadIdx.x;
    if (ctr->flags & kCtOverflowMask) return;
    const int base = img_info[img * kCtInfo + 1], nref = img_info[img * kCtInfo + 2];
    const int sbase = img_info[img * kCtInfo + 4];
    if (lane == 0) sm.flags = 0;
    __syncthreads();
    for (int i = blockIdx.x; i < nref; i += gridDim.x) {
        const int2 r = refs[base + i];
        if (r.y < 0) continue;
        const CtComp c = comps[r.x];
        const int n = (int)c.nv;
        const int2 *p = pts + c.off;
        if (n <= kPtsLds) {  // stage the vertices in LDS
            for (int i = lane; i < n; i += 64) sm.pts[i] = p[i];
            __syncthreads();
            p = sm.pts;
        }
        const double area = fabs((double)c.area2 * 0.5);
        const double per = perimeter_of(p, n, lane);
        const int width = c.x1 - c.x0 + 1;
        if (width > kHullCols) {
            if (lane == 0) atomicOr(&ctr->flags, kCtTooWide);
            return;
        }
        // detect_border_radius(contour, 0.02)
        double br = 0.0;
        if (dp_count(p, n, 0.02 * per, sm, lane) > 4) {
            const double ha = hull_area_of(p, n, c.x0, width, sm, lane);
            if (ha > 0) br = fmax(0.0, (1 - area / ha) * 50.0);
        }
        const int nv = dp_count(p, n, 0.04 * per, sm, lane);
        if (sm.flags) {
            if (lane == 0) atomicOr(&ctr->flags, kCtDpOverflow);
            return;
        }
        int type = LLFE_SHAPE_UNKNOWN;
        if (nv == 3) {
            type = LLFE_SHAPE_TRIANGLE;
        } else if (nv == 4) {
            type = LLFE_SHAPE_RECTANGLE;
        } else if (nv > 4 && per > 0) {
            const double four_pi = 4 * 3.141592653589793;
            const double circularity = four_pi * area / (per * per);
            type = circularity > 0.8 ? LLFE_SHAPE_CIRCLE : LLFE_SHAPE_POLYGON;
        }
        if (lane == 0) {
            llfe_shape s;
            s.type = type;
            s.x = c.x0;
            s.y = c.y0;
            s.width = width;
            s.height = c.y1 - c.y0 + 1;
            s.pad_ = 0;
            s.border_radius = br;
            s.area = area;
            shapes[sbase + r.y] = s;
        }
        __syncthreads();
    }
}

}  // namespace

CtCaps contours_default_caps(int n, int h, int w) {
    CtCaps c;
    c.comps = (int64_t)n * 1024 + 4096;
    c.pts = (int64_t)n * 16384 + 65536;
    c.refs = c.comps + (int64_t)n * kCtQuirkCap;
    c.shapes = (int64_t)n * 64 + 256;
    (void)h;
    (void)w;
    return c;
}

size_t contours_plane_words(int n, int h, int w) { return (size_t)n * h * words_per_row(w); }

hipError_t launch_contours(const uint64_t *bits, int n, int h, int w, const CtWork &wk, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    Geo g{h, w, words_per_row(w), tiles_x(w), tiles_x(w) * tiles_y(h), n};
    const size_t pw = contours_plane_words(n, h, w);
    hipError_t e;
    if ((e = hipMemsetAsync(wk.planes, 0, sizeof(uint64_t) * pw * 5, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(wk.ctr, 0, sizeof(CtCounters), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(wk.img_info, 0, sizeof(int) * kCtInfo * n, s)) != hipSuccess) return e;
    const dim3 grid((unsigned)std::min<int64_t>((int64_t)g.ntiles * n, 65536));  // tile loops
    hipLaunchKernelGGL(k_ct_local, grid, dim3(NT), 0, s, bits, g, wk.lab, wk.parent, wk.roots, wk.nroots);
    hipLaunchKernelGGL(k_ct_border, grid, dim3(128), 0, s, bits, g, wk.lab, wk.nroots, wk.parent);
    hipLaunchKernelGGL(k_ct_flatten, grid, dim3(NT), 0, s, g, wk.roots, wk.nroots, wk.parent);
    hipLaunchKernelGGL(k_ct_collect, grid, dim3(NT), 0, s, g, wk.roots, wk.nroots, wk.parent, wk.comps, wk.acc,
                       wk.planes + 4 * pw, wk.ctr, wk.img_info, wk.caps.comps);
    hipLaunchKernelGGL(k_ct_finalize, grid, dim3(NT), 0, s, g, wk.roots, wk.nroots, wk.parent);
    hipLaunchKernelGGL(k_ct_trace, dim3(kCtTraceBlocks), dim3(64), 0, s, bits, g, wk.comps, wk.caps.comps, wk.pts,
                       wk.caps.pts, wk.stage, wk.planes, wk.planes + pw, wk.ctr);
    hipLaunchKernelGGL(k_ct_scan, dim3(n), dim3(64), 0, s, bits, g, wk.lab, wk.parent, wk.planes, pw, wk.comps,
                       wk.caps.comps, wk.acc, wk.pts, wk.caps.pts, wk.refs, wk.caps.refs, wk.ctr, wk.img_info);
    hipLaunchKernelGGL(k_ct_bases, dim3(1), dim3(1024), 0, s, n, wk.img_info, wk.ctr, wk.caps.shapes);
    hipLaunchKernelGGL(k_ct_shapes, dim3(8, n), dim3(64), 0, s, wk.comps, wk.pts, wk.refs, wk.img_info, wk.ctr,
                       wk.shapes);
    return hipGetLastError();
}

}  // namespace llfe
