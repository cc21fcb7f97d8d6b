// Stencil front-end of the shapes + shadows path on gfx950.
//
// One 256-thread workgroup per 64x32 output tile stages a (32+14)x(64+14) BGR
// window (halo 7 = blur5 halo 2 + adaptive-mean halo 5) through LDS and derives,
// without touching HBM in between:
//   gray   = cvtColor(BGR2GRAY)                        shape pyc @L18, shadow pyc @L8
//   blur   = GaussianBlur(gray, (5,5), 0) 8U bit-exact shape pyc @L21, shadow pyc @L9
//   Canny  : Sobel3 (REPLICATE) -> |dx|+|dy| -> NMS    shape pyc @L24 (classes 0/1/2)
//   shadow : adaptiveThreshold GAUSSIAN_C 11, C=2, INV  shadow pyc @L17-24
//            mean = rint(CV_32F Gauss11(blur)) ; mask = blur - mean <= -2 ;
//            sum/count of blur under the mask -> one u64 atomic pair per tile.
// Only the class map (1 B/px) leaves the tile; hysteresis + dilate follow in
// separate launches (global connectivity).
#include <cstdlib>

#include "llfe_internal.h"

namespace llfe {
namespace {

constexpr int TW = kTileW, TH = kTileH;
constexpr int HG = 7;                       // gray halo
constexpr int GW = TW + 2 * HG, GH = TH + 2 * HG;
constexpr int BWD = TW + 10, BHT = TH + 10; // blurred region (halo 5)
constexpr int MW = TW + 2, MH = TH + 2;     // magnitude region (halo 1)
constexpr int NT = 256;

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ int reflect101(int p, int len) {
    // borderInterpolate(BORDER_REFLECT_101): gfedcb|abcdefgh|gfedcba
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// ---------------------------------------------------------------- interior tiles
// Tiles whose whole window lies inside the image (88 % of a 1080p frame) need no
// border handling: every stage works on 4 consecutive pixels per thread with dword /
// 8-byte / 16-byte LDS accesses and no index clamping.  Window columns start at
// tx0 - 8 (4-aligned), rows at ty0 - 7.
constexpr int FGW = TW + 16;      // gray columns   x in [tx0 - 8, tx0 + 72)
constexpr int FBW = TW + 12;      // hb/blur columns x in [tx0 - 6, tx0 + 70)
constexpr int FMH = TH + 2, FMW = TW + 2;

struct __align__(16) FastSmem {
    uint32_t g[GH][FGW / 4];          // gray, 4 per dword
    uint2 hb[GH][FBW / 4];            // horizontal blur5 sums (unscaled taps), 4 x u16 per entry
    uint32_t blur[BHT][FBW / 4];      // blurred gray rows y in [ty0 - 5, ty0 + 37)
    uint16_t md[FMH][FMW + 2];        // |dx|+|dy| | NMS direction << 12, tile + 1 halo
    float4 hf[BHT][TW / 4];           // CV_32F Gauss11 row pass
    uint2 red[NT / 64];               // per-wave shadow (sum, count)
};

__device__ __forceinline__ uint32_t byte_of(uint32_t w, int i) { return (w >> (8 * i)) & 255u; }

typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

template <bool BORDER>
__device__ void stencil_tile(FastSmem &sm, const uint8_t *__restrict__ src, int H, int W, int tx0, int ty0,
                                 uint8_t *__restrict__ cls, uint8_t *__restrict__ blurred_out,
                                 uint2 *tile_part, uint8_t *__restrict__ font_mask,
                                 const StencilParams &prm) {
    const int tid = threadIdx.x;
    // 1) gray: 4 BGR pixels (12 bytes, 3 dwords) -> one dword of gray.  Per pixel the
    //    (B, G) pair is one v_perm into packed u16 and Y = dot2((B, G), (1868, 9617)) +
    //    4899 R + 2^13, >> 14 (exact: every term is an integer < 2^32).
    if (BORDER) {
        // window pixels outside the image take the gray of their REFLECT_101 image
        // pixel: exact for the blur5 taps (<= 2 outside); deeper values are replaced
        // after stage 3 (REPLICATE of the blurred image)
        for (int u = tid; u < GH * FGW; u += NT) {
            const int row = u / FGW, c = u - row * FGW;
            const int Y = reflect101(ty0 - HG + row, H), X = reflect101(tx0 - 8 + c, W);
            const uint8_t *q = src + ((size_t)Y * W + X) * 3;
            ((uint8_t *)sm.g[row])[c] = (uint8_t)((q[0] * 1868u + q[1] * 9617u + q[2] * 4899u + 8192u) >> 14);
        }
    } else
    for (int u = tid; u < GH * (FGW / 4); u += NT) {
        const int row = u / (FGW / 4), q = u - row * (FGW / 4);
        const uint32_t *p = (const uint32_t *)(src + ((size_t)(ty0 - HG + row) * W + (tx0 - 8 + 4 * q)) * 3);
        const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];
        // v_perm selector bytes: 0-3 = second operand, 4-7 = first operand, 0x0c = 0
        const u16x2 bg0 = as_u16x2(__builtin_amdgcn_perm(0u, d0, 0x0c010c00u));
        const u16x2 bg1 = as_u16x2(__builtin_amdgcn_perm(d1, d0, 0x0c040c03u));
        const u16x2 bg2 = as_u16x2(__builtin_amdgcn_perm(0u, d1, 0x0c030c02u));
        const u16x2 bg3 = as_u16x2(__builtin_amdgcn_perm(0u, d2, 0x0c020c01u));
        const u16x2 wbg = {1868, 9617};
        const uint32_t y0 = __builtin_amdgcn_udot2(bg0, wbg, byte_of(d0, 2) * 4899u + 8192u, false) >> 14;
        const uint32_t y1 = __builtin_amdgcn_udot2(bg1, wbg, byte_of(d1, 1) * 4899u + 8192u, false) >> 14;
        const uint32_t y2 = __builtin_amdgcn_udot2(bg2, wbg, byte_of(d2, 0) * 4899u + 8192u, false) >> 14;
        const uint32_t y3 = __builtin_amdgcn_udot2(bg3, wbg, byte_of(d2, 3) * 4899u + 8192u, false) >> 14;
        sm.g[row][q] = y0 | (y1 << 8) | (y2 << 16) | (y3 << 24);
    }
    __syncthreads();
    if (font_mask) {
        // FontDetector.preprocess_image thresholds the gray image itself (no blur5): the
        // "blurred" rows are the gray rows y = ty0 - 5 + ly, x = tx0 - 6 + 4q .. (two
        // bytes into gray dword q)
        for (int u = tid; u < BHT * (FBW / 4); u += NT) {
            const int ly = u / (FBW / 4), q = u - ly * (FBW / 4);
            sm.blur[ly][q] = __builtin_amdgcn_perm(sm.g[ly + 2][q + 1], sm.g[ly + 2][q], 0x05040302u);
        }
        __syncthreads();
    } else {
    // 2) horizontal blur5 in packed u16 with the unscaled taps [1, 4, 6, 4, 1] (sum of a
    //    row <= 16 * 255): hb col c <-> x = tx0 - 6 + c; taps are gray cols c .. c + 4.
    //    (the 8U blur is (sum_ij w_i w_j g + 128) >> 8, so both passes fit in 16 bits)
    for (int u = tid; u < GH * (FBW / 4); u += NT) {
        const int row = u / (FBW / 4), q = u - row * (FBW / 4);
        const uint32_t w0 = sm.g[row][q], w1 = sm.g[row][q + 1];
        const u16x2 b01 = as_u16x2(__builtin_amdgcn_perm(0u, w0, 0x0c010c00u));
        const u16x2 b12 = as_u16x2(__builtin_amdgcn_perm(0u, w0, 0x0c020c01u));
        const u16x2 b23 = as_u16x2(__builtin_amdgcn_perm(0u, w0, 0x0c030c02u));
        const u16x2 b34 = as_u16x2(__builtin_amdgcn_perm(w1, w0, 0x0c040c03u));
        const u16x2 b45 = as_u16x2(__builtin_amdgcn_perm(0u, w1, 0x0c010c00u));
        const u16x2 b56 = as_u16x2(__builtin_amdgcn_perm(0u, w1, 0x0c020c01u));
        const u16x2 b67 = as_u16x2(__builtin_amdgcn_perm(0u, w1, 0x0c030c02u));
        const u16x2 four = {4, 4}, six = {6, 6};
        const u16x2 h01 = (b12 + b34) * four + (b01 + b45) + b23 * six;
        const u16x2 h23 = (b34 + b56) * four + (b23 + b67) + b45 * six;
        sm.hb[row][q] = make_uint2(as_u32(h01), as_u32(h23));
    }
    __syncthreads();
    // 3) vertical blur5 -> blur rows ly (y = ty0 - 5 + ly) from hb rows ly .. ly + 4
    for (int u = tid; u < BHT * (FBW / 4); u += NT) {
        const int ly = u / (FBW / 4), q = u - ly * (FBW / 4);
        u16x2 s01 = {128, 128}, s23 = {128, 128};
        const uint16_t kw[5] = {1, 4, 6, 4, 1};
#pragma unroll
        for (int r = 0; r < 5; r++) {
            const uint2 v = sm.hb[ly + r][q];
            const u16x2 k = {kw[r], kw[r]};
            s01 = as_u16x2(v.x) * k + s01;
            s23 = as_u16x2(v.y) * k + s23;
        }
        const u16x2 e8 = {8, 8};
        s01 = s01 >> e8;
        s23 = s23 >> e8;
        sm.blur[ly][q] = __builtin_amdgcn_perm(as_u32(s23), as_u32(s01), 0x06040200u);
    }
    __syncthreads();
    }
    if (BORDER) {
        // blurred values outside the image: REPLICATE (Sobel's and the CV_32F Gauss11's
        // border on the blurred image)
        for (int u = tid; u < BHT * FBW; u += NT) {
            const int ly = u / FBW, c = u - ly * FBW, Y = ty0 - 5 + ly, X = tx0 - 6 + c;
            if ((unsigned)Y >= (unsigned)H || (unsigned)X >= (unsigned)W) {
                const int sy = clampi(Y, 0, H - 1) - (ty0 - 5), sx = clampi(X, 0, W - 1) - (tx0 - 6);
                ((uint8_t *)sm.blur[ly])[c] = ((const uint8_t *)sm.blur[sy])[sx];
            }
        }
        __syncthreads();
    }
    // blur byte at tile-relative (row ly, col c) where c <-> x = tx0 - 6 + c
    auto BL = [&](int ly, int c) -> int { return (int)byte_of(sm.blur[ly][c >> 2], c & 3); };

    if (blurred_out) {
        for (int u = tid; u < TH * (TW / 4); u += NT) {
            const int y = u / (TW / 4), q = u - y * (TW / 4);
            uint32_t o = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) o |= (uint32_t)BL(y + 5, 4 * q + j + 6) << (8 * j);
            if (BORDER) {
                const int Y = ty0 + y, X = tx0 + 4 * q;
                if (Y < H)
                    for (int j = 0; j < 4 && X + j < W; j++) blurred_out[(size_t)Y * W + X + j] = (uint8_t)(o >> (8 * j));
            } else {
                *(uint32_t *)(blurred_out + (size_t)(ty0 + y) * W + tx0 + 4 * q) = o;
            }
        }
    }

    if (cls) {
        // 4) Sobel (no border inside), |dx|+|dy| and the NMS direction class, for the
        //    tile + 1 halo: md row my <-> y = ty0 - 1 + my (blur row my + 4), col mc <->
        //    x = tx0 - 1 + mc (blur col mc + 5)
        constexpr int TG22 = 13573;
        for (int u = tid; u < FMH * ((FMW + 3) / 4); u += NT) {
            const int my = u / ((FMW + 3) / 4), q = u - my * ((FMW + 3) / 4);
            int bv[3][6];
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const uint32_t a = sm.blur[my + 3 + r][q + 1], b2 = sm.blur[my + 3 + r][q + 2];
                // blur cols 4q + 4 .. 4q + 9 = mag cols 4q - 1 .. 4q + 4 around 4q .. 4q + 3
#pragma unroll
                for (int i = 0; i < 4; i++) bv[r][i] = (int)byte_of(a, i);
                bv[r][4] = (int)byte_of(b2, 0);
                bv[r][5] = (int)byte_of(b2, 1);
            }
            int gx[4], gy[4], m[4];
            bool need = false;  // the direction class matters only where m > LOW (stage 5)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                gx[j] = (bv[0][j + 2] + 2 * bv[1][j + 2] + bv[2][j + 2]) - (bv[0][j] + 2 * bv[1][j] + bv[2][j]);
                gy[j] = (bv[2][j] + 2 * bv[2][j + 1] + bv[2][j + 2]) - (bv[0][j] + 2 * bv[0][j + 1] + bv[0][j + 2]);
                m[j] = abs(gx[j]) + abs(gy[j]);
                need = need || m[j] > 50;
            }
            int dir[4] = {0, 0, 0, 0};
            if (need) {  // whole waves of flat / noise-only pixels skip the direction math
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int ax = abs(gx[j]), ay = abs(gy[j]) << 15, tg22x = ax * TG22;
                    if (ay < tg22x) dir[j] = 0;
                    else if (ay > tg22x + (ax << 16)) dir[j] = 1;
                    else dir[j] = (gx[j] ^ gy[j]) < 0 ? 2 : 3;
                }
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int mc = 4 * q + j;
                if (mc >= FMW) break;
                const bool out = BORDER && ((unsigned)(ty0 - 1 + my) >= (unsigned)H || (unsigned)(tx0 - 1 + mc) >= (unsigned)W);
                sm.md[my][mc] = out ? (uint16_t)0 : (uint16_t)(m[j] | (dir[j] << 12));  // Canny: no magnitude outside
            }
        }
        __syncthreads();
        // 5) NMS + double threshold on 4 consecutive pixels; one dword of classes out
        constexpr int LOW = 50, HIGH = 150;
        for (int u = tid; u < TH * (TW / 4); u += NT) {
            const int ty = u / (TW / 4), q = u - ty * (TW / 4);
            uint32_t o = 0x01010101u;  // class 1 (not an edge) unless m > LOW
            int mv[4];
            bool any = false;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                mv[j] = sm.md[ty + 1][4 * q + j + 1];
                any = any || (mv[j] & 4095) > LOW;
            }
            if (any)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int tx = 4 * q + j;
                const int v = mv[j];
                const int m = v & 4095, dir = v >> 12;
                uint32_t c = 1;
                if (m > LOW) {
                    bool keep;
                    if (dir == 0) {
                        keep = m > (sm.md[ty + 1][tx] & 4095) && m >= (sm.md[ty + 1][tx + 2] & 4095);
                    } else if (dir == 1) {
                        keep = m > (sm.md[ty][tx + 1] & 4095) && m >= (sm.md[ty + 2][tx + 1] & 4095);
                    } else {
                        const int sgn = dir == 2 ? -1 : 1;
                        keep = m > (sm.md[ty][tx + 1 - sgn] & 4095) && m > (sm.md[ty + 2][tx + 1 + sgn] & 4095);
                    }
                    if (keep) c = m > HIGH ? 2u : 0u;
                }
                o = (o & ~(255u << (8 * j))) | (c << (8 * j));
            }
            if (BORDER) {
                const int Y = ty0 + ty, X = tx0 + 4 * q;
                if (Y < H)
                    for (int j = 0; j < 4 && X + j < W; j++) cls[(size_t)Y * W + X + j] = (uint8_t)(o >> (8 * j));
            } else {
                *(uint32_t *)(cls + (size_t)(ty0 + ty) * W + tx0 + 4 * q) = o;
            }
        }
    }

    if (tile_part || font_mask) {
        // 6) CV_32F row pass (fma chain left -> right) for 4 consecutive x = tx0 + 4q + j
        //    on two rows at once (packed FP32: lane 0 = row ly, lane 1 = row ly + 1; each
        //    lane is the same fma chain as the scalar form): taps are blur cols
        //    4q + 1 + j .. 4q + 11 + j (dwords q .. q + 3)
        for (int u = tid; u < (BHT / 2) * (TW / 4); u += NT) {
            const int lp = u / (TW / 4), q = u - lp * (TW / 4), ly = 2 * lp;
            f32x2 bv[16];
#pragma unroll
            for (int d = 0; d < 4; d++) {
                const uint32_t wa = sm.blur[ly][q + d], wb = sm.blur[ly + 1][q + d];
#pragma unroll
                for (int i = 0; i < 4; i++) bv[4 * d + i] = f32x2{(float)byte_of(wa, i), (float)byte_of(wb, i)};
            }
            f32x2 out[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                f32x2 acc = {0.0f, 0.0f};
#pragma unroll
                for (int k = 0; k < 11; k++)
                    acc = __builtin_elementwise_fma(bv[1 + j + k], f32x2{prm.k11[k], prm.k11[k]}, acc);
                out[j] = acc;
            }
            sm.hf[ly][q] = make_float4(out[0].x, out[1].x, out[2].x, out[3].x);
            sm.hf[ly + 1][q] = make_float4(out[0].y, out[1].y, out[2].y, out[3].y);
        }
        __syncthreads();
        // 7) column pass (centre, then symmetric pairs inner -> outer), cvRound, mask;
        //    packed FP32 over column pairs (j, j + 1)
        uint32_t lsum = 0, lcnt = 0;
        for (int u = tid; u < TH * (TW / 4); u += NT) {
            const int ty = u / (TW / 4), q = u - ty * (TW / 4);
            const int ly = ty + 5;
            const float4 c0 = sm.hf[ly][q];
            const f32x2 w5 = {prm.k11[5], prm.k11[5]}, z = {0.0f, 0.0f};
            f32x2 s01 = __builtin_elementwise_fma(f32x2{c0.x, c0.y}, w5, z);
            f32x2 s23 = __builtin_elementwise_fma(f32x2{c0.z, c0.w}, w5, z);
#pragma unroll
            for (int d = 1; d <= 5; d++) {
                const float4 a = sm.hf[ly + d][q], b = sm.hf[ly - d][q];
                const f32x2 wd = {prm.k11[5 + d], prm.k11[5 + d]};
                s01 = __builtin_elementwise_fma(f32x2{a.x, a.y} + f32x2{b.x, b.y}, wd, s01);
                s23 = __builtin_elementwise_fma(f32x2{a.z, a.w} + f32x2{b.z, b.w}, wd, s23);
            }
            const float sj[4] = {s01.x, s01.y, s23.x, s23.y};
            const uint32_t bw = sm.blur[ly][q + 1], bw2 = sm.blur[ly][q + 2];
            // blur cols for x = tx0 + 4q + j are 4q + 6 + j: bytes 2, 3 of dword q + 1, 0, 1 of q + 2
            const int bv[4] = {(int)byte_of(bw, 2), (int)byte_of(bw, 3), (int)byte_of(bw2, 0), (int)byte_of(bw2, 1)};
            uint32_t mo = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                int mean = (int)__builtin_rintf(sj[j]);
                mean = clampi(mean, 0, 255);
                const bool in = !BORDER || (ty0 + ty < H && tx0 + 4 * q + j < W);
                if (in && bv[j] - mean <= -2) {
                    lsum += (unsigned)bv[j];
                    lcnt += 1;
                    mo |= 255u << (8 * j);
                }
            }
            if (font_mask) {  // adaptiveThreshold(..., THRESH_BINARY_INV, 11, 2) -> 255 / 0
                if (BORDER) {
                    const int Y = ty0 + ty, X = tx0 + 4 * q;
                    if (Y < H)
                        for (int j = 0; j < 4 && X + j < W; j++) font_mask[(size_t)Y * W + X + j] = (uint8_t)(mo >> (8 * j));
                } else {
                    *(uint32_t *)(font_mask + (size_t)(ty0 + ty) * W + tx0 + 4 * q) = mo;
                }
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {  // per wave: <= 64 x 8 x 4 x 255 < 2^32
            lsum += __shfl_xor(lsum, off);
            lcnt += __shfl_xor(lcnt, off);
        }
        // one (sum, count) per tile, no atomics: k_shadow_reduce adds the tiles up
        if ((tid & 63) == 0) sm.red[tid >> 6] = make_uint2(lsum, lcnt);
        __syncthreads();
        if (tid == 0 && tile_part) {
            uint2 r = sm.red[0];
#pragma unroll
            for (int w = 1; w < NT / 64; w++) {
                r.x += sm.red[w].x;
                r.y += sm.red[w].y;
            }
            *tile_part = r;
        }
    }
}

// grid (n): per-image totals of the tiles' (sum, count)
__global__ __launch_bounds__(256) void k_shadow_reduce(const uint2 *__restrict__ tile_part, int ntiles,
                                                       unsigned long long *__restrict__ shadow_sum,
                                                       unsigned long long *__restrict__ shadow_cnt) {
    __shared__ unsigned long long rs[4], rc[4];
    const int img = blockIdx.x, tid = threadIdx.x;
    unsigned long long a = 0, b = 0;
    for (int t = tid; t < ntiles; t += 256) {
        const uint2 v = tile_part[(size_t)img * ntiles + t];
        a += v.x;
        b += v.y;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off);
        b += __shfl_xor(b, off);
    }
    if ((tid & 63) == 0) {
        rs[tid >> 6] = a;
        rc[tid >> 6] = b;
    }
    __syncthreads();
    if (tid == 0) {
        shadow_sum[img] = rs[0] + rs[1] + rs[2] + rs[3];
        shadow_cnt[img] = rc[0] + rc[1] + rc[2] + rc[3];
    }
}

__global__ __launch_bounds__(NT) void k_stencil(const uint8_t *__restrict__ bgr, int H, int W, int ntx, int nty,
                                                uint8_t *__restrict__ cls, uint8_t *__restrict__ blurred_out,
                                                uint2 *__restrict__ tile_part, uint8_t *__restrict__ font_mask,
                                                StencilParams prm) {
    __shared__ FastSmem shm;
    const int tid = threadIdx.x;
    const int img = blockIdx.y;
    const int t = blockIdx.x;
    const int tx0 = (t % ntx) * TW, ty0 = (t / ntx) * TH;
    const uint8_t *src = bgr + (size_t)img * H * W * 3;
    const bool aligned =
        (((uintptr_t)bgr | (uintptr_t)cls | (uintptr_t)blurred_out | (uintptr_t)font_mask) & 3) == 0 && (W & 3) == 0;
    uint8_t *fm = font_mask ? font_mask + (size_t)img * H * W : nullptr;
    uint8_t *c = cls ? cls + (size_t)img * H * W : nullptr;
    uint8_t *bo = blurred_out ? blurred_out + (size_t)img * H * W : nullptr;
    uint2 *tp = tile_part ? tile_part + (size_t)img * ntx * nty + t : nullptr;
    if (aligned && tx0 >= 8 && ty0 >= HG && tx0 + TW + 8 <= W && ty0 + TH + HG <= H)
        stencil_tile<false>(shm, src, H, W, tx0, ty0, c, bo, tp, fm, prm);
    else
        stencil_tile<true>(shm, src, H, W, tx0, ty0, c, bo, tp, fm, prm);
}

}  // namespace

hipError_t launch_stencil(const uint8_t *bgr, int n, int h, int w, uint8_t *cls, uint8_t *blurred,
                          unsigned long long *shadow_sum, unsigned long long *shadow_cnt, uint2 *tile_part,
                          const StencilParams &p, hipStream_t s) {
    if (!blurred)
        return launch_stencil_stream(bgr, n, h, w, cls, shadow_sum, shadow_cnt, tile_part, p, s);
    int ntx = tiles_x(w), nty = tiles_y(h);
    dim3 grid(ntx * nty, n);
    hipLaunchKernelGGL(k_stencil, grid, dim3(NT), 0, s, bgr, h, w, ntx, nty, cls, blurred,
                       shadow_sum ? tile_part : nullptr, (uint8_t *)nullptr, p);
    if (shadow_sum)
        hipLaunchKernelGGL(k_shadow_reduce, dim3(n), dim3(256), 0, s, tile_part, ntx * nty, shadow_sum, shadow_cnt);
    return hipGetLastError();
}

hipError_t launch_font_binary(const uint8_t *bgr, int n, int h, int w, uint8_t *mask, const StencilParams &p,
                              hipStream_t s) {
    int ntx = tiles_x(w), nty = tiles_y(h);
    dim3 grid(ntx * nty, n);
    hipLaunchKernelGGL(k_stencil, grid, dim3(NT), 0, s, bgr, h, w, ntx, nty, (uint8_t *)nullptr, (uint8_t *)nullptr,
                       (uint2 *)nullptr, mask, p);
    return hipGetLastError();
}

}  // namespace llfe
