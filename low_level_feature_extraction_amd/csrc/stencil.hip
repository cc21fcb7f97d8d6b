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

struct __align__(16) StencilSmem {
    uint8_t gray[GH][GW];
    uint16_t hb[GH][BWD];
    uint8_t blur[BHT][BWD];
    uint16_t mag[MH][MW];
    float hf[BHT][TW];
};

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
    uint2 hb[GH][FBW / 4];            // horizontal blur5 sums, 4 x u16 per entry
    uint32_t blur[BHT][FBW / 4];      // blurred gray rows y in [ty0 - 5, ty0 + 37)
    uint16_t md[FMH][FMW + 2];        // |dx|+|dy| | NMS direction << 12, tile + 1 halo
    float4 hf[BHT][TW / 4];           // CV_32F Gauss11 row pass
};

__device__ __forceinline__ uint32_t byte_of(uint32_t w, int i) { return (w >> (8 * i)) & 255u; }

__device__ void stencil_interior(FastSmem &sm, const uint8_t *__restrict__ src, int H, int W, int tx0, int ty0,
                                 uint8_t *__restrict__ cls, uint8_t *__restrict__ blurred_out,
                                 unsigned long long *shadow_sum, unsigned long long *shadow_cnt,
                                 const StencilParams &prm) {
    const int tid = threadIdx.x;
    // 1) gray: 4 BGR pixels (12 bytes, 3 dwords) -> one dword of gray
    for (int u = tid; u < GH * (FGW / 4); u += NT) {
        const int row = u / (FGW / 4), q = u - row * (FGW / 4);
        const uint32_t *p = (const uint32_t *)(src + ((size_t)(ty0 - HG + row) * W + (tx0 - 8 + 4 * q)) * 3);
        const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];
        const uint32_t b[12] = {byte_of(d0, 0), byte_of(d0, 1), byte_of(d0, 2), byte_of(d0, 3),
                                byte_of(d1, 0), byte_of(d1, 1), byte_of(d1, 2), byte_of(d1, 3),
                                byte_of(d2, 0), byte_of(d2, 1), byte_of(d2, 2), byte_of(d2, 3)};
        uint32_t o = 0;
#pragma unroll
        for (int j = 0; j < 4; j++)
            o |= ((b[3 * j] * 1868u + b[3 * j + 1] * 9617u + b[3 * j + 2] * 4899u + 8192u) >> 14) << (8 * j);
        sm.g[row][q] = o;
    }
    __syncthreads();
    // 2) horizontal blur5: hb col c <-> x = tx0 - 6 + c; taps are gray cols c .. c + 4
    for (int u = tid; u < GH * (FBW / 4); u += NT) {
        const int row = u / (FBW / 4), q = u - row * (FBW / 4);
        const uint32_t w0 = sm.g[row][q], w1 = sm.g[row][q + 1];
        uint32_t b[8];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            b[i] = byte_of(w0, i);
            b[4 + i] = byte_of(w1, i);
        }
        uint32_t h[4];
#pragma unroll
        for (int j = 0; j < 4; j++) h[j] = 16u * (b[j] + b[j + 4]) + 64u * (b[j + 1] + b[j + 3]) + 96u * b[j + 2];
        sm.hb[row][q] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    }
    __syncthreads();
    // 3) vertical blur5 -> blur rows ly (y = ty0 - 5 + ly) from hb rows ly .. ly + 4
    for (int u = tid; u < BHT * (FBW / 4); u += NT) {
        const int ly = u / (FBW / 4), q = u - ly * (FBW / 4);
        uint32_t s[4] = {0, 0, 0, 0};
        const uint32_t kw[5] = {16u, 64u, 96u, 64u, 16u};
#pragma unroll
        for (int r = 0; r < 5; r++) {
            const uint2 v = sm.hb[ly + r][q];
            s[0] += kw[r] * (v.x & 0xFFFFu);
            s[1] += kw[r] * (v.x >> 16);
            s[2] += kw[r] * (v.y & 0xFFFFu);
            s[3] += kw[r] * (v.y >> 16);
        }
        uint32_t o = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) o |= ((s[j] + 32768u) >> 16) << (8 * j);
        sm.blur[ly][q] = o;
    }
    __syncthreads();
    // blur byte at tile-relative (row ly, col c) where c <-> x = tx0 - 6 + c
    auto BL = [&](int ly, int c) -> int { return (int)byte_of(sm.blur[ly][c >> 2], c & 3); };

    if (blurred_out) {
        for (int u = tid; u < TH * (TW / 4); u += NT) {
            const int y = u / (TW / 4), q = u - y * (TW / 4);
            uint32_t o = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) o |= (uint32_t)BL(y + 5, 4 * q + j + 6) << (8 * j);
            *(uint32_t *)(blurred_out + (size_t)(ty0 + y) * W + tx0 + 4 * q) = o;
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
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int mc = 4 * q + j;
                if (mc >= FMW) break;
                const int gx = (bv[0][j + 2] + 2 * bv[1][j + 2] + bv[2][j + 2]) - (bv[0][j] + 2 * bv[1][j] + bv[2][j]);
                const int gy = (bv[2][j] + 2 * bv[2][j + 1] + bv[2][j + 2]) - (bv[0][j] + 2 * bv[0][j + 1] + bv[0][j + 2]);
                const int m = abs(gx) + abs(gy);
                const int ax = abs(gx), ay = abs(gy) << 15, tg22x = ax * TG22;
                int dir;
                if (ay < tg22x) dir = 0;
                else if (ay > tg22x + (ax << 16)) dir = 1;
                else dir = (gx ^ gy) < 0 ? 2 : 3;
                sm.md[my][mc] = (uint16_t)(m | (dir << 12));
            }
        }
        __syncthreads();
        // 5) NMS + double threshold on 4 consecutive pixels; one dword of classes out
        constexpr int LOW = 50, HIGH = 150;
        for (int u = tid; u < TH * (TW / 4); u += NT) {
            const int ty = u / (TW / 4), q = u - ty * (TW / 4);
            uint32_t o = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int tx = 4 * q + j;
                const int v = sm.md[ty + 1][tx + 1];
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
                o |= c << (8 * j);
            }
            *(uint32_t *)(cls + (size_t)(ty0 + ty) * W + tx0 + 4 * q) = o;
        }
    }

    if (shadow_sum) {
        // 6) CV_32F row pass (fma chain left -> right) for 4 consecutive x = tx0 + 4q + j:
        //    taps are blur cols 4q + 1 + j .. 4q + 11 + j (dwords q .. q + 3)
        for (int u = tid; u < BHT * (TW / 4); u += NT) {
            const int ly = u / (TW / 4), q = u - ly * (TW / 4);
            float bvf[16];
#pragma unroll
            for (int d = 0; d < 4; d++) {
                const uint32_t w = sm.blur[ly][q + d];
#pragma unroll
                for (int i = 0; i < 4; i++) bvf[4 * d + i] = (float)byte_of(w, i);
            }
            float out[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                float s = 0.0f;
#pragma unroll
                for (int k = 0; k < 11; k++) s = __builtin_fmaf(bvf[1 + j + k], prm.k11[k], s);
                out[j] = s;
            }
            sm.hf[ly][q] = make_float4(out[0], out[1], out[2], out[3]);
        }
        __syncthreads();
        // 7) column pass (centre, then symmetric pairs inner -> outer), cvRound, mask
        unsigned long long lsum = 0, lcnt = 0;
        for (int u = tid; u < TH * (TW / 4); u += NT) {
            const int ty = u / (TW / 4), q = u - ty * (TW / 4);
            const int ly = ty + 5;
            const float4 c0 = sm.hf[ly][q];
            float s[4] = {__builtin_fmaf(c0.x, prm.k11[5], 0.0f), __builtin_fmaf(c0.y, prm.k11[5], 0.0f),
                          __builtin_fmaf(c0.z, prm.k11[5], 0.0f), __builtin_fmaf(c0.w, prm.k11[5], 0.0f)};
#pragma unroll
            for (int d = 1; d <= 5; d++) {
                const float4 a = sm.hf[ly + d][q], b = sm.hf[ly - d][q];
                s[0] = __builtin_fmaf(a.x + b.x, prm.k11[5 + d], s[0]);
                s[1] = __builtin_fmaf(a.y + b.y, prm.k11[5 + d], s[1]);
                s[2] = __builtin_fmaf(a.z + b.z, prm.k11[5 + d], s[2]);
                s[3] = __builtin_fmaf(a.w + b.w, prm.k11[5 + d], s[3]);
            }
            const uint32_t bw = sm.blur[ly][q + 1], bw2 = sm.blur[ly][q + 2];
            // blur cols for x = tx0 + 4q + j are 4q + 6 + j: bytes 2, 3 of dword q + 1, 0, 1 of q + 2
            const int bv[4] = {(int)byte_of(bw, 2), (int)byte_of(bw, 3), (int)byte_of(bw2, 0), (int)byte_of(bw2, 1)};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                int mean = (int)__builtin_rintf(s[j]);
                mean = clampi(mean, 0, 255);
                if (bv[j] - mean <= -2) {
                    lsum += (unsigned)bv[j];
                    lcnt += 1;
                }
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            lsum += __shfl_xor(lsum, off);
            lcnt += __shfl_xor(lcnt, off);
        }
        if ((tid & 63) == 0 && lcnt) {
            atomicAdd(shadow_sum, lsum);
            atomicAdd(shadow_cnt, lcnt);
        }
    }
}

union StencilShared {
    StencilSmem g;
    FastSmem f;
};

__global__ __launch_bounds__(NT) void k_stencil(const uint8_t *__restrict__ bgr, int H, int W, int ntx, int nty,
                                                uint8_t *__restrict__ cls, uint8_t *__restrict__ blurred_out,
                                                unsigned long long *__restrict__ shadow_sum,
                                                unsigned long long *__restrict__ shadow_cnt, StencilParams prm) {
    __shared__ StencilShared shm;
    const int tid = threadIdx.x;
    const int img = blockIdx.y;
    const int t = blockIdx.x;
    const int tx0 = (t % ntx) * TW, ty0 = (t / ntx) * TH;
    const uint8_t *src = bgr + (size_t)img * H * W * 3;
    const bool aligned = (((uintptr_t)bgr | (uintptr_t)cls | (uintptr_t)blurred_out) & 3) == 0 && (W & 3) == 0;
    if (aligned && tx0 >= 8 && ty0 >= HG && tx0 + TW + 8 <= W && ty0 + TH + HG <= H) {
        stencil_interior(shm.f, src, H, W, tx0, ty0, cls ? cls + (size_t)img * H * W : nullptr,
                         blurred_out ? blurred_out + (size_t)img * H * W : nullptr,
                         shadow_sum ? shadow_sum + img : nullptr, shadow_cnt ? shadow_cnt + img : nullptr, prm);
        return;
    }
    StencilSmem &sm = shm.g;

    // 1) BGR window -> gray (Y = (1868 B + 9617 G + 4899 R + 2^13) >> 14)
    for (int i = tid; i < GH * GW; i += NT) {
        int gy = i / GW, gx = i - gy * GW;
        int Y = ty0 - HG + gy, X = tx0 - HG + gx;
        uint8_t g = 0;
        if ((unsigned)Y < (unsigned)H && (unsigned)X < (unsigned)W) {
            const uint8_t *p = src + ((size_t)Y * W + X) * 3;
            unsigned b = p[0], gg = p[1], r = p[2];
            g = (uint8_t)((b * 1868u + gg * 9617u + r * 4899u + 8192u) >> 14);
        }
        sm.gray[gy][gx] = g;
    }
    __syncthreads();

    // 2) horizontal blur5 (REFLECT_101) for every in-image gray row of the window,
    //    at the (replicate-clamped) columns of the blurred region.
    for (int i = tid; i < GH * BWD; i += NT) {
        int gy = i / BWD, lx = i - gy * BWD;
        int Y = ty0 - HG + gy;
        uint16_t v = 0;
        if ((unsigned)Y < (unsigned)H) {
            int X = clampi(tx0 - 5 + lx, 0, W - 1);
            int c0 = reflect101(X - 2, W) - (tx0 - HG), c1 = reflect101(X - 1, W) - (tx0 - HG);
            int c2 = X - (tx0 - HG), c3 = reflect101(X + 1, W) - (tx0 - HG), c4 = reflect101(X + 2, W) - (tx0 - HG);
            const uint8_t *row = sm.gray[gy];
            v = (uint16_t)(16u * row[c0] + 64u * row[c1] + 96u * row[c2] + 64u * row[c3] + 16u * row[c4]);
        }
        sm.hb[gy][lx] = v;
    }
    __syncthreads();

    // 3) vertical blur5 -> blurred region; entry (ly,lx) holds blur(clamp(ty0-5+ly), clamp(tx0-5+lx))
    for (int i = tid; i < BHT * BWD; i += NT) {
        int ly = i / BWD, lx = i - ly * BWD;
        int Y = clampi(ty0 - 5 + ly, 0, H - 1);
        int r0 = reflect101(Y - 2, H) - (ty0 - HG), r1 = reflect101(Y - 1, H) - (ty0 - HG), r2 = Y - (ty0 - HG);
        int r3 = reflect101(Y + 1, H) - (ty0 - HG), r4 = reflect101(Y + 2, H) - (ty0 - HG);
        uint32_t s = 16u * sm.hb[r0][lx] + 64u * sm.hb[r1][lx] + 96u * sm.hb[r2][lx] + 64u * sm.hb[r3][lx] +
                     16u * sm.hb[r4][lx];
        uint32_t v = (s + 32768u) >> 16;
        sm.blur[ly][lx] = (uint8_t)(v > 255u ? 255u : v);
    }
    __syncthreads();

    if (blurred_out) {
        for (int i = tid; i < TH * TW; i += NT) {
            int y = i / TW, x = i - y * TW;
            int Y = ty0 + y, X = tx0 + x;
            if (Y < H && X < W) blurred_out[((size_t)img * H + Y) * W + X] = sm.blur[y + 5][x + 5];
        }
    }

    // blurred value at in-image global (Y, X) with |Y-ty0|,|X-tx0| in range
#define BLUR(Y, X) ((int)sm.blur[(Y) - (ty0 - 5)][(X) - (tx0 - 5)])

    if (cls) {
        // 4) |dx|+|dy| on the tile + 1 halo (0 outside the image: Canny's mag border)
        for (int i = tid; i < MH * MW; i += NT) {
            int my = i / MW, mx = i - my * MW;
            int y = ty0 - 1 + my, x = tx0 - 1 + mx;
            uint16_t m = 0;
            if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) {
                int ym = max(y - 1, 0), yp = min(y + 1, H - 1), xm = max(x - 1, 0), xp = min(x + 1, W - 1);
                int gx = (BLUR(ym, xp) + 2 * BLUR(y, xp) + BLUR(yp, xp)) - (BLUR(ym, xm) + 2 * BLUR(y, xm) + BLUR(yp, xm));
                int gy = (BLUR(yp, xm) + 2 * BLUR(yp, x) + BLUR(yp, xp)) - (BLUR(ym, xm) + 2 * BLUR(ym, x) + BLUR(ym, xp));
                m = (uint16_t)(abs(gx) + abs(gy));
            }
            sm.mag[my][mx] = m;
        }
        __syncthreads();

        // 5) non-maximum suppression + double threshold (50, 150) -> class
        constexpr int TG22 = 13573, LOW = 50, HIGH = 150;
        for (int i = tid; i < TH * TW; i += NT) {
            int ty = i / TW, tx = i - ty * TW;
            int y = ty0 + ty, x = tx0 + tx;
            if (y >= H || x >= W) continue;
            int m = sm.mag[ty + 1][tx + 1];
            uint8_t v = 1;
            if (m > LOW) {
                int ym = max(y - 1, 0), yp = min(y + 1, H - 1), xm = max(x - 1, 0), xp = min(x + 1, W - 1);
                int xs = (BLUR(ym, xp) + 2 * BLUR(y, xp) + BLUR(yp, xp)) - (BLUR(ym, xm) + 2 * BLUR(y, xm) + BLUR(yp, xm));
                int ys = (BLUR(yp, xm) + 2 * BLUR(yp, x) + BLUR(yp, xp)) - (BLUR(ym, xm) + 2 * BLUR(ym, x) + BLUR(ym, xp));
                int ax = abs(xs);
                int ay = abs(ys) << 15;
                int tg22x = ax * TG22;
                bool keep;
                if (ay < tg22x) {
                    keep = m > sm.mag[ty + 1][tx] && m >= sm.mag[ty + 1][tx + 2];
                } else {
                    int tg67x = tg22x + (ax << 16);
                    if (ay > tg67x) {
                        keep = m > sm.mag[ty][tx + 1] && m >= sm.mag[ty + 2][tx + 1];
                    } else {
                        int sgn = (xs ^ ys) < 0 ? -1 : 1;
                        keep = m > sm.mag[ty][tx + 1 - sgn] && m > sm.mag[ty + 2][tx + 1 + sgn];
                    }
                }
                if (keep) v = m > HIGH ? 2 : 0;
            }
            cls[((size_t)img * H + y) * W + x] = v;
        }
    }

    if (shadow_sum) {
        // 6) CV_32F row pass of the 11x11 Gaussian (REPLICATE): fma chain left->right
        for (int i = tid; i < BHT * TW; i += NT) {
            int ly = i / TW, tx = i - ly * TW;
            int x = min(tx0 + tx, W - 1);
            const uint8_t *row = sm.blur[ly];
            float s = 0.0f;
#pragma unroll
            for (int j = 0; j < 11; j++) {
                int c = clampi(x + j - 5, 0, W - 1) - (tx0 - 5);
                s = __builtin_fmaf((float)row[c], prm.k11[j], s);
            }
            sm.hf[ly][tx] = s;
        }
        __syncthreads();
        // 7) column pass: centre first, then symmetric pairs inner->outer; cvRound
        unsigned long long lsum = 0, lcnt = 0;
        for (int i = tid; i < TH * TW; i += NT) {
            int ty = i / TW, tx = i - ty * TW;
            int y = ty0 + ty, x = tx0 + tx;
            if (y >= H || x >= W) continue;
            int ly = y - (ty0 - 5);
            float s = __builtin_fmaf(sm.hf[ly][tx], prm.k11[5], 0.0f);
#pragma unroll
            for (int d = 1; d <= 5; d++) {
                float a = sm.hf[min(y + d, H - 1) - (ty0 - 5)][tx];
                float b = sm.hf[max(y - d, 0) - (ty0 - 5)][tx];
                s = __builtin_fmaf(a + b, prm.k11[5 + d], s);
            }
            int mean = (int)__builtin_rintf(s);
            mean = clampi(mean, 0, 255);
            int bv = BLUR(y, x);
            if (bv - mean <= -2) {
                lsum += (unsigned)bv;
                lcnt += 1;
            }
        }
        // wave reduce, then one atomic pair per wave
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            lsum += __shfl_xor(lsum, off);
            lcnt += __shfl_xor(lcnt, off);
        }
        if ((tid & 63) == 0 && lcnt) {
            atomicAdd(shadow_sum + img, lsum);
            atomicAdd(shadow_cnt + img, lcnt);
        }
    }
#undef BLUR
}

}  // namespace

hipError_t launch_stencil(const uint8_t *bgr, int n, int h, int w, uint8_t *cls, uint8_t *blurred,
                          unsigned long long *shadow_sum, unsigned long long *shadow_cnt, const StencilParams &p,
                          hipStream_t s) {
    int ntx = tiles_x(w), nty = tiles_y(h);
    dim3 grid(ntx * nty, n);
    hipLaunchKernelGGL(k_stencil, grid, dim3(NT), 0, s, bgr, h, w, ntx, nty, cls, blurred, shadow_sum, shadow_cnt, p);
    return hipGetLastError();
}

}  // namespace llfe
