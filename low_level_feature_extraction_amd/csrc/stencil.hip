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

__global__ __launch_bounds__(NT) void k_stencil(const uint8_t *__restrict__ bgr, int H, int W, int ntx, int nty,
                                                uint8_t *__restrict__ cls, uint8_t *__restrict__ blurred_out,
                                                unsigned long long *__restrict__ shadow_sum,
                                                unsigned long long *__restrict__ shadow_cnt, StencilParams prm) {
    __shared__ StencilSmem sm;
    const int tid = threadIdx.x;
    const int img = blockIdx.y;
    const int t = blockIdx.x;
    const int tx0 = (t % ntx) * TW, ty0 = (t / ntx) * TH;
    const uint8_t *src = bgr + (size_t)img * H * W * 3;

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
