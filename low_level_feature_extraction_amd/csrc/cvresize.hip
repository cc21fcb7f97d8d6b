// cv2.resize(image, new_size, interpolation) on u8 HWC images for the preprocessing
// modes of validate_and_preprocess_image (app/services/analyze/utils.py:118-143):
//   auto -> INTER_AREA, high_quality -> INTER_LANCZOS4, performance -> INTER_LINEAR.
//
// OpenCV 4.x imgproc/src/resize.cpp restated (oracle/llfe_oracle.c orc_cv_resize is the
// CPU statement the parity tests compare against):
//   * dsize == ssize: copy; LINEAR at exactly 2x2 runs as AREA;
//   * AREA, integer factors (resizeAreaFast_): 2x2 -> (a + b + c + d + 2) >> 2, other
//     factors cvRound(int sum * (1.f / area)), partial border cells cvRound(sum / count);
//   * AREA, other factors >= 1 (resizeArea_): computeResizeAreaTab weights (float), row
//     buffers accumulated in table order, then rows in table order, cvRound;
//   * LINEAR / CUBIC / LANCZOS4 / AREA-upscale (resizeGeneric_): 11-bit fixed-point
//     taps, int32 horizontal pass, vertical LANCZOS4 (sum + 2^21) >> 22, vertical LINEAR
//     VResizeLinearVec_32s8u ((S0 >> 4) * b0 >> 16) + ((S1 >> 4) * b1 >> 16) + 2 >> 2
//     for the row elements its 128-bit vector loops cover, FixedPtCast for the tail;
//     vertical CUBIC VResizeCubicVec_32s8u (float S3*b3, then S2*b2 + t, S1*b1 + t,
//     S0*b0 + t with b = beta / 2^22, rint, saturate; mul + add on the SSE baseline) for
//     the elements its loop covers (steps of 16), FixedPtCast for the tail.  CUBIC is the
//     small-image upscale of TextExtractor.preprocess_image (text_extractor.py:31-37).
// The tables are built on the host exactly as OpenCV builds them (double / float
// arithmetic, libm sin / cos for Lanczos); the kernels evaluate one output pixel per
// thread.  Not a hot path (no BASELINE configuration resizes): clarity over speed.
#include <cmath>
#include <cstring>
#include <vector>

#include "llfe_internal.h"

namespace llfe {
namespace {

constexpr int RT = 256;

__device__ __forceinline__ int sat8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
__device__ __forceinline__ int rint_sat8(float v) { return sat8((int)__builtin_rintf(v)); }

__global__ __launch_bounds__(RT) void k_cv_area_fast(const uint8_t *__restrict__ src, int h, int w, int cn,
                                                     uint8_t *__restrict__ dst, int oh, int ow, int fx, int fy) {
    const long long i = (long long)blockIdx.x * RT + threadIdx.x;
    if (i >= (long long)oh * ow) return;
    const int dy = (int)(i / ow), dx = (int)(i - (long long)dy * ow);
    uint8_t *D = dst + i * cn;
    const int sy0 = dy * fy, sx0 = dx * fx;
    if (sy0 >= h) {
        for (int c = 0; c < cn; c++) D[c] = 0;
        return;
    }
    const bool full = sy0 + fy <= h && dx < w / fx;
    const bool fast2 = fx == 2 && fy == 2 && (cn == 1 || cn == 3 || cn == 4);
    const float scale = 1.f / (float)(fx * fy);
    for (int c = 0; c < cn; c++) {
        int s = 0, count = 0;
        for (int yy = 0; yy < fy && sy0 + yy < h; yy++) {
            const uint8_t *R = src + ((size_t)(sy0 + yy) * w) * cn + c;
            for (int xx = 0; xx < fx && sx0 + xx < w; xx++) {
                s += R[(size_t)(sx0 + xx) * cn];
                count++;
            }
        }
        int v;
        if (full) v = fast2 ? (s + 2) >> 2 : rint_sat8((float)s * scale);
        else v = count ? rint_sat8((float)s / (float)count) : 0;
        D[c] = (uint8_t)v;
    }
}

// xt: [ow + 1] starts, then (si, alpha bits) pairs; yt likewise for rows
__global__ __launch_bounds__(RT) void k_cv_area(const uint8_t *__restrict__ src, int w, int cn,
                                                uint8_t *__restrict__ dst, int oh, int ow,
                                                const int32_t *__restrict__ xt, const int32_t *__restrict__ yt) {
    const long long i = (long long)blockIdx.x * RT + threadIdx.x;
    if (i >= (long long)oh * ow) return;
    const int dy = (int)(i / ow), dx = (int)(i - (long long)dy * ow);
    const int32_t *xp = xt + (ow + 1), *yp = yt + (oh + 1);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j = yt[dy]; j < yt[dy + 1]; j++) {
        const uint8_t *S = src + (size_t)yp[2 * j] * w * cn;
        const float beta = __int_as_float(yp[2 * j + 1]);
        float buf[4] = {0.f, 0.f, 0.f, 0.f};
        for (int k = xt[dx]; k < xt[dx + 1]; k++) {
            const int si = xp[2 * k];
            const float a = __int_as_float(xp[2 * k + 1]);
            for (int c = 0; c < cn && c < 4; c++) buf[c] = __fadd_rn(buf[c], __fmul_rn((float)S[si + c], a));
        }
        for (int c = 0; c < cn && c < 4; c++) acc[c] = __fadd_rn(acc[c], __fmul_rn(beta, buf[c]));
    }
    for (int c = 0; c < cn && c < 4; c++) dst[i * cn + c] = (uint8_t)rint_sat8(acc[c]);
}

// generic: xs = [xofs px (ow)] [alpha (ow * ks)], ys = [yofs (oh)] [beta (oh * ks)]
__global__ __launch_bounds__(RT) void k_cv_generic(const uint8_t *__restrict__ src, int h, int w, int cn,
                                                   uint8_t *__restrict__ dst, int oh, int ow, int ks, int xmin_px,
                                                   int xmax_px, int x_vec, const int32_t *__restrict__ xs,
                                                   const int32_t *__restrict__ ys) {
    const long long i = (long long)blockIdx.x * RT + threadIdx.x;
    if (i >= (long long)oh * ow) return;
    const int dy = (int)(i / ow), dx = (int)(i - (long long)dy * ow);
    const int sx = xs[dx];
    const int32_t *a = xs + ow + (size_t)dx * ks;
    const int sy0 = ys[dy];
    const int32_t *b = ys + oh + (size_t)dy * ks;
    const int half = ks / 2;
    int32_t hv[8][4];
    for (int k = 0; k < ks; k++) {
        const int row = min(max(sy0 - half + 1 + k, 0), h - 1);
        const uint8_t *S = src + (size_t)row * w * cn;
        for (int c = 0; c < cn && c < 4; c++) {
            int32_t v;
            if (ks == 2) {
                v = dx < xmax_px ? S[sx * cn + c] * a[0] + S[(sx + 1) * cn + c] * a[1] : S[sx * cn + c] * 2048;
            } else if (ks == 4) {
                v = 0;
                for (int j = 0; j < 4; j++) v += S[min(max(sx - 1 + j, 0), w - 1) * cn + c] * a[j];
            } else {
                v = 0;
                for (int j = 0; j < 8; j++) v += S[min(max(sx - 3 + j, 0), w - 1) * cn + c] * a[j];
            }
            hv[k][c] = v;
        }
    }
    (void)xmin_px;  // the clamped taps above equal OpenCV's border loop (cn-stepping clamp)
    for (int c = 0; c < cn && c < 4; c++) {
        int v;
        if (ks == 2) {
            const int x = dx * cn + c;
            if (x < x_vec) {
                const int s0 = min(max(hv[0][c] >> 4, -32768), 32767), s1 = min(max(hv[1][c] >> 4, -32768), 32767);
                int t = ((s0 * b[0]) >> 16) + ((s1 * b[1]) >> 16);
                t = min(max(t, -32768), 32767);
                v = sat8((t + 2) >> 2);
            } else {
                v = sat8((hv[0][c] * b[0] + hv[1][c] * b[1] + (1 << 21)) >> 22);
            }
        } else if (ks == 4) {
            if (dx * cn + c < x_vec) {
                const float sc = 1.f / (2048.f * 2048.f);
                float t = __fmul_rn((float)hv[3][c], (float)b[3] * sc);
                t = __fadd_rn(__fmul_rn((float)hv[2][c], (float)b[2] * sc), t);
                t = __fadd_rn(__fmul_rn((float)hv[1][c], (float)b[1] * sc), t);
                t = __fadd_rn(__fmul_rn((float)hv[0][c], (float)b[0] * sc), t);
                v = rint_sat8(t);
            } else {
                v = sat8((hv[0][c] * b[0] + hv[1][c] * b[1] + hv[2][c] * b[2] + hv[3][c] * b[3] + (1 << 21)) >> 22);
            }
        } else {
            uint32_t s = 0;
            for (int k = 0; k < 8; k++) s += (uint32_t)hv[k][c] * (uint32_t)b[k];
            v = sat8(((int32_t)s + (1 << 21)) >> 22);
        }
        dst[i * cn + c] = (uint8_t)v;
    }
}

// ------------------------------------------------------------------ host tables
inline int floor_f(float v) {
    int i = (int)v;
    return i - (i > v);
}
inline int floor_d(double v) {
    int i = (int)v;
    return i - (i > v);
}
inline int ceil_d(double v) {
    int i = (int)v;
    return i + (i < v);
}
inline int32_t sat_s16(float v) {
    long r = std::lrint(v);
    return (int32_t)(r < -32768 ? -32768 : (r > 32767 ? 32767 : r));
}
inline int32_t fbits(float f) {
    int32_t b;
    std::memcpy(&b, &f, 4);
    return b;
}

// interpolateCubic, A = -0.75 (float arithmetic)
void cubic(float x, float *coeffs) {
    const float A = -0.75f;
    coeffs[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
    coeffs[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
    coeffs[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
    coeffs[3] = 1.f - coeffs[0] - coeffs[1] - coeffs[2];
}

// interpolateLanczos4
void lanczos4(float x, float *coeffs) {
    static const double s45 = 0.70710678118654752440084436210485;
    static const double cs[8][2] = {{1, 0}, {-s45, -s45}, {0, 1}, {s45, -s45}, {-1, 0}, {s45, s45}, {0, -1}, {-s45, s45}};
    const double pi = 3.1415926535897932384626433832795;
    float sum = 0;
    const double y0 = -(x + 3) * pi * 0.25, s0 = std::sin(y0), c0 = std::cos(y0);
    for (int i = 0; i < 8; i++) {
        const float y0_ = (x + 3 - i);
        if (std::fabs(y0_) >= 1e-6f) {
            const double y = -y0_ * pi * 0.25;
            coeffs[i] = (float)((cs[i][0] * s0 + cs[i][1] * c0) / (y * y));
        } else {
            coeffs[i] = 1e30f;
        }
        sum += coeffs[i];
    }
    sum = 1.f / sum;
    for (int i = 0; i < 8; i++) coeffs[i] *= sum;
}

// computeResizeAreaTab as [dsize + 1] starts + (si, alpha) pairs (si in pixels * cn)
void area_tab(int ssize, int dsize, int cn, double scale, std::vector<int32_t> &out) {
    std::vector<int32_t> starts(dsize + 1), pairs;
    for (int dx = 0; dx < dsize; dx++) {
        starts[dx] = (int32_t)(pairs.size() / 2);
        const double f1 = dx * scale, f2 = f1 + scale;
        const double cell = std::min(scale, ssize - f1);
        int s1 = ceil_d(f1), s2 = floor_d(f2);
        s2 = std::min(s2, ssize - 1);
        s1 = std::min(s1, s2);
        if (s1 - f1 > 1e-3) {
            pairs.push_back((s1 - 1) * cn);
            pairs.push_back(fbits((float)((s1 - f1) / cell)));
        }
        for (int sx = s1; sx < s2; sx++) {
            pairs.push_back(sx * cn);
            pairs.push_back(fbits((float)(1.0 / cell)));
        }
        if (f2 - s2 > 1e-3) {
            pairs.push_back(s2 * cn);
            pairs.push_back(fbits((float)(std::min(std::min(f2 - s2, 1.), cell) / cell)));
        }
    }
    starts[dsize] = (int32_t)(pairs.size() / 2);
    out.insert(out.end(), starts.begin(), starts.end());
    out.insert(out.end(), pairs.begin(), pairs.end());
}

}  // namespace

int cv_resize_plan(int h, int w, int cn, int oh, int ow, int interp, CvResizePlan &p) {
    if (h <= 0 || w <= 0) return -1;
    return cv_resize_plan_scaled(h, w, cn, oh, ow, (double)ow / w, (double)oh / h, interp, p);
}

int cv_resize_plan_scaled(int h, int w, int cn, int oh, int ow, double inv_x, double inv_y, int interp,
                          CvResizePlan &p) {
    p = CvResizePlan{};
    p.h = h, p.w = w, p.cn = cn, p.oh = oh, p.ow = ow;
    if (h <= 0 || w <= 0 || oh <= 0 || ow <= 0 || cn <= 0 || cn > 4) return -1;
    if (interp != kCvInterLinear && interp != kCvInterArea && interp != kCvInterLanczos4 && interp != kCvInterCubic)
        return -1;
    if (oh == h && ow == w) {
        p.kind = CvResizePlan::COPY;
        return 0;
    }
    const double scale_x = 1. / inv_x, scale_y = 1. / inv_y;
    const int ix = (int)std::lrint(scale_x), iy = (int)std::lrint(scale_y);
    const bool fast = std::fabs(scale_x - ix) < 2.220446049250313e-16 && std::fabs(scale_y - iy) < 2.220446049250313e-16;
    if (interp == kCvInterLinear && fast && ix == 2 && iy == 2) interp = kCvInterArea;
    if (interp == kCvInterArea && scale_x >= 1 && scale_y >= 1) {
        if (fast) {
            p.kind = CvResizePlan::AREA_FAST;
            p.fx = ix, p.fy = iy;
        } else {
            p.kind = CvResizePlan::AREA;
            area_tab(w, ow, cn, scale_x, p.tab);
            p.ytab_off = (int64_t)p.tab.size();
            area_tab(h, oh, 1, scale_y, p.tab);
            // row table entries hold the row index (cn = 1)
        }
        return 0;
    }
    p.kind = CvResizePlan::GENERIC;
    const int ks = interp == kCvInterLanczos4 ? 8 : (interp == kCvInterCubic ? 4 : 2), ks2 = ks / 2;
    const bool area_mode = interp == kCvInterArea;
    const bool wide = interp == kCvInterLanczos4 || interp == kCvInterCubic;  // no sx / fx clamp
    p.ks = ks;
    std::vector<int32_t> xofs(ow), xa((size_t)ow * ks), yofs(oh), yb((size_t)oh * ks);
    float cbuf[8];
    int xmin = 0, xmax = ow;
    for (int dx = 0; dx < ow; dx++) {
        float fx;
        int sx;
        if (!area_mode) {
            fx = (float)((dx + 0.5) * scale_x - 0.5);
            sx = floor_f(fx);
            fx -= sx;
        } else {
            sx = floor_d(dx * scale_x);
            fx = (float)((dx + 1) - (sx + 1) * inv_x);
            fx = fx <= 0 ? 0.f : fx - floor_f(fx);
        }
        if (sx < ks2 - 1) {
            xmin = dx + 1;
            if (sx < 0 && !wide) fx = 0, sx = 0;
        }
        if (sx + ks2 >= w) {
            xmax = std::min(xmax, dx);
            if (sx >= w - 1 && !wide) fx = 0, sx = w - 1;
        }
        xofs[dx] = sx;
        if (interp == kCvInterLanczos4) lanczos4(fx, cbuf);
        else if (interp == kCvInterCubic) cubic(fx, cbuf);
        else cbuf[0] = 1.f - fx, cbuf[1] = fx;
        for (int k = 0; k < ks; k++) xa[(size_t)dx * ks + k] = sat_s16(cbuf[k] * 2048);
    }
    for (int dy = 0; dy < oh; dy++) {
        float fy;
        int sy;
        if (!area_mode) {
            fy = (float)((dy + 0.5) * scale_y - 0.5);
            sy = floor_f(fy);
            fy -= sy;
        } else {
            sy = floor_d(dy * scale_y);
            fy = (float)((dy + 1) - (sy + 1) * inv_y);
            fy = fy <= 0 ? 0.f : fy - floor_f(fy);
        }
        yofs[dy] = sy;
        if (interp == kCvInterLanczos4) lanczos4(fy, cbuf);
        else if (interp == kCvInterCubic) cubic(fy, cbuf);
        else cbuf[0] = 1.f - fy, cbuf[1] = fy;
        for (int k = 0; k < ks; k++) yb[(size_t)dy * ks + k] = sat_s16(cbuf[k] * 2048);
    }
    p.xmin = xmin, p.xmax = xmax;
    const int width = ow * cn;
    int xv = 0;
    while (xv <= width - 16) xv += 16;
    if (ks == 2)  // VResizeLinearVec_32s8u's second, 8-lane loop (VResizeCubicVec has one)
        while (xv < width - 8) xv += 8;
    p.x_vec = xv;
    p.tab.insert(p.tab.end(), xofs.begin(), xofs.end());
    p.tab.insert(p.tab.end(), xa.begin(), xa.end());
    p.ytab_off = (int64_t)p.tab.size();
    p.tab.insert(p.tab.end(), yofs.begin(), yofs.end());
    p.tab.insert(p.tab.end(), yb.begin(), yb.end());
    return 0;
}

hipError_t launch_cv_resize(const CvResizePlan &p, const uint8_t *src, uint8_t *dst, const int32_t *d_tab,
                            hipStream_t s) {
    const long long n = (long long)p.oh * p.ow;
    const unsigned blocks = (unsigned)((n + RT - 1) / RT);
    switch (p.kind) {
    case CvResizePlan::COPY:
        return hipMemcpyAsync(dst, src, (size_t)p.h * p.w * p.cn, hipMemcpyDeviceToDevice, s);
    case CvResizePlan::AREA_FAST:
        hipLaunchKernelGGL(k_cv_area_fast, dim3(blocks), dim3(RT), 0, s, src, p.h, p.w, p.cn, dst, p.oh, p.ow, p.fx,
                           p.fy);
        break;
    case CvResizePlan::AREA:
        hipLaunchKernelGGL(k_cv_area, dim3(blocks), dim3(RT), 0, s, src, p.w, p.cn, dst, p.oh, p.ow, d_tab,
                           d_tab + p.ytab_off);
        break;
    case CvResizePlan::GENERIC:
        hipLaunchKernelGGL(k_cv_generic, dim3(blocks), dim3(RT), 0, s, src, p.h, p.w, p.cn, dst, p.oh, p.ow, p.ks,
                           p.xmin, p.xmax, p.x_vec, d_tab, d_tab + p.ytab_off);
        break;
    }
    return hipGetLastError();
}

}  // namespace llfe
