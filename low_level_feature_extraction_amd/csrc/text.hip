// TextExtractor.preprocess_image (app/services/analyze/text_extractor.py:15-46) on gfx950:
//   gray = cvtColor(BGR2GRAY) (or the 1-channel image itself)
//   if h < 30 or w < 100: cv2.resize(gray, None, fx=s, fy=s, INTER_CUBIC),
//                          s = max(2, 300 / w, 100 / h)          (cvresize.hip)
//   _, binary = cv2.threshold(gray, 0, 255, THRESH_BINARY + THRESH_OTSU)
//   if np.mean(binary) > 127: binary = cv2.bitwise_not(binary)
// Otsu restates getThreshVal_Otsu_8u (imgproc/src/thresh.cpp, the non-IPP path): a
// 256-bin histogram (per-block LDS histograms merged with global atomics), then the
// sequential double-precision between-class-variance scan, first maximum, in one
// thread (256 dependent steps; the operation order is the reference's).  The inversion
// test mean > 127 is the exact integer test 255 * ones > 127 * n.  Not a hot path.
#include "llfe_internal.h"

namespace llfe {
namespace {

constexpr int TT = 256;

__global__ __launch_bounds__(TT) void k_text_gray(const uint8_t *__restrict__ img, long long n, int cn,
                                                  uint8_t *__restrict__ gray) {
    const long long i = (long long)blockIdx.x * TT + threadIdx.x;
    if (i >= n) return;
    const uint8_t *p = img + i * cn;
    gray[i] = cn >= 3 ? (uint8_t)((p[0] * 1868u + p[1] * 9617u + p[2] * 4899u + 8192u) >> 14) : p[0];
}

// hist[0..255] += counts of this block's pixels (hist zeroed by the caller)
__global__ __launch_bounds__(TT) void k_text_hist(const uint8_t *__restrict__ g, long long n,
                                                  unsigned long long *__restrict__ hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    for (long long i = (long long)blockIdx.x * TT + threadIdx.x; i < n; i += (long long)gridDim.x * TT)
        atomicAdd(&h[g[i]], 1u);
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

// hist[256] <- the Otsu threshold (one thread)
__global__ void k_text_otsu(unsigned long long *__restrict__ hist, long long n) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double mu = 0, scale = 1. / (double)(int)n;
    for (int i = 0; i < 256; i++) mu += i * (double)hist[i];
    mu *= scale;
    double mu1 = 0, q1 = 0, max_sigma = 0, max_val = 0;
    const double eps = 1.1920928955078125e-07;  // FLT_EPSILON
    for (int i = 0; i < 256; i++) {
        const double p_i = (double)hist[i] * scale;
        mu1 *= q1;
        q1 += p_i;
        const double q2 = 1. - q1;
        if (fmin(q1, q2) < eps || fmax(q1, q2) > 1. - eps) continue;
        mu1 = (mu1 + i * p_i) / q1;
        const double mu2 = (mu - q1 * mu1) / q2;
        const double sigma = q1 * q2 * (mu1 - mu2) * (mu1 - mu2);
        if (sigma > max_sigma) {
            max_sigma = sigma;
            max_val = i;
        }
    }
    hist[256] = (unsigned long long)max_val;
    hist[257] = 0;  // count of 255s, accumulated by k_text_binarize
}

__global__ __launch_bounds__(TT) void k_text_binarize(const uint8_t *__restrict__ g, long long n,
                                                      unsigned long long *__restrict__ hist, uint8_t *__restrict__ out) {
    const int t = (int)hist[256];
    unsigned c = 0;
    for (long long i = (long long)blockIdx.x * TT + threadIdx.x; i < n; i += (long long)gridDim.x * TT) {
        const bool on = g[i] > t;
        out[i] = on ? 255 : 0;
        c += on;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(&hist[257], (unsigned long long)c);
}

__global__ __launch_bounds__(TT) void k_text_invert(uint8_t *__restrict__ out, long long n,
                                                    const unsigned long long *__restrict__ hist) {
    if (!(255ull * hist[257] > 127ull * (unsigned long long)n)) return;  // np.mean(binary) > 127
    for (long long i = (long long)blockIdx.x * TT + threadIdx.x; i < n; i += (long long)gridDim.x * TT)
        out[i] = (uint8_t)(255 - out[i]);
}

inline unsigned grid_for(long long n) {
    const long long b = (n + TT - 1) / TT;
    return (unsigned)(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

}  // namespace

hipError_t launch_text_gray(const uint8_t *img, long long n, int cn, uint8_t *gray, hipStream_t s) {
    hipLaunchKernelGGL(k_text_gray, dim3((unsigned)((n + TT - 1) / TT)), dim3(TT), 0, s, img, n, cn, gray);
    return hipGetLastError();
}

hipError_t launch_text_otsu_binary(const uint8_t *g, long long n, unsigned long long *hist, uint8_t *out,
                                   hipStream_t s) {
    hipError_t e = hipMemsetAsync(hist, 0, sizeof(unsigned long long) * 258, s);
    if (e != hipSuccess) return e;
    const unsigned grid = grid_for(n);
    hipLaunchKernelGGL(k_text_hist, dim3(grid), dim3(TT), 0, s, g, n, hist);
    hipLaunchKernelGGL(k_text_otsu, dim3(1), dim3(64), 0, s, hist, n);
    hipLaunchKernelGGL(k_text_binarize, dim3(grid), dim3(TT), 0, s, g, n, hist, out);
    hipLaunchKernelGGL(k_text_invert, dim3(grid), dim3(TT), 0, s, out, n, hist);
    return hipGetLastError();
}

}  // namespace llfe
