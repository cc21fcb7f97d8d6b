// Pillow LANCZOS resample (libImaging/Resample.c semantics) for
// ImageProcessor.auto_process_image's thumbnail (image_processor.py:221-224).
//
// Coefficients are precomputed on the host in double exactly as Pillow's
// precompute_coeffs does and quantised to 22-bit fixed point; the device does the
// two separable int32 passes (horizontal first, u8 intermediate), which makes the
// result bit-identical to Pillow.  One thread per output byte-channel, rows mapped
// to blockIdx.y so that consecutive threads write consecutive bytes.
#include "llfe_internal.h"

namespace llfe {
namespace {

constexpr int PREC = 22;
constexpr int RT = 256;

__device__ __forceinline__ uint8_t clip8(int v) {
    v >>= PREC;
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// (blockIdx.z: image of a same-size batch; src_img / dst_img: bytes between images)
__global__ __launch_bounds__(RT) void k_resize_h(const uint8_t *__restrict__ src, int src_w, int ch, int row0,
                                                 uint8_t *__restrict__ dst, int out_w,
                                                 const int32_t *__restrict__ bounds,
                                                 const int32_t *__restrict__ coeffs, int ksize, long long src_img,
                                                 long long dst_img) {
    const int yy = blockIdx.y;
    src += (size_t)blockIdx.z * src_img;
    dst += (size_t)blockIdx.z * dst_img;
    const int i = blockIdx.x * RT + threadIdx.x;
    if (i >= out_w * ch) return;
    const int xx = i / ch, c = i - xx * ch;
    const int xmin = bounds[2 * xx], xmax = bounds[2 * xx + 1];
    const int32_t *k = coeffs + (size_t)xx * ksize;
    const uint8_t *row = src + ((size_t)(yy + row0) * src_w + xmin) * ch + c;
    int ss = 1 << (PREC - 1);
    for (int x = 0; x < xmax; x++) ss += (int)row[(size_t)x * ch] * k[x];
    dst[(size_t)yy * out_w * ch + i] = clip8(ss);
}

__global__ __launch_bounds__(RT) void k_resize_v(const uint8_t *__restrict__ src, int src_w, int ch,
                                                 uint8_t *__restrict__ dst, const int32_t *__restrict__ bounds,
                                                 const int32_t *__restrict__ coeffs, int ksize, long long src_img,
                                                 long long dst_img) {
    const int yy = blockIdx.y;
    src += (size_t)blockIdx.z * src_img;
    dst += (size_t)blockIdx.z * dst_img;
    const int i = blockIdx.x * RT + threadIdx.x;
    const int rowlen = src_w * ch;
    if (i >= rowlen) return;
    const int ymin = bounds[2 * yy], ymax = bounds[2 * yy + 1];
    const int32_t *k = coeffs + (size_t)yy * ksize;
    const uint8_t *col = src + (size_t)ymin * rowlen + i;
    int ss = 1 << (PREC - 1);
    for (int y = 0; y < ymax; y++) ss += (int)col[(size_t)y * rowlen] * k[y];
    dst[(size_t)yy * rowlen + i] = clip8(ss);
}

// Pillow Image.reduce((fx, fy), box) (libImaging/Reduce.c): box mean with
// out = ((sum + n/2) * floor(2^32 / (256 n))) >> 24, n = pixels in the (possibly
// clipped) box; used by thumbnail(..., reducing_gap=2.0) when the input is >= 4x the
// target in a dimension.
__global__ __launch_bounds__(RT) void k_reduce(const uint8_t *__restrict__ src, int src_w, int ch, int x0, int y0,
                                               int x1, int y1, int fx, int fy, uint8_t *__restrict__ dst, int out_w,
                                               long long src_img, long long dst_img) {
    const int yy = blockIdx.y;
    src += (size_t)blockIdx.z * src_img;
    dst += (size_t)blockIdx.z * dst_img;
    const int i = blockIdx.x * RT + threadIdx.x;
    if (i >= out_w * ch) return;
    const int xx = i / ch, c = i - xx * ch;
    const int ya = y0 + yy * fy, yb = min(y1, ya + fy);
    const int xa = x0 + xx * fx, xb = min(x1, xa + fx);
    const uint32_t n = (uint32_t)((yb - ya) * (xb - xa));
    const uint32_t mult = (uint32_t)(4294967296.0f / (float)(256u * n));
    uint32_t ss = n / 2;
    for (int y = ya; y < yb; y++)
        for (int x = xa; x < xb; x++) ss += src[((size_t)y * src_w + x) * ch + c];
    dst[(size_t)yy * out_w * ch + i] = (uint8_t)((ss * mult) >> 24);
}

}  // namespace

hipError_t launch_reduce(const uint8_t *src, int src_w, int ch, int x0, int y0, int x1, int y1, int fx, int fy,
                         uint8_t *dst, int out_w, int out_h, hipStream_t s, int n, long long src_img,
                         long long dst_img) {
    dim3 grid((out_w * ch + RT - 1) / RT, out_h, n);
    hipLaunchKernelGGL(k_reduce, grid, dim3(RT), 0, s, src, src_w, ch, x0, y0, x1, y1, fx, fy, dst, out_w, src_img,
                       dst_img);
    return hipGetLastError();
}

hipError_t launch_resize_h(const uint8_t *src, int src_h, int src_w, int ch, int row0, int rows, uint8_t *dst,
                           int out_w, const int32_t *bounds, const int32_t *coeffs, int ksize, hipStream_t s, int n,
                           long long src_img, long long dst_img) {
    (void)src_h;
    dim3 grid((out_w * ch + RT - 1) / RT, rows, n);
    hipLaunchKernelGGL(k_resize_h, grid, dim3(RT), 0, s, src, src_w, ch, row0, dst, out_w, bounds, coeffs, ksize,
                       src_img, dst_img);
    return hipGetLastError();
}

hipError_t launch_resize_v(const uint8_t *src, int src_w, int ch, uint8_t *dst, int out_h, const int32_t *bounds,
                           const int32_t *coeffs, int ksize, hipStream_t s, int n, long long src_img,
                           long long dst_img) {
    dim3 grid((src_w * ch + RT - 1) / RT, out_h, n);
    hipLaunchKernelGGL(k_resize_v, grid, dim3(RT), 0, s, src, src_w, ch, dst, bounds, coeffs, ksize, src_img,
                       dst_img);
    return hipGetLastError();
}

}  // namespace llfe
