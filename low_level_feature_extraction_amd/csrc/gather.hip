// Gather of separately allocated device images into one packed NHWC batch
// (llfe_submit_images: the request path's micro-batches, SURVEY.md 8f row 3 /
// app/api/v1/endpoints/analyze.py:63-129, where every request brings its own image).
//
// One launch per batch instead of a copy per image: grid.y = image, grid.x = slices of
// that image's bytes.  A packed image (row pitch = 3w) is one contiguous span, copied in
// 16-byte vectors when source, destination and span are 16-byte aligned (torch
// allocations and the workspace are; 1080p spans are 388,800 vectors); anything else
// (row pitch > 3w, odd sizes) goes row by row in bytes.  HBM-bound: 2 x 3P bytes per
// image.
#include "llfe_internal.h"

namespace llfe {
namespace {

constexpr int GT = 256;          // threads per workgroup
constexpr int kSlicesPerImage = 48;  // workgroups per image (512 images -> 24k workgroups)

__global__ __launch_bounds__(GT) void k_gather_images(const uint64_t *__restrict__ tab, int n, int h, int rowbytes,
                                                      uint8_t *__restrict__ dst) {
    const int img = blockIdx.y;
    const uint8_t *src = (const uint8_t *)(uintptr_t)tab[img];
    const int64_t pitch = (int64_t)tab[n + img];
    const int64_t span = (int64_t)h * rowbytes;
    uint8_t *out = dst + (int64_t)img * span;
    if (pitch == rowbytes && ((((uintptr_t)src) | ((uintptr_t)out) | (uintptr_t)span) & 15) == 0) {
        const int64_t nv = span >> 4;
        const int64_t per = (nv + gridDim.x - 1) / gridDim.x;
        const int64_t v0 = (int64_t)blockIdx.x * per, v1 = v0 + per < nv ? v0 + per : nv;
        const uint4 *s = (const uint4 *)src;
        uint4 *d = (uint4 *)out;
        int64_t v = v0 + threadIdx.x;
        // four vectors in flight per lane
        for (; v + 3 * GT < v1; v += 4 * GT) {
            const uint4 a = s[v], b = s[v + GT], c = s[v + 2 * GT], e = s[v + 3 * GT];
            d[v] = a;
            d[v + GT] = b;
            d[v + 2 * GT] = c;
            d[v + 3 * GT] = e;
        }
        for (; v < v1; v += GT) d[v] = s[v];
        return;
    }
    const int64_t per = (span + gridDim.x - 1) / gridDim.x;
    const int64_t e0 = (int64_t)blockIdx.x * per, e1 = e0 + per < span ? e0 + per : span;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += GT) {
        const int64_t y = e / rowbytes, x = e - y * rowbytes;
        out[e] = src[y * pitch + x];
    }
}

}  // namespace

hipError_t launch_gather_images(const uint64_t *tab, int n, int h, int w, uint8_t *dst, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_images, dim3(kSlicesPerImage, (unsigned)n), dim3(GT), 0, s, tab, n, h, 3 * w, dst);
    return hipGetLastError();
}

}  // namespace llfe
