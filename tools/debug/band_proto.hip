// Prototype: the Canny front of the stencil -- BGR2GRAY, GaussianBlur
// 5x5 and Sobel |dx|+|dy| -- with blur5 and Sobel as exact i8 MFMA products
// (v_mfma_i32_16x16x64_i8) over 16-row bands staged in LDS, against the VALU row-streaming
// kernel of libllfe (llfe_edge_classes: the same front plus NMS).
//
// Layout.  A wave owns a strip of 96 output columns and a segment of rows, and walks
// down it in bands of 16 rows.  Per band: gray of 16 new rows (VALU, as stencil_stream)
// goes to an LDS ring (stored as gray - 128, i8); blur5 of the band is, per 16-column
// tile, D[col][row] = sum_k A[col][k] B[k][row] where B is 16 rows x 64 bytes of the ring
// (lane (g, n): row n of the band shifted by the tap row of group g, 16 columns of the
// tile's 32-column window) and A the constant 5x5 weights (Toeplitz in the columns, the
// vertical weight of each group's tap row): three MFMAs cover the five tap rows; the
// i32 result + 32896 has b in byte 1.  b - 128 goes to a second ring; Sobel dx / dy
// of the band (one row behind) are four MFMAs over two B loads of that ring.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <vector>

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

namespace {

constexpr int OT = 6;          // output tiles per strip (96 columns)
constexpr int BT = OT + 1;     // b / m tiles: ring columns [8 + 16t, 24 + 16t)
constexpr int RS = 144;        // LDS row stride (128 ring columns = image x0 - 16 .. x0 + 112, padded)
constexpr int RING = 32;
constexpr int WAVES = 4;
constexpr int LDS_WAVE = 2 * RING * RS;
constexpr int SEG = 540;
#ifndef BP_MINW
#define BP_MINW 1
#endif
#ifndef BP_UNROLL
#define BP_UNROLL 7
#endif

struct Raw {
    uint32_t a, b, c;
};

__device__ __forceinline__ uint32_t byte_of(uint32_t w, int i) { return (w >> (8 * i)) & 255u; }
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 U(uint32_t v) { return __builtin_bit_cast(u16x2, v); }

__device__ __forceinline__ uint32_t gray4(Raw r) {
    const u16x2 bg0 = U(__builtin_amdgcn_perm(0u, r.a, 0x0c010c00u));
    const u16x2 bg1 = U(__builtin_amdgcn_perm(r.b, r.a, 0x0c040c03u));
    const u16x2 bg2 = U(__builtin_amdgcn_perm(0u, r.b, 0x0c030c02u));
    const u16x2 bg3 = U(__builtin_amdgcn_perm(0u, r.c, 0x0c020c01u));
    const u16x2 wbg = {1868, 9617};
    const uint32_t y0 = __builtin_amdgcn_udot2(bg0, wbg, byte_of(r.a, 2) * 4899u + 8192u, false) >> 14;
    const uint32_t y1 = __builtin_amdgcn_udot2(bg1, wbg, byte_of(r.b, 1) * 4899u + 8192u, false) >> 14;
    const uint32_t y2 = __builtin_amdgcn_udot2(bg2, wbg, byte_of(r.c, 0) * 4899u + 8192u, false) >> 14;
    const uint32_t y3 = __builtin_amdgcn_udot2(bg3, wbg, byte_of(r.c, 3) * 4899u + 8192u, false) >> 14;
    return y0 | (y1 << 8) | (y2 << 16) | (y3 << 24);
}

__device__ __forceinline__ int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// the i8 A operand of lane l for a 16 x (4 groups x 16) product: row m = l & 15, group g
// = l >> 4; fill(m, g, j) -> weight
template <typename F>
__device__ __forceinline__ i32x4 make_a(F fill) {
    const int l = __lane_id(), m = l & 15, g = l >> 4;
    int8_t a[16];
#pragma unroll
    for (int j = 0; j < 16; j++) a[j] = (int8_t)fill(m, g, j);
    i32x4 v;
    __builtin_memcpy(&v, a, 16);
    return v;
}

// group g of a B operand: tap row dr(g) of the pair (dra, drb), window half g >> 1
//   g = 0: (dra, half 0), 1: (drb, half 0), 2: (dra, half 1), 3: (drb, half 1)
// (lanes 0-15 and 20-27 of one ds_read_b128 bank group then read 16 distinct rows)
__device__ __forceinline__ int grp_half(int g) { return g >> 1; }
__device__ __forceinline__ bool grp_second(int g) { return g & 1; }

__device__ __forceinline__ i32x4 lds_b128(const uint8_t *p) { return *(const i32x4 *)p; }

template <bool EDGE, bool DEBUG_M>
__device__ __forceinline__ void band_body(uint8_t *gring, uint8_t *bring, const uint8_t *__restrict__ img, int H, int W,
                                          int x0, int ya, int yb, uint8_t *__restrict__ cimg,
                                          uint16_t *__restrict__ mimg) {
    const int lane = __lane_id();
    const int n = lane & 15, g = lane >> 4;
    const int xr0 = x0 - 16;  // image column of ring column 0
    // ---- constant A operands
    // blur: output column m of the tile sits at window column 8 + m; horizontal tap
    // index c - m - 6 (c = 16 * half + j); vertical weights of the tap pair
    const int wv[5] = {1, 4, 6, 4, 1};
    auto blurA = [&](int dra, int drb) {
        return make_a([&](int m, int gg, int j) {
            const int c = 16 * grp_half(gg) + j, h = c - m - 6;
            const int dr = grp_second(gg) ? drb : dra;
            if (h < 0 || h > 4 || dr > 2) return 0;
            return wv[dr + 2] * wv[h];
        });
    };
    const i32x4 A0 = blurA(-2, -1), A1 = blurA(0, 1), A2 = blurA(2, 9);
    // Sobel: output m at window column 8 + m, horizontal tap c - m - 7 in [0, 2]
    auto sobA = [&](int wa, int wb, bool dx) {
        return make_a([&](int m, int gg, int j) {
            const int c = 16 * grp_half(gg) + j, h = c - m - 7;
            if (h < 0 || h > 2) return 0;
            const int w = grp_second(gg) ? wb : wa;
            return dx ? w * (h - 1) : w * (h == 1 ? 2 : 1);
        });
    };
    const i32x4 GX1 = sobA(1, 2, true), GX2 = sobA(1, 0, true);  // B1 = (y-1, y), B2 = (y+1, -)
    const i32x4 GY1 = sobA(-1, 0, false), GY2 = sobA(1, 0, false);

    auto ring_row = [](int y) { return (y + 4 * RING) & (RING - 1); };
    // ---- gray as an i8 MFMA: D[px][row] = sum_k A[px][k] B[k][row], B = 48 BGR bytes
    // (- 128) of 16 pixels of the row (lane groups 0-2, 16 bytes each; group 3 unused),
    // A = the BGR2GRAY weights split into base-128 digits (1868 = 14*128 + 76, 9617 =
    // 75*128 + 17, 4899 = 38*128 + 35): v = 128 * hi + lo + 2^21 + 8192, gray = v >> 14
    auto grayA = [&](bool hi) {
        return make_a([&](int m, int gg, int j) {
            const int c = 16 * gg + j;
            if (c >= 48 || c / 3 != m) return 0;
            const int ch = c % 3;
            const int wh[3] = {14, 75, 38}, wl[3] = {76, 17, 35};
            return hi ? wh[ch] : wl[ch];
        });
    };
    const i32x4 GH = grayA(true), GL = grayA(false);
    // B operand of gray tile u (16 pixels at image column xr0 + 16 u) for row y of lane n
    auto gray_b = [&](int y, int u) -> i32x4 {
        const int yy = y + n;
        const int sy = ((unsigned)yy < (unsigned)H) ? yy : reflect101(yy, H);
        const uint8_t *row = img + (size_t)sy * W * 3;
        const int px0 = xr0 + 16 * u;
        if (g == 3) return i32x4{0, 0, 0, 0};
        if (!EDGE || (px0 >= 0 && px0 + 16 <= W)) {
            const i32x4 v = *(const i32x4 *)(row + (size_t)px0 * 3 + 16 * g);
            return v ^ (int)0x80808080;
        }
        uint8_t bb[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int c = 16 * g + j;
            bb[j] = row[(size_t)reflect101(px0 + c / 3, W) * 3 + c % 3] ^ 0x80;
        }
        i32x4 v;
        __builtin_memcpy(&v, bb, 16);
        return v;
    };
    auto gray_tile = [&](int y, int u, i32x4 bv) {
        i32x4 hi = {0, 0, 0, 0}, lo = {2105344, 2105344, 2105344, 2105344};
        hi = __builtin_amdgcn_mfma_i32_16x16x64_i8(GH, bv, hi, 0, 0, 0);
        lo = __builtin_amdgcn_mfma_i32_16x16x64_i8(GL, bv, lo, 0, 0, 0);
        uint32_t t[4];
#pragma unroll
        for (int r = 0; r < 4; r++) t[r] = ((uint32_t)hi[r] << 7) + (uint32_t)lo[r] >> 6;  // gray in byte 1
        const uint32_t p01 = __builtin_amdgcn_perm(t[1], t[0], 0x0c0c0501u);
        const uint32_t p23 = __builtin_amdgcn_perm(t[3], t[2], 0x0c0c0501u);
        *(uint32_t *)(gring + ring_row(y + n) * RS + 16 * u + 4 * g) =
            __builtin_amdgcn_perm(p23, p01, 0x05040100u) ^ 0x80808080u;
    };
    auto gray_band = [&](int y, int rows16) {  // gray of rows [y, y + 16)
#pragma unroll
        for (int u = 0; u < 8; u++) gray_tile(y, u, gray_b(y, u));
    };
    const int Y0 = ya - 14;
    gray_band(Y0 - 14, 16);  // rows Y0-14 .. Y0+1 (only Y0-2 .. Y0+1 are used)
    for (int Y = Y0; Y - 1 < yb; Y += 16) {
        gray_band(Y + 2, 16);
        // ---- blur5 of rows [Y, Y + 16)
        const uint8_t *gA = gring + 16 * grp_half(g) + ring_row(Y + n + (grp_second(g) ? -1 : -2)) * RS;
        const uint8_t *gB = gring + 16 * grp_half(g) + ring_row(Y + n + (grp_second(g) ? 1 : 0)) * RS;
        const uint8_t *gC = gring + 16 * grp_half(g) + ring_row(Y + n + 2) * RS;
        uint8_t *bw = bring + ring_row(Y + n) * RS + 8 + 4 * g;
#pragma unroll BP_UNROLL
        for (int t = 0; t < BT; t++) {
            const i32x4 B0 = lds_b128(gA + 16 * t), B1 = lds_b128(gB + 16 * t), B2 = lds_b128(gC + 16 * t);
            i32x4 acc = {32896, 32896, 32896, 32896};
            acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, B0, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, B1, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A2, B2, acc, 0, 0, 0);
            // b = byte 1 of each; pack the lane's 4 columns, store b - 128
            const uint32_t p01 = __builtin_amdgcn_perm((uint32_t)acc[1], (uint32_t)acc[0], 0x0c0c0501u);
            const uint32_t p23 = __builtin_amdgcn_perm((uint32_t)acc[3], (uint32_t)acc[2], 0x0c0c0501u);
            *(uint32_t *)(bw + 16 * t) = __builtin_amdgcn_perm(p23, p01, 0x05040100u) ^ 0x80808080u;
        }
        // (REPLICATE of b beyond the image's columns / rows: not in this prototype)
        // ---- Sobel of rows [Y - 1, Y + 15)
        const int ys = Y - 1 + n;
        const uint8_t *b1 = bring + 16 * grp_half(g) + ring_row(ys + (grp_second(g) ? 0 : -1)) * RS;
        const uint8_t *b2 = bring + 16 * grp_half(g) + ring_row(ys + 1) * RS;
        const bool row_ok = ys >= ya && ys < yb;
        uint8_t *crow = cimg + (size_t)ys * W + x0 - 8 + 4 * g;
#pragma unroll BP_UNROLL
        for (int t = 0; t < BT; t++) {
            const i32x4 B1 = lds_b128(b1 + 16 * t), B2 = lds_b128(b2 + 16 * t);
            i32x4 gx = {2048, 2048, 2048, 2048}, gy = {2048, 2048, 2048, 2048};
            gx = __builtin_amdgcn_mfma_i32_16x16x64_i8(GX1, B1, gx, 0, 0, 0);
            gy = __builtin_amdgcn_mfma_i32_16x16x64_i8(GY1, B1, gy, 0, 0, 0);
            gx = __builtin_amdgcn_mfma_i32_16x16x64_i8(GX2, B2, gx, 0, 0, 0);
            gy = __builtin_amdgcn_mfma_i32_16x16x64_i8(GY2, B2, gy, 0, 0, 0);
            uint32_t m[4];
#pragma unroll
            for (int r = 0; r < 4; r++) m[r] = __sad(gy[r], 2048, __sad(gx[r], 2048, 0u));
            // tile 0 / BT-1 hold output columns in lane groups 2-3 / 0-1 only
            const bool col_ok = (t == 0 ? g >= 2 : (t == BT - 1 ? g < 2 : true));
            const int xc = x0 - 8 + 16 * t + 4 * g;
            if (DEBUG_M) {
                if (row_ok && col_ok)
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        if (xc + r < W) mimg[(size_t)ys * W + xc + r] = (uint16_t)m[r];
            } else if (row_ok && col_ok && (!EDGE || xc + 4 <= W)) {
                uint32_t o = 0;
#pragma unroll
                for (int r = 0; r < 4; r++) o |= (m[r] > 50u ? 0u : 1u) << (8 * r);
                *(uint32_t *)(crow + 16 * t) = o;
            }
        }
    }
}

template <bool DEBUG_M>
__global__ __launch_bounds__(64 * WAVES, BP_MINW) void k_band_front(const uint8_t *__restrict__ bgr, int H, int W, int strips,
                                                           int segs, int total_waves, uint8_t *__restrict__ cls,
                                                           uint16_t *__restrict__ mdbg) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wl = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int wid = blockIdx.x * WAVES + wl;
    if (wid >= total_waves) return;
    uint8_t *gring = smem + wl * LDS_WAVE;
    uint8_t *bring = gring + RING * RS;
    const int strip = wid % strips;
    const int rest = wid / strips;
    const int seg = rest % segs;
    const int img_i = rest / segs;
    const uint8_t *img = bgr + (size_t)img_i * H * W * 3;
    const int x0 = strip * 16 * OT;
    const int ya = seg * SEG, yb = min(H, ya + SEG);
    const bool interior = x0 - 16 >= 0 && x0 + 112 <= W && (W & 3) == 0;
    uint8_t *cimg = cls + (size_t)img_i * H * W;
    uint16_t *mimg = DEBUG_M ? mdbg + (size_t)img_i * H * W : nullptr;
#ifdef BP_NOEDGE
    if (interior) band_body<false, DEBUG_M>(gring, bring, img, H, W, x0, ya, yb, cimg, mimg);
#else
    if (interior)
        band_body<false, DEBUG_M>(gring, bring, img, H, W, x0, ya, yb, cimg, mimg);
    else
        band_body<true, DEBUG_M>(gring, bring, img, H, W, x0, ya, yb, cimg, mimg);
#endif
}

// synthetic 1080p-like images: gradient + rectangles + noise
__global__ void k_synth(uint8_t *out, int n, int H, int W) {
    const size_t P = (size_t)H * W;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (size_t)n * P; i += (size_t)gridDim.x * blockDim.x) {
        const int im = (int)(i / P);
        const int y = (int)((i % P) / W), x = (int)(i % W);
        uint32_t h = (uint32_t)i * 2654435761u ^ (uint32_t)im * 40503u;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        const int noise = (int)(h & 7) - 3;
        int v = (x * 255) / W;
        if (((x / (60 + 17 * (im % 5))) + (y / (45 + 13 * (im % 7)))) % 3 == 0) v = 40 + 30 * (im % 6);
        for (int c = 0; c < 3; c++) {
            int q = v + noise * (c + 1) + 20 * c;
            out[i * 3 + c] = (uint8_t)std::min(255, std::max(0, q));
        }
    }
}

// CPU reference: gray, blur5 (REFLECT_101), Sobel (REPLICATE), m
void ref_m(const uint8_t *bgr, int H, int W, std::vector<uint16_t> &m) {
    auto r101 = [](int p, int len) {
        if (len == 1) return 0;
        while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
        return p;
    };
    std::vector<uint8_t> g((size_t)H * W), b((size_t)H * W);
    for (size_t i = 0; i < (size_t)H * W; i++)
        g[i] = (uint8_t)((bgr[3 * i] * 1868 + bgr[3 * i + 1] * 9617 + bgr[3 * i + 2] * 4899 + 8192) >> 14);
    const int w5[5] = {1, 4, 6, 4, 1};
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            int s = 0;
            for (int i = 0; i < 5; i++)
                for (int j = 0; j < 5; j++) s += w5[i] * w5[j] * g[(size_t)r101(y + i - 2, H) * W + r101(x + j - 2, W)];
            b[(size_t)y * W + x] = (uint8_t)((s + 128) >> 8);
        }
    m.assign((size_t)H * W, 0);
    auto B = [&](int y, int x) { return (int)b[(size_t)std::min(std::max(y, 0), H - 1) * W + std::min(std::max(x, 0), W - 1)]; };
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            const int gx = (B(y - 1, x + 1) + 2 * B(y, x + 1) + B(y + 1, x + 1)) - (B(y - 1, x - 1) + 2 * B(y, x - 1) + B(y + 1, x - 1));
            const int gy = (B(y + 1, x - 1) + 2 * B(y + 1, x) + B(y + 1, x + 1)) - (B(y - 1, x - 1) + 2 * B(y - 1, x) + B(y - 1, x + 1));
            m[(size_t)y * W + x] = (uint16_t)(std::abs(gx) + std::abs(gy));
        }
}

}  // namespace

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 512, H = 1080, W = 1920;
    const int strips = (W + 16 * OT - 1) / (16 * OT), segs = (H + SEG - 1) / SEG;
    const int waves = N * strips * segs, blocks = (waves + WAVES - 1) / WAVES;
    uint8_t *d_img, *d_cls;
    uint16_t *d_m;
    CHK(hipMalloc(&d_img, (size_t)N * H * W * 3));
    CHK(hipMalloc(&d_cls, (size_t)N * H * W));
    CHK(hipMalloc(&d_m, (size_t)2 * H * W * 2));
    hipLaunchKernelGGL(k_synth, dim3(4096), dim3(256), 0, 0, d_img, N, H, W);
    CHK(hipDeviceSynchronize());
    const size_t lds = (size_t)WAVES * LDS_WAVE;
    // ---- validation of m on 2 images (interior columns / rows only in this prototype)
    CHK(hipMemset(d_m, 0xff, (size_t)2 * H * W * 2));
    const int vw = 2 * strips * segs;
    hipLaunchKernelGGL(k_band_front<true>, dim3((vw + WAVES - 1) / WAVES), dim3(64 * WAVES), lds, 0, d_img, H, W,
                       strips, segs, vw, d_cls, d_m);
    CHK(hipDeviceSynchronize());
    std::vector<uint8_t> h_img((size_t)2 * H * W * 3);
    std::vector<uint16_t> h_m((size_t)2 * H * W);
    CHK(hipMemcpy(h_img.data(), d_img, h_img.size(), hipMemcpyDeviceToHost));
    CHK(hipMemcpy(h_m.data(), d_m, h_m.size() * 2, hipMemcpyDeviceToHost));
    long bad = 0, checked = 0;
    for (int i = 0; i < 2; i++) {
        std::vector<uint16_t> ref;
        ref_m(h_img.data() + (size_t)i * H * W * 3, H, W, ref);
        for (int y = 1; y < H - 1; y++)
            for (int x = 16; x < W - 16; x++) {
                const size_t k = (size_t)y * W + x;
                checked++;
                if (h_m[(size_t)i * H * W + k] != ref[k]) {
                    if (bad < 5)
                        printf("mismatch img %d y %d x %d: got %d want %d\n", i, y, x, h_m[(size_t)i * H * W + k], ref[k]);
                    bad++;
                }
            }
    }
    printf("validation: %ld / %ld interior pixels differ\n", bad, checked);
    // ---- timing: band prototype
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; rep++)
        hipLaunchKernelGGL(k_band_front<false>, dim3(blocks), dim3(64 * WAVES), lds, 0, d_img, H, W, strips, segs, waves,
                           d_cls, d_m);
    CHK(hipDeviceSynchronize());
    const int R = 10;
    CHK(hipEventRecord(e0, 0));
    for (int rep = 0; rep < R; rep++)
        hipLaunchKernelGGL(k_band_front<false>, dim3(blocks), dim3(64 * WAVES), lds, 0, d_img, H, W, strips, segs, waves,
                           d_cls, d_m);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("band front (gray+blur5+Sobel+m, MFMA): %.3f ms per %d images\n", ms / R, N);
    // ---- timing: libllfe's row-streaming kernel, cls only (gray+blur5+Sobel+NMS)
    void *h = dlopen(argc > 2 ? argv[2] : "low_level_feature_extraction_amd/libllfe.so", RTLD_NOW);
    if (!h) {
        printf("no libllfe: %s\n", dlerror());
        return 0;
    }
    typedef int (*init_t)(int, void **);
    typedef int (*edge_t)(void *, const uint8_t *, uint8_t *, int, int, int, void *);
    auto init = (init_t)dlsym(h, "llfe_init");
    auto edge = (edge_t)dlsym(h, "llfe_edge_classes");
    void *ctx = nullptr;
    if (init(0, &ctx) != 0) {
        printf("llfe_init failed\n");
        return 0;
    }
    for (int rep = 0; rep < 2; rep++) edge(ctx, d_img, d_cls, N, H, W, nullptr);
    auto t0 = std::chrono::steady_clock::now();
    for (int rep = 0; rep < R; rep++) edge(ctx, d_img, d_cls, N, H, W, nullptr);
    auto t1 = std::chrono::steady_clock::now();
    printf("libllfe k_stencil_stream<cls> (gray+blur5+Sobel+NMS, VALU): %.3f ms per %d images (host-timed, incl. sync)\n",
           std::chrono::duration<double, std::milli>(t1 - t0).count() / R, N);
    return 0;
}
