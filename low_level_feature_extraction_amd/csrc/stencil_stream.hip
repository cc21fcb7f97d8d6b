// Row-streaming stencil front-end of the shapes + shadows path on gfx950.
//
// Replaces, per pixel, the native work of
//   gray   = cvtColor(BGR2GRAY)                        shape pyc @L18, shadow pyc @L8
//   blur   = GaussianBlur(gray, (5,5), 0) 8U bit-exact shape pyc @L21, shadow pyc @L9
//   Canny  : Sobel3 (REPLICATE) -> |dx|+|dy| -> NMS    shape pyc @L24 (classes 0/1/2)
//   shadow : adaptiveThreshold GAUSSIAN_C 11, C=2, INV  shadow pyc @L17-24
//            mean = rint(CV_32F Gauss11(blur)), mask = blur - mean <= -2,
//            sum / count of blur under the mask
// with the same arithmetic as the tiled kernel (stencil.hip) and the oracle.
//
// Layout.  One wave owns a vertical strip of 256 columns (64 lanes x 4 pixels, one
// packed dword of gray / blur per lane) and marches down a segment of rows.  Of the 64
// lanes, 2 on each side are halo (8 columns): every horizontal neighbour a pixel
// needs -- blur5 +-2, Sobel / NMS +-1, Gauss11 +-5 on the blurred row -- comes from lanes
// L-2 .. L+2 through DPP wave shifts, so 240 columns per wave are exact (1920 = 8 x
// 240).  Vertical neighbours live in registers, in rings whose lengths divide the
// 12-step unroll of the row loop (gray rows 6, blurred rows 6, CV_32F row-pass results 12,
// magnitude rows 3), so every ring slot is a fixed register and no step moves ring data.
// One BGR row is loaded per step, five steps ahead, straight into a per-wave LDS ring of 6
// rows (round 6: 12-byte direct-to-LDS loads, a counted vmcnt wait before a row is read;
// the round-5 kernel held 3 input rows in VGPRs, two steps ahead); each pixel is read from
// HBM once plus a 10/216-row halo (the 16/256-column halo of neighbouring strips hits L2);
// no barriers, no halo recomputation beyond those margins.
//
// Per step (blur row c = clamp(t, 0, H-1) enters; REPLICATE of the blurred image):
//   gray row reflect101(c + 2) -> vertical then horizontal blur5 (exact integer, any
//   order: (sum w_i w_j g + 128) >> 8 in packed u16) -> blur ring
//   CV_32F row pass of the blurred row (fma chain left -> right) -> Gauss ring
//   Sobel on blurred rows t-2..t (packed i16) -> |dx|+|dy| | dir << 12 -> magnitude ring
//   NMS of row t-2 from magnitude rows t-3..t-1 -> class map row t-2
//   column pass (centre, then symmetric pairs inner -> outer) of row t-5, rint,
//   mask, masked sum / count
#include <algorithm>

#include "llfe_internal.h"

namespace llfe {
namespace {

__device__ __constant__ constexpr float kGauss11[11] = {LLFE_GAUSS11_F32};

// (analysis builds only, -DLLFE_ST_MARK: stage markers in the ISA for the per-stage
// instruction table of tools/stencil_isa.py)
// ST_PIN(x) materialises a stage's result before the next marker, so code motion cannot
// sink the stage's instructions into a later one
#if LLFE_ST_MARK
#define ST_MARK(name) do { __builtin_amdgcn_sched_barrier(0); asm volatile(";@st " #name); __builtin_amdgcn_sched_barrier(0); } while (0)
#define ST_PIN(x) asm volatile("" : "+v"(x))
#define ST_RARE() asm volatile(";@rare")
#else
#define ST_RARE()
#define ST_MARK(name)
#define ST_PIN(x)
#endif

constexpr int kLanesOut = 60;               // lanes 2 .. 61 produce output
constexpr int kStripW = 4 * kLanesOut;      // 240 output columns per wave
constexpr int kHalo = 8;                    // columns left of the strip's first output
#ifndef LLFE_ST_WPB
#define LLFE_ST_WPB 4
#endif
constexpr int kWavesPerBlock = LLFE_ST_WPB;

typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef int16_t i16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 U(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ i16x2 I(uint32_t v) { return __builtin_bit_cast(i16x2, v); }
__device__ __forceinline__ uint32_t W32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t W32(i16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t byte_of(uint32_t w, int i) { return (w >> (8 * i)) & 255u; }

// DPP wave shifts: from_left(v) in lane L is v of lane L-1; from_right(v) of lane L+1
// (bound_ctrl: the lanes shifted in at the wave's ends read 0 -- they are halo lanes)
__device__ __forceinline__ uint32_t from_left(uint32_t v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, true); }
__device__ __forceinline__ uint32_t from_right(uint32_t v) { return __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, true); }
// (hi16 of a, lo16 of b) -> the u16 pair straddling two adjacent dwords a, b
__device__ __forceinline__ uint32_t mid16(uint32_t a, uint32_t b) { return __builtin_amdgcn_alignbit(b, a, 16); }

__device__ __forceinline__ int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

struct Raw {
    uint32_t a, b, c;
};

// 4 BGR pixels of row y at the lane's columns: one aligned 12-byte load when the whole
// wave is inside the image (wave-uniform `fast`), else 12 byte loads from the
// REFLECT_101 columns precomputed in coff (byte offsets within a row)
__device__ __forceinline__ Raw load_px(const uint8_t *__restrict__ img, int y, int W, int x, bool fast,
                                       const uint32_t coff[4]) {
    const uint8_t *row = img + (size_t)y * W * 3;  // 64-bit: h * w * 3 may pass 2^31
    Raw r;
    if (fast) {
        const uint32_t *p = (const uint32_t *)(row + (uint32_t)(x * 3));
        // plain (not non-temporal) loads: the neighbouring strips' 16-column halo then
        // comes from L2 (PMC FETCH_SIZE -6 %: 1.02x the 3P input instead of 1.08x)
        r.a = p[0];
        r.b = p[1];
        r.c = p[2];
    } else {
        uint32_t v[3] = {0, 0, 0};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint8_t *q = row + coff[j];
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const int k = 3 * j + c;
                v[k >> 2] |= (uint32_t)q[c] << (8 * (k & 3));
            }
        }
        r.a = v[0];
        r.b = v[1];
        r.c = v[2];
    }
    return r;
}

// Y = (B*1868 + G*9617 + R*4899 + 2^13) >> 14 for the 4 pixels -> packed u8x4
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

// {1, 1} the optimiser cannot see: min(sub_sat(a, b), 1) with a visible 1 is folded into
// a per-half compare (a > b), which gfx950 has only for one u16 at a time -- two v_cmp, two
// v_cndmask and a v_perm instead of one v_pk_min_u16 per pair (ISA, tools/stencil_isa.py)
__device__ __forceinline__ uint32_t opaque_ones() {
    uint32_t v;
    asm("s_mov_b32 %0, 0x10001" : "=s"(v));
    return v;
}

__device__ __forceinline__ uint32_t lo2(uint32_t g) { return __builtin_amdgcn_perm(0u, g, 0x0c010c00u); }  // bytes 0,1 -> u16x2
__device__ __forceinline__ uint32_t hi2(uint32_t g) { return __builtin_amdgcn_perm(0u, g, 0x0c030c02u); }  // bytes 2,3 -> u16x2

// blur5 of the lane's 4 columns from the 5 gray rows (vertical taps unscaled, then the
// horizontal taps with the neighbours' vertical sums; (sum + 128) >> 8 -- exact)
__device__ __forceinline__ uint32_t blur4(uint32_t g0, uint32_t g1, uint32_t g2, uint32_t g3, uint32_t g4) {
    const u16x2 four = {4, 4}, six = {6, 6};
    const u16x2 vlo = (U(lo2(g1)) + U(lo2(g3))) * four + (U(lo2(g0)) + U(lo2(g4))) + U(lo2(g2)) * six;
    const u16x2 vhi = (U(hi2(g1)) + U(hi2(g3))) * four + (U(hi2(g0)) + U(hi2(g4))) + U(hi2(g2)) * six;
    const uint32_t A = from_left(W32(vhi));   // cols c-2, c-1
    const uint32_t B = W32(vlo), C = W32(vhi);
    const uint32_t D = from_right(W32(vlo));  // cols c+4, c+5
    const u16x2 pm1 = U(mid16(A, B)), p1 = U(mid16(B, C)), p3 = U(mid16(C, D));
    const u16x2 r128 = {128, 128}, e8 = {8, 8};
    const u16x2 hlo = ((pm1 + p1) * four + (U(A) + U(C)) + U(B) * six + r128) >> e8;
    const u16x2 hhi = ((p1 + p3) * four + (U(B) + U(D)) + U(C) * six + r128) >> e8;
    return __builtin_amdgcn_perm(W32(hhi), W32(hlo), 0x06040200u);
}

// Sobel (3x3, on REPLICATE'd blurred rows b0 above, b1, b2 below) -> |dx|+|dy| and the
// Canny NMS direction class (0 horizontal, 1 vertical, 2 / 3 diagonals) as
// m | dir << 12 in two u16x2 dwords (cols c0 c1 | c2 c3)
// `live`: the lane holds output columns.  Only those decide whether the wave's row needs the
// direction classes and NMS: the halo lanes 0 / 63 read zeros past the wave's edge (DPP
// bound_ctrl), so their magnitudes are not the image's and would make every row look like it
// has a candidate (round 4 / early round 5: the direction + NMS code ran on every row).
__device__ __forceinline__ bool sobel4(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t &mlo, uint32_t &mhi,
                                       bool live) {
    const u16x2 two = {2, 2};
    const u16x2 vs_lo = U(lo2(b0)) + U(lo2(b2)) + U(lo2(b1)) * two;  // [1 2 1] vertical
    const u16x2 vs_hi = U(hi2(b0)) + U(hi2(b2)) + U(hi2(b1)) * two;
    const u16x2 vd_lo = U(lo2(b2)) - U(lo2(b0));                       // [-1 0 1] vertical
    const u16x2 vd_hi = U(hi2(b2)) - U(hi2(b0));
    const uint32_t sL = from_left(W32(vs_hi)), sR = from_right(W32(vs_lo));
    const uint32_t dL = from_left(W32(vd_hi)), dR = from_right(W32(vd_lo));
    // gx(c) = vs(c+1) - vs(c-1); gy(c) = vd(c-1) + 2 vd(c) + vd(c+1)
    const i16x2 gx_lo = I(mid16(W32(vs_lo), W32(vs_hi))) - I(mid16(sL, W32(vs_lo)));
    const i16x2 gx_hi = I(mid16(W32(vs_hi), sR)) - I(mid16(W32(vs_lo), W32(vs_hi)));
    const i16x2 t2 = {2, 2};
    const i16x2 gy_lo = I(mid16(dL, W32(vd_lo))) + I(mid16(W32(vd_lo), W32(vd_hi))) + I(W32(vd_lo)) * t2;
    const i16x2 gy_hi = I(mid16(W32(vd_lo), W32(vd_hi))) + I(mid16(W32(vd_hi), dR)) + I(W32(vd_hi)) * t2;
    const i16x2 z = {0, 0};
    const i16x2 ax_lo = __builtin_elementwise_max(gx_lo, z - gx_lo), ax_hi = __builtin_elementwise_max(gx_hi, z - gx_hi);
    const i16x2 ay_lo = __builtin_elementwise_max(gy_lo, z - gy_lo), ay_hi = __builtin_elementwise_max(gy_hi, z - gy_hi);
    const i16x2 m_lo = ax_lo + ay_lo, m_hi = ax_hi + ay_hi;
    uint32_t lo = W32(m_lo), hi = W32(m_hi);
    // the direction class matters only where m > LOW (the NMS below): computed, without
    // branches, only when some lane of the wave has such a pixel
    constexpr int LOW = 50, TG22 = 13573;
    const bool need = live && ((int)m_lo.x > LOW || (int)m_lo.y > LOW || (int)m_hi.x > LOW || (int)m_hi.y > LOW);
    const bool wave_need = __ballot(need) != 0;
    if (wave_need) {
        ST_MARK(direction);
        const int gxs[4] = {gx_lo.x, gx_lo.y, gx_hi.x, gx_hi.y};
        const int gys[4] = {gy_lo.x, gy_lo.y, gy_hi.x, gy_hi.y};
        const int axs[4] = {ax_lo.x, ax_lo.y, ax_hi.x, ax_hi.y};
        const int ays[4] = {ay_lo.x, ay_lo.y, ay_hi.x, ay_hi.y};
        uint32_t d[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int ax = axs[j], ay = ays[j] << 15, tg22x = ax * TG22;
            // 0 if ay < tg22x, else 1 if ay > tg22x + ax * 2^16, else 2 / 3 by the signs --
            // as arithmetic on 0/1 flags, so the compiler emits no branches
            const uint32_t diag = 3u - (uint32_t)((gxs[j] ^ gys[j]) < 0);
            const uint32_t ge = (uint32_t)(ay >= tg22x), steep = (uint32_t)(ay > tg22x + (ax << 16));
            d[j] = ge * (diag - steep * (diag - 1u));
        }
        lo |= (d[0] << 12) | (d[1] << 28);
        hi |= (d[2] << 12) | (d[3] << 28);
        ST_MARK(direction_end);
    }
    mlo = lo;
    mhi = hi;
    return wave_need;  // some pixel of the wave's row has m > LOW (a Canny candidate)
}

// Canny NMS + double threshold of the lane's 4 pixels of the middle magnitude row;
// a = above, m = middle, b = below (lo = cols c0 c1, hi = c2 c3, m | dir << 12).  Called
// by the whole wave (DPP).  In packed u16 on the (c0, c1) and (c2, c3) pairs: the four
// directions' thresholds -- keep iff m >= T with
//   dir 0 (left / right):           T = max(left + 1, right)
//   dir 1 (up / down):              T = max(up + 1, down)
//   dir 2 (up-right / down-left):   T = max(up-right, down-left) + 1
//   dir 3 (up-left / down-right):   T = max(up-left, down-right) + 1
// (the second neighbour takes >= for 0 / 1, > for the diagonals), then the pixel's own
// threshold picked by v_bfi on its two direction bits, max'ed with LOW + 1, and the class
// from saturating subtractions -- no per-pixel unpacking, compares or selects.
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }
__device__ __forceinline__ uint32_t nms4(uint32_t alo, uint32_t ahi, uint32_t mlo, uint32_t mhi, uint32_t blo,
                                         uint32_t bhi) {
    constexpr uint32_t MK = 0x0FFF0FFFu;
    const uint32_t A0 = alo & MK, A1 = ahi & MK, M0 = mlo & MK, M1 = mhi & MK, B0 = blo & MK, B1 = bhi & MK;
    // the neighbour lanes' dwords: cols (c-2, c-1) from the left, (c+4, c+5) from the right
    const uint32_t Ap = from_left(A1), An = from_right(A0), Mp = from_left(M1), Mn = from_right(M0),
                   Bp = from_left(B1), Bn = from_right(B0);
    const u16x2 one = {1, 1}, low1 = {51, 51}, high1 = {151, 151}, one_o = U(opaque_ones());
    auto cls2 = [&](uint32_t Ac, uint32_t AL, uint32_t AR, uint32_t Mc, uint32_t ML, uint32_t MR, uint32_t Bc,
                    uint32_t BL, uint32_t BR, uint32_t mraw) {
        const u16x2 t0 = __builtin_elementwise_max(U(ML) + one, U(MR));
        const u16x2 t1 = __builtin_elementwise_max(U(Ac) + one, U(Bc));
        const u16x2 t2 = __builtin_elementwise_max(U(AR), U(BL)) + one;
        const u16x2 t3 = __builtin_elementwise_max(U(AL), U(BR)) + one;
        const u16x2 z = {0, 0};
        const uint32_t m0 = W32(z - U((mraw >> 12) & 0x00010001u));  // dir bit 0 -> 0xffff per half
        const uint32_t m1 = W32(z - U((mraw >> 13) & 0x00010001u));  // dir bit 1
        const uint32_t T = bsel(m1, bsel(m0, W32(t3), W32(t2)), bsel(m0, W32(t1), W32(t0)));
        const u16x2 Tm = __builtin_elementwise_max(U(T), low1);
        const u16x2 nk = __builtin_elementwise_min(__builtin_elementwise_sub_sat(Tm, U(Mc)), one_o);    // 1: suppressed
        const u16x2 ns = __builtin_elementwise_min(__builtin_elementwise_sub_sat(high1, U(Mc)), one_o); // 1: not strong
        const uint32_t k2 = (W32(nk) | W32(ns)) ^ 0x00010001u;  // kept and strong
        return W32(nk) | (k2 + k2);                             // 1 suppressed, 2 strong, 0 weak
    };
    const uint32_t mid_a = mid16(A0, A1), mid_m = mid16(M0, M1), mid_b = mid16(B0, B1);
    const uint32_t c0 = cls2(A0, mid16(Ap, A0), mid_a, M0, mid16(Mp, M0), mid_m, B0, mid16(Bp, B0), mid_b, mlo);
    const uint32_t c1 = cls2(A1, mid_a, mid16(A1, An), M1, mid_m, mid16(M1, Mn), B1, mid_b, mid16(B1, Bn), mhi);
    return __builtin_amdgcn_perm(c1, c0, 0x06040200u);
}

// CV_32F Gauss11 row pass (s = 0; s = fma(x[k-5], k[k], s) left -> right) of the lane's
// 4 columns of one blurred row B; taps reach lanes L-2 .. L+2.  Packed FP32: columns c0
// and c2 share one v_pk_fma_f32 chain (operand pairs (x[k], x[k+2])), c1 and c3 the
// other ((x[k+1], x[k+3])) -- each lane of a pair is its own exact fma chain, in order
__device__ __forceinline__ void rowpass4(uint32_t B, const float *__restrict__ k11, f32x2 &o02, f32x2 &o13) {
    const uint32_t l1 = from_left(B), l2 = from_left(l1), r1 = from_right(B), r2 = from_right(r1);
    // taps for column c0 + j: bytes (c0 - 5 + j) .. (c0 + 5 + j); index 0 = c0 - 5
    float x[14];
    x[0] = (float)byte_of(l2, 3);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        x[1 + i] = (float)byte_of(l1, i);
        x[5 + i] = (float)byte_of(B, i);
        x[9 + i] = (float)byte_of(r1, i);
    }
    x[13] = (float)byte_of(r2, 0);
    f32x2 a = {0.0f, 0.0f}, b = {0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < 11; k++) {
        const f32x2 w = {k11[k], k11[k]};
        a = __builtin_elementwise_fma(f32x2{x[k], x[k + 2]}, w, a);
        b = __builtin_elementwise_fma(f32x2{x[k + 1], x[k + 3]}, w, b);
    }
    o02 = a;
    o13 = b;
}

#ifndef LLFE_ST_MINW
#define LLFE_ST_MINW 4
#endif
#ifndef LLFE_ST_LPT
#define LLFE_ST_LPT 0
#endif
#ifndef LLFE_ST_QD
#define LLFE_ST_QD 3  // input-row ring length: rows are loaded QD - 1 steps before use (divides 12)
#endif
#ifndef LLFE_ST_LDSQ
#define LLFE_ST_LDSQ 6  // > 0: input rows through a per-wave LDS ring of this depth (divides 12), loaded
                        // LDSQ - 1 steps ahead by direct-to-LDS loads (buffer loads with range checks
                        // for border waves; byte loads for unaligned rows); 0: the Q VGPR ring
                        // (rows two steps ahead; 2.60-2.65 vs 2.32-2.38 ms per 512 x 1080p, round 6)
#endif
#ifndef LLFE_ST_HOTROW
#define LLFE_ST_HOTROW 0  // (timing experiments only: every step loads the segment's first row, L2-hot)
#endif
#ifndef LLFE_ST_NOSTORE
#define LLFE_ST_NOSTORE 0  // (timing experiments only: no class-map stores, wrong results)
#endif
#ifndef LLFE_ST_STORE_AUX
#define LLFE_ST_STORE_AUX 2  // the class-map stores' cache policy (2: non-temporal)
#endif
// One wave's work item: strip x segment of one image.  `wid` is wave-uniform (an SGPR):
// every per-wave quantity below -- strip, segment, row bounds, border flags -- then stays
// scalar and its branches cost no exec masking.
template <bool CLS, bool SHD>
__device__ __forceinline__ void stencil_wave(int wid, const uint8_t *__restrict__ bgr, int H, int W, int strips,
                                             int segs, int seg_rows, int vec, uint8_t *__restrict__ cls,
                                             uint2 *__restrict__ wave_part, const StencilParams &prm) {
    const int lane = threadIdx.x & 63;
    const int strip = wid % strips;
    const int rest = wid / strips;
    const int seg = rest % segs;
    const int img_i = rest / segs;
    const uint8_t *img = prm.img_tab ? (const uint8_t *)prm.img_tab[img_i] : bgr + (size_t)img_i * H * W * 3;
    uint8_t *cimg = CLS ? cls + (size_t)img_i * H * W : nullptr;
    // the image's class map as a buffer (H * W < 2^31 bytes: valid_dims)
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(cimg, (short)0, CLS ? H * W : 0, 0x00020000);
    const int ya = seg * seg_rows, yb = min(H, ya + seg_rows);
    const int x = strip * kStripW - kHalo + 4 * lane;  // the lane's first column
    const bool out_lane = lane >= 2 && lane < 2 + kLanesOut && x < W;
    const bool out_fast = out_lane && vec && x + 4 <= W;
    // wave covers the left / right image border: gray columns outside are REFLECT_101'd
    // (byte loads), blurred columns outside REPLICATE'd; interior waves load 12 aligned
    // bytes per lane
    const int xw0 = strip * kStripW - kHalo, xw1 = xw0 + 256;
    const bool edge_l = xw0 < 0, edge_r = xw1 > W;
    const bool edge = edge_l || edge_r;
    const bool fast = vec && !edge;  // wave-uniform
    uint32_t coff[4];
#pragma unroll
    for (int j = 0; j < 4; j++) coff[j] = (uint32_t)(reflect101(x + j, W) * 3);
    // blurred bytes of column 0 / W-1 (REPLICATE) come from these lanes
    const int lane0 = (0 - xw0) >> 2, laneW = (W - 1 - xw0) >> 2;
    uint32_t rep_l = 0, rep_r = 0;  // bytes of the lane left of column 0 / right of W-1
    // per-column "inside the image" masks for the magnitude (Canny: no magnitude outside)
    uint32_t in_lo = 0xffffffffu, in_hi = 0xffffffffu;
    uint32_t in_02 = 0x00010001u, in_13 = 0x00010001u;  // the same, 1 per u16 half, columns (0, 2) / (1, 3)
    if (edge) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (x + j < 0) rep_l |= 255u << (8 * j);
            if (x + j >= W) rep_r |= 255u << (8 * j);
        }
        in_lo = ((unsigned)x < (unsigned)W ? 0xffffu : 0u) | ((unsigned)(x + 1) < (unsigned)W ? 0xffff0000u : 0u);
        in_hi = ((unsigned)(x + 2) < (unsigned)W ? 0xffffu : 0u) | ((unsigned)(x + 3) < (unsigned)W ? 0xffff0000u : 0u);
        in_02 = ((unsigned)x < (unsigned)W ? 1u : 0u) | ((unsigned)(x + 2) < (unsigned)W ? 0x10000u : 0u);
        in_13 = ((unsigned)(x + 1) < (unsigned)W ? 1u : 0u) | ((unsigned)(x + 3) < (unsigned)W ? 0x10000u : 0u);
    }
    // the CV_32F 11-tap Gaussian (ksize 11, sigma 0: OpenCV's getGaussianKernel, computed in
    // double and rounded to float) as constants, not kernel arguments: the compiler can
    // rematerialise them instead of holding 11 SGPRs through the loop (the kernel is at the
    // SGPR limit).  llfe_create checks prm.k11 against this table (kGauss11).
    const float *k11 = kGauss11;

    // Row steps t (one blurred row enters per step; the loop is unrolled kU = 12 times and
    // every ring's length divides 12, so each ring slot is a fixed register and no step
    // moves ring data -- round 4's 11-row unroll shifted its gray / input / magnitude rings
    // by register moves every step):
    //   input rows  LDS ring qr[6] (LLFE_ST_LDSQ; Q[3] in VGPRs without it): virtual row
    //                      v = t + QD + 1 issued at step t, consumed at step t + QD - 1
    //   gray rows   G[6]   virtual row v = t + 2 converted at step t, slot v % 6 (gray row
    //                      reflect101(v): blur row t reads virtual rows t - 2 .. t + 2)
    //   blurred     bring[6]: row t, slot t % 6 (read back to row t - 5); CV_32F row pass
//               ra / rb[12]: row t, slot t % 12 (the column pass reads rows t - 10 .. t)
    //   magnitude   Mlo / Mhi / Mc[3]: row t - 1 (computed at step t), slot t % 3
    // Steps t0 - 6, t0 - 5 only issue loads, t0 - 4 .. t0 - 1 also convert gray rows; from
    // max(t0, 0) on a step computes its blurred row.  REPLICATE of the blurred image: rows
    // t >= H copy row t - 1; rows -5 .. -1 (the first segment) are filled with row 0 when it
    // is computed, at step 0, before anything reads them.
    constexpr int kU = 12;
#if LLFE_ST_LDSQ
    constexpr int QD = LLFE_ST_LDSQ;
    // this wave's ring: QD rows of 64 lanes x 16 bytes -- a 12-byte direct-to-LDS load puts lane
    // l's bytes at l * 16, not l * 12 (measured, tools/debug/glds_probe.hip)
    __shared__ __attribute__((aligned(16))) uint32_t qring[kWavesPerBlock][QD][256];
    uint32_t(*const qr)[256] = qring[__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))];
    // border waves load the window's raw row (x * 3 .. x * 3 + 11 per lane) through a buffer
    // resource, so lanes left of column 0 / past the image's end read zeros instead of
    // faulting, and take each pixel's REFLECT_101 column from the row in LDS (byte offsets
    // within the window; every column a needed lane reflects to lies in it, others clamp)
    // (32-bit buffer offsets: border waves of images of 2^31 bytes or more take the byte path)
    const bool small_img = (long long)H * W * 3 < 0x7fffffffll;
    const __amdgpu_buffer_rsrc_t irs =
        __builtin_amdgcn_make_buffer_rsrc((void *)img, (short)0, small_img ? H * W * 3 : 0, 0x00020000);
    // LDS byte offset of each of the lane's REFLECT_101 columns in the ring row (column c of the
    // window, d = c - xw0: lane d >> 2 at 16 B a lane, pixel d & 3 at 3 B a pixel); only border
    // waves read them, out-of-window columns of lanes no output needs clamp to the row
    // (held in coff, whose byte offsets only the unaligned-row path reads)
    if (vec && small_img) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int d = min(max(reflect101(x + j, W) - xw0, 0), 255);
            coff[j] = (uint32_t)((d >> 2) * 16 + (d & 3) * 3);
        }
    }
#else
    constexpr int QD = LLFE_ST_QD;
#endif
    static_assert(kU % QD == 0, "the input ring's length must divide the unroll");
    const int t0 = ya - 5, t_end = yb + 5, ts = t0 - 6 - (QD - 3), tf = max(t0, 0);
    const int tb0 = ts >= 0 ? ts - ts % kU : -(((-ts) + kU - 1) / kU) * kU;  // floor to a multiple of kU
#if !LLFE_ST_LDSQ
    Raw Q[QD];
#endif
    uint32_t G[6], bring[6], Mlo[3], Mhi[3];
    bool Mc[3];
    f32x2 ra[kU], rb[kU];
#pragma unroll
    for (int k = 0; k < kU; k++) ra[k] = rb[k] = f32x2{0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < 6; k++) G[k] = bring[k] = 0;
#pragma unroll
    for (int k = 0; k < QD; k++) {
#if LLFE_ST_LDSQ
        qr[k][4 * lane] = qr[k][4 * lane + 1] = qr[k][4 * lane + 2] = 0u;
#else
        Q[k] = Raw{0u, 0u, 0u};
#endif
    }
#pragma unroll
    for (int k = 0; k < 3; k++) {
        Mlo[k] = Mhi[k] = 0;
        Mc[k] = false;
    }
    uint32_t lsum = 0, lcnt = 0;
    // hysteresis tile flags (prm.tflag): an output lane whose NMS row holds a class != 1
    // pixel sets its 64 x 64 tile's byte (measured against OR-ing a ballot per row and
    // storing once per 64-row band: the per-row stores cost the stencil nothing, the band
    // flushes +90 us per 512 x 1080p through their register pressure)
    const int tf_ntx = (W + 63) >> 6;
    uint8_t *const tf_img = CLS && prm.tflag ? prm.tflag + (size_t)img_i * ((H + 63) >> 6) * tf_ntx : nullptr;

    for (int tb = tb0; tb < t_end; tb += kU) {
#pragma unroll
        for (int k = 0; k < kU; k++) {
            const int t = tb + k;
            if (t >= ts && t < t_end) {  // (no break: the loop must unroll so ring slots are registers)
            ST_MARK(load);
#if LLFE_ST_LDSQ
            if (t + QD - 1 < t_end) {
                const int yl = reflect101(t + QD + 1, H);
                uint32_t *const slot = &qr[(k + QD - 1) % QD][0];
                if (fast) {
                    __builtin_amdgcn_global_load_lds((const void *)(img + (size_t)yl * W * 3 + (uint32_t)(x * 3)),
                                                     (void *)slot, 12, 0, 0);
                } else if (vec && small_img) {
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(irs, (__attribute__((address_space(3))) void *)slot, 12,
                                                             yl * W * 3 + x * 3, 0, 0, 0);
                } else {  // unaligned rows: byte loads (REFLECT_101 columns), written now
                    const Raw r = load_px(img, yl, W, x, false, coff);
                    slot[4 * lane] = r.a;
                    slot[4 * lane + 1] = r.b;
                    slot[4 * lane + 2] = r.c;
                }
            }
            if (t >= ts + QD - 1) {
                ST_MARK(gray);
                // the direct-to-LDS row issued QD - 1 steps ago has landed once at most QD - 2
                // younger vector-memory operations are outstanding (they complete in order;
                // the compiler does not track these loads)
                if (vec) __builtin_amdgcn_s_waitcnt(((QD - 2) & 15) | (7 << 4) | (15 << 8) | (((QD - 2) >> 4) << 14));
                Raw cur;
                if (edge && vec && small_img) {
                    // (32-bit LDS addresses: with generic pointers the compiler hoisted a 64-bit
                    // address per byte and slot out of the loop and spilled 100 VGPRs)
                    const uint32_t rbase = (uint32_t)(uintptr_t)&qr[k % QD][0];
                    uint32_t v[3] = {0u, 0u, 0u};
#pragma unroll
                    for (int j = 0; j < 4; j++)
#pragma unroll
                        for (int c = 0; c < 3; c++) {
                            const int q = 3 * j + c;
                            v[q >> 2] |= (uint32_t)(*(const __attribute__((address_space(3))) uint8_t *)(uintptr_t)(rbase + coff[j] + c))
                                           << (8 * (q & 3));
                        }
                    cur = Raw{v[0], v[1], v[2]};
                } else {
                    const uint32_t *qs = &qr[k % QD][4 * lane];
                    cur = Raw{qs[0], qs[1], qs[2]};
                }
                uint32_t g = gray4(cur);
#else
            if (t + QD - 1 < t_end)
                Q[(k + QD - 1) % QD] = load_px(img, LLFE_ST_HOTROW ? ya : reflect101(t + QD + 1, H), W, x, fast, coff);
            if (t >= ts + QD - 1) {
                ST_MARK(gray);
                uint32_t g = gray4(Q[k % QD]);
#endif
                ST_PIN(g);
                G[(k + 2) % 6] = g;
            }
            if (t >= tf) {
            // ---- blurred row t: computed (0 <= t < H) or REPLICATE'd (t >= H)
            ST_MARK(blur5);
            uint32_t B = blur4(G[(k + 4) % 6], G[(k + 5) % 6], G[k % 6], G[(k + 1) % 6], G[(k + 2) % 6]);
            ST_PIN(B);
            ST_MARK(edge);
            if (edge) {  // REPLICATE the blurred image beyond columns 0 / W-1
                ST_RARE();
                const uint32_t bl = byte_of(__builtin_amdgcn_readlane(B, max(lane0, 0) & 63), 0) * 0x01010101u;
                const uint32_t br = byte_of(__builtin_amdgcn_readlane(B, min(laneW, 63) & 63), (W - 1 - xw0) & 3) * 0x01010101u;
                B = (B & ~(rep_l | rep_r)) | (bl & rep_l) | (br & rep_r);
            }
            if (t >= H) {  // (t >= 0 here)
                ST_RARE();
                B = bring[(k + 5) % 6];
            }
            bring[k % 6] = B;
            if (t == 0 && t0 < 0) {  // rows -5 .. -1 of the first segment
                ST_RARE();
#pragma unroll
                for (int j = 1; j <= 5; j++) bring[(k + 6 - j) % 6] = B;
            }
            ST_MARK(gauss_row);
            if (SHD) {
                rowpass4(B, k11, ra[k], rb[k]);  // (of the copied row past H: the same values)
                ST_PIN(ra[k]);
                ST_PIN(rb[k]);
                if (t == 0 && t0 < 0) {
                    ST_RARE();
#pragma unroll
                    for (int j = 1; j <= 5; j++) {
                        ra[(k + kU - j) % kU] = ra[k];
                        rb[(k + kU - j) % kU] = rb[k];
                    }
                }
            }
            if (CLS && t >= ya) {
                // ---- magnitude row t-1 from blurred rows t-2, t-1, t
                ST_MARK(sobel);
                uint32_t lo, hi;
                const bool cand = sobel4(bring[(k + 4) % 6], bring[(k + 5) % 6], B, lo, hi, out_lane);
                ST_PIN(lo);
                ST_PIN(hi);
                const bool row_in = (unsigned)(t - 1) < (unsigned)H;
                Mlo[k % 3] = row_in ? (lo & in_lo) : 0u;
                Mhi[k % 3] = row_in ? (hi & in_hi) : 0u;
                Mc[k % 3] = cand && row_in;
                // ---- NMS of row t-2 from magnitude rows t-3, t-2, t-1 (class 1 for the
                // whole row when no pixel of the wave's row is a candidate)
                const int yn = t - 2;
                ST_MARK(nms);
                if (yn >= ya && yn < yb) {
                    const int ia = (k + 1) % 3, im = (k + 2) % 3, ib = k % 3;
                    uint32_t o = 0x01010101u;
                    if (Mc[im]) {
                        o = nms4(Mlo[ia], Mhi[ia], Mlo[im], Mhi[im], Mlo[ib], Mhi[ib]);
                        if (tf_img && out_lane && o != 0x01010101u) tf_img[(yn >> 6) * tf_ntx + (x >> 6)] = 1;
                    }
                    ST_PIN(o);
                    ST_MARK(store);
                    if (LLFE_ST_NOSTORE) {
                    } else if (out_fast) {
                        // buffer store: row offset yn * W in an SGPR, the lane's column x in a
                        // VGPR that never changes -- no per-lane 64-bit address per step
                        __builtin_amdgcn_raw_buffer_store_b32(o, crs, (uint32_t)x, yn * W, LLFE_ST_STORE_AUX);
                    } else if (out_lane) {
                        uint8_t *const dst = cimg + ((size_t)yn * W + x);
#pragma unroll
                        for (int j = 0; j < 4; j++)
                            if (x + j < W) dst[j] = (uint8_t)(o >> (8 * j));
                    }
                }
            }
            ST_MARK(gauss_col);
            if (SHD) {
                // ---- Gauss11 column pass of row t-5, mean, mask, masked sum / count
                const int yg = t - 5;
                if (yg >= ya && yg < yb) {
                    const int kc = (k + kU - 5) % kU;
                    const f32x2 w5 = {k11[5], k11[5]};
                    // (the symmetric pairs summed first: the packed adds then never feed the
                    // next instruction, which on gfx950 costs an s_nop)
                    f32x2 pa[5], pb[5];
#pragma unroll
                    for (int d = 1; d <= 5; d++) {
                        const int kp = (kc + d) % kU, kq = (kc + kU - d) % kU;
                        pa[d - 1] = ra[kp] + ra[kq];
                        pb[d - 1] = rb[kp] + rb[kq];
                    }
                    f32x2 s01 = ra[kc] * w5, s23 = rb[kc] * w5;
#pragma unroll
                    for (int d = 1; d <= 5; d++) {
                        const f32x2 wd = {k11[5 + d], k11[5 + d]};
                        s01 = __builtin_elementwise_fma(pa[d - 1], wd, s01);
                        s23 = __builtin_elementwise_fma(pb[d - 1], wd, s23);
                    }
                    // mean = saturate(rint(s)) (0 <= s <= 255 + rounding, so rint(s) <= 255).
                    // s + 2^23 rounds to 2^23 + rint(s) (round-half-even, spacing 1 in
                    // [2^23, 2^24)), so the low 16 bits of the sum are the mean; then two
                    // pixels per u16 pair: mask = min(sat(mean - (b + 1)), 1) (b + 2 <= mean),
                    // sum += b . mask and count += 1 . mask by v_dot2_u32_u16
                    ST_PIN(s01);
                    ST_PIN(s23);
                    ST_MARK(mean_mask_sum);
                    const f32x2 two23 = {8388608.0f, 8388608.0f};
                    // (ring pairs, and so s01 / s23 here, hold columns (c0, c2) and (c1, c3))
                    const f32x2 q01 = s01 + two23, q23 = s23 + two23;
                    const uint32_t mean01 = __builtin_amdgcn_perm(__float_as_uint(q01.y), __float_as_uint(q01.x), 0x05040100u);
                    const uint32_t mean23 = __builtin_amdgcn_perm(__float_as_uint(q23.y), __float_as_uint(q23.x), 0x05040100u);
                    const uint32_t bw = bring[(k + 1) % 6];  // row t - 5
                    const u16x2 one = {1, 1};
                    const u16x2 b01 = U(__builtin_amdgcn_perm(0u, bw, 0x0c020c00u));  // bytes 0, 2
                    const u16x2 b23 = U(__builtin_amdgcn_perm(0u, bw, 0x0c030c01u));  // bytes 1, 3
                    const u16x2 one_o = U(opaque_ones());
                    uint32_t m01 = W32(__builtin_elementwise_min(__builtin_elementwise_sub_sat(U(mean01), b01 + one), one_o));
                    uint32_t m23 = W32(__builtin_elementwise_min(__builtin_elementwise_sub_sat(U(mean23), b23 + one), one_o));
                    // halo lanes are dropped after the loop; only border waves have output
                    // lanes with columns past W
                    if (edge) {
                        ST_RARE();
                        m01 &= in_02;
                        m23 &= in_13;
                    }
                    lsum = __builtin_amdgcn_udot2(b01, U(m01), lsum, false);
                    lsum = __builtin_amdgcn_udot2(b23, U(m23), lsum, false);
                    lcnt = __builtin_amdgcn_udot2(U(m01), one, lcnt, false);
                    lcnt = __builtin_amdgcn_udot2(U(m23), one, lcnt, false);
                }
            }
            }  // t >= tf
            ST_MARK(step_end);
            }
        }
    }
    if (SHD) {
        if (!out_lane) lsum = lcnt = 0;  // halo lanes (and lanes wholly past W)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {  // <= 240 x 4096 x 255 < 2^32 per wave
            lsum += __shfl_xor(lsum, off);
            lcnt += __shfl_xor(lcnt, off);
        }
        if (lane == 0) wave_part[wid] = make_uint2(lsum, lcnt);
    }
}

// static form: wave i of the grid runs item i (blocks of kWavesPerBlock waves)
template <bool CLS, bool SHD>
__global__ __launch_bounds__(64 * kWavesPerBlock, LLFE_ST_MINW) void k_stencil_stream(
    const uint8_t *__restrict__ bgr, int H, int W, int strips, int segs, int seg_rows, int total_waves, int vec,
    uint8_t *__restrict__ cls, uint2 *__restrict__ wave_part, StencilParams prm) {
    int wid = blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (wid >= total_waves) return;  // whole wave leaves
#if LLFE_ST_LPT
    // (experiment) LPT dispatch order: the border strips (0 and strips - 1) of every (image,
    // segment) first -- their byte loads make them the longest items -- then the interior
    if (strips > 2) {
        const int n_edge = 2 * (total_waves / strips);
        if (wid < n_edge) {
            wid = (wid >> 1) * strips + ((wid & 1) ? strips - 1 : 0);
        } else {
            const int r = wid - n_edge, inner = strips - 2;
            wid = (r / inner) * strips + 1 + r % inner;
        }
    }
#endif
    stencil_wave<CLS, SHD>(wid, bgr, H, W, strips, segs, seg_rows, vec, cls, wave_part, prm);
}

// per image: sum of its waves' (sum, count)
__global__ __launch_bounds__(256) void k_stream_shadow_reduce(const uint2 *__restrict__ part, int per_img,
                                                              unsigned long long *__restrict__ shadow_sum,
                                                              unsigned long long *__restrict__ shadow_cnt) {
    __shared__ unsigned long long rs[4], rc[4];
    const int img = blockIdx.x, tid = threadIdx.x;
    unsigned long long a = 0, b = 0;
    for (int t = tid; t < per_img; t += 256) {
        const uint2 v = part[(size_t)img * per_img + t];
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

void stream_geometry(int h, int w, int &strips, int &segs, int &seg_rows) {
    strips = (w + kStripW - 1) / kStripW;
    // ~216-row segments (40 waves per 1080p image, 16 fill rows per segment).  Measured after
    // round 5's candidate-lane fix (profiles/r5/r5p/, isolated 512 x 1080p): 270 rows 2.81 ms,
    // 216 2.60-2.63, 180 2.63-2.64, 135 2.75-2.78, 108 2.58-2.61 (round 2, when every row ran
    // the NMS code, 270 was the best)
#ifndef LLFE_ST_SEG
#define LLFE_ST_SEG 216
#endif
    segs = std::max(1, (h + LLFE_ST_SEG - 1) / LLFE_ST_SEG);
    seg_rows = (h + segs - 1) / segs;
    segs = (h + seg_rows - 1) / seg_rows;
}

}  // namespace

size_t stencil_stream_parts(int n, int h, int w) {
    int strips, segs, seg_rows;
    stream_geometry(h, w, strips, segs, seg_rows);
    return (size_t)n * strips * segs;
}

hipError_t launch_stencil_stream(const uint8_t *bgr, int n, int h, int w, uint8_t *cls,
                                 unsigned long long *shadow_sum, unsigned long long *shadow_cnt, uint2 *wave_part,
                                 const StencilParams &p, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int strips, segs, seg_rows;
    stream_geometry(h, w, strips, segs, seg_rows);
    const long long waves = (long long)n * strips * segs;
    const int vec = ((((uintptr_t)bgr | (uintptr_t)cls) & 3) == 0 && (w & 3) == 0) ? 1 : 0;
    const bool shd = shadow_sum != nullptr;
    const int blocks = (int)((waves + kWavesPerBlock - 1) / kWavesPerBlock);
    if (cls && shd)
        hipLaunchKernelGGL((k_stencil_stream<true, true>), dim3(blocks), dim3(64 * kWavesPerBlock), 0, s, bgr, h, w,
                           strips, segs, seg_rows, (int)waves, vec, cls, wave_part, p);
    else if (cls)
        hipLaunchKernelGGL((k_stencil_stream<true, false>), dim3(blocks), dim3(64 * kWavesPerBlock), 0, s, bgr, h,
                           w, strips, segs, seg_rows, (int)waves, vec, cls, wave_part, p);
    else if (shd)
        hipLaunchKernelGGL((k_stencil_stream<false, true>), dim3(blocks), dim3(64 * kWavesPerBlock), 0, s, bgr, h,
                           w, strips, segs, seg_rows, (int)waves, vec, cls, wave_part, p);
    if (shd)
        hipLaunchKernelGGL(k_stream_shadow_reduce, dim3(n), dim3(256), 0, s, wave_part, strips * segs, shadow_sum,
                           shadow_cnt);
    return hipGetLastError();
}

}  // namespace llfe
