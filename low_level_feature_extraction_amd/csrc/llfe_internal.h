// Internal declarations shared by the HIP kernel files and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/llfe.h"

namespace llfe {

// ---------------------------------------------------------------- stencils
// Output tile of the fused stencil front-end (gray -> blur5 -> {Canny NMS,
// adaptive Gaussian mean}); 256 threads per tile.
constexpr int kTileW = 64;
constexpr int kTileH = 32;

// getGaussianKernel(11, 0, CV_32F) (gauss_kernel_f32(11) in llfe_api.cpp, checked equal at
// llfe_create): the row-streaming stencil takes these as constants
#define LLFE_GAUSS11_F32                                                                                     \
    0x1.20c256p-7f, 0x1.bcb86ap-6f, 0x1.0ab50ap-4f, 0x1.f2464cp-4f, 0x1.6a7e1ep-3f, 0x1.9ac20ap-3f,          \
        0x1.6a7e1ep-3f, 0x1.f2464cp-4f, 0x1.0ab50ap-4f, 0x1.bcb86ap-6f, 0x1.20c256p-7f

struct StencilParams {
    float k11[11];  // CV_32F GaussianBlur 11x11 sigma 0 kernel (adaptiveThreshold)
    // (row-streaming kernel, with cls) n x ceil(h / 64) x ceil(w / 64) bytes, zeroed by the
    // caller: set to 1 for every 64 x 64 hysteresis tile holding a class != 1 pixel
    uint8_t *tflag;
    // (row-streaming kernel) image i at img_tab[i] instead of bgr + i * h * w * 3 -- the
    // separately allocated device images of llfe_submit_images, no gather; null: packed
    const uint64_t *img_tab;
};

// shape pyc @L18-24 + shadow pyc @L8-21 for a packed NHWC batch.
//   cls (may be null): n x h x w u8, 0 weak / 1 suppressed / 2 strong
//   blurred (may be null): n x h x w u8 (parity of GaussianBlur 5x5)
//   shadow_sum/shadow_cnt (may be null): per image u64 accumulators (zeroed by caller)
// shadow_sum / shadow_cnt (when non-null) need tile_part scratch of stencil_parts(n, h, w)
// entries.  Without `blurred` the row-streaming kernel runs (launch_stencil_stream).
hipError_t launch_stencil(const uint8_t *bgr, int n, int h, int w, uint8_t *cls, uint8_t *blurred,
                          unsigned long long *shadow_sum, unsigned long long *shadow_cnt, uint2 *tile_part,
                          const StencilParams &p, hipStream_t s);

// The row-streaming form of launch_stencil's cls / shadow outputs (stencil_stream.hip;
// one wave per 240-column strip and row segment, DPP neighbours, register rings).
// wave_part: stencil_stream_parts(n, h, w) entries of scratch when shadows are wanted.
size_t stencil_stream_parts(int n, int h, int w);
hipError_t launch_stencil_stream(const uint8_t *bgr, int n, int h, int w, uint8_t *cls,
                                 unsigned long long *shadow_sum, unsigned long long *shadow_cnt, uint2 *wave_part,
                                 const StencilParams &p, hipStream_t s);

// FontDetector.preprocess_image (font_detector.py:17-37): gray -> adaptiveThreshold(
// GAUSSIAN_C, THRESH_BINARY_INV, 11, 2) -> n x h x w u8 255 / 0 (the stencil kernel
// with the Gaussian mean taken over the gray image instead of the blurred one)
hipError_t launch_font_binary(const uint8_t *bgr, int n, int h, int w, uint8_t *mask, const StencilParams &p,
                              hipStream_t s);

// Canny hysteresis as connected components + dilate(3x3) + bit-pack (hysteresis.hip).
// Workspace: lab n*h*w u16; parent/sroot/roots over hysteresis_ids() entries; nroots
// per tile.  bits: n x h x words_per_row u64 (bit x&63 of word x>>6), mask_u8 optional.
struct HystWork {
    uint16_t *lab;
    int *parent;
    uint8_t *sroot;
    uint16_t *roots;
    int *nroots;
    uint32_t *tstrong;  // per tile TP / 32 words (the promoted local roots)
    uint64_t *ebits;    // n x h x words_per_row, edges before the dilate
    const uint8_t *tflag;  // (may be null) the stencil's tile flags (StencilParams::tflag)
    int *ftlist;           // the tiles to label (flagged ones, or every tile without tflag),
    int *ftcount;          // their count and a work counter (two ints)
    int *pflag;            // per ftlist entry: the tile has a root promoted by the global unions
};
size_t hysteresis_ids(int n, int h, int w);    // >= the GPU contour pass's ids as well
size_t hysteresis_tiles(int n, int h, int w);  // hysteresis tiles (<= n * tiles_x * tiles_y)
size_t hysteresis_tile_words();                // tstrong words per hysteresis tile
hipError_t launch_hysteresis_dilate(const uint8_t *cls, int n, int h, int w, const HystWork &wk, uint64_t *bits,
                                    uint8_t *mask_u8, hipStream_t s);
// the same connected components without the dilation: Canny's 0 / 255 edges (llfe_canny)
hipError_t launch_canny_edges(const uint8_t *cls, int n, int h, int w, const HystWork &wk, uint8_t *edges_u8,
                              hipStream_t s);
// 3x3 dilate (max filter) of n u8 images (llfe_dilate3)
hipError_t launch_dilate3_u8(const uint8_t *src, int n, int h, int w, uint8_t *dst, hipStream_t s);

// External contours + shape records on the GPU (contours_gpu.hip).  Reuses the
// hysteresis workspace (lab, parent, roots, nroots) once the dilated mask exists.
struct CtComp {  // one outer border: a component's (or a border started elsewhere)
    uint32_t key;    // raster key y * W + x of the start pixel
    int32_t img;
    uint32_t nv;     // CHAIN_APPROX_SIMPLE vertices at pts[off, off + nv)
    uint32_t off;
    int64_t area2;   // signed twice contourArea (shoelace, exact)
    uint16_t x0, y0, x1, y1;  // bounding box (inclusive)
};
static_assert(sizeof(CtComp) == 32, "CtComp is 32 bytes");
struct CtCounters {
    unsigned int comps, refs;
    unsigned long long pts;
    unsigned int flags, quirks, shapes, pad;
};
constexpr unsigned kCtOverflowComps = 1, kCtOverflowPts = 2, kCtOverflowRefs = 4, kCtOverflowShapes = 8;
constexpr unsigned kCtBadTrace = 16, kCtTooWide = 32, kCtDpOverflow = 64;
constexpr unsigned kCtOverflowMask = 15;  // capacity flags: the host grows and reruns
constexpr int kCtInfo = 5;       // per image: components, ref base, contours, kept, shape base
constexpr int kCtQuirkCap = 64;  // borders per image started away from a first pixel
constexpr int kCtTraceBlocks = 2048, kCtStage = 8192;  // border-following waves, vertices staged per wave
constexpr int kCtMaxWidth = 4096;   // GPU contours: widest image (hull columns in LDS)
constexpr int kCtMaxHeight = 65535; // and tallest (16-bit y in the hull candidates)
struct CtCaps {
    int64_t comps, pts, refs, shapes;
};
struct CtWork {
    uint16_t *lab;
    int *parent;
    uint16_t *roots;
    int *nroots;
    uint64_t *planes;  // 5 bit planes of contours_plane_words(): visited, right-bound, Q visited, Q right, first
    CtComp *comps;     // caps.comps
    uint8_t *acc;      // caps.comps
    int2 *pts;         // caps.pts
    int2 *refs;        // caps.refs: (component slot, shape index or -1) in start order
    int2 *stage;       // kCtTraceBlocks * kCtStage vertex staging
    CtCounters *ctr;
    int *img_info;     // n * kCtInfo
    llfe_shape *shapes;  // caps.shapes
    CtCaps caps;
};
CtCaps contours_default_caps(int n, int h, int w);
size_t contours_plane_words(int n, int h, int w);
hipError_t launch_contours(const uint64_t *bits, int n, int h, int w, const CtWork &wk, hipStream_t s);

inline int words_per_row(int w) { return (w + 63) / 64; }
inline int tiles_x(int w) { return (w + kTileW - 1) / kTileW; }
inline int tiles_y(int h) { return (h + kTileH - 1) / kTileH; }
inline size_t stencil_parts(int n, int h, int w) {
    const size_t a = (size_t)n * tiles_x(w) * tiles_y(h), b = stencil_stream_parts(n, h, w);
    return a > b ? a : b;
}

// Global index of image i of a launch (per-image noise streams and k-means seeds, so
// results do not depend on batching): base + i, or idx[i] (device) when a ragged batch
// or a caller's index list gives images non-consecutive indices.
struct ImgIndex {
    long long base;
    const long long *idx;
    __host__ __device__ long long at(int i) const { return idx ? idx[i] : base + i; }
    ImgIndex shifted(int i0) const { return ImgIndex{base + i0, idx ? idx + i0 : nullptr}; }
};

// ---------------------------------------------------------------- colours
constexpr int kMaxK = 5;                     // the cube-table k-means (n_colors <= 5)
constexpr int kMaxColors = LLFE_MAX_COLORS;  // the generic k-means (k_kmeans_big) up to this
constexpr int kAttempts = 10;
constexpr int kParts = 64;         // key partitions by red quarter r >> 2
constexpr int kCubesPerPart = 4096;  // 64 x 64 cubes of 4x4x4 per partition

struct KmeansAttemptOut {
    double compactness;
    float centers[kMaxColors][3];
    int32_t counts[kMaxColors];
    int32_t iters;
    int32_t pad;
    uint64_t bytes;  // algorithmic bytes this attempt read (keys, cube table)
    // workgroup timeline (s_memrealtime, 100 MHz) and placement, for LLFE_KM_TRACE
    uint64_t t_start, t_pp, t_lloyd, t_end;  // start, k-means++ done, Lloyd done, end
    uint32_t hw_id, xcc_id;
    uint32_t pp_pts, n_cubes;  // colours k-means++ read one by one; cube count
    uint64_t t_sel;            // k-means++ time in the selection scans (ticks)
    uint64_t ll_pts;           // colours Lloyd labelled one by one (all sweeps)
    uint64_t t_sw;             // Lloyd time in the labelling sweeps (ticks)
    uint64_t drift_hist;       // Lloyd iterations by largest centre move (8 x u8 bins)
    uint64_t qtot;             // sum of |p|^2 over the image's colours (k-means++ -> Lloyd launch)
    uint64_t t_lstart;         // Lloyd launch: start of the attempt's workgroup
    uint32_t hw_id2, xcc_id2;  // ... and its placement
    float pp_centers[kMaxK][3];  // the k-means++ centres (cube-table path; llfe_kmeans_attempts)
};

struct KmeansImageOut {
    int32_t k;
    int32_t counts[kMaxColors];
    uint8_t centers_rgb[kMaxColors][3];
    uint8_t pad[4];
    int64_t n_unique;
    double compactness;
    uint64_t bytes;  // algorithmic bytes read, summed over the attempts (roofline)
};

// k-means pruning by 4x4x4 colour cubes: one 16-byte entry per occupied cube holds its
// occupancy mask and the exact sums of its colours.  A cube whose whole box provably
// has one label (margin test) is accumulated from its sums; the colours of the others
// are enumerated from the mask and labelled one by one -- OpenCV's labels either way.
struct CubeEnt {
    uint64_t mask;  // bit i*16 + j*4 + b: colour (4R + i, 4G + j, 4B + b) is present
    uint32_t id;    // R << 12 | G << 6 | B (cube = [4R, 4R+3] x [4G, 4G+3] x [4B, 4B+3]) in bits 0..17,
                    // sum over the cube's colours u = colour - origin of |u|^2 (<= 1728) in bits 18..28
    uint32_t sums;  // count (<= 64) | sum u_r << 7 | sum u_g << 15 | sum u_b << 23 (each <= 192)
};
static_assert(sizeof(CubeEnt) == 16, "CubeEnt is one 16-byte load");
constexpr int kMaxCubes = 1 << 18;
// 4 x 8 x 8 cells: the (up to) four cubes (R, 2 G2 + j, 2 B2 + c), j, c in {0, 1}, of one
// partition, consecutive in the cube table (cube order within a partition is (G2, B2, j, c)).
// The Lloyd sweeps test a cell first (one margin test for up to four cubes); only the cubes
// of a failing cell are tested one by one.
constexpr int kCellsPerPart = 1024;  // 32 x 32 cells per partition
struct CellEnt {
    uint32_t id;     // R << 10 | G2 << 5 | B2 (cell = [4R, 4R+3] x [8G2, 8G2+7] x [8B2, 8B2+7]) in bits
                     // 0..15, (cubes - 1) in bits 16..17, colour count (<= 256) in bits 18..26
    uint32_t first;  // index of its first cube in the image's cube table
    uint32_t sums;   // sum over its colours u = colour - cell origin: u_r (<= 768) | u_g << 10 | u_b << 21
                     // (each <= 1792)
    uint32_t s2;     // sum of |u|^2 (<= 27392)
};
static_assert(sizeof(CellEnt) == 16, "CellEnt is one 16-byte load");
// 4 x 16 x 16 super-cells (round 6): the (up to) four cells (R, 2 G4 + j, 2 B4 + c) of one
// partition; in the cell table (G2, B2) order they are two pairs, (j = 0, c = 0..1) at first0
// and (j = 1, c = 0..1) at first1.  The Lloyd sweep tests them before their cells.
constexpr int kSupsPerPart = 256;  // 16 x 16 super-cells per partition
struct SupEnt {
    uint32_t id;     // R << 8 | G4 << 4 | B4 in bits 0..13, cells of the j = 0 pair (0..2) in bits 14..15,
                     // of the j = 1 pair in bits 16..17, colour count (<= 1024) in bits 18..28, bit 18 of
                     // s2 in bit 29
    uint32_t first;  // first0 | first1 << 16: the pairs' first cell indices in the image's cell table
    uint32_t srg;    // sum over its colours u = colour - origin: u_r (<= 3072) | u_g << 12 (<= 15360)
    uint32_t sb;     // sum of u_b (<= 15360) | bits 0..17 of s2 << 14; s2 = sum of |u|^2 (<= 1024 x 459 < 2^19)
};
static_assert(sizeof(SupEnt) == 16, "SupEnt is one 16-byte load");
struct KmeansCubes {
    const CubeEnt *cubes;   // per image (cube_stride) entries, partition by partition (nullptr: no pruning)
    int64_t cube_stride;
    const int32_t *n_cubes;
    const uint32_t *part_uq;  // per image: unique colours per red-quarter partition (kParts)
    const CellEnt *cells;     // per image (cell_stride) cells in partition / cell order
    const int32_t *n_cells;
    int64_t cell_stride;      // min(cube_stride, kParts * kCellsPerPart): an image has <= 65536 cells
    // Segmented keys (k_uq_part's layout, no key gather): when part_hist is set, the keys
    // passed to launch_kmeans hold each image's partitions at the prefix of part_hist (the
    // partitions' pixel counts: partition R's unique keys at [sum_{r<R} hist_r, + uq_R)),
    // not contiguously; part_uq gives the unique counts.
    const uint32_t *part_hist;
    const SupEnt *sups;       // per image (sup_stride) super-cells in partition order (nullptr: none)
    const int32_t *n_sups;
    int64_t sup_stride;
};
// Unique colours (unique.hip), all per image with stride key_stride (u32 keys):
//   keys:    pixels -> noised keys into `raw`, partition histogram `hist` (n x 64, zeroed)
//   scatter: raw -> `part` grouped by partition (`cursor` n x 64, zeroed)
//   part:    per (image, partition): sorted unique keys -> `skeys` (may alias raw),
//            cube entries -> `seg_cubes` (n x 64 x 4096), cells -> `seg_cells` (n x 64 x 1024),
//            counts -> uq, cc, cl (n x 64)
//   gather:  contiguous sorted keys -> `keys` (may alias part), cube table -> `cubes`,
//            cell table -> `cells` (first cube indices made image-global), n_unique, n_cubes,
//            n_cells
// noise: the caller's parity noise (n x P x 3 int8) or null -> the launch's noise field
// (noise_field_pixels(P) bytes at `field`, written by launch_uq_noise; unique.hip)
int64_t noise_field_pixels(int64_t P);
hipError_t launch_uq_noise(const int8_t *noise, int8_t *field, int64_t P, uint64_t seed, hipStream_t s);
// steps of 4096 pixels per image (k_uq_scatter's segments; its run table is n x steps x 64 u32)
int64_t uq_steps(int64_t P);
int64_t uq_tab_words(int64_t P);  // k_uq_scatter's run table, u32 words per image
// img_tab (may be null): image i at img_tab[i] instead of bgr + i * h * w * 3
hipError_t launch_uq_scatter(const uint8_t *bgr, const uint64_t *img_tab, const int8_t *noise, const int8_t *field,
                             int n, int h, int w,
                             uint64_t seed, ImgIndex index, int64_t key_stride, uint32_t *hist, uint32_t *tab,
                             uint32_t *seg, hipStream_t s);
hipError_t launch_uq_part(const uint32_t *seg, int n, int64_t key_stride, int64_t P, const uint32_t *hist,
                          const uint32_t *tab, uint32_t *skeys, CubeEnt *seg_cubes, CellEnt *seg_cells,
                          uint32_t *uq, uint32_t *cc, uint32_t *cl, uint32_t *cs, hipStream_t s);
hipError_t launch_uq_gather(const uint32_t *skeys, int n, int64_t key_stride, const uint32_t *hist, const uint32_t *uq,
                            const uint32_t *cc, const uint32_t *cl, const uint32_t *cs, const CubeEnt *seg_cubes,
                            const CellEnt *seg_cells, uint32_t *keys, CubeEnt *cubes,
                            CellEnt *cells, SupEnt *sups, int64_t cube_stride, int64_t cell_stride, int64_t sup_stride,
                            int64_t *n_unique, int32_t *n_cubes, int32_t *n_cells, int32_t *n_sups, bool copy_keys,
                            hipStream_t s);

// per image: K = min(n_colors, U); attempts run as separate workgroups
// (ordered largest U first), then a finalize kernel picks the best attempt.
// cv::RNG state of image i = splitmix64(seed + index.at(i)), 0 -> 0xffffffff
// order: n + 2 ints (the LPT order, then the work-queue counters of the cube path)
hipError_t launch_kmeans(const uint32_t *keys, int64_t key_stride, const int64_t *n_unique, int n, int n_colors,
                         uint64_t seed, ImgIndex index, int32_t *order, uint32_t *scratch, int64_t scratch_stride,
                         KmeansAttemptOut *attempts, KmeansImageOut *out, const KmeansCubes &cubes,
                         hipStream_t s);
// the same in 512-thread workgroups, two per CU (kmeans.hip built a second time with
// LLFE_KM_WIDE): launch_kmeans calls it when every attempt of the batch fits the GPU at once
hipError_t launch_kmeans_wide(const uint32_t *keys, int64_t key_stride, const int64_t *n_unique, int n, int n_colors,
                              uint64_t seed, ImgIndex index, int32_t *order, uint32_t *scratch, int64_t scratch_stride,
                              KmeansAttemptOut *attempts, KmeansImageOut *out, const KmeansCubes &cubes,
                              hipStream_t s);
// K in (kMaxK, kMaxColors]: the general-K attempts (kmeans_big.hip) in the order of
// k_kmeans_order, into the same attempt records (launch_kmeans calls it)
hipError_t launch_kmeans_big(const uint32_t *keys, int64_t key_stride, const int64_t *n_unique, int n, int n_colors,
                             uint64_t seed, ImgIndex index, const int32_t *order, uint32_t *scratch,
                             int64_t scratch_stride, KmeansAttemptOut *attempts, hipStream_t s);
// u32 scratch per (image, attempt) for k-means++ step sums
int64_t kmeans_scratch_stride(int64_t key_stride);
constexpr int kMaxKmeansBatch = 4096;

// ---------------------------------------------------------------- resize
// Pillow LANCZOS / reduce (resize.hip) on n same-size images, src_img / dst_img bytes apart
hipError_t launch_resize_h(const uint8_t *src, int src_h, int src_w, int ch, int row0, int rows, uint8_t *dst,
                           int out_w, const int32_t *bounds, const int32_t *coeffs, int ksize, hipStream_t s,
                           int n = 1, long long src_img = 0, long long dst_img = 0);
hipError_t launch_resize_v(const uint8_t *src, int src_w, int ch, uint8_t *dst, int out_h, const int32_t *bounds,
                           const int32_t *coeffs, int ksize, hipStream_t s, int n = 1, long long src_img = 0,
                           long long dst_img = 0);
hipError_t launch_reduce(const uint8_t *src, int src_w, int ch, int x0, int y0, int x1, int y1, int fx, int fy,
                         uint8_t *dst, int out_w, int out_h, hipStream_t s, int n = 1, long long src_img = 0,
                         long long dst_img = 0);

// cv2.resize for the preprocessing modes (cvresize.hip); OpenCV interpolation codes
constexpr int kCvInterLinear = 1, kCvInterCubic = 2, kCvInterArea = 3, kCvInterLanczos4 = 4;
struct CvResizePlan {
    enum Kind { COPY, AREA_FAST, AREA, GENERIC } kind = COPY;
    int h = 0, w = 0, cn = 0, oh = 0, ow = 0;
    int fx = 1, fy = 1;                      // AREA_FAST integer factors
    int ks = 2, xmin = 0, xmax = 0, x_vec = 0;  // GENERIC: taps, border columns, vector stop
    std::vector<int32_t> tab;                // coefficient tables (x part, then y part)
    int64_t ytab_off = 0;
};
// host: OpenCV's tables for (h, w, cn) -> (oh, ow); 0 ok, -1 unsupported
int cv_resize_plan(int h, int w, int cn, int oh, int ow, int interp, CvResizePlan &p);
// the same with cv::resize's inverse scales given (dsize empty: the caller's fx, fy)
int cv_resize_plan_scaled(int h, int w, int cn, int oh, int ow, double inv_x, double inv_y, int interp,
                          CvResizePlan &p);
hipError_t launch_cv_resize(const CvResizePlan &p, const uint8_t *src, uint8_t *dst, const int32_t *d_tab,
                            hipStream_t s);

// TextExtractor.preprocess_image (text.hip): gray of n pixels (cn 1, 3 or 4); Otsu
// binary of n gray pixels; hist = 258 u64 of device scratch (threshold in hist[256])
hipError_t launch_text_gray(const uint8_t *img, long long n, int cn, uint8_t *gray, hipStream_t s);
hipError_t launch_text_otsu_binary(const uint8_t *g, long long n, unsigned long long *hist, uint8_t *out,
                                   hipStream_t s);

// llfe_submit_images (gather.hip): n device images of h x w x 3 u8 -> one packed batch;
// tab (device) = n source addresses, then n row pitches in bytes
hipError_t launch_gather_images(const uint64_t *tab, int n, int h, int w, uint8_t *dst, hipStream_t s);

}  // namespace llfe
