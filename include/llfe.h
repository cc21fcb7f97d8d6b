/*
 * llfe.h -- C ABI of libllfe.so, the MI355X (gfx950) batched image-feature backend.
 *
 * This is the drop-in boundary behind the reference's Python call sites
 * (Kira7dn/Low_Level_Feature_Extraction @ 2025-05-23).  The reference has no FFI of
 * its own -- its "plugin" surface is a set of static Python methods bound by direct
 * import in app/api/v1/endpoints/analyze.py:15-26 -- so each entry point below names
 * the reference function whose native work it replaces.  The Python mirror of those
 * methods lives in low_level_feature_extraction_amd/ and reaches this ABI via ctypes
 * (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - plain pointers and sizes only; no torch / numpy types.
 *   - images are BGR, 8-bit, H x W x 3, rows contiguous (stride W*3), batches are
 *     packed N x H x W x 3 (NHWC) with one shared H, W.
 *   - "device" pointers live on the ctx's device (e.g. a torch tensor's data_ptr());
 *     "host" pointers are ordinary CPU memory.
 *   - every call returns LLFE_OK (0) or a negative LLFE_ERR_* code; no exception
 *     crosses the ABI; llfe_last_error(ctx) returns a message for the last failure.
 *   - a ctx is bound to one device and is not thread-safe; use one ctx per host
 *     thread per GPU.  `stream` is a hipStream_t (NULL = the legacy default stream).
 *   - calls are synchronous with respect to their host outputs: when a function
 *     returns, every host output it wrote is valid.
 */
#ifndef LLFE_H
#define LLFE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LLFE_ABI_VERSION 3
/* most k-means centres per image (extract_colors(n_colors=...) accepts 1 .. LLFE_MAX_COLORS) */
#define LLFE_MAX_COLORS 32

#define LLFE_OK 0
#define LLFE_ERR_INVALID (-1)
#define LLFE_ERR_HIP (-2)
#define LLFE_ERR_CAPACITY (-3)
#define LLFE_ERR_OOM (-4)
#define LLFE_ERR_UNSUPPORTED (-5)

/* feature mask bits (FeatureType colors / shapes / shadows) */
#define LLFE_FEATURE_COLORS 1u
#define LLFE_FEATURE_SHAPES 2u
#define LLFE_FEATURE_SHADOWS 4u

/* shape type codes (ShapeAnalyzer.analyze_shapes @L159-172 type strings) */
#define LLFE_SHAPE_UNKNOWN 0
#define LLFE_SHAPE_TRIANGLE 1
#define LLFE_SHAPE_RECTANGLE 2
#define LLFE_SHAPE_CIRCLE 3
#define LLFE_SHAPE_POLYGON 4

/* validate_and_preprocess_image modes (app/services/analyze/utils.py:22-28) */
#define LLFE_PRE_NONE 0
#define LLFE_PRE_AUTO 1
#define LLFE_PRE_HIGH_QUALITY 2
#define LLFE_PRE_PERFORMANCE 3

typedef struct llfe_ctx llfe_ctx;
typedef void *llfe_stream; /* hipStream_t */

typedef struct {
    const uint8_t *data;   /* N x H x W x 3 BGR u8 */
    int32_t n, height, width;
    int32_t on_device;     /* 1: device pointer, 0: host pointer */
    /* optional "parity mode" noise: N x H x W x 3 int8 in RGB channel order, i.e.
     * exactly np.random.normal(0, 0.5, (H*W, 3)).astype(np.int8) per image
     * (color_extractor.py:224).  NULL -> on-device counter-based (hashed) noise of the same
     * distribution. */
    const int8_t *noise;
    int32_t noise_on_device;
    int32_t n_colors;      /* extract_colors(n_colors=...) in [1, LLFE_MAX_COLORS]; 0 -> 5 (the default) */
    int64_t index_base;    /* global index of image 0 (seeds are per global index) */
    const int64_t *indices; /* optional (host): global index of each image, overriding
                               index_base + i -- results stay those of each image's own index
                               whatever the batching (a request's image keeps its seeds) */
} llfe_batch;

typedef struct {
    /* colors: _get_dominant_colors + bincount (color_extractor.py:174-236) */
    int32_t n_colors;          /* centres written: K = min(n_colors, U) when K > 1; when K <= 1
                                  (n_colors = 1 or U <= 1) the reference returns every unique
                                  colour with labels [0]*U (color_extractor.py:185-186): here
                                  the first min(U, 5) in np.unique order, counts [U, 0, ...] */
    int32_t counts[LLFE_MAX_COLORS];         /* np.bincount(labels) per centre, k-means order */
    uint8_t centers_rgb[LLFE_MAX_COLORS][3]; /* centers.astype(np.uint8), k-means order */
    uint8_t pad_[4];
    int64_t n_unique;          /* len(np.unique(pixels, axis=0)) */
    double compactness;        /* best cv2.kmeans compactness */
    /* shadows: processed[thresh == 255] sum / size (shadow pyc @L21-24) */
    uint64_t shadow_sum;
    uint64_t shadow_count;
    /* shapes: slice [shape_offset, shape_offset + n_shapes) of the shapes array */
    int64_t shape_offset;
    int32_t n_shapes;
    int32_t n_contours;        /* external contours before the area >= 100 filter */
    /* the reference-shaped summaries, made on the host half of the call in C (no Python):
     * extract_colors' palette rules on the centres / counts above (color_extractor.py:
     * 231-284: most frequent first, '#rrggbb', '#ffffff' / '#000000' dropped, primary, three
     * accents, background by the primary's luminance, is_light_color :67-71) and
     * analyze_shadow_level's level (shadow pyc @L21-31) */
    char primary[8];           /* NUL-terminated; "" when colors were not requested */
    char background[8];        /* "#FFFFFF" or "#000000" (the reference's upper case) */
    char accent[3][8];
    int32_t shadow_level;      /* 0 Low, 1 Moderate, 2 High; -1 when shadows were not requested */
    int32_t pad2_;
} llfe_image_result;

typedef struct {
    int32_t type; /* LLFE_SHAPE_* */
    int32_t x, y, width, height;
    int32_t pad_;
    double border_radius;
    double area;
} llfe_shape;

/* per-kernel timing collected with hipEvents on the launch stream while profiling
 * is enabled (bench.py's roofline numbers) */
typedef struct {
    char name[32];
    int64_t launches;
    double total_ms;
    double bytes;  /* algorithmic HBM bytes attributed to those launches */
} llfe_kernel_stat;

/* one k-means attempt of the last llfe_process_batch (diagnostics, llfe_kmeans_attempts):
 * cv2.kmeans' attempt a (color_extractor.py:192-196) -- its k-means++ centres, the centres
 * and cluster sizes after Lloyd, the Lloyd iterations and the compactness */
typedef struct {
    float pp_centers[5][3];
    float centers[5][3];
    int32_t counts[5];
    int32_t iters;
    double compactness;
} llfe_kmeans_attempt;

/* ---- context ---------------------------------------------------------- */
int llfe_init(int device, llfe_ctx **out);
int llfe_destroy(llfe_ctx *ctx);
const char *llfe_last_error(llfe_ctx *ctx);
int llfe_abi_version(void);
/* file path of the HIP runtime (libamdhip64) the library is bound to.  Device pointers
 * and `stream` handles passed in must come from this same runtime: a process that
 * also uses PyTorch-ROCm loads libllfe after torch, so both share torch's runtime. */
const char *llfe_hip_runtime(void);
/* host threads a new ctx gives its contour pool: the process's share of the usable CPUs
 * -- LLFE_RANK_CPUS when the rank was pinned to its GPU's NUMA node (placement.py), else
 * (affinity mask and cgroup quota) / LOCAL_WORLD_SIZE -- at most 16; LLFE_HOST_THREADS
 * overrides.  Host only. */
int llfe_default_host_threads(void);
/* enable (1) / disable (0) event timing; enabling resets the statistics */
int llfe_set_profiling(llfe_ctx *ctx, int enable);
/* llfe_process_batch runs the colour path on a second stream beside shapes / shadows
 * (1, the default) or everything in order on one stream (0: isolated kernel timings) */
int llfe_set_concurrency(llfe_ctx *ctx, int enable);
/* where llfe_process_batch / llfe_collect_batch run findContours + the shape loop of
 * ShapeAnalyzer.analyze_shapes (shape pyc @L140-181): LLFE_CONTOURS_HOST (default) on the
 * context's host thread pool from the bit-packed mask copied back, overlapping the
 * GPU's k-means; LLFE_CONTOURS_GPU on the GPU (contours_gpu.hip; images up to 4096 wide
 * and 65535 tall, wider ones stay on the host).  Identical results either way.  Initial
 * mode: GPU when the process has fewer than 4 host cores (hardware threads /
 * LOCAL_WORLD_SIZE), else host; LLFE_CONTOURS=host|gpu overrides. */
#define LLFE_CONTOURS_HOST 0
#define LLFE_CONTOURS_GPU 1
/* diagnostic: GPU mode, with every chunk then redone by the host fallback that a chunk
 * the GPU tracer flags as unsupported takes (tests exercise that path with it) */
#define LLFE_CONTOURS_GPU_FORCE_FALLBACK 2
int llfe_set_contour_mode(llfe_ctx *ctx, int mode);
int llfe_get_contour_mode(llfe_ctx *ctx); /* the current mode (or < 0) */
/* batches llfe_submit_batch keeps in flight, each on its own workspace and streams: 2 or
 * 3 (LLFE_INFLIGHT sets a new context's depth, default 2); only with none in flight.  One
 * device pass's workspace is sized within LLFE_WORKSPACE_GB (default 24) per slot, so the
 * device memory held grows with the depth. */
int llfe_set_inflight(llfe_ctx *ctx, int32_t depth);
int llfe_get_inflight(llfe_ctx *ctx); /* the current depth (or < 0) */
/* copies up to cap entries, returns the number of kernels with statistics */
int llfe_kernel_stats(llfe_ctx *ctx, llfe_kernel_stat *out, int32_t cap);
/* host contour pool (LLFE_CONTOURS_HOST), always counted: wall milliseconds the pool spent
 * in contour passes, images traced and the pool's thread count since the last reset
 * (reset != 0 clears after reading).  busy_ms / elapsed wall time near 1 means a
 * workload is bound by the host pool, not the GPU. */
int llfe_host_contour_stats(llfe_ctx *ctx, double *busy_ms, int64_t *images, int32_t *threads, int32_t reset);

/* ---- whole hot path ----------------------------------------------------
 * Replaces, per image of the batch:
 *   ColorExtractor.extract_colors native work  (color_extractor.py:217-236)
 *   ShapeAnalyzer.analyze_shapes               (shape pyc @L125-189)
 *   ShadowAnalyzer.analyze_shadow_level stats  (shadow pyc @L12-24)
 * results[n] host; shapes[shape_capacity] host; *shapes_needed = total shapes
 * (LLFE_ERR_CAPACITY when it exceeds shape_capacity; results are still valid). */
int llfe_process_batch(llfe_ctx *ctx, const llfe_batch *batch, uint32_t features, uint64_t seed,
                       llfe_image_result *results, llfe_shape *shapes, int64_t shape_capacity,
                       int64_t *shapes_needed, llfe_stream stream);

/* One image of a ragged batch: H x W BGR u8 pixels, rows of W * 3 bytes row_stride bytes
 * apart (0: packed), in host or device memory. */
typedef struct {
    const uint8_t *data;
    int32_t height, width;
    int64_t row_stride;
    int32_t on_device;
    int32_t noise_on_device;
    /* optional parity-mode noise of this image after preprocessing (H' x W' x 3 int8, RGB
     * order, as llfe_batch.noise); give it for every image of the call or for none */
    const int8_t *noise;
} llfe_image_desc;

/* llfe_process_batch for a ragged batch: every image its own size, row
 * stride and memory, plus validate_and_preprocess_image's resize rule applied on the GPU
 * first (preprocessing = LLFE_PRE_NONE / AUTO / HIGH_QUALITY / PERFORMANCE, utils.py:
 * 118-143: INTER_AREA above 2000 px / LANCZOS4 above 4000 / LINEAR above 1000).  Images
 * of one (preprocessed) size share device passes; image i keeps global index
 * index_base + i, so its results equal a one-image call's.  results[i] belongs to
 * images[i]; its shapes are shapes[results[i].shape_offset ...] (LLFE_ERR_CAPACITY and
 * *shapes_needed as llfe_process_batch).  Synchronous. */
int llfe_process_images(llfe_ctx *ctx, const llfe_image_desc *images, int32_t n, uint32_t features,
                        int32_t preprocessing, int32_t n_colors, uint64_t seed, int64_t index_base,
                        llfe_image_result *results, llfe_shape *shapes, int64_t shape_capacity,
                        int64_t *shapes_needed, llfe_stream stream);

/* Asynchronous form (serving loops): llfe_submit_batch enqueues the device work of one
 * batch (n <= one device pass) and returns a ticket; llfe_collect_batch (tickets in
 * submission order) waits for it, traces contours and fills results / shapes exactly as
 * llfe_process_batch would.  At most two batches are in flight; batch k + 1 runs on the
 * second workspace, so its kernels start in the tail of batch k's k-means.  The input
 * (and parity noise) must stay valid until the ticket is collected.  On
 * LLFE_ERR_CAPACITY the ticket stays collectable with a larger shapes buffer. */
int llfe_submit_batch(llfe_ctx *ctx, const llfe_batch *batch, uint32_t features, uint64_t seed, llfe_stream stream,
                      int64_t *ticket);
int llfe_collect_batch(llfe_ctx *ctx, int64_t ticket, llfe_image_result *results, llfe_shape *shapes,
                       int64_t shape_capacity, int64_t *shapes_needed);

/* llfe_submit_batch for n separately allocated images of ONE size (the request path:
 * concurrent /analyze requests -- app/api/v1/endpoints/analyze.py:63-129, one image per
 * request -- sharing one launch, MicroBatcher).  The images (host or device, any row
 * stride, no parity noise) are gathered on the submit's stream into the in-flight
 * slot's own input buffer (device sources: one gather kernel; host sources: 2-D
 * copies), then run exactly as llfe_submit_batch; image i carries global index
 * indices[i] (its noise / k-means seeds), so its results equal a one-image call's.
 * Collect with llfe_collect_batch.  The sources must stay valid until the ticket is
 * collected; the library keeps its own copy of `images` and `indices`. */
int llfe_submit_images(llfe_ctx *ctx, const llfe_image_desc *images, int32_t n, uint32_t features, int32_t n_colors,
                       uint64_t seed, const int64_t *indices, llfe_stream stream, int64_t *ticket);
/* images of h x w one device pass takes: the largest n llfe_submit_batch /
 * llfe_submit_images accept (the workspace budget, LLFE_WORKSPACE_GB); < 0 on bad sizes */
int llfe_batch_capacity(int32_t h, int32_t w);

/* ---- stage entry points (parity tests; device in/out unless noted) ------
 * The ones that use the context's workspace (llfe_shape_mask, llfe_canny,
 * llfe_shadow_stats, llfe_color_unique, llfe_kmeans, llfe_find_contours_gpu,
 * llfe_shapes_from_masks_gpu) and llfe_process_images return LLFE_ERR_INVALID while a
 * batch submitted with llfe_submit_batch is not yet collected. */
/* gray = cvtColor(BGR2GRAY); out = GaussianBlur(gray, (5,5), 0)
 * (shape pyc @L18-21, shadow pyc @L8-9) */
int llfe_gray_blur5(llfe_ctx *ctx, const uint8_t *bgr, uint8_t *blurred, int32_t n, int32_t h, int32_t w,
                    llfe_stream stream);
/* dilate(Canny(blur5(gray), 50, 150), ones(3,3)) as 0/255 u8 (shape pyc @L6-30) */
int llfe_shape_mask(llfe_ctx *ctx, const uint8_t *bgr, uint8_t *mask, int32_t n, int32_t h, int32_t w,
                    llfe_stream stream);
/* Canny(blur5(gray), 50, 150) as 0/255 u8: the shape mask before its dilation */
int llfe_canny(llfe_ctx *ctx, const uint8_t *bgr, uint8_t *edges, int32_t n, int32_t h, int32_t w,
               llfe_stream stream);
/* dilate(src, ones(3,3)) of n h x w u8 images (any values; out-of-image never wins);
 * src and dst must not alias */
int llfe_dilate3(llfe_ctx *ctx, const uint8_t *src, uint8_t *dst, int32_t n, int32_t h, int32_t w,
                 llfe_stream stream);
/* Canny NMS classes before hysteresis: 0 weak, 1 suppressed, 2 strong */
int llfe_edge_classes(llfe_ctx *ctx, const uint8_t *bgr, uint8_t *classes, int32_t n, int32_t h, int32_t w,
                      llfe_stream stream);
/* FontDetector.preprocess_image (app/services/analyze/font_detector.py:17-37):
 * adaptiveThreshold(cvtColor(BGR2GRAY), 255, GAUSSIAN_C, THRESH_BINARY_INV, 11, 2) as
 * 0/255 u8; bgr and mask are device pointers (n x h x w x 3 / n x h x w). */
int llfe_font_binary(llfe_ctx *ctx, const uint8_t *bgr, uint8_t *mask, int32_t n, int32_t h, int32_t w,
                     llfe_stream stream);
/* TextExtractor.preprocess_image (app/services/analyze/text_extractor.py:15-46): gray
 * (cvtColor BGR2GRAY for 3 / 4 channels, the image itself for 1), INTER_CUBIC upscale by
 * max(2, 300 / w, 100 / h) when h < 30 or w < 100, Otsu THRESH_BINARY, bitwise_not when
 * mean(binary) > 127.  img: device h x w x channels u8; out: device out_h x out_w u8
 * (llfe_text_size); *threshold (host, may be NULL) receives Otsu's threshold. */
int llfe_text_binary(llfe_ctx *ctx, const uint8_t *img, int32_t h, int32_t w, int32_t channels, uint8_t *out,
                     int32_t *threshold, llfe_stream stream);
/* output size of llfe_text_binary: returns 1 when the image is upscaled, 0 when not
 * (text_extractor.py:31-37; saturate_cast<int> of w * scale, h * scale), negative for
 * invalid sizes or an upscaled side past INT32_MAX. Host only. */
int llfe_text_size(int32_t h, int32_t w, int32_t *out_h, int32_t *out_w);
/* sums[n], counts[n] host: adaptive-threshold shadow statistics (shadow pyc @L15-21) */
int llfe_shadow_stats(llfe_ctx *ctx, const uint8_t *bgr, uint64_t *sums, uint64_t *counts, int32_t n, int32_t h,
                      int32_t w, llfe_stream stream);
/* noise + np.unique(axis=0) (color_extractor.py:220-225,177).  keys: device
 * n x (h*w) u32 (R<<16|G<<8|B ascending, first n_unique[i] valid); n_unique host. */
int llfe_color_unique(llfe_ctx *ctx, const llfe_batch *batch, uint64_t seed, uint32_t *keys, int64_t *n_unique,
                      llfe_stream stream);
/* cv2.kmeans(float32(keys->RGB), K=min(n_colors,U), None, (EPS+MAX_ITER,200,0.2), 10,
 * KMEANS_PP_CENTERS) per image (color_extractor.py:189-197).  keys device
 * (n x key_stride), n_points host; results host (colour fields only). */
int llfe_kmeans(llfe_ctx *ctx, const uint32_t *keys, int64_t key_stride, const int64_t *n_points, int32_t n,
                int32_t n_colors, uint64_t seed, int64_t index_base, llfe_image_result *results,
                llfe_stream stream);
/* extract_colors' palette rules alone (color_extractor.py:231-284; host, no context):
 * k centres (RGB u8) and counts in k-means order -> r's primary / background / accent, as
 * llfe_process_batch fills them (the other fields of r are left as they are). */
int llfe_palette_rules(const uint8_t *centers_rgb, const int32_t *counts, int32_t k, llfe_image_result *r);
/* Diagnostics: the 10 attempt records (llfe_kmeans_attempt) of each of the first n images
 * of the last chunk of the last llfe_process_batch on this context (n <= its size), for
 * n_colors <= 5 (the cube-table k-means), into out[n * 10] (host).  Replaces nothing in the
 * reference: cv2.kmeans only returns the best attempt (color_extractor.py:194). */
int llfe_kmeans_attempts(llfe_ctx *ctx, int32_t n, llfe_kmeans_attempt *out);
/* Pillow Image.resize(size, LANCZOS, box) on u8 HWC (image_processor.py:221-224).
 * box may be NULL (whole image). src/dst device. */
int llfe_resize_lanczos_pil(llfe_ctx *ctx, const uint8_t *src, int32_t h, int32_t w, int32_t ch, uint8_t *dst,
                            int32_t out_h, int32_t out_w, const double *box, llfe_stream stream);
/* Pillow Image.reduce((fx, fy)) box averaging of a device u8 HWC image; dst holds
 * ceil(h/fy) x ceil(w/fx) x ch bytes. */
int llfe_reduce_pil(llfe_ctx *ctx, const uint8_t *src, int32_t h, int32_t w, int32_t ch, int32_t fx, int32_t fy,
                    uint8_t *dst, llfe_stream stream);
/* cv2.resize(src, (out_w, out_h), interpolation=...) on a device u8 HWC image (ch <= 4)
 * -- the downscale of validate_and_preprocess_image (app/services/analyze/utils.py:
 * 118-143): LLFE_CV_INTER_AREA for "auto", LLFE_CV_INTER_LANCZOS4 for "high_quality",
 * LLFE_CV_INTER_LINEAR for "performance".  dst holds out_h x out_w x ch bytes. */
#define LLFE_CV_INTER_LINEAR 1
#define LLFE_CV_INTER_CUBIC 2
#define LLFE_CV_INTER_AREA 3
#define LLFE_CV_INTER_LANCZOS4 4
int llfe_resize_cv(llfe_ctx *ctx, const uint8_t *src, int32_t h, int32_t w, int32_t ch, uint8_t *dst, int32_t out_h,
                   int32_t out_w, int32_t interpolation, llfe_stream stream);
/* validate_and_preprocess_image's size rule (utils.py:118-143, Python float
 * semantics): returns 1 with (out_w, out_h, interpolation) when `mode` (LLFE_PRE_*)
 * resizes a w x h image, 0 when it does not. Host only. */
int llfe_preprocess_size(int32_t w, int32_t h, int32_t mode, int32_t *out_w, int32_t *out_h, int32_t *interpolation);
/* PIL Image.thumbnail size rule (preserve_aspect_ratio): returns 1 and the new size
 * when a resize happens, 0 when (w, h) already fits (max_w, max_h). Host only. */
int llfe_thumbnail_size(int32_t w, int32_t h, int32_t max_w, int32_t max_h, int32_t *out_w, int32_t *out_h);
/* ImageProcessor.auto_process_image resize step (image_processor.py:221-224):
 * thumbnail((max_w, max_h), LANCZOS) incl. reducing_gap=2.0's reduce() pre-pass, on a
 * device u8 HWC image.  dst (device) needs out_h * out_w * ch <= dst_capacity bytes. */
int llfe_thumbnail_pil(llfe_ctx *ctx, const uint8_t *src, int32_t h, int32_t w, int32_t ch, int32_t max_w,
                       int32_t max_h, uint8_t *dst, int64_t dst_capacity, int32_t *out_h, int32_t *out_w,
                       llfe_stream stream);
/* the same for n same-size device images packed n x h x w x ch -> n x out_h x out_w x ch
 * (ImageProcessor.auto_process_image over a batch: one launch sequence per pass) */
int llfe_thumbnail_pil_batch(llfe_ctx *ctx, const uint8_t *src, int32_t n, int32_t h, int32_t w, int32_t ch,
                             int32_t max_w, int32_t max_h, uint8_t *dst, int64_t dst_capacity, int32_t *out_h,
                             int32_t *out_w, llfe_stream stream);
/* host-side external contours (findContours RETR_EXTERNAL/CHAIN_APPROX_SIMPLE,
 * shape pyc @L140) on a host u8 mask; points x,y pairs; offsets[n_contours+1].
 * Returns the number of contours, or LLFE_ERR_CAPACITY with *needed_points set. */
int llfe_find_contours(const uint8_t *mask, int32_t h, int32_t w, int32_t *points, int64_t points_capacity,
                       int32_t *offsets, int32_t offsets_capacity, int64_t *needed_points);
/* ShapeAnalyzer.detect_border_radius(contour, epsilon_factor) (shape pyc @L32-61)
 * on one contour (x,y int32 pairs). */
double llfe_border_radius(const int32_t *points, int32_t n, double epsilon_factor);
/* one iteration of the analyze_shapes loop (shape pyc @L146-181): returns 1 and fills
 * *out when contourArea >= 100, 0 when the contour is dropped. */
int llfe_classify_contour(const int32_t *points, int32_t n, llfe_shape *out);
/* host-side shape records from a host u8 mask (the analyze_shapes loop). */
int llfe_shapes_from_mask(const uint8_t *mask, int32_t h, int32_t w, llfe_shape *shapes, int32_t capacity,
                          int32_t *n_contours);
/* The same two on the GPU path the batch uses (contours_gpu.hip: components, border
 * following from first pixels, the raster-scan replay, geometry), from host u8 masks
 * of width <= 4096.  llfe_find_contours_gpu: as llfe_find_contours (cv2 order).
 * llfe_shapes_from_masks_gpu: n masks; per image n_shapes / n_contours, shape records
 * concatenated (LLFE_ERR_CAPACITY with *needed when capacity is short). */
int llfe_find_contours_gpu(llfe_ctx *ctx, const uint8_t *mask, int32_t h, int32_t w, int32_t *points,
                           int64_t points_capacity, int32_t *offsets, int32_t offsets_capacity,
                           int64_t *needed_points);
int llfe_shapes_from_masks_gpu(llfe_ctx *ctx, const uint8_t *masks, int32_t n, int32_t h, int32_t w,
                               llfe_shape *shapes, int64_t capacity, int32_t *n_shapes, int32_t *n_contours,
                               int64_t *needed);

/* ---- host decode (cv2.imdecode(buf, IMREAD_COLOR), utils.py:108-109 and
 * image_processor.py:208-211).  Host only, no ctx.  IMREAD_COLOR semantics: BGR u8.
 * PNG (native decoder): alpha dropped, grey expanded, palette looked up, 16-bit -> high
 * byte, critical-chunk CRCs checked.  JPEG (system libjpeg-turbo via dlopen, OpenCV's
 * settings: ISLOW IDCT, fancy upsampling, JCS_EXT_BGR out).  Images above
 * LLFE_MAX_PIXELS (default 2^30, cv2's CV_IO_MAX_IMAGE_PIXELS) are refused before
 * anything is allocated.  LLFE_ERR_UNSUPPORTED hands an image back to the caller's
 * other decoder: interlaced / sub-byte-depth PNG, CMYK / YCCK JPEG, JPEG with an EXIF
 * orientation other than 1, other formats; corrupt data is LLFE_ERR_INVALID. */
/* size of a PNG from its IHDR; LLFE_ERR_CAPACITY (size still written) above the pixel limit */
int llfe_png_info(const uint8_t *data, uint64_t size, int32_t *width, int32_t *height);
/* n PNGs of one size into out_bgr (n x height x width x 3, host), `threads` host
 * threads.  status[i] per image (LLFE_OK, LLFE_ERR_UNSUPPORTED, LLFE_ERR_INVALID, or
 * LLFE_ERR_CAPACITY when its size differs); returns the first non-OK status. */
int llfe_decode_png_batch(const uint8_t *const *data, const uint64_t *sizes, int32_t n, int32_t height,
                          int32_t width, uint8_t *out_bgr, int32_t *status, int32_t threads);
/* the same two for PNG and JPEG, by signature (LLFE_ERR_UNSUPPORTED for other formats) */
int llfe_image_info(const uint8_t *data, uint64_t size, int32_t *width, int32_t *height);
int llfe_decode_batch(const uint8_t *const *data, const uint64_t *sizes, int32_t n, int32_t height, int32_t width,
                      uint8_t *out_bgr, int32_t *status, int32_t threads);
/* which codecs the host decoders run: "png=libdeflate|zlib;jpeg=libjpeg.so.8|pillow"
 * (NUL-terminated into buf; LLFE_ERR_CAPACITY if cap is too small) */
int llfe_decoder_info(char *buf, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* LLFE_H */
