"""CPU ORACLE for the llfe hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker / CPU baseline.  The product
(``low_level_feature_extraction_amd``) never imports it.

It wraps ``oracle/liborc.so`` (the C restatement in ``llfe_oracle.c``) and adds the
pure-Python result assembly that the reference performs in Python:

* ``color_palette``     -- ColorExtractor.extract_colors steps 4-8
                           (app/services/analyze/color_extractor.py:231-284, helpers :39-71)
* ``shadow_level``      -- ShadowAnalyzer.analyze_shadow_level (shadow pyc @L21-31)
* ``classify_shapes``   -- ShapeAnalyzer.analyze_shapes loop (shape pyc @L144-189) and
                           detect_border_radius (@L32-61)
* ``thumbnail_size``    -- PIL.Image.thumbnail size rule used by
                           ImageProcessor.auto_process_image (image_processor.py:221-224)
* ``preprocess_size``   -- validate_and_preprocess_image resize rule (utils.py:118-143)

Parity status: Pillow LANCZOS + np.unique + NumPy noise are pinned
against the real libraries in this container; the OpenCV-backed stages are "parity
unpinned" against OpenCV (no cv2 anywhere, no reference tests) and pinned only by KATs.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liborc.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "llfe_oracle.c")
        ):
            build()
        L = C.CDLL(_LIB_PATH)
        u8p = C.POINTER(C.c_uint8)
        L.orc_kmeans.restype = C.c_double
        L.orc_kmeans_ex.restype = C.c_double
        L.orc_contour_area.restype = C.c_double
        L.orc_arc_length.restype = C.c_double
        L.orc_convex_hull_area.restype = C.c_double
        L.orc_color_unique.restype = C.c_int64
        L.orc_cvrng_next.restype = C.c_uint32
        del u8p
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _chk_bgr(bgr: np.ndarray) -> np.ndarray:
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    assert bgr.ndim == 3 and bgr.shape[2] == 3, bgr.shape
    return bgr


# --------------------------------------------------------------------------- stencils
def set_fma(on: bool):
    """Oracle arithmetic mode (parity-risk probe only): True = FMA (AVX2 OpenCV build,
    the default and what the device reproduces), False = separate mul + add (SSE2 build)."""
    lib().orc_set_fma(1 if on else 0)


def bgr2gray(bgr):
    bgr = _chk_bgr(bgr)
    h, w = bgr.shape[:2]
    out = np.empty((h, w), np.uint8)
    lib().orc_bgr2gray(_p(bgr), h, w, _p(out))
    return out


def blur5(gray):
    gray = np.ascontiguousarray(gray, np.uint8)
    out = np.empty_like(gray)
    lib().orc_blur5(_p(gray), _p(out), gray.shape[0], gray.shape[1])
    return out


def gaussian_kernel_fixed8(n):
    out = np.empty(n, np.int32)
    lib().orc_gaussian_kernel_fixed8(n, _p(out))
    return out


def gaussian_kernel_float(n):
    out = np.empty(n, np.float32)
    lib().orc_gaussian_kernel_float(n, _p(out))
    return out


def gauss_float_mean(gray, ksize=11):
    gray = np.ascontiguousarray(gray, np.uint8)
    out = np.empty_like(gray)
    lib().orc_gauss_float_mean(_p(gray), _p(out), gray.shape[0], gray.shape[1], ksize)
    return out


def adaptive_threshold_inv(gray, block=11, idelta=2, maxval=255):
    gray = np.ascontiguousarray(gray, np.uint8)
    out = np.empty_like(gray)
    lib().orc_adaptive_threshold_inv(_p(gray), _p(out), gray.shape[0], gray.shape[1], block, idelta, C.c_uint8(maxval))
    return out


def sobel3(gray):
    gray = np.ascontiguousarray(gray, np.uint8)
    dx = np.empty(gray.shape, np.int16)
    dy = np.empty(gray.shape, np.int16)
    lib().orc_sobel3(_p(gray), _p(dx), _p(dy), gray.shape[0], gray.shape[1])
    return dx, dy


def canny_nms(gray, low=50, high=150):
    """0 = candidate (weak), 1 = suppressed, 2 = strong (OpenCV's Canny map values)."""
    gray = np.ascontiguousarray(gray, np.uint8)
    out = np.empty_like(gray)
    lib().orc_canny_nms(_p(gray), _p(out), gray.shape[0], gray.shape[1], low, high)
    return out


def canny(gray, low=50, high=150):
    gray = np.ascontiguousarray(gray, np.uint8)
    out = np.empty_like(gray)
    lib().orc_canny(_p(gray), _p(out), gray.shape[0], gray.shape[1], low, high)
    return out


def dilate3(img):
    img = np.ascontiguousarray(img, np.uint8)
    out = np.empty_like(img)
    lib().orc_dilate3(_p(img), _p(out), img.shape[0], img.shape[1])
    return out


def shape_mask(bgr):
    bgr = _chk_bgr(bgr)
    h, w = bgr.shape[:2]
    out = np.empty((h, w), np.uint8)
    lib().orc_shape_mask(_p(bgr), h, w, _p(out))
    return out


def shadow_stats(bgr):
    bgr = _chk_bgr(bgr)
    s = C.c_uint64()
    c = C.c_uint64()
    lib().orc_shadow_stats(_p(bgr), bgr.shape[0], bgr.shape[1], C.byref(s), C.byref(c))
    return int(s.value), int(c.value)


# --------------------------------------------------------------------------- contours
def find_contours_external(mask):
    """List of (n,2) int32 arrays, in OpenCV's RETR_EXTERNAL output order."""
    mask = np.ascontiguousarray(mask, np.uint8)
    pts = C.POINTER(C.c_int)()
    off = C.POINTER(C.c_int)()
    L = lib()
    n = L.orc_find_contours_external(_p(mask), mask.shape[0], mask.shape[1], C.byref(pts), C.byref(off))
    offs = [off[i] for i in range(n + 1)]
    total = offs[-1]
    flat = np.ctypeslib.as_array(pts, shape=(max(total, 1) * 2,))[: total * 2].copy() if total else np.zeros(0, np.int32)
    L.orc_free(pts)
    L.orc_free(off)
    flat = flat.reshape(-1, 2).astype(np.int32)
    return [flat[offs[i]: offs[i + 1]] for i in range(n)]


def contour_area(c):
    c = np.ascontiguousarray(c, np.int32)
    return lib().orc_contour_area(_p(c), len(c))


def arc_length(c, closed=True):
    c = np.ascontiguousarray(c, np.int32)
    return lib().orc_arc_length(_p(c), len(c), int(closed))


def approx_poly_dp(c, eps, closed=True):
    c = np.ascontiguousarray(c, np.int32)
    out = np.empty((max(len(c), 1) + 1, 2), np.int32)
    n = lib().orc_approx_poly_dp(_p(c), len(c), C.c_double(eps), int(closed), _p(out))
    return out[:n].copy()


def convex_hull_area(c):
    c = np.ascontiguousarray(c, np.int32)
    return lib().orc_convex_hull_area(_p(c), len(c))


def bounding_rect(c):
    c = np.ascontiguousarray(c, np.int32)
    r = np.empty(4, np.int32)
    lib().orc_bounding_rect(_p(c), len(c), _p(r))
    return tuple(int(v) for v in r)


def detect_border_radius(contour, epsilon_factor=0.02):
    """shape pyc @L32-61."""
    epsilon = epsilon_factor * arc_length(contour, True)
    approx = approx_poly_dp(contour, epsilon, True)
    if len(approx) > 4:
        hull_area = convex_hull_area(contour)
        contour_area_ = contour_area(contour)
        if hull_area > 0:
            border_radius = (1 - contour_area_ / hull_area) * 50.0
            return max(0.0, border_radius)
    return 0.0


def classify_contour(contour):
    """Body of the analyze_shapes loop (shape pyc @L146-181); None when area < 100."""
    if contour_area(contour) < 100:
        return None
    x, y, w, h = bounding_rect(contour)
    border_radius = detect_border_radius(contour)
    epsilon = 0.04 * arc_length(contour, True)
    approx = approx_poly_dp(contour, epsilon, True)
    shape_type = "unknown"
    if len(approx) == 3:
        shape_type = "triangle"
    elif len(approx) == 4:
        _aspect_ratio = w / float(h)  # computed and unused in the reference
        shape_type = "rectangle"
    elif len(approx) > 4:
        area = contour_area(contour)
        perimeter = arc_length(contour, True)
        if perimeter > 0:
            circularity = 4 * np.pi * area / perimeter ** 2
            shape_type = "circle" if circularity > 0.8 else "polygon"
    return {
        "type": shape_type,
        "x": int(x),
        "y": int(y),
        "width": int(w),
        "height": int(h),
        "border_radius": border_radius,
        "area": contour_area(contour),
    }


def analyze_shapes(bgr):
    """ShapeAnalyzer.analyze_shapes (shape pyc @L125-189) on a BGR u8 image."""
    bgr = _chk_bgr(bgr)
    mask = shape_mask(bgr)
    contours = find_contours_external(mask)
    shapes = []
    for c in contours:
        r = classify_contour(c)
        if r is not None:
            shapes.append(r)
    return {
        "shapes": shapes,
        "total_shapes": len(shapes),
        "metadata": {"image_width": bgr.shape[1], "image_height": bgr.shape[0]},
    }


# --------------------------------------------------------------------------- shadows
def shadow_level_from_stats(mask_sum, mask_count):
    """shadow pyc @L21-31 given sum/count of processed[thresh == 255]."""
    if mask_count == 0:
        return "Low"
    avg_darkness = 255 - np.float64(mask_sum) / np.float64(mask_count)
    if avg_darkness < 30:
        return "Low"
    elif avg_darkness < 60:
        return "Moderate"
    return "High"


def analyze_shadow_level(bgr):
    s, c = shadow_stats(bgr)
    return shadow_level_from_stats(s, c)


# --------------------------------------------------------------------------- colours
def numpy_noise(n_pixels, seed):
    """np.random.normal(0, 0.5, (P, 3)).astype(np.int8) from a seeded legacy
    RandomState -- the exact stream color_extractor.py:224 draws (RGB order)."""
    rs = np.random.RandomState(seed)
    return rs.normal(0, 0.5, (n_pixels, 3)).astype(np.int8)


def device_noise(n_pixels, seed, index):
    """The product's production noise for the image with global ``index`` under batch
    ``seed`` (no caller noise; unique.hip), restated in llfe_oracle.c
    ``orc_device_noise``: (n_pixels, 3) int8 in RGB order, the layout of numpy_noise."""
    out = np.empty((max(int(n_pixels), 0), 3), np.int8)
    lib().orc_device_noise(C.c_int64(int(n_pixels)), C.c_uint64(int(seed) & MASK64), C.c_int64(int(index)), _p(out))
    return out


def color_unique(bgr, noise=None):
    bgr = _chk_bgr(bgr)
    h, w = bgr.shape[:2]
    keys = np.empty(max(h * w, 1), np.uint32)
    nz = None if noise is None else np.ascontiguousarray(noise, np.int8).reshape(-1)
    u = lib().orc_color_unique(_p(bgr), h, w, None if nz is None else _p(nz), _p(keys))
    return keys[:u].copy()


def kmeans(data, K, attempts=10, max_count=200, eps=0.2, rng_state=0xFFFFFFFF):
    data = np.ascontiguousarray(data, np.float32)
    N = data.shape[0]
    labels = np.empty(N, np.int32)
    centers = np.empty((K, 3), np.float32)
    counts = np.empty(K, np.int32)
    iters = np.empty(attempts, np.int32)
    c = lib().orc_kmeans(_p(data), N, K, max_count, C.c_double(eps), attempts, C.c_uint64(rng_state),
                         _p(labels), _p(centers), _p(counts), _p(iters))
    return c, labels, centers, counts, iters


def kmeans_attempts(keys, K, rng_state, exact_sums=False, attempts=10):
    """Every attempt of cv2.kmeans on the unique colours ``keys`` (packed RGB, np.unique
    order; llfe_oracle.c orc_kmeans_ex): per attempt its k-means++ centres, final centres
    (float32, before astype(uint8)), counters, compactness, iterations and the centres after
    each Lloyd update.  exact_sums: the device's exact int64 cluster sums instead of
    OpenCV's sequential float32 ones (kmeans.hip / DESIGN.md §5)."""
    keys = np.asarray(keys, np.uint32)
    data = np.ascontiguousarray(np.stack([(keys >> 16) & 255, (keys >> 8) & 255, keys & 255], -1), np.float32)
    N = data.shape[0]
    labels = np.empty(N, np.int32)
    best = np.empty((K, 3), np.float32)
    bcnt = np.empty(K, np.int32)
    iters = np.empty(attempts, np.int32)
    pp = np.zeros((attempts, K, 3), np.float32)
    cen = np.zeros((attempts, K, 3), np.float32)
    cnt = np.zeros((attempts, K), np.int32)
    comp = np.zeros(attempts, np.float64)
    it = np.full((attempts, 100, K, 3), np.nan, np.float32)
    c = lib().orc_kmeans_ex(_p(data), N, K, 200, C.c_double(0.2), attempts, C.c_uint64(rng_state), int(exact_sums),
                            _p(labels), _p(best), _p(bcnt), _p(iters), _p(pp), _p(cen), _p(cnt), _p(comp), _p(it))
    return {"compactness": c, "labels": labels, "centers": best, "counts": bcnt, "iters": iters, "pp": pp,
            "att_centers": cen, "att_counts": cnt, "att_compactness": comp, "iter_centers": it}


def dominant_colors(bgr, noise=None, n_colors=5, rng_state=0xFFFFFFFF):
    """_get_dominant_colors on the noised RGB pixels. Returns (centers_rgb u8 (K,3),
    counts (K,), n_unique, compactness); counts = np.bincount(labels)."""
    bgr = _chk_bgr(bgr)
    h, w = bgr.shape[:2]
    cap = max(n_colors, 5)
    centers = np.zeros((cap, 3), np.uint8)
    counts = np.zeros(cap, np.int32)
    nu = C.c_int64()
    comp = C.c_double()
    nz = None if noise is None else np.ascontiguousarray(noise, np.int8).reshape(-1)
    k = lib().orc_dominant_colors(_p(bgr), h, w, None if nz is None else _p(nz), n_colors, C.c_uint64(rng_state),
                                  _p(centers), _p(counts), C.byref(nu), C.byref(comp))
    return centers[:k].copy(), counts[:k].copy(), int(nu.value), float(comp.value)


def rgb_to_hex(rgb):
    return "#{:02x}{:02x}{:02x}".format(rgb[0], rgb[1], rgb[2])


def hex_to_rgb(hex_color):
    hex_color = hex_color.lstrip("#")
    return tuple(int(hex_color[i:i + 2], 16) for i in (0, 2, 4))


def is_light_color(rgb):
    r, g, b = [x / 255.0 for x in rgb]
    luminance = 0.2126 * r + 0.7152 * g + 0.0722 * b
    return luminance > 0.6


def color_palette(centers_rgb, counts):
    """color_extractor.py:231-284 given centres (already in k-means order) and the
    per-centre bincount.  Uses a stable descending order; equal counts are
    unordered in the reference (host-SIMD argsort), tests compare them as sets."""
    centers = np.asarray(centers_rgb, np.uint8).reshape(-1, 3)
    counts = np.asarray(counts)
    if len(centers) > 1:
        order = np.argsort(-counts, kind="stable")
        centers = centers[order]
    hex_colors = [rgb_to_hex(tuple(int(v) for v in c)) for c in centers]
    hex_colors = [c for c in hex_colors if c.lower() not in ["#ffffff", "#000000"]]
    if not hex_colors:
        bg = "#000000" if is_light_color((255, 255, 255)) else "#FFFFFF"
        return {"primary": bg, "background": bg, "accent": [bg] * 3}
    primary = hex_colors[0]
    accent = [c for c in hex_colors if c != primary][:3]
    while len(accent) < 3:
        accent.append(accent[-1] if accent else primary)
    bg = "#FFFFFF" if not is_light_color(hex_to_rgb(primary)) else "#000000"
    return {"primary": primary, "background": bg, "accent": accent[:3]}


# --------------------------------------------------------------------------- resize
def thumbnail_size(w, h, max_w=1920, max_h=1080):
    """PIL Image.thumbnail's preserve_aspect_ratio; None when no resize happens."""
    x, y = math.floor(max_w), math.floor(max_h)
    if x >= w and y >= h:
        return None
    aspect = w / h

    def round_aspect(number, key):
        return max(min(math.floor(number), math.ceil(number), key=key), 1)

    if x / y >= aspect:
        x = round_aspect(y * aspect, key=lambda n: abs(aspect - n / y))
    else:
        y = round_aspect(x / aspect, key=lambda n: 0 if n == 0 else abs(aspect - x / n))
    return x, y


def pil_resize_lanczos(img, out_w, out_h, box=None):
    img = np.ascontiguousarray(img, np.uint8)
    if img.ndim == 2:
        img = img[:, :, None]
    h, w, ch = img.shape
    out = np.empty((out_h, out_w, ch), np.uint8)
    b = None
    if box is not None:
        b = np.asarray(box, np.float64)
    lib().orc_pil_resize_lanczos(_p(img), h, w, ch, _p(out), out_h, out_w, None if b is None else _p(b))
    return out


def pil_reduce(img, fx, fy):
    img = np.ascontiguousarray(img, np.uint8)
    if img.ndim == 2:
        img = img[:, :, None]
    h, w, ch = img.shape
    out = np.empty(((h + fy - 1) // fy, (w + fx - 1) // fx, ch), np.uint8)
    lib().orc_pil_reduce(_p(img), h, w, ch, fx, fy, _p(out))
    return out


def pil_thumbnail(img, max_w=1920, max_h=1080, reducing_gap=2.0):
    """PIL Image.thumbnail((max_w, max_h), LANCZOS) restated: size rule, reduce()
    pre-pass when the input is >= 2 * reducing_gap x the target, then resize with the
    fractional box left by the reduction."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape[:2]
    size = thumbnail_size(w, h, max_w, max_h)
    if size is None:
        return img
    ow, oh = size
    fx = int(w / ow / reducing_gap) or 1
    fy = int(h / oh / reducing_gap) or 1
    box = None
    if fx > 1 or fy > 1:
        img = pil_reduce(img, fx, fy)
        box = (0.0, 0.0, w / fx, h / fy)
    return pil_resize_lanczos(img, ow, oh, box)


def preprocess_size(w, h, mode):
    """utils.py:118-143: (new_w, new_h, interpolation) or None when no resize."""
    limits = {"auto": (2000, "area"), "high_quality": (4000, "lanczos4"), "performance": (1000, "linear")}
    if mode not in limits:
        return None
    max_dim, interp = limits[mode]
    if max(h, w) > max_dim:
        scale = max_dim / max(h, w)
        return int(w * scale), int(h * scale), interp
    return None


CV_INTER = {"linear": 1, "cubic": 2, "area": 3, "lanczos4": 4}


def cv_resize(img, out_w, out_h, interp):
    """cv2.resize(img, (out_w, out_h), interpolation=INTER_<interp>) on u8 (H, W[, C]),
    restated in llfe_oracle.c (utils.py:118-143)."""
    img = np.ascontiguousarray(img, np.uint8)
    squeeze = img.ndim == 2
    if squeeze:
        img = img[:, :, None]
    h, w, ch = img.shape
    out = np.empty((out_h, out_w, ch), np.uint8)
    code = CV_INTER[interp] if isinstance(interp, str) else int(interp)
    if lib().orc_cv_resize(_p(img), h, w, ch, _p(out), out_h, out_w, code) != 0:
        raise ValueError(f"cv_resize: unsupported {interp!r} {w}x{h} -> {out_w}x{out_h}")
    return out[:, :, 0] if squeeze else out


def cv_resize_scaled(img, fx, fy, interp):
    """cv2.resize(img, None, fx=fx, fy=fy, interpolation=...): dsize = saturate_cast<int>
    of w * fx, h * fy and the given factors as the inverse scales."""
    img = np.ascontiguousarray(img, np.uint8)
    squeeze = img.ndim == 2
    if squeeze:
        img = img[:, :, None]
    h, w, ch = img.shape
    out_w, out_h = int(np.rint(w * fx)), int(np.rint(h * fy))
    out = np.empty((out_h, out_w, ch), np.uint8)
    code = CV_INTER[interp] if isinstance(interp, str) else int(interp)
    if lib().orc_cv_resize_scaled(_p(img), h, w, ch, _p(out), out_h, out_w, C.c_double(fx), C.c_double(fy),
                                  code) != 0:
        raise ValueError(f"cv_resize_scaled: unsupported {interp!r} {w}x{h} x ({fx}, {fy})")
    return out[:, :, 0] if squeeze else out


def otsu_threshold(gray) -> int:
    """cv2.threshold(gray, 0, 255, THRESH_BINARY + THRESH_OTSU)[0] (non-IPP path)."""
    g = np.ascontiguousarray(gray, np.uint8)
    return int(lib().orc_otsu_threshold(_p(g), C.c_longlong(g.size)))


def text_size(h, w):
    """Output size (h, w) of TextExtractor.preprocess_image (text_extractor.py:31-37)."""
    oh, ow = C.c_int(), C.c_int()
    lib().orc_text_size(h, w, C.byref(oh), C.byref(ow), None)
    return oh.value, ow.value


def text_binary(img):
    """TextExtractor.preprocess_image (text_extractor.py:15-46) restated in llfe_oracle.c:
    (binary u8 image, Otsu threshold)."""
    img = np.ascontiguousarray(img, np.uint8)
    if img.ndim == 2:
        img = img[:, :, None]
    h, w, cn = img.shape
    oh, ow = text_size(h, w)
    out = np.empty((oh, ow), np.uint8)
    t = lib().orc_text_binary(_p(img), h, w, cn, _p(out))
    return out, int(t)


def preprocess(img, mode):
    """validate_and_preprocess_image's resize step on a decoded BGR image."""
    plan = preprocess_size(img.shape[1], img.shape[0], mode)
    if plan is None:
        return img
    return cv_resize(img, plan[0], plan[1], plan[2])


# --------------------------------------------------------------------------- seeds
MASK64 = (1 << 64) - 1


def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & MASK64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def image_rng_state(seed, index):
    """Per-image cv::RNG state used by the product's k-means for batch item
    ``index``; 0 maps to cv::RNG's default 0xffffffff."""
    s = splitmix64((seed + index) & MASK64)
    return s if s else 0xFFFFFFFF
