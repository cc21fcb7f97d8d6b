"""Known-answer and independent-restatement tests for the OpenCV-backed oracle stages.

OpenCV is not importable anywhere in this pipeline and the reference ships no tests or
fixtures for these stages, so these stages are "parity unpinned" against OpenCV itself
(DESIGN.md §Oracle).  What pins them here:

* hand-derived known answers (documented OpenCV constants and values anyone can check
  with cv2: cvtColor of pure B/G/R = 29/150/76, getGaussianKernel(5, 0) fixed point
  = [1,4,6,4,1]*16, ...);
* a second, independent NumPy/SciPy restatement of each stage, compared bit-exactly on
  random inputs (separable fixed-point blur, float separable blur with emulated FMA,
  Sobel, 8-connected hysteresis via scipy.ndimage.label, 3x3 dilation).
"""
import math

import numpy as np
import pytest
from scipy import ndimage


def _rng(seed):
    return np.random.default_rng(seed)


def _smooth_image(seed, h, w, levels=255):
    r = _rng(seed)
    a = r.random((h // 8 + 2, w // 8 + 2))
    a = ndimage.zoom(a, 8, order=1)[:h, :w]
    a = (a - a.min()) / max(a.max() - a.min(), 1e-9) * levels
    return a.astype(np.uint8)


# --------------------------------------------------------------------------- gray
def test_bgr2gray_known_values(orc):
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0]]], np.uint8)
    assert orc.bgr2gray(px).tolist() == [[29, 150, 76, 255, 0]]


def test_bgr2gray_formula(orc):
    bgr = _rng(1).integers(0, 256, (37, 53, 3), dtype=np.uint8)
    b, g, r = (bgr[..., i].astype(np.int64) for i in range(3))
    want = ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)
    np.testing.assert_array_equal(orc.bgr2gray(bgr), want)


# --------------------------------------------------------------------------- gaussian kernels
def test_gaussian_kernels(orc):
    assert orc.gaussian_kernel_fixed8(5).tolist() == [16, 64, 96, 64, 16]
    k11 = orc.gaussian_kernel_fixed8(11)
    assert k11.sum() == 256 and (k11 == k11[::-1]).all()
    kf = orc.gaussian_kernel_float(11).astype(np.float64)
    sigma = 0.3 * ((11 - 1) * 0.5 - 1) + 0.8  # = 2.0 (getGaussianKernel, sigma <= 0)
    x = np.arange(11) - 5
    g = np.exp(-x * x / (2 * sigma * sigma))
    np.testing.assert_allclose(kf, g / g.sum(), rtol=2e-6)
    assert abs(kf.sum() - 1) < 1e-6


def _reflect101(i, n):
    if n == 1:
        return np.zeros_like(i)
    i = np.abs(i)
    return np.where(i >= n, 2 * (n - 1) - i, i)


def _blur5_np(g):
    h, w = g.shape
    k = np.array([16, 64, 96, 64, 16], np.int64)
    xi = _reflect101(np.arange(w)[:, None] + np.arange(-2, 3)[None, :], w)
    yi = _reflect101(np.arange(h)[:, None] + np.arange(-2, 3)[None, :], h)
    g = g.astype(np.int64)
    rows = (g[:, xi] * k).sum(-1)  # (h, w)
    full = (rows[yi, :] * k[None, :, None]).sum(1)
    return ((full + (1 << 15)) >> 16).astype(np.uint8)


@pytest.mark.parametrize("shape", [(1, 1), (1, 7), (2, 2), (5, 3), (31, 47), (64, 64)])
def test_blur5_matches_numpy(orc, shape):
    g = _rng(shape[0] * 100 + shape[1]).integers(0, 256, shape, dtype=np.uint8)
    np.testing.assert_array_equal(orc.blur5(g), _blur5_np(g))


def test_blur5_impulse(orc):
    g = np.zeros((9, 9), np.uint8)
    g[4, 4] = 255
    out = orc.blur5(g).astype(np.int64)
    k = np.array([1, 4, 6, 4, 1])
    want = (np.outer(k, k) * 255 * 256 + (1 << 15)) >> 16
    np.testing.assert_array_equal(out[2:7, 2:7], want)
    assert out.sum() == out[2:7, 2:7].sum()


# --------------------------------------------------------------------------- adaptive threshold
def _fma32(a, b, c):
    # a*b is exact in float64 for float32 operands; one rounding of the sum to f32 (the
    # double rounding f64->f32 differs from a true fma only on ties, ~2^-29 per op)
    return (a.astype(np.float64) * np.float64(b) + c.astype(np.float64)).astype(np.float32)


def _gauss_float_mean_np(src, k):
    h, w = src.shape
    r = len(k) // 2
    x = src.astype(np.float32)
    s = np.zeros((h, w), np.float32)
    for j in range(len(k)):
        idx = np.clip(np.arange(w) + j - r, 0, w - 1)
        s = _fma32(x[:, idx], k[j], s)
    t = s
    s = _fma32(t, k[r], np.zeros_like(t))
    for d in range(1, r + 1):
        a = t[np.clip(np.arange(h) + d, 0, h - 1)]
        b = t[np.clip(np.arange(h) - d, 0, h - 1)]
        s = _fma32((a + b).astype(np.float32), k[r + d], s)
    return np.clip(np.rint(s), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("shape", [(1, 1), (3, 17), (40, 33), (64, 80)])
def test_gauss_float_mean_matches_numpy(orc, shape):
    g = _rng(7 + shape[1]).integers(0, 256, shape, dtype=np.uint8)
    k = orc.gaussian_kernel_float(11)
    np.testing.assert_array_equal(orc.gauss_float_mean(g), _gauss_float_mean_np(g, k))


def test_adaptive_threshold_kats(orc):
    flat = np.full((20, 20), 173, np.uint8)
    assert orc.adaptive_threshold_inv(flat).max() == 0  # src - mean = 0 > -2
    dot = flat.copy()
    dot[10, 10] = 20
    t = orc.adaptive_threshold_inv(dot)
    assert t[10, 10] == 255 and t.sum() == 255  # only the dark pixel is below its mean
    g = _rng(3).integers(0, 256, (30, 30), dtype=np.uint8)
    mean = orc.gauss_float_mean(g)
    want = np.where(g.astype(int) - mean.astype(int) <= -2, 255, 0)
    np.testing.assert_array_equal(orc.adaptive_threshold_inv(g), want)


def test_shadow_stats_composition(orc):
    bgr = _rng(11).integers(0, 256, (48, 64, 3), dtype=np.uint8)
    b = orc.blur5(orc.bgr2gray(bgr))
    t = orc.adaptive_threshold_inv(b)
    s, c = orc.shadow_stats(bgr)
    assert c == int((t == 255).sum()) and s == int(b[t == 255].astype(np.int64).sum())


def test_shadow_level_thresholds(orc):
    f = orc.shadow_level_from_stats
    assert f(0, 0) == "Low"
    assert f(226 * 10, 10) == "Low"          # darkness 29
    assert f(225 * 10, 10) == "Moderate"     # darkness 30
    assert f(196 * 10, 10) == "Moderate"     # darkness 59
    assert f(195 * 10, 10) == "High"         # darkness 60
    assert f(3 * 255 + 254, 4) == "Low"      # darkness 0.25


# --------------------------------------------------------------------------- canny
def test_sobel_matches_numpy(orc):
    g = _rng(5).integers(0, 256, (23, 31), dtype=np.uint8)
    h, w = g.shape
    p = np.pad(g.astype(np.int32), 1, mode="edge")
    dx = (p[:-2, 2:] + 2 * p[1:-1, 2:] + p[2:, 2:]) - (p[:-2, :-2] + 2 * p[1:-1, :-2] + p[2:, :-2])
    dy = (p[2:, :-2] + 2 * p[2:, 1:-1] + p[2:, 2:]) - (p[:-2, :-2] + 2 * p[:-2, 1:-1] + p[:-2, 2:])
    gx, gy = orc.sobel3(g)
    np.testing.assert_array_equal(gx, dx)
    np.testing.assert_array_equal(gy, dy)


def test_canny_vertical_step(orc):
    g = np.zeros((32, 32), np.uint8)
    g[:, 10:] = 200
    e = orc.canny(g)
    # |dx| = 800 at x = 9 and x = 10; NMS keeps m > left && m >= right -> x = 9 only
    want = np.zeros_like(e)
    want[:, 9] = 255
    np.testing.assert_array_equal(e, want)


def test_canny_horizontal_step(orc):
    g = np.zeros((32, 32), np.uint8)
    g[12:, :] = 200
    want = np.zeros_like(g)
    want[11, :] = 255  # vertical direction: m > up && m >= down
    np.testing.assert_array_equal(orc.canny(g), want)


def test_canny_weak_gradient_dropped(orc):
    g = np.zeros((16, 16), np.uint8)
    g[:, 8:] = 10  # |dx| = 40 < low threshold 50
    assert orc.canny(g).max() == 0


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_hysteresis_is_8conn_components_with_a_strong_pixel(orc, seed):
    g = _smooth_image(seed, 96, 128)
    g = np.clip(g.astype(int) + _rng(seed + 50).integers(-12, 13, g.shape), 0, 255).astype(np.uint8)
    cls = orc.canny_nms(g)
    cand = cls != 1
    lab, n = ndimage.label(cand, structure=np.ones((3, 3), int))
    strong_labels = np.unique(lab[cls == 2])
    want = np.where(np.isin(lab, strong_labels[strong_labels > 0]), 255, 0)
    np.testing.assert_array_equal(orc.canny(g), want)
    assert (cls == 2).any() and (cls == 0).any()


def test_dilate_matches_scipy(orc):
    m = (_rng(9).random((41, 57)) > 0.97).astype(np.uint8) * 255
    want = ndimage.grey_dilation(m, size=(3, 3), mode="constant", cval=0)
    np.testing.assert_array_equal(orc.dilate3(m), want)
    g = _rng(10).integers(0, 256, (13, 17), dtype=np.uint8)
    np.testing.assert_array_equal(orc.dilate3(g), ndimage.grey_dilation(g, size=(3, 3), mode="nearest"))


def test_shape_mask_composition(orc):
    bgr = _rng(12).integers(0, 256, (40, 50, 3), dtype=np.uint8)
    want = orc.dilate3(orc.canny(orc.blur5(orc.bgr2gray(bgr))))
    np.testing.assert_array_equal(orc.shape_mask(bgr), want)


# --------------------------------------------------------------------------- contours + geometry
def test_rectangle_contour(orc):
    m = np.zeros((20, 30), np.uint8)
    m[3:9, 5:17] = 255  # x 5..16, y 3..8
    cs = orc.find_contours_external(m)
    assert len(cs) == 1
    assert cs[0].tolist() == [[5, 3], [5, 8], [16, 8], [16, 3]]
    assert orc.contour_area(cs[0]) == 11 * 5
    assert orc.arc_length(cs[0]) == 2 * (11 + 5)
    assert orc.bounding_rect(cs[0]) == (5, 3, 12, 6)


def test_contour_degenerate_shapes(orc):
    m = np.zeros((10, 10), np.uint8)
    m[4, 6] = 1
    assert [c.tolist() for c in orc.find_contours_external(m)] == [[[6, 4]]]
    m = np.zeros((10, 10), np.uint8)
    m[2, 1:8] = 1
    assert [c.tolist() for c in orc.find_contours_external(m)] == [[[1, 2], [7, 2]]]
    assert orc.find_contours_external(np.zeros((5, 5), np.uint8)) == []
    full = np.ones((4, 6), np.uint8)  # touches every border (1-px zero pad)
    assert orc.find_contours_external(full)[0].tolist() == [[0, 0], [0, 3], [5, 3], [5, 0]]


def test_contours_external_only_and_order(orc):
    m = np.zeros((40, 40), np.uint8)
    m[2:6, 2:6] = 1            # discovered first (top)
    m[10:30, 10:30] = 1        # ring with a hole containing a blob
    m[14:26, 14:26] = 0
    m[18:22, 18:22] = 1
    cs = orc.find_contours_external(m)
    assert len(cs) == 2  # the inner blob is not external
    # OpenCV returns contours in reverse discovery order
    assert orc.bounding_rect(cs[0]) == (10, 10, 20, 20)
    assert orc.bounding_rect(cs[1]) == (2, 2, 4, 4)


def test_area_and_arclength_numpy(orc):
    r = _rng(21)
    for _ in range(20):
        n = int(r.integers(1, 30))
        c = r.integers(-50, 50, (n, 2)).astype(np.int32)
        x, y = c[:, 0].astype(float), c[:, 1].astype(float)
        area = abs(np.sum(np.roll(x, 1) * y - x * np.roll(y, 1))) / 2 if n >= 3 else 0.0
        assert orc.contour_area(c) == pytest.approx(area, abs=1e-9)
        d = np.diff(np.vstack([c, c[:1]]), axis=0).astype(np.float32)
        per = float(np.sum(np.sqrt((d * d).sum(1)).astype(np.float32), dtype=np.float64)) if n > 1 else 0.0
        assert orc.arc_length(c) == pytest.approx(per, rel=1e-6)


def test_approx_poly_dp_kats(orc):
    # square with collinear points on every edge -> 4 corners
    sq = [(0, 0), (0, 5), (0, 10), (5, 10), (10, 10), (10, 5), (10, 0), (5, 0)]
    assert len(orc.approx_poly_dp(np.array(sq), 0.5)) == 4
    tri = [(0, 0), (10, 0), (20, 0), (10, 15)]
    assert len(orc.approx_poly_dp(np.array(tri), 1.0)) == 3
    # small eps keeps every vertex of a convex octagon
    ang = np.arange(8) * 2 * np.pi / 8
    octo = np.stack([np.round(50 + 40 * np.cos(ang)), np.round(50 + 40 * np.sin(ang))], 1).astype(np.int32)
    assert len(orc.approx_poly_dp(octo, 1.0)) == 8


def test_convex_hull_area(orc):
    pts = np.array([(0, 0), (0, 10), (5, 5), (10, 10), (10, 0)], np.int32)  # notch at (5,5)
    assert orc.convex_hull_area(pts) == 100.0
    assert orc.contour_area(pts) == 75.0


def _disc(h, w, cy, cx, r):
    yy, xx = np.mgrid[:h, :w]
    return (((yy - cy) ** 2 + (xx - cx) ** 2) <= r * r).astype(np.uint8)


def test_classify_contour_kats(orc):
    m = np.zeros((60, 80), np.uint8)
    m[10:40, 5:55] = 1
    (c,) = orc.find_contours_external(m)
    s = orc.classify_contour(c)
    assert s["type"] == "rectangle" and s["border_radius"] == 0.0
    assert (s["x"], s["y"], s["width"], s["height"]) == (5, 10, 50, 30) and s["area"] == 49 * 29
    (c,) = orc.find_contours_external(_disc(100, 100, 50, 50, 30))
    s = orc.classify_contour(c)
    assert s["type"] == "circle" and s["border_radius"] > 0
    m = np.zeros((30, 30), np.uint8)
    m[5:12, 5:12] = 1  # area 36 < 100
    (c,) = orc.find_contours_external(m)
    assert orc.classify_contour(c) is None
    m = np.zeros((80, 80), np.uint8)
    for y in range(10, 70):  # right triangle
        m[y, 10:10 + (y - 10)] = 1
    (c,) = orc.find_contours_external(m)
    assert orc.classify_contour(c)["type"] == "triangle"


# --------------------------------------------------------------------------- k-means + RNG
def test_cv_rng_matches_mwc(orc):
    import ctypes as C

    st = C.c_uint64(0xFFFFFFFF)
    s = 0xFFFFFFFF
    for _ in range(1000):
        s = ((s & 0xFFFFFFFF) * 4164903690 + (s >> 32)) & ((1 << 64) - 1)
        assert orc.lib().orc_cvrng_next(C.byref(st)) == (s & 0xFFFFFFFF)


def test_kmeans_separated_clusters(orc):
    r = _rng(4)
    means = np.array([[20, 20, 20], [200, 30, 40], [40, 220, 60], [90, 90, 230], [250, 250, 10]], np.float32)
    data = np.concatenate([m + r.integers(-3, 4, (100 + 20 * i, 3)) for i, m in enumerate(means)]).astype(np.float32)
    comp, labels, centers, counts, iters = orc.kmeans(data, 5)
    assert sorted(counts.tolist()) == [100, 120, 140, 160, 180]
    for k in range(5):
        pts = data[labels == k]
        np.testing.assert_allclose(centers[k], pts.mean(0), atol=1e-3)
    d = data - centers[labels]
    assert comp == pytest.approx(float((d.astype(np.float64) ** 2).sum()), rel=1e-5)
    assert (iters >= 1).all() and (iters <= 100).all()


def test_kmeans_fewer_points_than_clusters_paths(orc):
    data = np.array([[1, 2, 3], [1, 2, 3], [9, 9, 9]], np.float32)
    comp, labels, centers, counts, _ = orc.kmeans(data, 2)
    assert comp == 0.0 and sorted(counts.tolist()) == [1, 2]
    one = np.array([[5, 6, 7]], np.float32)
    comp, labels, centers, counts, _ = orc.kmeans(one, 1)
    assert comp == 0.0 and centers[0].tolist() == [5, 6, 7]


def test_dominant_colors_small_palette(orc):
    bgr = np.zeros((20, 20, 3), np.uint8)
    bgr[:, :10] = (255, 0, 0)
    bgr[:, 10:] = (0, 0, 255)
    bgr[:5, :5] = (0, 255, 0)
    centers, counts, nu, _ = orc.dominant_colors(bgr, None, 5)
    assert nu == 3 and len(centers) == 3  # K = min(5, n_unique)
    got = {tuple(c.tolist()): int(n) for c, n in zip(centers, counts)}
    # np.unique -> kmeans on UNIQUE colours: every centre is one colour, count 1
    assert set(got) == {(0, 0, 255), (255, 0, 0), (0, 255, 0)} and set(got.values()) == {1}


def test_color_palette_rules(orc):
    pal = orc.color_palette(np.array([[255, 255, 255], [10, 20, 30], [200, 200, 200]]), [5, 3, 1])
    assert pal == {"primary": "#0a141e", "background": "#FFFFFF", "accent": ["#c8c8c8", "#c8c8c8", "#c8c8c8"]}
    pal = orc.color_palette(np.array([[255, 255, 255], [0, 0, 0]]), [1, 1])
    assert pal == {"primary": "#000000", "background": "#000000", "accent": ["#000000"] * 3}
    pal = orc.color_palette(np.array([[240, 240, 240]]), [1])
    assert pal["background"] == "#000000" and pal["accent"] == ["#f0f0f0"] * 3


def test_preprocess_and_seed_helpers(orc):
    assert orc.preprocess_size(1920, 1080, "auto") is None
    assert orc.preprocess_size(3840, 2160, "auto") == (2000, 1125, "area")
    assert orc.preprocess_size(3840, 2160, "high_quality") is None
    assert orc.preprocess_size(1920, 1080, "performance") == (1000, 562, "linear")
    assert orc.preprocess_size(5000, 5000, "none") is None
    assert orc.image_rng_state(0, 0) == orc.splitmix64(0) != 0
    assert orc.splitmix64(0) == 0xE220A8397B1DCDAF
    assert math.isclose(orc.thumbnail_size(3840, 2160)[0], 1920)


# --------------------------------------------------------------------------- cv2.resize
# utils.py:118-143 (validate_and_preprocess_image): AREA / LANCZOS4 / LINEAR downscales.
# A second restatement in NumPy (float32 scalars for OpenCV's float steps, int64 for its
# fixed point) checked bit-exactly against llfe_oracle.c, plus hand-derived answers.
def _np_area_tab(ssize, dsize, scale):
    tab = []
    for dx in range(dsize):
        f1 = dx * scale
        f2 = f1 + scale
        cell = min(scale, ssize - f1)
        s1, s2 = math.ceil(f1), math.floor(f2)
        s2 = min(s2, ssize - 1)
        s1 = min(s1, s2)
        if s1 - f1 > 1e-3:
            tab.append((dx, s1 - 1, np.float32((s1 - f1) / cell)))
        for s in range(s1, s2):
            tab.append((dx, s, np.float32(1.0 / cell)))
        if f2 - s2 > 1e-3:
            tab.append((dx, s2, np.float32(min(min(f2 - s2, 1.0), cell) / cell)))
    return tab


def _np_lanczos4(x):
    x = np.float32(x)
    s45 = 0.70710678118654752440084436210485
    cs = [(1, 0), (-s45, -s45), (0, 1), (s45, -s45), (-1, 0), (s45, s45), (0, -1), (-s45, s45)]
    y0 = -float(np.float32(x + np.float32(3))) * math.pi * 0.25
    s0, c0 = math.sin(y0), math.cos(y0)
    c = []
    tot = np.float32(0)
    for i in range(8):
        yi = np.float32(np.float32(x + np.float32(3)) - np.float32(i))
        if abs(yi) >= np.float32(1e-6):
            y = -float(yi) * math.pi * 0.25
            v = np.float32((cs[i][0] * s0 + cs[i][1] * c0) / (y * y))
        else:
            v = np.float32(1e30)
        c.append(v)
        tot = np.float32(tot + v)
    inv = np.float32(np.float32(1) / tot)
    return [np.float32(v * inv) for v in c]


def _s16(v):
    return int(np.clip(np.rint(np.float32(v)), -32768, 32767))


def _np_cv_resize(img, ow, oh, interp):
    h, w, cn = img.shape
    sx_, sy_ = w / ow, h / oh  # = 1 / ((double)dsize / ssize) up to the last ulp; recomputed below
    inv_x, inv_y = ow / w, oh / h
    scale_x, scale_y = 1.0 / inv_x, 1.0 / inv_y
    ix, iy = int(round(scale_x)), int(round(scale_y))
    fast = abs(scale_x - ix) < 2.220446049250313e-16 and abs(scale_y - iy) < 2.220446049250313e-16
    if interp == "linear" and fast and ix == 2 and iy == 2:
        interp = "area"
    if interp == "area":
        if fast:
            out = np.zeros((oh, ow, cn), np.uint8)
            for dy in range(oh):
                for dx in range(ow):
                    blk = img[dy * iy:(dy + 1) * iy, dx * ix:(dx + 1) * ix].astype(np.int64)
                    s = blk.sum(axis=(0, 1))
                    if ix == 2 and iy == 2:
                        out[dy, dx] = (s + 2) >> 2
                    else:
                        out[dy, dx] = np.clip(np.rint(s.astype(np.float32) * np.float32(1.0 / np.float32(ix * iy))),
                                              0, 255)
            return out
        S = img.astype(np.float32)
        buf = np.zeros((h, ow, cn), np.float32)
        for dx, sx, a in _np_area_tab(w, ow, scale_x):
            buf[:, dx] = buf[:, dx] + S[:, sx] * a
        acc = np.zeros((oh, ow, cn), np.float32)
        for dy, sy, b in _np_area_tab(h, oh, scale_y):
            acc[dy] = acc[dy] + b * buf[sy]
        return np.clip(np.rint(acc), 0, 255).astype(np.uint8)
    ks = 8 if interp == "lanczos4" else 2

    def coeffs(d, scale, n):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = math.floor(f)
        f = np.float32(f - np.float32(s))
        if ks == 2 and s >= n - 1:
            s, f = n - 1, np.float32(0)
        c = _np_lanczos4(f) if ks == 8 else [np.float32(1) - f, f]
        return s, [_s16(np.float32(v * np.float32(2048))) for v in c]

    xs = [coeffs(dx, scale_x, w) for dx in range(ow)]
    ys = [coeffs(dy, scale_y, h) for dy in range(oh)]
    I = img.astype(np.int64)
    # horizontal pass for every source row: (h, ow, cn)
    hor = np.zeros((h, ow, cn), np.int64)
    for dx, (sx, a) in enumerate(xs):
        for j in range(ks):
            col = min(max(sx - (ks // 2 - 1) + j, 0), w - 1)
            hor[:, dx] += I[:, col] * a[j]
    width = ow * cn
    x_vec = 0
    while x_vec <= width - 16:
        x_vec += 16
    while x_vec < width - 8:
        x_vec += 8
    out = np.zeros((oh, ow * cn), np.int64)
    for dy, (sy, b) in enumerate(ys):
        rows = [hor[min(max(sy - (ks // 2 - 1) + k, 0), h - 1)].reshape(-1) for k in range(ks)]
        if ks == 8:
            v = sum(r * bk for r, bk in zip(rows, b))
            out[dy] = (v + (1 << 21)) >> 22
        else:
            scal = (rows[0] * b[0] + rows[1] * b[1] + (1 << 21)) >> 22
            t = ((np.clip(rows[0] >> 4, -32768, 32767) * b[0]) >> 16) + ((np.clip(rows[1] >> 4, -32768, 32767) * b[1]) >> 16)
            vec = (np.clip(t, -32768, 32767) + 2) >> 2
            idx = np.arange(width)
            out[dy] = np.where(idx < x_vec, vec, scal)
    return np.clip(out, 0, 255).astype(np.uint8).reshape(oh, ow, cn)


RESIZE_CASES = [  # (h, w, oh, ow): exact 2x, 3x, fractional, tall, wide, odd
    (40, 60, 20, 30), (45, 66, 15, 22), (97, 131, 40, 57), (120, 50, 77, 32), (33, 200, 9, 61),
    (64, 64, 21, 21), (101, 103, 100, 102), (18, 26, 7, 13),
]


@pytest.mark.parametrize("interp", ["area", "linear", "lanczos4"])
@pytest.mark.parametrize("h,w,oh,ow", RESIZE_CASES)
def test_cv_resize_numpy_restatement(orc, interp, h, w, oh, ow):
    img = _rng(h * 7 + w).integers(0, 256, (h, w, 3), dtype=np.uint8)
    if interp != "area":
        img = np.stack([_smooth_image(h + w + c, h, w) for c in range(3)], -1)
    got = orc.cv_resize(img, ow, oh, interp)
    exp = _np_cv_resize(img, ow, oh, interp)
    assert np.array_equal(got, exp)


def test_cv_resize_known_answers(orc):
    # INTER_AREA 2x2 (and INTER_LINEAR at exactly 2x, which OpenCV runs as AREA):
    # (a + b + c + d + 2) >> 2 -- 1+2+3+4 = 10 -> 3, 0+0+0+2 = 2 -> 1, 255*4 -> 255
    x = np.array([[1, 2, 0, 0, 255, 255], [3, 4, 0, 2, 255, 255]], np.uint8)[:, :, None]
    assert orc.cv_resize(x, 3, 1, "area")[:, :, 0].tolist() == [[3, 1, 255]]
    assert orc.cv_resize(x, 3, 1, "linear")[:, :, 0].tolist() == [[3, 1, 255]]
    # INTER_AREA 3x3: cvRound(sum * (1.f / 9)); 13 / 9 = 1.44 -> 1, 14 / 9 = 1.56 -> 2
    y = np.zeros((3, 6), np.uint8)
    y[0, 0], y[0, 1] = 9, 4
    y[0, 3], y[2, 5] = 9, 5
    assert orc.cv_resize(y[:, :, None], 2, 1, "area")[:, :, 0].tolist() == [[1, 2]]
    # INTER_LINEAR at 4x: fx = 4 dx + 1.5 -> taps (4dx + 1, 4dx + 2) with 1024 / 1024
    z = np.tile(np.arange(16, dtype=np.uint8) * 10, (4, 1))[:, :, None]
    assert orc.cv_resize(z, 4, 1, "linear")[:, :, 0].tolist() == [[15, 55, 95, 135]]
    # constant images stay constant for every mode and size
    for interp in ("area", "linear", "lanczos4"):
        c = np.full((37, 53, 3), 201, np.uint8)
        assert (orc.cv_resize(c, 17, 11, interp) == 201).all()
    # LANCZOS4 at integer phase (fx = 0) is a copy of the centre tap
    assert _np_lanczos4(0.0)[3] == np.float32(1.0)


def test_cv_resize_preprocess_modes(orc):
    img = _rng(3).integers(0, 256, (1100, 700, 3), dtype=np.uint8)
    assert orc.preprocess(img, "auto") is img and orc.preprocess(img, "none") is img
    out = orc.preprocess(img, "performance")
    assert out.shape == (1000, int(700 * (1000 / 1100)), 3)
