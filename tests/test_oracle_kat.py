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
