"""TextExtractor.preprocess_image (app/services/analyze/text_extractor.py:15-46), §8f row 4.

CPU: the oracle's restatement (oracle/llfe_oracle.c orc_text_binary: BGR2GRAY, the
INTER_CUBIC upscale of small images, getThreshVal_Otsu_8u, the mean > 127 inversion)
against hand-derived known answers and a second, independent NumPy restatement written
here.  Parity against OpenCV itself is unpinned (no cv2 in this pipeline; the reference
ships no fixtures for this path; opencv-python may take IPP's Otsu / resize paths, the
restatement follows OpenCV's own C++ code with its SSE-baseline vector rounding).
GPU: llfe_text_binary and llfe_resize_cv(INTER_CUBIC) bit-exact vs the oracle.
"""
import math

import numpy as np
import pytest


def _rng(seed):
    return np.random.default_rng(seed)


# ------------------------------------------------------- independent NumPy restatement
def np_cubic_coeffs(x):
    x = np.float32(x)
    A = np.float32(-0.75)
    one = np.float32(1)
    c0 = ((A * (x + one) - np.float32(5) * A) * (x + one) + np.float32(8) * A) * (x + one) - np.float32(4) * A
    c1 = ((A + np.float32(2)) * x - (A + np.float32(3))) * x * x + one
    y = one - x
    c2 = ((A + np.float32(2)) * y - (A + np.float32(3))) * y * y + one
    c3 = one - c0 - c1 - c2
    return [c0, c1, c2, c3]


def np_taps(n_out, scale):
    ofs, coef = [], []
    for d in range(n_out):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = math.floor(f)
        f = np.float32(f - np.float32(s))
        ofs.append(s)
        coef.append([int(np.rint(np.float32(c * np.float32(2048)))) for c in np_cubic_coeffs(f)])
    return ofs, coef


def np_resize_cubic(g, oh, ow, inv_x, inv_y):
    """resizeGeneric_ with HResizeCubic / VResizeCubic (+ VResizeCubicVec_32s8u for the
    elements of its 16-wide loop) on a 2-D u8 image."""
    h, w = g.shape
    xo, xa = np_taps(ow, 1.0 / inv_x)
    yo, yb = np_taps(oh, 1.0 / inv_y)
    g = g.astype(np.int64)
    xv = (ow // 16) * 16
    out = np.zeros((oh, ow), np.uint8)
    for dy in range(oh):
        rows = []
        for k in range(4):
            S = g[min(max(yo[dy] - 1 + k, 0), h - 1)]
            rows.append([sum(int(S[min(max(xo[dx] - 1 + j, 0), w - 1)]) * xa[dx][j] for j in range(4))
                         for dx in range(ow)])
        b = yb[dy]
        sc = np.float32(1.0 / (2048 * 2048))
        bf = [np.float32(np.float32(bk) * sc) for bk in b]
        for x in range(ow):
            if x < xv:
                t = np.float32(rows[3][x]) * bf[3]
                t = np.float32(np.float32(rows[2][x]) * bf[2]) + t
                t = np.float32(np.float32(rows[1][x]) * bf[1]) + t
                t = np.float32(np.float32(rows[0][x]) * bf[0]) + t
                v = int(np.rint(t))
            else:
                v = (rows[0][x] * b[0] + rows[1][x] * b[1] + rows[2][x] * b[2] + rows[3][x] * b[3] + (1 << 21)) >> 22
            out[dy, x] = min(max(v, 0), 255)
    return out


def np_otsu(g):
    hist = np.bincount(g.ravel(), minlength=256)
    n = g.size
    scale = 1.0 / n
    mu = 0.0
    for i in range(256):
        mu += i * float(hist[i])
    mu *= scale
    mu1 = q1 = max_sigma = 0.0
    max_val = 0
    eps = float(np.finfo(np.float32).eps)
    for i in range(256):
        p_i = hist[i] * scale
        mu1 *= q1
        q1 += p_i
        q2 = 1.0 - q1
        if min(q1, q2) < eps or max(q1, q2) > 1.0 - eps:
            continue
        mu1 = (mu1 + i * p_i) / q1
        mu2 = (mu - q1 * mu1) / q2
        sigma = q1 * q2 * (mu1 - mu2) * (mu1 - mu2)
        if sigma > max_sigma:
            max_sigma, max_val = sigma, i
    return max_val


def np_text_binary(img):
    img = np.asarray(img, np.uint8)
    if img.ndim == 3 and img.shape[2] > 1:
        b = img.astype(np.uint32)
        gray = ((b[..., 0] * 1868 + b[..., 1] * 9617 + b[..., 2] * 4899 + 8192) >> 14).astype(np.uint8)
    else:
        gray = img.reshape(img.shape[0], img.shape[1])
    h, w = gray.shape
    if h < 30 or w < 100:
        s = max(2, 300 / w, 100 / h)
        gray = np_resize_cubic(gray, int(np.rint(h * s)), int(np.rint(w * s)), s, s)
    t = np_otsu(gray)
    binary = np.where(gray > t, 255, 0).astype(np.uint8)
    if np.mean(binary) > 127:
        binary = 255 - binary
    return binary, t


# ------------------------------------------------------------------------ CPU tests
def test_cubic_coefficients_known_values():
    assert [float(c) for c in np_cubic_coeffs(0.0)] == [0.0, 1.0, 0.0, 0.0]
    assert [float(c) for c in np_cubic_coeffs(0.5)] == [-0.09375, 0.59375, 0.59375, -0.09375]


@pytest.mark.parametrize("h,w,s", [(13, 17, 2.5), (20, 50, 6.0), (29, 99, 100 / 29), (1, 1, 2.0), (5, 40, 7.5),
                                   (3, 200, 100 / 3)])
def test_oracle_cubic_vs_numpy(orc, h, w, s):
    g = _rng(h * 1000 + w).integers(0, 256, (h, w), dtype=np.uint8)
    ref = np_resize_cubic(g, int(np.rint(h * s)), int(np.rint(w * s)), s, s)
    assert np.array_equal(orc.cv_resize_scaled(g, s, s, "cubic"), ref)


def test_cubic_integer_upscale_of_constant(orc):
    g = np.full((7, 9), 77, np.uint8)
    assert (orc.cv_resize_scaled(g, 2.0, 2.0, "cubic") == 77).all()


def test_otsu_known_answers(orc):
    two = np.array([[10] * 30 + [200] * 70], np.uint8)
    assert orc.otsu_threshold(two) == 10  # every split in [10, 199] ties; first maximum
    assert orc.otsu_threshold(np.full((5, 5), 128, np.uint8)) == 0  # one class: all bins skipped
    three = np.array([[0] * 50 + [100] * 25 + [255] * 25], np.uint8)
    assert orc.otsu_threshold(three) == np_otsu(three)


@pytest.mark.parametrize("seed", range(6))
def test_otsu_vs_numpy(orc, seed):
    r = _rng(seed)
    g = np.clip(np.concatenate([r.normal(60 + 10 * seed, 20, 3000), r.normal(180, 30, 2000)]), 0, 255)
    g = g.astype(np.uint8).reshape(50, 100)
    assert orc.otsu_threshold(g) == np_otsu(g)


@pytest.mark.parametrize("h,w,c", [(20, 50, 3), (29, 99, 3), (30, 100, 3), (12, 140, 1), (64, 80, 4), (1, 1, 3),
                                   (31, 257, 3)])
def test_oracle_text_binary_vs_numpy(orc, h, w, c):
    r = _rng(h * 7 + w + c)
    img = r.integers(0, 256, (h, w, c), dtype=np.uint8)
    img[h // 3: 2 * h // 3, w // 4: w // 2] //= 4  # a dark "text" block
    out, t = orc.text_binary(img)
    ref, rt = np_text_binary(img if c > 1 else img[:, :, 0])
    assert t == rt
    assert np.array_equal(out, ref)


def test_text_size_rule(orc):
    from low_level_feature_extraction_amd.backend import text_size

    for h, w in [(20, 50), (29, 99), (30, 100), (30, 99), (29, 100), (1, 1), (5, 300), (1000, 10), (100, 3)]:
        if h < 30 or w < 100:
            s = max(2, 300 / w, 100 / h)
            exp = (int(np.rint(h * s)), int(np.rint(w * s)))
        else:
            exp = (h, w)
        assert text_size(h, w) == exp == orc.text_size(h, w)


def test_text_size_rejects_overflow():
    from low_level_feature_extraction_amd.backend import text_size

    with pytest.raises(ValueError):
        text_size(1, 30_000_000)  # scale 100: 3e9 columns
    with pytest.raises(ValueError):
        text_size(0, 10)
    assert text_size(1, 20_000_000) == (100, 2_000_000_000)


def test_text_binary_inverts_mostly_white(orc):
    img = np.full((40, 120, 3), 250, np.uint8)
    img[10:20, 10:60] = 5  # dark text on a light page: the page binarises to 255 (mean >
    out, t = orc.text_binary(img)  # 127), so the reference flips it -- page 0, text 255
    assert out.mean() <= 127 and out[15, 20] == 255 and out[0, 0] == 0


# ------------------------------------------------------------------------ GPU tests
@pytest.mark.gpu
@pytest.mark.parametrize("h,w,c", [(20, 50, 3), (29, 99, 3), (30, 100, 3), (12, 140, 1), (64, 80, 4), (1, 1, 3),
                                   (31, 257, 3), (5, 300, 3), (480, 640, 3), (17, 23, 1)])
def test_gpu_text_binary_vs_oracle(backend, orc, h, w, c):
    r = _rng(h * 31 + w + c)
    img = r.integers(0, 256, (h, w, c), dtype=np.uint8)
    img[h // 3: 2 * h // 3, w // 4: w // 2] //= 3
    out, t = backend.text_binary(img)
    ref, rt = orc.text_binary(img)
    assert t == rt
    assert np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.gpu
def test_gpu_text_extractor_dropin(orc):
    from low_level_feature_extraction_amd.text_extractor import TextExtractor

    img = np.full((24, 90, 3), 240, np.uint8)
    img[8:16, 10:70] = 20
    out = TextExtractor.preprocess_image(img)
    assert np.array_equal(out, orc.text_binary(img)[0])
    assert out.shape == orc.text_size(24, 90)
    gray = img[:, :, 1].copy()
    assert np.array_equal(TextExtractor.preprocess_image(gray), orc.text_binary(gray)[0])


@pytest.mark.gpu
@pytest.mark.parametrize("h,w,c,oh,ow", [(13, 17, 1, 40, 33), (20, 50, 3, 120, 300), (64, 48, 4, 100, 77),
                                         (9, 200, 1, 27, 600)])
def test_gpu_resize_cubic_vs_oracle(backend, orc, h, w, c, oh, ow):
    img = _rng(oh + ow).integers(0, 256, (h, w, c), dtype=np.uint8)
    out = backend.resize_cv(img, ow, oh, "cubic").cpu().numpy()
    assert np.array_equal(out, orc.cv_resize(img, ow, oh, "cubic"))
