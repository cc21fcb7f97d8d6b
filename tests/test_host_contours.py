"""Product host geometry (csrc/contours.cpp through the C ABI) vs the oracle.

findContours(RETR_EXTERNAL, CHAIN_APPROX_SIMPLE) + the per-contour classification of
ShapeAnalyzer.analyze_shapes (shape pyc @L144-189) run on the host in libllfe, fed with
the GPU's bit-packed mask; here they are fed with masks built on the CPU (random,
structured, and the oracle's own shape masks of synthetic UI/photo images)."""
import numpy as np
import pytest
from scipy import ndimage

from low_level_feature_extraction_amd import backend as B


def _masks():
    r = np.random.default_rng(123)
    out = {
        "empty": np.zeros((17, 23), np.uint8),
        "full": np.full((9, 14), 255, np.uint8),
        "pixel": np.pad(np.full((1, 1), 255, np.uint8), ((3, 4), (5, 2))),
        "one_row": (r.random((1, 64)) > 0.5).astype(np.uint8) * 255,
        "one_col": (r.random((64, 1)) > 0.5).astype(np.uint8) * 255,
        "sparse": (r.random((60, 80)) > 0.9).astype(np.uint8),
        "dense": (r.random((60, 80)) > 0.4).astype(np.uint8) * 7,
    }
    blobs = ndimage.gaussian_filter(r.random((200, 300)), 4)
    out["blobs"] = (blobs > np.quantile(blobs, 0.6)).astype(np.uint8) * 255
    rings = np.zeros((120, 160), np.uint8)
    yy, xx = np.mgrid[:120, :160]
    for cy, cx, r0 in [(40, 40, 30), (80, 110, 25), (20, 130, 12)]:
        d = np.hypot(yy - cy, xx - cx)
        rings[(d <= r0) & (d >= r0 - 3)] = 255
        rings[d <= r0 / 3] = 255
    out["rings"] = rings
    return out


MASKS = _masks()


@pytest.mark.parametrize("name", sorted(MASKS))
def test_find_contours_matches_oracle(orc, name):
    m = MASKS[name]
    got = B.find_contours(m)
    want = orc.find_contours_external(m)
    assert len(got) == len(want)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("name", sorted(MASKS))
def test_shapes_from_mask_matches_oracle(orc, name):
    m = MASKS[name]
    want = [s for s in (orc.classify_contour(c) for c in orc.find_contours_external(m)) if s is not None]
    got = B.shapes_from_mask(m)
    assert got == want


@pytest.mark.parametrize("kind,seed", [("ui", 0), ("ui", 1), ("photo", 2), ("photo", 3)])
def test_shapes_on_oracle_masks_of_synthetic_images(orc, kind, seed):
    from low_level_feature_extraction_amd.synth import synth_numpy

    bgr = synth_numpy(seed, 180, 320, seed=99, kind=kind)
    m = orc.shape_mask(bgr)
    want = orc.analyze_shapes(bgr)["shapes"]
    assert B.shapes_from_mask(m) == want
    for c in orc.find_contours_external(m)[:50]:
        assert B.classify_contour(c) == orc.classify_contour(c)
        assert B.border_radius(c) == orc.detect_border_radius(c)


def test_contour_capacity_growth(orc):
    # more points than the binding's initial 64K capacity -> CAPACITY error path + retry
    m = np.zeros((700, 700), np.uint8)
    m[1::3, 1::3] = 1  # 233*233 isolated pixels = 54289 one-point contours
    m[::2, 0] = 1
    got = B.find_contours(m)
    want = orc.find_contours_external(m)
    assert len(got) == len(want) > 50000
    assert all((a == b).all() for a, b in zip(got, want))
