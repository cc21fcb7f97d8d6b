"""extract_colors' palette rules made in C on the host half of a batch call
(llfe_palette_rules / llfe_image_result, color_extractor.py:231-284) against the Python
restatement ColorExtractor._palette, and the directly built ColorFeatures against the
validated model.  Host only."""
import ctypes as C

import numpy as np
import pytest

from low_level_feature_extraction_amd import _lib as L
from low_level_feature_extraction_amd.color_extractor import ColorExtractor, _validated, palette_features


def _c_palette(centers, counts):
    r = L.LlfeImageResult()
    centers = np.ascontiguousarray(centers, np.uint8).reshape(-1, 3)
    counts = np.ascontiguousarray(counts, np.int32)
    assert L.lib().llfe_palette_rules(centers.ctypes.data, counts.ctypes.data, len(counts), C.byref(r)) == 0
    return r.primary.decode(), r.background.decode(), [bytes(a).split(b"\0")[0].decode() for a in r.accent]


def _cases():
    rng = np.random.default_rng(7)
    out = []
    for k in range(1, 6):
        for _ in range(200):
            c = rng.integers(0, 256, (k, 3))
            # white / black / repeated centres and count ties in a fraction of the cases
            if rng.random() < 0.3:
                c[rng.integers(0, k)] = 255
            if rng.random() < 0.3:
                c[rng.integers(0, k)] = 0
            if rng.random() < 0.2 and k > 1:
                c[1] = c[0]
            n = rng.integers(0, 4, k) if rng.random() < 0.5 else rng.integers(0, 10**6, k)
            out.append((c, n))
    out += [(np.array([[255, 255, 255]]), np.array([7])), (np.array([[0, 0, 0], [255, 255, 255]]), np.array([3, 3])),
            (np.array([[200, 200, 200]]), np.array([1])), (np.array([[10, 10, 10]] * 5), np.array([1, 2, 3, 4, 5]))]
    return out


def test_c_palette_equals_python_rules():
    for c, n in _cases():
        want = ColorExtractor._palette(c, n)
        got = _c_palette(c, n)
        assert got == (want.primary, want.background, want.accent), (c.tolist(), n.tolist())


@pytest.mark.parametrize("args", [("#0a141e", "#FFFFFF", ["#28323c"] * 3), ("#000000", "#000000", ["#000000"] * 3),
                                  ("#ffee00", "#000000", ["#010203", "#a0b0c0", "#a0b0c0"])])
def test_direct_colorfeatures_equal_validated(args):
    a, b = palette_features(*args), _validated(*args)
    assert a == b and a.model_dump() == b.model_dump() and a.model_dump_json() == b.model_dump_json()
    assert type(a) is type(b)


def test_assemble_batch_matches_per_record_rules():
    """pipeline.assemble_batch (the serving loop's batch assembly: dispatch resolved once per
    batch) builds, per record and in `features` order, what the reference's per-feature calls
    return -- from the C-made palette / shadow level when present, else by the Python rules;
    unknown feature names are skipped, as assemble() always did."""
    from low_level_feature_extraction_amd.backend import ImageFeatures
    from low_level_feature_extraction_amd.models import FeatureType
    from low_level_feature_extraction_amd.pipeline import assemble, assemble_batch, shadow_level

    cen = np.array([[10, 20, 30], [200, 210, 220], [255, 255, 255]], np.uint8)
    cnt = np.array([5, 9, 1], np.int64)
    shapes = [{"type": "rectangle", "x": 1, "y": 2, "width": 3, "height": 4, "border_radius": 0.0, "area": 12.0}]
    made = ImageFeatures(cen, cnt, 15, 1.0, 800, 10, shapes, 1, 64, 32,
                         palette=("#c8d2dc", "#000000", ["#0a141e", "#0a141e", "#0a141e"]), shadow_level="Moderate")
    bare = ImageFeatures(cen, cnt, 15, 1.0, 800, 10, shapes, 1, 64, 32)
    feats = ["shadows", FeatureType.COLORS if hasattr(FeatureType, "COLORS") else "colors", "shapes", "text"]
    out = assemble_batch([made, bare], feats)
    assert [list(o) for o in out] == [["shadows", "colors", "shapes"]] * 2
    assert out[0]["shadows"] == {"shadow_level": "Moderate"}
    assert out[1]["shadows"] == {"shadow_level": shadow_level(800, 10)}
    assert out[0]["colors"] == out[1]["colors"] == ColorExtractor._palette(cen, cnt)
    assert out[0]["shapes"] == {"shapes": shapes, "total_shapes": 1, "metadata": {"image_width": 64, "image_height": 32}}
    assert out[0]["shapes"]["shapes"] is not shapes  # a new list per result, as analyze_shapes returns
    assert assemble(made, feats) == out[0]
