"""CPU-side behaviour of the drop-in services (no GPU): input normalisation quirks,
palette assembly, schemas, shadow levels, preprocessing rules, decoding, and that the
compute entry points refuse to run without the HIP backend (no CPU fallback)."""
import asyncio
import io

import numpy as np
import pytest
from PIL import Image

from low_level_feature_extraction_amd import (ColorExtractor, ColorFeatures, FeatureType, PreprocessingMode,
                                              ShadowAnalyzer, ShapeAnalyzer, validate_and_preprocess_image)
from low_level_feature_extraction_amd.decode import DecodeError, decode_bgr
from low_level_feature_extraction_amd.pipeline import shadow_level
from low_level_feature_extraction_amd import _lib as L
from low_level_feature_extraction_amd.utils import preprocess_decoded, preprocess_size

PI = ColorExtractor._process_image


def _no_gpu():
    import torch

    return not torch.cuda.is_available()


# --------------------------------------------------------------------------- _process_image
def test_process_image_defaults():
    d = np.zeros((100, 100, 3), np.uint8)
    for bad in (None, np.zeros((0,), np.uint8), np.array(5, np.uint8), np.arange(10, dtype=np.uint8), "x", 3.0,
                np.zeros((5, 5), np.float64), np.zeros((5, 5), np.int8), np.zeros((6, 6, 3), np.int32)):
        np.testing.assert_array_equal(PI(bad), d)


def test_process_image_layouts():
    r = np.random.default_rng(0)
    bgr = r.integers(0, 256, (10, 12, 3), dtype=np.uint8)
    np.testing.assert_array_equal(PI(bgr), bgr[:, :, ::-1])                       # BGR2RGB
    g = r.integers(0, 256, (10, 12), dtype=np.uint8)
    np.testing.assert_array_equal(PI(g), np.repeat(g[:, :, None], 3, 2))           # GRAY2RGB
    bgra = r.integers(0, 256, (10, 12, 4), dtype=np.uint8)
    np.testing.assert_array_equal(PI(bgra), bgra[:, :, 2::-1])                     # BGRA2RGB, alpha dropped
    flat = bgr.reshape(-1)[: 6 * 6 * 3]
    np.testing.assert_array_equal(PI(flat), flat.reshape(6, 6, 3)[:, :, ::-1])    # square 1-D reshape
    chw = r.integers(0, 256, (3, 10, 12), dtype=np.uint8)                          # <= 4 rows: (C,H,W) guess
    np.testing.assert_array_equal(PI(chw), np.transpose(chw, (1, 2, 0))[:, :, ::-1])
    tall = r.integers(0, 256, (4, 7, 3), dtype=np.uint8)  # a real 4-row BGR image is transposed too
    assert PI(tall).shape == (7, 3, 3)
    many = r.integers(0, 256, (10, 12, 6), dtype=np.uint8)
    np.testing.assert_array_equal(PI(many), many[..., :3])                         # > 4 channels: first 3
    f = r.random((8, 9, 3)).astype(np.float32)
    np.testing.assert_array_equal(PI(f), (f[:, :, ::-1] * 255).clip(0, 255).astype(np.uint8))
    u16 = r.integers(0, 65536, (8, 9, 3), dtype=np.uint16)
    np.testing.assert_array_equal(PI(u16), u16[:, :, ::-1].astype(np.uint8))      # wraps, as astype does
    four_d = np.zeros((2, 5, 6, 3), np.uint8)
    assert PI(four_d).shape == (2, 5, 6, 3)                                        # passes through


def test_process_image_pil():
    rgba = Image.new("RGBA", (4, 3), (10, 20, 30, 0))
    np.testing.assert_array_equal(PI(rgba), np.full((3, 4, 3), 255, np.uint8))    # composited on white
    half = Image.new("RGBA", (2, 2), (0, 0, 0, 255))
    np.testing.assert_array_equal(PI(half), np.zeros((2, 2, 3), np.uint8))
    la = Image.new("L", (5, 4), 77)
    np.testing.assert_array_equal(PI(la), np.full((4, 5, 3), 77, np.uint8))
    rgb = Image.new("RGB", (5, 4), (1, 2, 3))
    assert PI(rgb)[0, 0].tolist() == [1, 2, 3]


# --------------------------------------------------------------------------- palette + schema
def test_palette_matches_oracle_rules(orc):
    r = np.random.default_rng(5)
    for _ in range(200):
        k = int(r.integers(1, 6))
        centers = r.integers(0, 256, (k, 3)).astype(np.uint8)
        if r.random() < 0.3:
            centers[r.integers(0, k)] = (255, 255, 255) if r.random() < 0.5 else (0, 0, 0)
        counts = r.permutation(np.arange(1, k + 1) * 7)
        got = ColorExtractor._palette(centers, counts)
        want = orc.color_palette(centers, counts)
        assert (got.primary, got.background, got.accent) == (want["primary"], want["background"], want["accent"])
        assert got.metadata["success"] is True
    # equal counts (kept in k-means order, np.argsort(kind="stable")), repeated colours,
    # all-white / all-black palettes, zero counts
    for _ in range(300):
        k = int(r.integers(1, 9))
        centers = r.integers(0, 256, (k, 3)).astype(np.uint8)
        for j in range(k):
            u = r.random()
            if u < 0.15:
                centers[j] = (255, 255, 255)
            elif u < 0.3:
                centers[j] = (0, 0, 0)
            elif u < 0.4:
                centers[j] = centers[0]
        counts = r.integers(0, 4, k)
        got = ColorExtractor._palette(centers, counts)
        want = orc.color_palette(centers, counts)
        assert (got.primary, got.background, got.accent) == (want["primary"], want["background"], want["accent"])


def test_helpers():
    assert ColorExtractor.rgb_to_hex((255, 0, 16)) == "#ff0010"
    assert ColorExtractor.hex_to_rgb("#ff0010") == (255, 0, 16)
    assert ColorExtractor.is_light_color((255, 255, 255)) and not ColorExtractor.is_light_color((0, 0, 0))
    assert ColorExtractor.get_contrast_ratio("#000000", "#ffffff") == pytest.approx(21.0)


def test_color_features_schema():
    """Rules read from app/api/v1/models/analyze.py:157-204 (hex pattern on primary /
    background, per-item validator on accent, from_dict keeping three metadata keys)."""
    ok = ColorFeatures(primary="#0a141e", background="#FFF", accent=["#abc", "#ABCDEF"], metadata={})
    assert ok.model_dump()["accent"] == ["#abc", "#ABCDEF"]
    assert ColorFeatures(primary=None, background=None).accent == []
    for bad in ({"primary": "0a141e"}, {"primary": "#0a141"}, {"background": "#GGGGGG"}, {"accent": ["#12"]},
                {"accent": ["#123456", "red"]}, {"accent": ["#1234567"]}):
        with pytest.raises(Exception):
            ColorFeatures(**bad)
    fd = ColorFeatures.from_dict({"primary": "#123", "metadata": {"timestamp": 5.0, "x": 1}})
    assert fd.metadata == {"success": True, "timestamp": 5.0, "processing_time": 0.0}
    assert [f.value for f in FeatureType][:3] == ["colors", "text", "fonts"]


def test_legacy_color_palette_alias():
    """color_extractor.py:16-35: ColorPalette is a ColorFeatures with a schema example."""
    from low_level_feature_extraction_amd import ColorPalette
    from low_level_feature_extraction_amd.color_extractor import ColorPalette as CP

    assert CP is ColorPalette and issubclass(ColorPalette, ColorFeatures)
    p = ColorPalette(primary="#1a73e8", background="#f8f9fa", accent=["#0d47a1"], metadata={"success": True})
    assert p.primary == "#1a73e8" and isinstance(p, ColorFeatures)
    with pytest.raises(Exception):
        ColorPalette(primary="blue")
    assert ColorPalette.model_json_schema()["example"]["primary"] == "#1a73e8"


def test_extract_colors_without_gpu_reports_failure():
    if not _no_gpu():
        pytest.skip("GPU present")
    res = ColorExtractor.extract_colors(np.zeros((8, 8, 3), np.uint8))
    assert res.metadata["success"] is False and res.primary == "#000000"
    assert res.accent == ["#666666", "#999999", "#CCCCCC"]


def test_analyzers_raise_without_gpu():
    if not _no_gpu():
        pytest.skip("GPU present")
    img = np.zeros((16, 16, 3), np.uint8)
    with pytest.raises(Exception):
        ShapeAnalyzer.analyze_shapes(img)
    with pytest.raises(Exception):
        ShadowAnalyzer.analyze_shadow_level(img)


# --------------------------------------------------------------------------- shadows
def test_shadow_level_matches_oracle(orc):
    r = np.random.default_rng(8)
    for _ in range(500):
        c = int(r.integers(0, 50))
        s = int(r.integers(0, 256 * max(c, 1))) if c else 0
        s = min(s, 255 * c)
        assert shadow_level(s, c) == orc.shadow_level_from_stats(s, c)


# --------------------------------------------------------------------------- preprocessing
@pytest.mark.parametrize("wh", [(1920, 1080), (3840, 2160), (2001, 10), (10, 2001), (4001, 3000), (1001, 1001),
                                (999, 999), (12000, 7), (1000, 1000), (2000, 2000)])
@pytest.mark.parametrize("mode", ["none", "auto", "high_quality", "performance", "bogus"])
def test_preprocess_size_matches_oracle(orc, wh, mode):
    got = preprocess_size(*wh, mode)
    want = orc.preprocess_size(*wh, mode)
    if want is None:
        assert got is None
    else:
        assert got[:2] == want[:2] and got[2].lower().endswith(want[2].upper().lower())


def test_preprocess_modes_enum():
    assert [m.value for m in PreprocessingMode] == ["none", "auto", "high_quality", "performance"]
    img = np.zeros((10, 2100, 3), np.uint8)
    assert preprocess_decoded(img, "none") is img
    assert preprocess_decoded(img[:, :2000], "auto") is not None  # no resize needed: no GPU needed
    try:
        import torch

        if torch.cuda.is_available():
            return
    except ImportError:
        pass
    with pytest.raises(L.LlfeError):  # a resize needs the HIP backend: no CPU fallback
        preprocess_decoded(img, "auto")


def _png(arr, mode=None):
    buf = io.BytesIO()
    Image.fromarray(arr, mode).save(buf, format="PNG") if mode else Image.fromarray(arr).save(buf, format="PNG")
    return buf.getvalue()


def test_validate_and_preprocess_image():
    rgb = np.random.default_rng(1).integers(0, 256, (20, 30, 3), dtype=np.uint8)
    out = asyncio.run(validate_and_preprocess_image(_png(rgb), "r1", "auto"))
    np.testing.assert_array_equal(out, rgb[:, :, ::-1])
    from fastapi import HTTPException

    with pytest.raises(HTTPException) as ei:
        asyncio.run(validate_and_preprocess_image(b"not an image", "r2", "auto"))
    assert ei.value.status_code == 400
    big = np.zeros((10, 2100, 3), np.uint8)
    import torch

    if not torch.cuda.is_available():  # the resize runs on the GPU only: fails loudly here
        with pytest.raises(HTTPException) as ei:
            asyncio.run(validate_and_preprocess_image(_png(big), "r3", "auto"))
        assert ei.value.status_code == 400 and "llfe" in ei.value.detail
    assert asyncio.run(validate_and_preprocess_image(_png(big), "r4", "none")).shape == (10, 2100, 3)


# --------------------------------------------------------------------------- decode
def test_decode_bgr_modes():
    r = np.random.default_rng(2)
    rgb = r.integers(0, 256, (9, 11, 3), dtype=np.uint8)
    np.testing.assert_array_equal(decode_bgr(_png(rgb)), rgb[:, :, ::-1])
    rgba = r.integers(0, 256, (9, 11, 4), dtype=np.uint8)
    np.testing.assert_array_equal(decode_bgr(_png(rgba)), rgba[:, :, 2::-1])        # alpha dropped
    g = r.integers(0, 256, (9, 11), dtype=np.uint8)
    np.testing.assert_array_equal(decode_bgr(_png(g)), np.repeat(g[:, :, None], 3, 2))
    g16 = r.integers(0, 65536, (9, 11), dtype=np.uint16)
    buf = io.BytesIO()
    Image.fromarray(g16).save(buf, format="PNG")
    np.testing.assert_array_equal(decode_bgr(buf.getvalue()), np.repeat((g16 >> 8).astype(np.uint8)[:, :, None], 3, 2))
    pal = Image.fromarray(rgb).convert("P", palette=Image.Palette.ADAPTIVE, colors=8)
    buf = io.BytesIO()
    pal.save(buf, format="PNG")
    np.testing.assert_array_equal(decode_bgr(buf.getvalue()), np.asarray(pal.convert("RGB"))[:, :, ::-1])
    for bad in (b"", b"\x89PNG\r\n\x1a\n garbage", b"hello"):
        with pytest.raises(DecodeError):
            decode_bgr(bad)


def test_decode_jpeg_exif_orientation():
    a = np.zeros((8, 16, 3), np.uint8)
    a[:, :8] = 255
    im = Image.fromarray(a)
    exif = Image.Exif()
    exif[0x0112] = 6  # rotate 90 CW on display
    buf = io.BytesIO()
    im.save(buf, format="JPEG", exif=exif, quality=95)
    out = decode_bgr(buf.getvalue())
    assert out.shape == (16, 8, 3)
