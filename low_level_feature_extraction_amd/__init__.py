"""MI355X (gfx950) batched image-feature backend for Kira7dn/Low_Level_Feature_Extraction.

Drop-in replacements for the reference's hot-path services:

    ImageProcessor.auto_process_image   (app/services/analyze/image_processor.py)
    validate_and_preprocess_image       (app/services/analyze/utils.py)
    ColorExtractor.extract_colors       (app/services/analyze/color_extractor.py)
    ShapeAnalyzer.analyze_shapes        (app/services/shape_analyzer)
    ShadowAnalyzer.analyze_shadow_level (app/services/shadow_analyzer)
    FontDetector.detect_font            (app/services/analyze/font_detector.py)

plus batched entry points (``run_batch``, ``*_batch``).  All per-pixel work runs in
libllfe.so (HIP kernels for gfx950, C ABI in include/llfe.h); there is no CPU fallback.
"""
from .color_extractor import ColorExtractor, ColorPalette
from .font_detector import FontDetector
from .image_processor import ImageProcessor
from .models import ColorFeatures, FeatureType, FontFeatures
from .shadow_analyzer import ShadowAnalyzer
from .shape_analyzer import ShapeAnalyzer
from .utils import PreprocessingMode, validate_and_preprocess_image


def run_batch(images, features=("colors", "shapes", "shadows"), seed=None, noise=None):
    from .pipeline import run_batch as _rb

    return _rb(images, features, seed=seed, noise=noise)


__all__ = [
    "ColorExtractor",
    "ColorFeatures",
    "ColorPalette",
    "FeatureType",
    "FontDetector",
    "FontFeatures",
    "ImageProcessor",
    "PreprocessingMode",
    "ShadowAnalyzer",
    "ShapeAnalyzer",
    "run_batch",
    "validate_and_preprocess_image",
]
