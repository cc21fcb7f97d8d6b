"""Batched hot path with reference-shaped results.

``run_batch(images, features)`` groups images by size, runs each group through
``llfe_process_batch`` and assembles, per image, exactly what the reference's
per-image calls return:

* ``colors``  -> ColorFeatures      (ColorExtractor.extract_colors, color_extractor.py:204-300)
* ``shapes``  -> {"shapes", "total_shapes", "metadata"}  (ShapeAnalyzer.analyze_shapes @L184-189)
* ``shadows`` -> {"shadow_level": "Low" | "Moderate" | "High"}  (analyze_shadow_level
  @L21-31; wrapped in a dict because UnifiedAnalysisResponse rejects a bare str)
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence

import numpy as np

from .backend import Backend, feature_mask  # noqa: F401  (feature_mask validates names)
from .color_extractor import ColorExtractor, palette_features


def shadow_level(mask_sum: int, mask_count: int) -> str:
    """shadow pyc @L22-31: empty mask -> Low; avg_darkness = 255 - mean(shadow pixels)."""
    if mask_count == 0:
        return "Low"
    avg_darkness = 255 - np.float64(mask_sum) / np.float64(mask_count)
    if avg_darkness < 30:
        return "Low"
    if avg_darkness < 60:
        return "Moderate"
    return "High"


def shapes_result(r) -> dict:
    return {"shapes": list(r.shapes), "total_shapes": len(r.shapes),
            "metadata": {"image_width": r.width, "image_height": r.height}}


def _colors_result(r):
    p = getattr(r, "palette", None)
    return palette_features(*p) if p else ColorExtractor._palette(r.centers_rgb, r.counts)


def _shadows_result(r):
    lv = getattr(r, "shadow_level", None)
    return {"shadow_level": lv if lv is not None else shadow_level(r.shadow_sum, r.shadow_count)}


_MAKERS = {"colors": _colors_result, "shapes": shapes_result, "shadows": _shadows_result}


def assemble(r, features: Iterable[str]) -> dict:
    """The reference-shaped results of one image.  The palette strings and the shadow level
    come made from libllfe's host half (C, off the GIL; llfe_image_result), so this only
    builds the objects; records without them (none from the batch entry points) take the
    Python rules."""
    return assemble_batch([r], features)[0]


def assemble_batch(recs, features: Iterable[str]) -> list:
    """assemble() over a batch of records, the feature dispatch resolved once."""
    makers = [(f, _MAKERS[f]) for f in (getattr(f, "value", f) for f in features) if f in _MAKERS]
    return [{f: mk(r) for f, mk in makers} for r in recs]


def run_batch(images, features: Sequence[str] = ("colors", "shapes", "shadows"), seed: Optional[int] = None,
              noise=None, backend: Optional[Backend] = None, raw: bool = False, n_colors: int = 5,
              index_base: Optional[int] = None, preprocessing: str = "none") -> List[dict]:
    """images: N x H x W x 3 BGR uint8 array / torch tensor, or a list of H x W x 3
    arrays of any sizes.  Returns one dict per image, in input order.  ``index_base``
    fixes the global index of image 0 (the per-image noise / k-means seeds); by default
    the process counter hands out fresh indices.  ``preprocessing`` (lists only):
    validate_and_preprocess_image's resize mode, applied on the GPU before the features."""
    from . import color_extractor as ce

    be = backend or Backend.get()
    feats = tuple(getattr(f, "value", f) for f in features)
    feature_mask(feats)
    if seed is None:
        seed = ce._SEED
    if isinstance(images, np.ndarray) and images.ndim == 4 or hasattr(images, "data_ptr"):
        n = int(images.shape[0])
        base = ce._next_index(n) if index_base is None else int(index_base)
        res = be.process(images, feats, seed=seed, noise=noise, index_base=base, n_colors=n_colors)
        return res if raw else assemble_batch(res, feats)
    # a list of images of any sizes: one ragged llfe_process_images call (size groups
    # share device passes; every image keeps its own global index)
    imgs = [im if hasattr(im, "data_ptr") else np.asarray(im, np.uint8) for im in images]
    for im in imgs:
        if len(im.shape) != 3 or im.shape[2] != 3:
            raise ValueError(f"expected H x W x 3 BGR uint8 images, got {tuple(im.shape)}")
    base = ce._next_index(len(imgs)) if index_base is None else int(index_base)
    nz = None
    if noise is not None:
        nz = [np.asarray(noise[i], np.int8).reshape(-1, 3) for i in range(len(imgs))]
    res = be.process_images(imgs, feats, seed=seed, noise=nz, index_base=base, n_colors=n_colors,
                            preprocessing=preprocessing)
    out = res if raw else assemble_batch(res, feats)
    return out  # type: ignore[return-value]
