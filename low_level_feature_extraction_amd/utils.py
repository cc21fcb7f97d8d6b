"""Drop-in validate_and_preprocess_image (app/services/analyze/utils.py:90-152).

Decode on the host (cv2.imdecode IMREAD_COLOR semantics, decode.py), then the
mode-dependent downscale of utils.py:118-143:

    none          -> no resize
    auto          -> INTER_AREA     when max(h, w) > 2000
    high_quality  -> INTER_LANCZOS4 when max(h, w) > 4000
    performance   -> INTER_LINEAR   when max(h, w) > 1000

with new_size = (int(w * s), int(h * s)), s = max_dim / max(h, w) (the size rule is
llfe_preprocess_size in the C ABI).  The resize itself runs on the GPU
(llfe_resize_cv: OpenCV's fixed-point / area tables, csrc/cvresize.hip).  No BASELINE
configuration triggers a resize (1920 < 2000, 3840 < 4000).
"""
from __future__ import annotations

import logging
from enum import Enum

import numpy as np

from .decode import DecodeError, decode_bgr

logger = logging.getLogger(__name__)

_LIMITS = {"auto": (2000, "INTER_AREA"), "high_quality": (4000, "INTER_LANCZOS4"),
           "performance": (1000, "INTER_LINEAR")}


class PreprocessingMode(str, Enum):
    NONE = "none"
    AUTO = "auto"
    HIGH_QUALITY = "high_quality"
    PERFORMANCE = "performance"


_CODE = {"INTER_LINEAR": 1, "INTER_AREA": 3, "INTER_LANCZOS4": 4}


def preprocess_size(w: int, h: int, preprocessing: str):
    """-> (new_w, new_h, interpolation name) or None (utils.py:118-143)."""
    from . import backend

    plan = backend.preprocess_size(w, h, preprocessing)
    if plan is None:
        return None
    return plan[0], plan[1], _LIMITS[preprocessing][1]


def preprocess_decoded(image: np.ndarray, preprocessing: str, device: int = 0) -> np.ndarray:
    """The mode resize of utils.py:118-143 on a decoded BGR image (GPU; the HIP
    extension must be present -- there is no CPU fallback)."""
    h, w = image.shape[:2]
    plan = preprocess_size(w, h, preprocessing)
    if plan is None:
        return image
    from .backend import Backend

    out = Backend.get(device).resize_cv(image, plan[0], plan[1], _CODE[plan[2]])
    return out.cpu().numpy()


def _http_exception(status_code: int, detail: str):
    try:
        from fastapi import HTTPException

        return HTTPException(status_code=status_code, detail=detail)
    except ImportError:  # pragma: no cover - fastapi absent
        return ValueError(detail)


async def validate_and_preprocess_image(image_bytes: bytes, request_id: str, preprocessing: str) -> np.ndarray:
    try:
        try:
            image = decode_bgr(image_bytes)
        except DecodeError:
            raise _http_exception(400, "Failed to decode image. The file may be corrupted or in an unsupported format.")
        return preprocess_decoded(image, preprocessing)
    except Exception as e:
        logger.error(f"Error in validate_and_preprocess_image: {str(e)}", exc_info=True)
        raise _http_exception(400, f"Image validation or preprocessing failed: {str(e)}")
