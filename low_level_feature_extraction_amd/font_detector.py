"""Drop-in FontDetector (app/services/analyze/font_detector.py:8-171), SURVEY.md §8f row 4.

preprocess_image -- cvtColor(BGR2GRAY) + adaptiveThreshold(GAUSSIAN_C, THRESH_BINARY_INV,
11, 2) (:17-37) -- runs on the GPU (llfe_font_binary: the stencil kernel with the CV_32F
11x11 Gaussian mean over the gray image, bit-exact vs the oracle).  Region detection
(findContours RETR_EXTERNAL + boundingRect + the aspect / height filter, :40-67) runs on
the host contour code of the shapes path; the remaining heuristics (:69-171) are the
reference's, restated: font size = int(0.75 h), weight from the region's mean gray,
family "Arial", confidence 0.8, and ``detect_font`` returns None when no region is found
or on any error.
"""
from __future__ import annotations

import logging
from typing import List, Optional, Tuple

import numpy as np

from .models import FontFeatures

logger = logging.getLogger(__name__)


def _gray(bgr: np.ndarray) -> np.ndarray:
    """cvtColor(BGR2GRAY) 8U: (1868 B + 9617 G + 4899 R + 2^13) >> 14 (exact integers)."""
    b = bgr.astype(np.uint32)
    return ((b[..., 0] * 1868 + b[..., 1] * 9617 + b[..., 2] * 4899 + 8192) >> 14).astype(np.uint8)


class FontDetector:
    COMMON_FONTS = [
        "Arial", "Helvetica", "Roboto", "Open Sans", "Lato",
        "Montserrat", "Times New Roman", "Georgia", "Courier New",
        "Verdana", "Tahoma", "Trebuchet MS", "Impact",
    ]

    @staticmethod
    def preprocess_image(image: np.ndarray) -> np.ndarray:
        """H x W x 3 BGR u8 -> H x W u8 binary (255 = darker than the local mean - 2)."""
        from .backend import Backend

        img = np.ascontiguousarray(image, np.uint8)
        return Backend.get().font_binary(img[None]).cpu().numpy()[0]

    @staticmethod
    def preprocess_batch(images) -> np.ndarray:
        """N x H x W x 3 batch (numpy or device tensor) -> N x H x W binaries (host)."""
        from .backend import Backend

        return Backend.get().font_binary(images).cpu().numpy()

    @staticmethod
    def detect_text_regions(image: np.ndarray) -> List[Tuple[int, int, int, int]]:
        """Bounding boxes of the external contours with 0.1 < w/h < 15 and h > 8, in
        findContours order (font_detector.py:39-67)."""
        from .backend import find_contours

        regions = []
        for c in find_contours(np.ascontiguousarray(image, np.uint8)):
            x0, y0 = c.min(axis=0)
            x1, y1 = c.max(axis=0)
            x, y, w, h = int(x0), int(y0), int(x1 - x0 + 1), int(y1 - y0 + 1)
            aspect_ratio = w / float(h)
            if 0.1 < aspect_ratio < 15 and h > 8:
                regions.append((x, y, w, h))
        return regions

    @staticmethod
    def estimate_font_size(region_height: int) -> int:
        return int(region_height * 0.75)

    @staticmethod
    def estimate_font_weight(region: np.ndarray) -> str:
        if len(region.shape) > 2:
            region = _gray(region)
        avg_intensity = np.mean(region)
        if avg_intensity >= 250:
            return "Light"
        elif avg_intensity > 190:
            return "Regular"
        return "Bold"

    @staticmethod
    def identify_font_family(region: np.ndarray) -> str:
        return "Arial"  # the reference's placeholder (font_detector.py:160-171)

    @classmethod
    def _from_binary(cls, image: np.ndarray, binary: np.ndarray) -> Optional[FontFeatures]:
        text_regions = cls.detect_text_regions(binary)
        if not text_regions:
            return None
        x, y, w, h = max(text_regions, key=lambda r: r[2] * r[3])
        text_region = image[y:y + h, x:x + w]
        return FontFeatures(font_family=cls.identify_font_family(text_region),
                            font_size=float(cls.estimate_font_size(h)),
                            font_style=cls.estimate_font_weight(text_region), confidence=0.8)

    @classmethod
    def detect_font(cls, image: np.ndarray) -> Optional[FontFeatures]:
        try:
            return cls._from_binary(image, cls.preprocess_image(image))
        except Exception as e:
            logging.error(f"Error in font detection: {str(e)}")
            return None

    @classmethod
    def detect_font_batch(cls, images) -> list:
        """detect_font over an N x H x W x 3 batch with one GPU launch."""
        imgs = np.ascontiguousarray(np.asarray(images), np.uint8)
        try:
            binaries = cls.preprocess_batch(imgs)
        except Exception as e:
            logging.error(f"Error in font detection: {str(e)}")
            return [None] * len(imgs)
        out = []
        for img, b in zip(imgs, binaries):
            try:
                out.append(cls._from_binary(img, b))
            except Exception as e:
                logging.error(f"Error in font detection: {str(e)}")
                out.append(None)
        return out
