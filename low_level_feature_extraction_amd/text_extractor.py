"""Drop-in TextExtractor preprocessing (app/services/analyze/text_extractor.py:15-46),
SURVEY.md §8f row 4.

``preprocess_image`` -- cvtColor(BGR2GRAY), the INTER_CUBIC upscale of small images
(h < 30 or w < 100: scale max(2, 300 / w, 100 / h)), Otsu THRESH_BINARY and the
``mean > 127`` inversion -- runs on the GPU (``llfe_text_binary``: text.hip and the
cubic mode of cvresize.hip), bit-exact vs the oracle's restatement of OpenCV
(oracle/llfe_oracle.c ``orc_text_binary``).  OCR itself (``extract_text``'s
pytesseract calls, :48-205) is not on the accelerated path: a maintainer keeps the
reference's ``extract_text`` and binds its ``cls.preprocess_image`` to this one
(INTEGRATION.md).
"""
from __future__ import annotations

from typing import Iterable, List

import numpy as np


class TextExtractor:
    @classmethod
    def preprocess_image(cls, image) -> np.ndarray:
        """H x W x 3 BGR (or H x W gray, or H x W x 4 BGRA) uint8 -> binary uint8 image,
        black text on white (text_extractor.py:15-46)."""
        from .backend import Backend

        img = image if hasattr(image, "data_ptr") else np.ascontiguousarray(image, np.uint8)
        out, _ = Backend.get().text_binary(img)
        return out.cpu().numpy()

    @classmethod
    def preprocess_images(cls, images: Iterable) -> List[np.ndarray]:
        """preprocess_image over a list of images of any sizes (one context, in order)."""
        return [cls.preprocess_image(im) for im in images]

    @staticmethod
    def otsu_threshold(image) -> int:
        """The threshold cv2.threshold(gray, 0, 255, THRESH_BINARY + THRESH_OTSU) picks
        for the (upscaled) gray image of preprocess_image."""
        from .backend import Backend

        img = image if hasattr(image, "data_ptr") else np.ascontiguousarray(image, np.uint8)
        return Backend.get().text_binary(img)[1]
