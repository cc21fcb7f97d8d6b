"""Drop-in ImageProcessor.auto_process_image (app/services/analyze/image_processor.py:185-232).

decode (host) -> BGR2RGB -> PIL thumbnail((max_width, max_height), LANCZOS) -> RGB2BGR.
The Lanczos resample (and Pillow's reducing_gap reduce() pre-pass for inputs >= 4x the
target) runs on the GPU through libllfe and is bit-identical to Pillow.  The channel
swaps commute with the per-channel resample, so the GPU works on BGR directly.

The reference's other ImageProcessor helpers (load_image, resize_image, compress_image,
convert_to_webp, lazy_load_image, convert_format) are file/format I/O outside the hot
path and are not part of this backend.
"""
from __future__ import annotations

import logging

import numpy as np

from .decode import DecodeError, decode_bgr

logger = logging.getLogger(__name__)


class ImageProcessor:
    @staticmethod
    def auto_process_image(image_bytes: bytes, max_width: int = 1920, max_height: int = 1080,
                           quality: int = 85) -> np.ndarray:
        """-> H' x W' x 3 uint8 BGR; raises ValueError("Image processing error: ...")."""
        try:
            try:
                image = decode_bgr(image_bytes)
            except DecodeError:
                raise ValueError("Failed to decode image")
            from .backend import Backend, thumbnail_size

            h, w = image.shape[:2]
            if thumbnail_size(w, h, max_width, max_height) is None:
                return image
            return Backend.get().thumbnail_pil(image, max_width, max_height).cpu().numpy()
        except Exception as e:
            logger.error(f"Image processing failed: {str(e)}")
            raise ValueError(f"Image processing error: {str(e)}")

    @staticmethod
    def auto_process_images(images_bytes, max_width: int = 1920, max_height: int = 1080) -> list:
        """Batched auto_process_image: host decode on the decode pool, then one GPU
        thumbnail launch sequence per group of equally sized images
        (llfe_thumbnail_pil_batch).  Returns arrays in input order; an input that fails
        to decode gets the ValueError auto_process_image would raise, in its place."""
        from .backend import Backend, thumbnail_size
        from .decode import decode_many

        decoded = decode_many(list(images_bytes))
        out: list = [None] * len(decoded)
        groups: dict = {}
        for i, im in enumerate(decoded):
            if isinstance(im, Exception):
                out[i] = ValueError("Image processing error: Failed to decode image")
            elif thumbnail_size(im.shape[1], im.shape[0], max_width, max_height) is None:
                out[i] = im
            else:
                groups.setdefault(im.shape, []).append(i)
        be = Backend.get() if groups else None
        for shape, idx in groups.items():
            res = be.thumbnail_pil_batch(np.stack([decoded[i] for i in idx]), max_width, max_height).cpu().numpy()
            for j, i in enumerate(idx):
                out[i] = res[j]
        return out
