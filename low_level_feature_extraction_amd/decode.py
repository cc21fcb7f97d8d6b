"""Host-side image decoding with cv2.imdecode(buf, IMREAD_COLOR) semantics.

Decoding stays on the host (north star); the reference decodes with OpenCV at
image_processor.py:208-211 and utils.py:108-109.  IMREAD_COLOR yields an 8-bit,
3-channel BGR array: alpha is dropped (not composited), grey and palette images are
expanded, 16-bit samples are scaled by >> 8, and JPEG EXIF orientation is applied.
Pillow (the reference's other imaging dependency) does the byte-level decoding here.
"""
from __future__ import annotations

import io

import numpy as np


class DecodeError(ValueError):
    pass


def decode_bgr(image_bytes: bytes) -> np.ndarray:
    """-> H x W x 3 uint8 BGR, or raises DecodeError (cv2.imdecode returned None)."""
    from PIL import Image, ImageOps, UnidentifiedImageError

    if not image_bytes:
        raise DecodeError("Failed to decode image")
    try:
        im = Image.open(io.BytesIO(image_bytes))
        im.load()
    except (UnidentifiedImageError, OSError, ValueError, SyntaxError) as e:
        raise DecodeError("Failed to decode image") from e
    if im.format == "JPEG":
        im = ImageOps.exif_transpose(im)
    mode = im.mode
    if mode in ("I;16", "I;16B", "I;16L", "I"):
        a = np.asarray(im)
        if a.dtype != np.uint16:
            a = np.clip(a, 0, 65535).astype(np.uint16)
        g = (a >> 8).astype(np.uint8)
        rgb = np.repeat(g[:, :, None], 3, axis=2)
    elif mode == "RGB":
        rgb = np.asarray(im)
    elif mode in ("RGBA", "RGBX", "RGBa"):
        rgb = np.asarray(im)[:, :, :3]
    elif mode in ("L", "1", "P", "PA", "LA", "CMYK", "YCbCr", "HSV", "LAB", "F"):
        if mode == "LA":
            im = im.getchannel("L")
        elif mode == "PA":
            im = im.convert("RGBA")
        rgb = np.asarray(im.convert("RGB"))[:, :, :3]
    else:
        rgb = np.asarray(im.convert("RGB"))
    return np.ascontiguousarray(rgb[:, :, ::-1])
