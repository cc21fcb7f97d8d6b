"""Host-side image decoding with cv2.imdecode(buf, IMREAD_COLOR) semantics.

Decoding stays on the host (north star); the reference decodes with OpenCV at
image_processor.py:208-211 and utils.py:108-109.  IMREAD_COLOR yields an 8-bit,
3-channel BGR array: alpha is dropped (not composited), grey and palette images are
expanded, 16-bit samples are scaled by >> 8, and JPEG EXIF orientation is applied.

PNG and JPEG go through libllfe's native host decoders (``llfe_decode_batch``:
csrc/png_decode.cpp, and csrc/jpeg_decode.cpp over the system libjpeg-turbo with
OpenCV's settings), fanned out over native threads; what they hand back (interlaced
PNG, CMYK JPEG, EXIF-rotated JPEG, other formats) is decoded with Pillow.  Images
above ``MAX_PIXELS`` (cv2's CV_IO_MAX_IMAGE_PIXELS, 2^30) fail like cv2.imdecode does.
"""
from __future__ import annotations

import io
import threading as _threading

import numpy as np


class DecodeError(ValueError):
    pass


_PNG_SIG = b"\x89PNG\r\n\x1a\n"
MAX_PIXELS = 1 << 30  # cv2 CV_IO_MAX_IMAGE_PIXELS (libllfe: LLFE_MAX_PIXELS)
_ERR_CAPACITY = -3


def _is_native(b) -> bool:
    return b[:8] == _PNG_SIG or b[:3] == b"\xff\xd8\xff"


def _native(blobs, h, w, out, threads) -> list:
    """libllfe's host decoders (PNG / JPEG, llfe_decode_batch) over all blobs into
    out[i]; other formats get LLFE_ERR_UNSUPPORTED.  Returns the per-image status list."""
    import ctypes as C

    from . import _lib

    L = _lib.lib()
    n = len(blobs)
    keep = [C.c_char_p(b) if _is_native(b) else None for b in blobs]
    ptrs = (C.c_void_p * n)(*[C.cast(k, C.c_void_p) if k is not None else None for k in keep])
    sizes = (C.c_uint64 * n)(*[len(b) for b in blobs])
    status = (C.c_int32 * n)()
    L.llfe_decode_batch(ptrs, sizes, n, h, w, out.ctypes.data, status, int(threads))
    del keep
    return list(status)


def decoder_info() -> str:
    """Codecs the native decoders run on this host: "png=libdeflate|zlib;jpeg=..."."""
    import ctypes as C

    from . import _lib

    buf = C.create_string_buffer(128)
    _lib.lib().llfe_decoder_info(buf, 128)
    return buf.value.decode()


def _image_size(b):
    """(h, w) of a PNG / JPEG from its header, None for other formats or unreadable
    headers; DecodeError above MAX_PIXELS (cv2.imdecode returns None there)."""
    import ctypes as C

    from . import _lib

    if not _is_native(b):
        return None
    w, h = C.c_int32(), C.c_int32()
    rc = _lib.lib().llfe_image_info(b, len(b), C.byref(w), C.byref(h))
    if rc == _ERR_CAPACITY:
        raise DecodeError(f"Failed to decode image: {w.value}x{h.value} exceeds {MAX_PIXELS} pixels")
    if rc != 0:
        return None
    return h.value, w.value


# Serialises _pillow_open: warnings.catch_warnings saves / restores the process-global
# filter list and the retry below swaps Image.MAX_IMAGE_PIXELS, so two decode threads
# inside it at once could leave either changed.  Image.open only parses the header.
_PIL_OPEN_LOCK = _threading.Lock()


def _pillow_open(Image, image_bytes: bytes):
    """Image.open under cv2.imdecode's size limit (MAX_PIXELS) instead of Pillow's
    decompression-bomb guard (2 x MAX_IMAGE_PIXELS, ~179 MP by default), leaving that
    process-global guard and the warning filters as they were: the warning between the
    two Pillow limits is suppressed locally, and only an image Pillow refuses outright is
    opened again with the limit raised for that one call.  All of it under one lock, so
    concurrent decode threads neither interleave the filter save / restore nor see each
    other's raised limit."""
    import warnings

    with _PIL_OPEN_LOCK, warnings.catch_warnings():
        warnings.simplefilter("ignore", Image.DecompressionBombWarning)
        try:
            return Image.open(io.BytesIO(image_bytes))
        except Image.DecompressionBombError:
            pass
        old = Image.MAX_IMAGE_PIXELS
        Image.MAX_IMAGE_PIXELS = MAX_PIXELS  # (the MAX_PIXELS check of the caller still applies)
        try:
            return Image.open(io.BytesIO(image_bytes))
        finally:
            Image.MAX_IMAGE_PIXELS = old


def decode_bgr(image_bytes: bytes) -> np.ndarray:
    """-> H x W x 3 uint8 BGR, or raises DecodeError (cv2.imdecode returned None)."""
    from PIL import Image, ImageOps, UnidentifiedImageError

    if not image_bytes:
        raise DecodeError("Failed to decode image")
    hw = _image_size(image_bytes)
    if hw is not None:  # native PNG / JPEG path; anything it does not take goes through Pillow
        out = np.empty((1, hw[0], hw[1], 3), np.uint8)
        if _native([image_bytes], hw[0], hw[1], out, 1)[0] == 0:
            return out[0]
    # cv2.imdecode accepts up to CV_IO_MAX_IMAGE_PIXELS; Pillow's decompression-bomb
    # check would refuse images above 2 * MAX_IMAGE_PIXELS (~179 MP by default) at open
    try:
        im = _pillow_open(Image, image_bytes)
        if im.width * im.height > MAX_PIXELS:
            raise DecodeError(f"Failed to decode image: {im.width}x{im.height} exceeds {MAX_PIXELS} pixels")
        im.load()
    except (UnidentifiedImageError, OSError, ValueError, SyntaxError, Image.DecompressionBombError) as e:
        if isinstance(e, DecodeError):
            raise
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


# ---------------------------------------------------------------------------- batches
# at ~10k 1080p images/s per node the host decode, not the GPU, is
# the end-to-end bound, so decoding fans out over a thread pool (Pillow's codecs release
# the GIL) and writes straight into the NHWC batch that goes to the device.
_POOL = None
_POOL_LOCK = _threading.Lock()


def usable_cores() -> int:
    """CPUs this process may run on (affinity mask, capped by a cgroup v2 cpu.max quota)."""
    import os

    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def default_decode_threads() -> int:
    """The rank's share of the host cores: the set placement.bind() pinned it to
    (LLFE_RANK_CPUS), else usable cores / LOCAL_WORLD_SIZE (one process per GPU shares the
    node's cores); LLFE_DECODE_THREADS overrides."""
    import os

    env = os.environ.get("LLFE_DECODE_THREADS")
    if env and int(env) > 0:
        return int(env)
    rank_cpus = os.environ.get("LLFE_RANK_CPUS")
    if rank_cpus and int(rank_cpus) > 0:
        return min(int(rank_cpus), 64)
    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
    return max(1, min(usable_cores() // local, 64))


def _pool(workers=None):
    global _POOL
    from concurrent.futures import ThreadPoolExecutor

    with _POOL_LOCK:
        want = workers or default_decode_threads()
        if _POOL is None or _POOL._max_workers != want:
            if _POOL is not None:
                _POOL.shutdown(wait=False)
            _POOL = ThreadPoolExecutor(max_workers=want, thread_name_prefix="llfe-decode")
        return _POOL


def decode_many(blobs, workers=None) -> list:
    """decode_bgr over a thread pool; returns arrays or DecodeError instances, in order."""

    def one(b):
        try:
            return decode_bgr(b)
        except DecodeError as e:
            return e

    return list(_pool(workers).map(one, blobs))


def decode_batch(blobs, out=None, workers=None) -> np.ndarray:
    """Decode equally sized images into one N x H x W x 3 BGR uint8 batch (``out`` if
    given, e.g. a pinned host tensor's numpy view).  Raises DecodeError naming the first
    image that fails or whose size differs from the first image's."""
    blobs = [bytes(b) for b in blobs]
    if not blobs:
        raise DecodeError("empty batch")
    hw = _image_size(blobs[0])
    first = None if hw is not None else decode_bgr(blobs[0])
    h, w = hw if hw is not None else first.shape[:2]
    if out is None:
        out = np.empty((len(blobs), h, w, 3), np.uint8)
    if out.shape != (len(blobs), h, w, 3) or out.dtype != np.uint8 or not out.flags.c_contiguous:
        raise ValueError(f"out must be a C-contiguous {(len(blobs), h, w, 3)} uint8 array, got {out.shape} {out.dtype}")
    todo = list(range(len(blobs)))
    if hw is not None:  # PNG / JPEG batch: native decoders, Pillow for whatever they leave
        st = _native(blobs, h, w, out, workers or default_decode_threads())
        todo = [i for i, s_ in enumerate(st) if s_ != 0]
    else:
        out[0] = first
        todo = todo[1:]

    def one(i):
        try:
            im = decode_bgr(blobs[i])
        except DecodeError:
            return f"image {i}: Failed to decode image"
        if im.shape[:2] != (h, w):
            return f"image {i}: size {im.shape[1]}x{im.shape[0]} differs from {w}x{h}"
        out[i] = im
        return None

    errs = [e for e in _pool(workers).map(one, todo) if e] if todo else []
    if errs:
        raise DecodeError(errs[0])
    return out
