"""Drop-in ColorExtractor (app/services/analyze/color_extractor.py) on the MI355X backend.

Call signatures and result semantics are those of the reference:

* ``extract_colors(image, n_colors=5) -> ColorFeatures`` (:203-300) never raises; on
  any error it returns the default palette with ``metadata.success = False``.
* ``_process_image`` (:74-171) keeps the reference's input normalisation, including
  its quirks (CHW guess for images <= 4 px tall, 100x100 black default on failure).
* The native work -- BGR->RGB, int8(N(0, 0.5)) noise, ``np.unique(axis=0)``,
  ``cv2.kmeans`` -- runs on the GPU through libllfe (colour bitmap + 10-attempt k-means);
  palette assembly (:231-284) is host Python, as in the reference.

The reference draws its noise from the process-global NumPy RNG and its k-means seeds
from OpenCV's process-global ``theRNG()``, so repeated calls differ.  Here every call
takes a fresh global image index (``index_base``) under a process seed
(``LLFE_SEED``, default random), which gives the same run-to-run behaviour; pass
``seed=`` to the batch API for reproducible results.
"""
from __future__ import annotations

import itertools
import os
import threading
from typing import List, Optional, Union

import numpy as np

from ._lib import MAX_COLORS
from .models import ColorFeatures

try:
    from PIL import Image
except ImportError:  # pragma: no cover
    Image = None

_SEED = int(os.environ.get("LLFE_SEED", str(int.from_bytes(os.urandom(8), "little"))))
_COUNTER = itertools.count()
_CLOCK = threading.Lock()


def _next_index(n: int = 1) -> int:
    """Reserve ``n`` consecutive global image indices; returns the first."""
    global _COUNTER
    with _CLOCK:
        first = next(_COUNTER)
        if n > 1:
            _COUNTER = itertools.count(first + n)
    return first


def _backend():
    from .backend import Backend

    return Backend.get()


class ColorPalette(ColorFeatures):
    """Legacy palette type of the reference module (color_extractor.py:16-35), kept so
    ``from ...color_extractor import ColorPalette`` still resolves after the import swap:
    a ColorFeatures with a schema example and nothing else."""

    model_config = {"json_schema_extra": {"example": {
        "primary": "#1a73e8", "background": "#f8f9fa", "accent": ["#0d47a1", "#64b5f6"],
        "metadata": {"success": True, "timestamp": 0.0, "processing_time": 0.0}}}}


def _md():
    return {"success": True, "timestamp": 0.0, "processing_time": 0.0}


def _validated(primary, background, accent) -> ColorFeatures:
    return ColorFeatures(primary=primary, background=background, accent=accent, metadata=_md())


def _direct(primary, background, accent) -> ColorFeatures:
    # what model_construct does for this model, without its per-field bookkeeping (1.3 vs
    # 4.7 us per image here): libllfe's palette rules only produce '#rrggbb' strings, so the
    # validators (pattern, accent list) have nothing to reject
    o = ColorFeatures.__new__(ColorFeatures)
    object.__setattr__(o, "__dict__", {"primary": primary, "background": background, "accent": accent,
                                       "metadata": _md()})
    # (its own set: pydantic may add names to one instance's fields_set)
    object.__setattr__(o, "__pydantic_fields_set__", set(_FIELDS))
    object.__setattr__(o, "__pydantic_extra__", None)
    object.__setattr__(o, "__pydantic_private__", None)
    return o


_FIELDS = {"primary", "background", "accent", "metadata"}
_TRUSTED = None


def palette_features(primary: str, background: str, accent: list) -> ColorFeatures:
    """ColorFeatures from a palette libllfe made in C (llfe_image_result.primary / background
    / accent: the rules of color_extractor.py:231-284).  Built directly when that gives an
    instance equal to the validated model (checked once per process: ==, model_dump, JSON);
    otherwise through the validators."""
    global _TRUSTED
    if _TRUSTED is None:
        try:
            a, b = _validated("#0a141e", "#FFFFFF", ["#28323c", "#28323c", "#28323c"]), \
                _direct("#0a141e", "#FFFFFF", ["#28323c", "#28323c", "#28323c"])
            _TRUSTED = _direct if (a == b and a.model_dump() == b.model_dump()
                                   and a.model_dump_json() == b.model_dump_json()) else _validated
        except Exception:  # a model this shortcut does not fit (another pydantic major)
            _TRUSTED = _validated
    return _TRUSTED(primary, background, accent)


class ColorExtractor:
    # ------------------------------------------------------------ helpers (:39-71)
    @staticmethod
    def rgb_to_hex(rgb: tuple) -> str:
        return "#{:02x}{:02x}{:02x}".format(rgb[0], rgb[1], rgb[2])

    @staticmethod
    def hex_to_rgb(hex_color: str) -> tuple:
        hex_color = hex_color.lstrip("#")
        return tuple(int(hex_color[i:i + 2], 16) for i in (0, 2, 4))

    @staticmethod
    def get_contrast_ratio(color1: str, color2: str) -> float:
        def lum(c: str) -> float:
            r, g, b = (int(c[i:i + 2], 16) / 255.0 for i in (1, 3, 5) if len(c) >= 6)
            r = r / 12.92 if r <= 0.03928 else ((r + 0.055) / 1.055) ** 2.4
            g = g / 12.92 if g <= 0.03928 else ((g + 0.055) / 1.055) ** 2.4
            b = b / 12.92 if b <= 0.03928 else ((b + 0.055) / 1.055) ** 2.4
            return 0.2126 * r + 0.7152 * g + 0.0722 * b

        l1, l2 = lum(color1), lum(color2)
        hi, lo = (l1, l2) if l1 > l2 else (l2, l1)
        return (hi + 0.05) / (lo + 0.05)

    @staticmethod
    def is_light_color(rgb: tuple) -> bool:
        r, g, b = [x / 255.0 for x in rgb]
        return 0.2126 * r + 0.7152 * g + 0.0722 * b > 0.6

    # ------------------------------------------------------------ input normalisation
    @staticmethod
    def _process_image(image) -> np.ndarray:
        """-> H x W x 3 uint8 RGB (reference :74-171)."""
        default = np.zeros((100, 100, 3), dtype=np.uint8)
        if image is None:
            return default
        if Image is not None and isinstance(image, Image.Image):
            try:
                arr = np.array(image)
                if arr.size == 0:
                    return default
                if image.mode == "RGBA":
                    bg = Image.new("RGB", image.size, (255, 255, 255))
                    bg.paste(image, mask=image.split()[3])
                    arr = np.array(bg)
                elif image.mode != "RGB":
                    arr = np.array(image.convert("RGB"))
                return arr.astype(np.uint8)
            except Exception:
                return default
        if isinstance(image, np.ndarray):
            try:
                if image.size == 0:
                    return default
                img = image.copy()
                if img.ndim == 0:
                    return default
                if img.ndim == 1:
                    side = int(np.sqrt(len(img) / 3))
                    if side * side * 3 == len(img):
                        img = img.reshape((side, side, 3))
                    else:
                        return default
                # cv2.cvtColor accepts 8U / 16U / 32F only; anything else raises -> default
                cvt_ok = img.dtype in (np.uint8, np.uint16, np.float32)
                if img.ndim == 2:
                    if not cvt_ok:
                        return default
                    img = np.repeat(img[:, :, None], 3, axis=2)          # GRAY2RGB
                elif img.ndim == 3:
                    if img.shape[0] <= 4:
                        img = np.transpose(img, (1, 2, 0))
                    c = img.shape[2]
                    if c in (1, 3, 4) and not cvt_ok:
                        return default
                    if c == 1:
                        img = np.repeat(img, 3, axis=2)                     # GRAY2RGB
                    elif c == 3:
                        img = img[:, :, ::-1]                               # BGR2RGB
                    elif c == 4:
                        img = img[:, :, 2::-1]                              # BGRA2RGB
                    else:
                        img = img[..., :3]
                # ndim >= 4 passes through unconverted, as in the reference
                if img.dtype != np.uint8:
                    if np.issubdtype(img.dtype, np.floating):
                        img = (img * 255).clip(0, 255).astype(np.uint8)
                    else:
                        img = img.astype(np.uint8)
                return np.ascontiguousarray(img)
            except Exception:
                return default
        return default

    # ------------------------------------------------------------ k-means (:174-201)
    @staticmethod
    def _get_dominant_colors(pixels: np.ndarray, n_colors: int, seed: Optional[int] = None) -> tuple:
        """(centers uint8 (K,3), labels) for already-noised RGB rows.  ``labels`` holds
        the per-cluster membership counts as np.repeat(arange(K), counts) -- the only
        use the reference makes of them is np.bincount (:232)."""
        px = np.ascontiguousarray(np.asarray(pixels, np.uint8).reshape(-1, 3))
        bgr = np.ascontiguousarray(px[:, ::-1]).reshape(1, -1, 3)
        zero = np.zeros(bgr.size, np.int8)
        idx = _next_index()
        if not 1 <= int(n_colors) <= MAX_COLORS:
            raise ValueError(f"the MI355X backend supports n_colors in [1, {MAX_COLORS}]")
        r = _backend().process(bgr[None], ("colors",), seed=_SEED if seed is None else seed, noise=zero,
                               index_base=idx, n_colors=int(n_colors))[0]
        centers = r.centers_rgb
        labels = np.repeat(np.arange(len(r.counts)), r.counts)
        return centers, labels

    # ------------------------------------------------------------ palette (:231-284)
    @staticmethod
    def _palette(centers: np.ndarray, counts: np.ndarray) -> ColorFeatures:
        # (plain Python lists: the serving loop assembles 512 of these per step, and
        # per-element NumPy scalars cost ~4x the whole rule set)
        rows = np.asarray(centers, np.uint8).reshape(-1, 3).tolist()
        if len(rows) > 1:
            cnt = np.asarray(counts).reshape(-1).tolist()
            # np.argsort(-counts) (:233-234); stable, equal counts keep k-means order
            rows = [rows[k] for k in sorted(range(len(cnt)), key=lambda k: -cnt[k])]
        hex_colors = ["#%02x%02x%02x" % (c[0], c[1], c[2]) for c in rows]  # rgb_to_hex (:39-41)
        hex_colors = [c for c in hex_colors if c not in ("#ffffff", "#000000")]  # (already lower case)
        md = {"success": True, "timestamp": 0.0, "processing_time": 0.0}
        if not hex_colors:
            bg = "#000000" if ColorExtractor.is_light_color((255, 255, 255)) else "#FFFFFF"
            return ColorFeatures(primary=bg, background=bg, accent=[bg] * 3, metadata=md)
        primary = hex_colors[0]
        accent = [c for c in hex_colors if c != primary][:3]
        while len(accent) < 3:
            accent.append(accent[-1] if accent else primary)
        bg = "#FFFFFF" if not ColorExtractor.is_light_color(ColorExtractor.hex_to_rgb(primary)) else "#000000"
        return ColorFeatures(primary=primary, background=bg, accent=accent[:3], metadata=md)

    @staticmethod
    def _error(e: Exception) -> ColorFeatures:
        return ColorFeatures(primary="#000000", background="#FFFFFF", accent=["#666666", "#999999", "#CCCCCC"],
                             metadata={"success": False, "error": str(e), "timestamp": 0.0, "processing_time": 0.0})

    # ------------------------------------------------------------ public API
    @staticmethod
    def extract_colors(image: Union[np.ndarray, "Image.Image"], n_colors: int = 5) -> ColorFeatures:
        try:
            rgb = ColorExtractor._process_image(image)
            pixels = rgb.reshape(-1, 3)  # raises for sizes not divisible by 3, as at :221
            if rgb.ndim == 3 and rgb.shape[2] == 3:
                bgr = np.ascontiguousarray(rgb[:, :, ::-1])
            else:  # odd layouts the reference flattens anyway: one row of pixels
                bgr = np.ascontiguousarray(pixels[:, ::-1]).reshape(1, -1, 3)
            k = int(n_colors)
            if k <= 1:
                return ColorExtractor._unique_palette(bgr)
            if k > MAX_COLORS:
                raise ValueError(f"the MI355X backend supports n_colors <= {MAX_COLORS}")
            r = _backend().process(bgr[None], ("colors",), seed=_SEED, index_base=_next_index(), n_colors=k)[0]
            return palette_features(*r.palette) if r.palette else ColorExtractor._palette(r.centers_rgb, r.counts)
        except Exception as e:  # the reference never raises from extract_colors
            return ColorExtractor._error(e)

    @staticmethod
    def _unique_palette(bgr: np.ndarray) -> ColorFeatures:
        """n_colors <= 1 (:185-186): the reference skips k-means and returns every
        unique colour with labels [0]*U, so the palette is the first unique colours in
        np.unique order (counts [U, 0, ...]; ties kept in order)."""
        keys, nu = _backend().color_unique(bgr[None], seed=_SEED, index_base=_next_index())
        u = int(nu[0])
        head = keys[0, : min(u, 8)].cpu().numpy().astype(np.uint32)
        centers = np.stack([(head >> 16) & 255, (head >> 8) & 255, head & 255], 1).astype(np.uint8)
        counts = np.zeros(len(centers), np.int64)
        if len(counts):
            counts[0] = u
        return ColorExtractor._palette(centers, counts)

    @staticmethod
    def extract_colors_batch(images: List[np.ndarray], n_colors: int = 5, seed: Optional[int] = None,
                             noise=None, index_base: Optional[int] = None) -> List[ColorFeatures]:
        """Batched extract_colors for same-size BGR uint8 images (N x H x W x 3 array or a
        list).  Mixed sizes are grouped; ``noise`` (parity mode) is the per-image
        np.random.normal(0, 0.5, (H*W, 3)).astype(np.int8) stream."""
        from .pipeline import run_batch

        res = run_batch(images, ("colors",), seed=seed, noise=noise, n_colors=n_colors, index_base=index_base)
        return [r["colors"] for r in res]
