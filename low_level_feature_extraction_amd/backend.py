"""Device-side entry points over the C ABI (one context per GPU per host thread).

``Backend`` owns an ``llfe_ctx`` for one device and exposes the batch pipeline and the
stage functions with numpy / torch arguments.  Device memory for host inputs is
handled by the library itself (``on_device = 0``); torch tensors already on the GPU are
passed by pointer together with torch's current HIP stream, so no copy is made.

Nothing in this module computes features on the CPU: a missing ``libllfe.so`` or a
missing GPU raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L

FEATURE_BITS = {"colors": L.FEATURE_COLORS, "shapes": L.FEATURE_SHAPES, "shadows": L.FEATURE_SHADOWS}


SHADOW_LEVELS = ("Low", "Moderate", "High")  # llfe_image_result.shadow_level 0 / 1 / 2


def feature_mask(features) -> int:
    m = 0
    for f in features:
        f = getattr(f, "value", f)
        if f not in FEATURE_BITS:
            raise ValueError(f"unknown feature {f!r}")
        m |= FEATURE_BITS[f]
    return m


@dataclass
class ImageFeatures:
    """Per-image output of the batched hot path (pre-assembly)."""

    centers_rgb: np.ndarray  # (K, 3) uint8, k-means order
    counts: np.ndarray       # (K,) unique colours per centre
    n_unique: int
    compactness: float
    shadow_sum: int
    shadow_count: int
    shapes: list = field(default_factory=list)
    n_contours: int = 0
    width: int = 0
    height: int = 0
    # made in C on the host half of collect / process (llfe_image_result): extract_colors'
    # palette (primary, background, [3 accents]) and analyze_shadow_level's level
    palette: tuple | None = None
    shadow_level: str | None = None


def _torch():
    import torch

    return torch


def _is_torch(x) -> bool:
    try:
        import torch
    except ImportError:  # pragma: no cover
        return False
    return isinstance(x, torch.Tensor)


def text_size(h: int, w: int):
    """Output (height, width) of TextExtractor.preprocess_image (llfe_text_size)."""
    oh, ow = C.c_int32(0), C.c_int32(0)
    if L.lib().llfe_text_size(int(h), int(w), C.byref(oh), C.byref(ow)) < 0:
        raise ValueError(f"text_size: invalid {h}x{w}")
    return oh.value, ow.value


class Backend:
    _instances: dict = {}
    _ilock = threading.Lock()

    def __init__(self, device: int | None = None):
        if device is None:
            device = int(os.environ.get("LLFE_DEVICE", os.environ.get("LOCAL_RANK", "0")))
        self.device = device
        # PyTorch-ROCm ships its own HIP runtime (torch/lib/libamdhip64.so) beside the
        # /opt/rocm one libllfe links: torch's must initialise first, or its later
        # lazy init finds "no HIP GPUs" once libllfe holds the device
        try:
            import torch

            if torch.cuda.is_available():
                torch.cuda.init()
        except ImportError:  # pragma: no cover
            pass
        self._lib = L.lib()
        ctx = C.c_void_p()
        rc = self._lib.llfe_init(device, C.byref(ctx))
        if rc != L.LLFE_OK:
            raise L.LlfeError(rc, f"llfe_init(device={device}) failed (no HIP device available?)")
        self.ctx = ctx
        self._lock = threading.RLock()  # (re-entered by submit -> _call)

    @classmethod
    def get(cls, device: int | None = None) -> "Backend":
        if device is None:
            device = int(os.environ.get("LLFE_DEVICE", os.environ.get("LOCAL_RANK", "0")))
        key = (device, threading.get_ident())
        with cls._ilock:
            b = cls._instances.get(key)
            if b is None:
                b = cls._instances[key] = Backend(device)
            return b

    @classmethod
    def release(cls, backend: "Backend"):
        """Drop a thread's cached context (``get``) and free its device workspaces -- for a
        thread that is about to end, e.g. MicroBatcher's worker at close()."""
        with cls._ilock:
            for key, b in list(cls._instances.items()):
                if b is backend:
                    del cls._instances[key]
        backend.close()

    def close(self):
        if self.ctx:
            with self._lock:
                self._lib.llfe_destroy(self.ctx)
                self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ profiling
    def set_profiling(self, enable: bool):
        self._call("llfe_set_profiling", int(bool(enable)))

    def set_concurrency(self, enable: bool):
        """Colour path on a second stream beside shapes / shadows (default) or all kernels
        in order on one stream (isolated kernel timings)."""
        self._call("llfe_set_concurrency", int(bool(enable)))

    def set_contour_mode(self, mode: str):
        """"host" (default): findContours + shape geometry on the host pool while the GPU
        runs k-means; "gpu": on the GPU (contours_gpu.hip).  Identical results."""
        self._call("llfe_set_contour_mode", CONTOUR_MODES[mode])

    @property
    def inflight(self) -> int:
        """Batches ``submit`` keeps in flight (2 or 3; llfe_set_inflight)."""
        return self._call("llfe_get_inflight")

    @inflight.setter
    def inflight(self, depth: int):
        self._call("llfe_set_inflight", int(depth))

    def contour_mode(self) -> str:
        m = self._call("llfe_get_contour_mode")
        return {v: k for k, v in CONTOUR_MODES.items()}[m]

    def kernel_stats(self) -> dict:
        """{kernel: {"launches", "total_ms", "bytes"}} accumulated while profiling."""
        arr = (L.LlfeKernelStat * 64)()
        n = self._call("llfe_kernel_stats", arr, 64)
        return {arr[i].name.decode(): {"launches": int(arr[i].launches), "total_ms": float(arr[i].total_ms),
                                       "bytes": float(arr[i].bytes)} for i in range(min(n, 64))}

    def host_contour_stats(self, reset: bool = False) -> dict:
        """Host contour pool: busy wall ms, images traced and threads since the last reset."""
        ms, imgs, th = C.c_double(0), C.c_int64(0), C.c_int32(0)
        self._call("llfe_host_contour_stats", C.byref(ms), C.byref(imgs), C.byref(th), int(reset))
        return {"busy_ms": ms.value, "images": int(imgs.value), "threads": int(th.value)}

    # ------------------------------------------------------------------ helpers
    def _chk(self, rc):
        return L.check(self.ctx, rc)

    def _call(self, fn: str, *args):
        """self._lib.<fn>(ctx, *args) under the context lock, checked.  A ctx is not
        thread-safe (llfe.h): its scratch buffers are shared by every entry point, so a
        stage call from a request thread must not run beside a batch on the
        MicroBatcher thread."""
        with self._lock:
            return self._chk(getattr(self._lib, fn)(self.ctx, *args))

    def _stream(self, t=None):
        if t is not None and _is_torch(t) and t.is_cuda:
            torch = _torch()
            return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
        return C.c_void_p(0)

    @staticmethod
    def _batch_view(images):
        """-> (pointer, n, h, w, on_device, keepalive)"""
        if _is_torch(images):
            t = images
            if t.dtype != _torch().uint8 or t.dim() != 4 or t.shape[-1] != 3:
                raise ValueError(f"expected N x H x W x 3 uint8 tensor, got {tuple(t.shape)} {t.dtype}")
            t = t.contiguous()
            return t.data_ptr(), t.shape[0], t.shape[1], t.shape[2], int(t.is_cuda), t
        a = np.ascontiguousarray(images, dtype=np.uint8)
        if a.ndim == 3:
            a = a[None]
        if a.ndim != 4 or a.shape[-1] != 3:
            raise ValueError(f"expected N x H x W x 3 uint8 array, got {a.shape}")
        return a.ctypes.data, a.shape[0], a.shape[1], a.shape[2], 0, a

    @staticmethod
    def _noise_view(noise, n, h, w):
        if noise is None:
            return None, 0, None
        if _is_torch(noise):
            t = noise.contiguous()
            if t.numel() != n * h * w * 3:
                raise ValueError("noise must hold N*H*W*3 int8 values")
            return t.data_ptr(), int(t.is_cuda), t
        a = np.ascontiguousarray(noise, dtype=np.int8)
        if a.size != n * h * w * 3:
            raise ValueError("noise must hold N*H*W*3 int8 values")
        return a.ctypes.data, 0, a

    # ------------------------------------------------------------------ hot path
    def process(self, images, features=("colors", "shapes", "shadows"), seed: int = 0, noise=None,
                index_base: int = 0, n_colors: int = 5) -> list:
        """Run the batched hot path. ``images``: N x H x W x 3 BGR uint8 (numpy host
        array or torch tensor, host or GPU).  Returns a list of ImageFeatures."""
        ptr, n, h, w, on_dev, keep = self._batch_view(images)
        nptr, n_on_dev, nkeep = self._noise_view(noise, n, h, w)
        mask = feature_mask(features)
        b = L.LlfeBatch(C.c_void_p(ptr), n, h, w, on_dev, C.c_void_p(nptr) if nptr else None, n_on_dev,
                        int(n_colors), index_base)
        results = (L.LlfeImageResult * max(n, 1))()
        cap = max(64 * n, 64)
        needed = C.c_int64(0)
        stream = self._stream(keep)
        with self._lock:
            while True:
                shapes = (L.LlfeShape * cap)()
                rc = self._lib.llfe_process_batch(self.ctx, C.byref(b), mask, C.c_uint64(seed & (2**64 - 1)), results,
                                                  shapes, cap, C.byref(needed), stream)
                if rc == L.LLFE_ERR_CAPACITY and needed.value > cap:
                    cap = int(needed.value)
                    continue
                self._chk(rc)
                break
        out = self._convert(results, shapes, n, mask, w, h)
        del keep, nkeep
        return out

    def process_images(self, images, features=("colors", "shapes", "shadows"), seed: int = 0, noise=None,
                       index_base: int = 0, n_colors: int = 5, preprocessing: str = "none") -> list:
        """Ragged batch through llfe_process_images: ``images`` is a list of H x W x 3 BGR
        uint8 images of any sizes -- numpy arrays (host) or torch tensors (host or GPU;
        rows may be strided, pixels must be packed) -- with validate_and_preprocess_image's
        resize rule (``preprocessing``: none / auto / high_quality / performance; other
        names do not resize, as in utils.py:116-143) applied on the GPU first.  Image i
        keeps global index index_base + i.  ``noise``: one parity-noise array per image of
        its preprocessed size, or None.  Returns ImageFeatures in input order."""
        n = len(images)
        mode = PRE_MODES.get(preprocessing, 0)
        descs = (L.LlfeImageDesc * max(n, 1))()
        keep, sizes = [], []
        for i, im in enumerate(images):
            if _is_torch(im):
                t = im
                if t.dtype != _torch().uint8 or t.dim() != 3 or t.shape[2] != 3:
                    raise ValueError(f"image {i}: expected H x W x 3 uint8, got {tuple(t.shape)} {t.dtype}")
                if t.stride(2) != 1 or t.stride(1) != 3 or t.stride(0) < 3 * t.shape[1]:
                    t = t.contiguous()  # pixels not packed, or rows overlap (stride 0): one copy
                ptr, h, w, stride, dev = t.data_ptr(), t.shape[0], t.shape[1], t.stride(0), int(t.is_cuda)
            else:
                t = np.asarray(im)
                if t.dtype != np.uint8 or t.ndim != 3 or t.shape[2] != 3:
                    raise ValueError(f"image {i}: expected H x W x 3 uint8, got {t.shape} {t.dtype}")
                if t.strides[2] != 1 or t.strides[1] != 3 or t.strides[0] < 3 * t.shape[1]:
                    t = np.ascontiguousarray(t)
                ptr, h, w, stride, dev = t.ctypes.data, t.shape[0], t.shape[1], t.strides[0], 0
            keep.append(t)
            descs[i].data, descs[i].height, descs[i].width = ptr, h, w
            descs[i].row_stride, descs[i].on_device = stride, dev
            plan = preprocess_size(w, h, preprocessing)
            oh, ow = (plan[1], plan[0]) if plan else (h, w)
            sizes.append((ow, oh))
            if noise is not None:
                nptr, n_on_dev, nk = self._noise_view(noise[i], 1, oh, ow)
                keep.append(nk)
                descs[i].noise, descs[i].noise_on_device = nptr, n_on_dev
        mask = feature_mask(features)
        results = (L.LlfeImageResult * max(n, 1))()
        cap = max(64 * n, 64)
        needed = C.c_int64(0)
        stream = self._stream(next((t for t in keep if _is_torch(t) and t.is_cuda), None))
        with self._lock:
            while True:
                shapes = (L.LlfeShape * cap)()
                rc = self._lib.llfe_process_images(self.ctx, descs, n, mask, mode, int(n_colors),
                                                   C.c_uint64(seed & (2**64 - 1)), index_base, results, shapes, cap,
                                                   C.byref(needed), stream)
                if rc == L.LLFE_ERR_CAPACITY and needed.value > cap:
                    cap = int(needed.value)
                    continue
                self._chk(rc)
                break
        out = self._convert(results, shapes, n, mask, [sz[0] for sz in sizes], [sz[1] for sz in sizes])
        del keep
        return out

    @staticmethod
    def _convert(results, shapes, n, mask, w, h) -> list:
        # bulk conversion through numpy views of the ctypes arrays (per-field ctypes
        # access would cost ~20 us per image while the GPU waits for the next batch)
        R = np.ctypeslib.as_array(results)[:n]
        ncol = R["n_colors"].tolist()
        cen = R["centers_rgb"].copy()
        cnt = R["counts"].astype(np.int64)
        nu, comp = R["n_unique"].tolist(), R["compactness"].tolist()
        ssum, scnt = R["shadow_sum"].tolist(), R["shadow_count"].tolist()
        off, nsh, ncont = R["shape_offset"].tolist(), R["n_shapes"].tolist(), R["n_contours"].tolist()
        pal = [None] * n
        if mask & L.FEATURE_COLORS and n:
            def strs(f, shape):  # char[8] fields (numpy: 8 x S1) -> NUL-stripped bytes
                return np.ascontiguousarray(R[f]).view("S8").reshape(shape).tolist()

            pr, bg, ac = strs("primary", n), strs("background", n), strs("accent", (n, 3))
            pal = [(p.decode(), b.decode(), [a[0].decode(), a[1].decode(), a[2].decode()])
                   for p, b, a in zip(pr, bg, ac)]
        lv = [None] * n
        if mask & L.FEATURE_SHADOWS and n:
            lv = [SHADOW_LEVELS[v] for v in R["shadow_level"].tolist()]
        recs = []
        if mask & L.FEATURE_SHAPES and n:
            tot = max(o + c for o, c in zip(off, nsh))
            S = np.ctypeslib.as_array(shapes)[:tot]
            names = L.SHAPE_TYPES
            recs = [{"type": names[t], "x": x, "y": y, "width": ww, "height": hh, "border_radius": br, "area": ar}
                    for t, x, y, ww, hh, br, ar in zip(S["type"].tolist(), S["x"].tolist(), S["y"].tolist(),
                                                       S["width"].tolist(), S["height"].tolist(),
                                                       S["border_radius"].tolist(), S["area"].tolist())]
        ws = w if isinstance(w, list) else [w] * n
        hs = h if isinstance(h, list) else [h] * n
        out = [ImageFeatures(cen[i, :ncol[i]], cnt[i, :ncol[i]], nu[i], comp[i], ssum[i], scnt[i],
                             recs[off[i]:off[i] + nsh[i]] if recs else [], ncont[i], ws[i], hs[i], pal[i], lv[i])
               for i in range(n)]
        return out

    # ------------------------------------------------------------------ async batches
    def submit(self, images, features=("colors", "shapes", "shadows"), seed: int = 0, noise=None,
               index_base: int = 0, n_colors: int = 5) -> int:
        """Enqueue one batch (llfe_submit_batch) and return its ticket; at most
        ``inflight`` (default 2) in flight.  Results: ``collect(ticket)``, in submission order."""
        ptr, n, h, w, on_dev, keep = self._batch_view(images)
        nptr, n_on_dev, nkeep = self._noise_view(noise, n, h, w)
        mask = feature_mask(features)
        b = L.LlfeBatch(C.c_void_p(ptr), n, h, w, on_dev, C.c_void_p(nptr) if nptr else None, n_on_dev,
                        int(n_colors), index_base)
        ticket = C.c_int64(0)
        self._call("llfe_submit_batch", C.byref(b), mask, C.c_uint64(seed & (2**64 - 1)), self._stream(keep),
                   C.byref(ticket))
        if not hasattr(self, "_inflight"):
            self._inflight = {}
        self._inflight[ticket.value] = (n, h, w, mask, keep, nkeep, b)  # inputs stay alive
        return ticket.value

    _DESC_DTYPE = None

    def batch_capacity(self, h: int, w: int) -> int:
        """Images of h x w one ``submit`` / ``submit_images`` launch takes."""
        return L.check(self.ctx, self._lib.llfe_batch_capacity(int(h), int(w)))

    def submit_images(self, images, features=("colors", "shapes", "shadows"), seed: int = 0, indices=None,
                      n_colors: int = 5) -> int:
        """llfe_submit_images: n separately allocated H x W x 3 BGR uint8 images of one size
        (torch tensors on the device, or host arrays; rows may be strided, pixels packed),
        gathered into one launch, image i under global index ``indices[i]``.  Same ticket /
        ``collect`` / in-flight rules as ``submit``; the images must stay alive until then
        (the backend holds references)."""
        n = len(images)
        if n < 1:
            raise ValueError("submit_images needs at least one image")
        if Backend._DESC_DTYPE is None:
            Backend._DESC_DTYPE = np.dtype(L.LlfeImageDesc)
        descs = np.zeros(n, Backend._DESC_DTYPE)
        keep = []
        ptr, hh, ww, st, dev = [], [], [], [], []
        u8 = None
        for i, im in enumerate(images):
            if _is_torch(im):
                # (few attribute calls per image: at serving rates this loop holds the GIL
                # once per request; a strided tensor is packed by one copy)
                if u8 is None:
                    u8 = _torch().uint8
                shp = im.shape
                if len(shp) != 3 or shp[2] != 3 or im.dtype != u8:
                    raise ValueError(f"image {i}: expected H x W x 3 uint8, got {tuple(shp)} {im.dtype}")
                t = im if im.is_contiguous() else im.contiguous()
                ptr.append(t.data_ptr())
                st.append(3 * shp[1])
                dev.append(1 if t.is_cuda else 0)
                hh.append(shp[0])
                ww.append(shp[1])
                keep.append(t)
            else:
                t = np.asarray(im)
                if t.dtype != np.uint8 or t.ndim != 3 or t.shape[2] != 3:
                    raise ValueError(f"image {i}: expected H x W x 3 uint8, got {t.shape} {t.dtype}")
                if t.strides[2] != 1 or t.strides[1] != 3 or t.strides[0] < 3 * t.shape[1]:
                    t = np.ascontiguousarray(t)
                ptr.append(t.ctypes.data)
                st.append(t.strides[0])
                dev.append(0)
                hh.append(t.shape[0])
                ww.append(t.shape[1])
                keep.append(t)
        descs["data"], descs["height"], descs["width"] = ptr, hh, ww
        descs["row_stride"], descs["on_device"] = st, dev
        idx = np.ascontiguousarray(np.arange(n) if indices is None else indices, dtype=np.int64)
        if idx.shape != (n,):
            raise ValueError("indices must hold one global index per image")
        mask = feature_mask(features)
        ticket = C.c_int64(0)
        stream = self._stream(next((t for t in keep if _is_torch(t) and t.is_cuda), None))
        self._call("llfe_submit_images", descs.ctypes.data, n, mask, int(n_colors), C.c_uint64(seed & (2**64 - 1)),
                   idx.ctypes.data, stream, C.byref(ticket))
        if not hasattr(self, "_inflight"):
            self._inflight = {}
        self._inflight[ticket.value] = (n, hh, ww, mask, keep, idx, descs)
        return ticket.value

    def collect(self, ticket: int) -> list:
        n, h, w, mask, keep, nkeep, b = self._inflight[ticket]
        results = (L.LlfeImageResult * max(n, 1))()
        cap = max(64 * n, 64)
        needed = C.c_int64(0)
        with self._lock:
            while True:
                shapes = (L.LlfeShape * cap)()
                rc = self._lib.llfe_collect_batch(self.ctx, C.c_int64(ticket), results, shapes, cap, C.byref(needed))
                if rc == L.LLFE_ERR_CAPACITY and needed.value > cap:
                    cap = int(needed.value)
                    continue
                self._chk(rc)
                break
        del self._inflight[ticket]
        return self._convert(results, shapes, n, mask, w, h)

    # ------------------------------------------------------------------ stages (device tensors)
    def _dev_batch(self, images):
        torch = _torch()
        if not _is_torch(images):
            images = torch.from_numpy(np.ascontiguousarray(images, np.uint8))
        if images.dim() == 3:
            images = images[None]
        return images.to(f"cuda:{self.device}").contiguous()

    def gray_blur5(self, images):
        torch = _torch()
        x = self._dev_batch(images)
        n, h, w, _ = x.shape
        out = torch.empty((n, h, w), dtype=torch.uint8, device=x.device)
        self._call("llfe_gray_blur5", x.data_ptr(), out.data_ptr(), n, h, w, self._stream(x))
        return out

    def edge_classes(self, images):
        torch = _torch()
        x = self._dev_batch(images)
        n, h, w, _ = x.shape
        out = torch.empty((n, h, w), dtype=torch.uint8, device=x.device)
        self._call("llfe_edge_classes", x.data_ptr(), out.data_ptr(), n, h, w, self._stream(x))
        return out

    def font_binary(self, images):
        """FontDetector.preprocess_image on the GPU: n x h x w u8 0/255 device tensor."""
        torch = _torch()
        x = self._dev_batch(images)
        n, h, w, _ = x.shape
        out = torch.empty((n, h, w), dtype=torch.uint8, device=x.device)
        self._call("llfe_font_binary", x.data_ptr(), out.data_ptr(), n, h, w, self._stream(x))
        return out

    def text_binary(self, image):
        """TextExtractor.preprocess_image on the GPU (text_extractor.py:15-46): one
        H x W [x C] uint8 image (C = 1, 3 BGR or 4 BGRA) -> (out_h x out_w 0/255 device
        tensor, Otsu threshold)."""
        torch = _torch()
        x = image if _is_torch(image) else torch.from_numpy(np.ascontiguousarray(image, np.uint8))
        x = x.to(f"cuda:{self.device}").contiguous()
        if x.dim() == 2:
            x = x[:, :, None]
        h, w, ch = x.shape
        oh, ow = text_size(h, w)
        out = torch.empty((oh, ow), dtype=torch.uint8, device=x.device)
        t = C.c_int32(0)
        self._call("llfe_text_binary", x.data_ptr(), h, w, ch, out.data_ptr(), C.byref(t),
                                             self._stream(x))
        return out, int(t.value)

    def shape_mask(self, images):
        torch = _torch()
        x = self._dev_batch(images)
        n, h, w, _ = x.shape
        out = torch.empty((n, h, w), dtype=torch.uint8, device=x.device)
        self._call("llfe_shape_mask", x.data_ptr(), out.data_ptr(), n, h, w, self._stream(x))
        return out

    def canny(self, images):
        """Canny(blur5(gray), 50, 150) of the shapes path, before its dilation: n x h x w
        u8 0/255 device tensor."""
        torch = _torch()
        x = self._dev_batch(images)
        n, h, w, _ = x.shape
        out = torch.empty((n, h, w), dtype=torch.uint8, device=x.device)
        self._call("llfe_canny", x.data_ptr(), out.data_ptr(), n, h, w, self._stream(x))
        return out

    def dilate3(self, masks):
        """dilate(masks, ones(3, 3)) of an n x h x w (or h x w) u8 batch on the GPU."""
        torch = _torch()
        x = masks if _is_torch(masks) else torch.from_numpy(np.ascontiguousarray(masks, np.uint8))
        x = x.to(f"cuda:{self.device}").contiguous()
        if x.dim() == 2:
            x = x[None]
        n, h, w = x.shape
        out = torch.empty_like(x)
        self._call("llfe_dilate3", x.data_ptr(), out.data_ptr(), n, h, w, self._stream(x))
        return out

    def find_contours_gpu(self, mask: np.ndarray) -> list:
        """findContours(RETR_EXTERNAL, CHAIN_APPROX_SIMPLE) of one host u8 mask on the GPU
        contour path (the one llfe_process_batch uses) -> list of (n,2) int32, cv2 order."""
        m = np.ascontiguousarray(mask, np.uint8)
        h, w = m.shape
        cap = 1 << 16
        while True:
            pts = np.empty((cap, 2), np.int32)
            offs = np.empty(cap + 1, np.int32)
            need = C.c_int64(0)
            with self._lock:
                nc = self._lib.llfe_find_contours_gpu(self.ctx, m.ctypes.data, h, w, pts.ctypes.data, cap,
                                                      offs.ctypes.data, cap + 1, C.byref(need))
            if nc == L.LLFE_ERR_CAPACITY:
                cap = max(int(need.value), cap * 2)
                continue
            self._chk(min(nc, 0))
            return [pts[offs[i]:offs[i + 1]].copy() for i in range(nc)]

    def shapes_from_masks_gpu(self, masks: np.ndarray):
        """analyze_shapes' records for n host u8 masks (n x h x w) on the GPU contour path
        -> (list of per-image shape dict lists, n_contours np.int32[n])."""
        m = np.ascontiguousarray(masks, np.uint8)
        n, h, w = m.shape
        cap = max(64, 16 * n)
        while True:
            arr = (L.LlfeShape * cap)()
            ns = np.zeros(n, np.int32)
            nc = np.zeros(n, np.int32)
            need = C.c_int64(0)
            with self._lock:
                rc = self._lib.llfe_shapes_from_masks_gpu(self.ctx, m.ctypes.data, n, h, w, arr, cap, ns.ctypes.data,
                                                          nc.ctypes.data, C.byref(need))
            if rc == L.LLFE_ERR_CAPACITY:
                cap = int(need.value)
                continue
            self._chk(rc)
            out, k = [], 0
            for i in range(n):
                out.append([{"type": L.SHAPE_TYPES[s.type], "x": int(s.x), "y": int(s.y), "width": int(s.width),
                             "height": int(s.height), "border_radius": float(s.border_radius),
                             "area": float(s.area)} for s in arr[k:k + ns[i]]])
                k += int(ns[i])
            return out, nc

    def shadow_stats(self, images):
        x = self._dev_batch(images)
        n, h, w, _ = x.shape
        sums = np.zeros(n, np.uint64)
        cnts = np.zeros(n, np.uint64)
        self._call("llfe_shadow_stats", x.data_ptr(), sums.ctypes.data, cnts.ctypes.data, n, h, w,
                                              self._stream(x))
        return sums, cnts

    def color_unique(self, images, seed=0, noise=None, index_base=0):
        """-> (keys device tensor n x h*w int32 view of u32, n_unique np.int64[n])"""
        torch = _torch()
        x = self._dev_batch(images)
        n, h, w, _ = x.shape
        nz = None
        if noise is not None:
            nz = torch.as_tensor(np.ascontiguousarray(noise, np.int8)).to(x.device).contiguous()
        keys = torch.empty((n, h * w), dtype=torch.int32, device=x.device)
        nu = np.zeros(n, np.int64)
        b = L.LlfeBatch(C.c_void_p(x.data_ptr()), n, h, w, 1, C.c_void_p(nz.data_ptr()) if nz is not None else None,
                        1, 0, index_base)
        self._call("llfe_color_unique", C.byref(b), C.c_uint64(seed), keys.data_ptr(),
                                              nu.ctypes.data, self._stream(x))
        return keys, nu

    def kmeans(self, keys, n_points, n_colors=5, seed=0, index_base=0):
        """keys: device int32 tensor (n, stride) of packed RGB keys; n_points np.int64[n]."""
        n = keys.shape[0]
        n_points = np.ascontiguousarray(n_points, np.int64)
        res = (L.LlfeImageResult * max(n, 1))()
        self._call("llfe_kmeans", keys.data_ptr(), keys.shape[1], n_points.ctypes.data, n, n_colors,
                                        C.c_uint64(seed), index_base, res, self._stream(keys))
        out = []
        for i in range(n):
            r = res[i]
            k = r.n_colors
            centers = np.array([[r.centers_rgb[j][c] for c in range(3)] for j in range(k)], np.uint8).reshape(-1, 3)
            out.append((centers, np.array([r.counts[j] for j in range(k)], np.int64), float(r.compactness)))
        return out

    def kmeans_attempts(self, n):
        """Diagnostics (llfe_kmeans_attempts): the 10 k-means attempts of each of the first n
        images of the last process() chunk -> list of n lists of dicts (pp_centers, centers
        float32 K x 3 before the uint8 truncation, counts, iters, compactness)."""
        out = (L.LlfeKmeansAttempt * max(n * 10, 1))()
        self._call("llfe_kmeans_attempts", n, out)
        recs = []
        for i in range(n):
            row = []
            for a in range(10):
                r = out[i * 10 + a]
                row.append({"pp_centers": np.array([[r.pp_centers[k][j] for j in range(3)] for k in range(5)], np.float32),
                            "centers": np.array([[r.centers[k][j] for j in range(3)] for k in range(5)], np.float32),
                            "counts": np.array(list(r.counts), np.int64), "iters": int(r.iters),
                            "compactness": float(r.compactness)})
            recs.append(row)
        return recs

    def resize_lanczos_pil(self, image, out_w, out_h, box=None):
        """Pillow LANCZOS resize of one H x W x C uint8 image (torch GPU tensor or numpy)."""
        torch = _torch()
        x = image if _is_torch(image) else torch.from_numpy(np.ascontiguousarray(image, np.uint8))
        x = x.to(f"cuda:{self.device}").contiguous()
        if x.dim() == 2:
            x = x[:, :, None]
        h, w, ch = x.shape
        out = torch.empty((out_h, out_w, ch), dtype=torch.uint8, device=x.device)
        bx = None
        if box is not None:
            bx = (C.c_double * 4)(*[float(v) for v in box])
        self._call("llfe_resize_lanczos_pil", x.data_ptr(), h, w, ch, out.data_ptr(), out_h, out_w,
                                                    bx, self._stream(x))
        return out


    def reduce_pil(self, image, fx, fy):
        torch = _torch()
        x = image if _is_torch(image) else torch.from_numpy(np.ascontiguousarray(image, np.uint8))
        x = x.to(f"cuda:{self.device}").contiguous()
        if x.dim() == 2:
            x = x[:, :, None]
        h, w, ch = x.shape
        out = torch.empty(((h + fy - 1) // fy, (w + fx - 1) // fx, ch), dtype=torch.uint8, device=x.device)
        self._call("llfe_reduce_pil", x.data_ptr(), h, w, ch, fx, fy, out.data_ptr(),
                                            self._stream(x))
        return out

    def resize_cv(self, image, out_w, out_h, interpolation):
        """cv2.resize(image, (out_w, out_h), interpolation) of one H x W [x C] uint8 image
        (validate_and_preprocess_image, utils.py:118-143); interpolation is an OpenCV
        code or one of "linear" / "area" / "lanczos4"."""
        torch = _torch()
        code = CV_INTER[interpolation] if isinstance(interpolation, str) else int(interpolation)
        x = image if _is_torch(image) else torch.from_numpy(np.ascontiguousarray(image, np.uint8))
        x = x.to(f"cuda:{self.device}").contiguous()
        squeeze = x.dim() == 2
        if squeeze:
            x = x[:, :, None]
        h, w, ch = x.shape
        out = torch.empty((out_h, out_w, ch), dtype=torch.uint8, device=x.device)
        self._call("llfe_resize_cv", x.data_ptr(), h, w, ch, out.data_ptr(), out_h, out_w, code,
                                           self._stream(x))
        return out[:, :, 0] if squeeze else out

    def thumbnail_pil(self, image, max_w=1920, max_h=1080):
        """PIL thumbnail((max_w, max_h), LANCZOS) of one H x W x C uint8 image."""
        torch = _torch()
        x = image if _is_torch(image) else torch.from_numpy(np.ascontiguousarray(image, np.uint8))
        x = x.to(f"cuda:{self.device}").contiguous()
        squeeze = x.dim() == 2
        if squeeze:
            x = x[:, :, None]
        h, w, ch = x.shape
        out = torch.empty(h * w * ch, dtype=torch.uint8, device=x.device)
        oh, ow = C.c_int32(0), C.c_int32(0)
        self._call("llfe_thumbnail_pil", x.data_ptr(), h, w, ch, max_w, max_h, out.data_ptr(),
                                               out.numel(), C.byref(oh), C.byref(ow), self._stream(x))
        out = out[: oh.value * ow.value * ch].view(oh.value, ow.value, ch)
        return out[:, :, 0] if squeeze else out

    def thumbnail_pil_batch(self, images, max_w=1920, max_h=1080):
        """PIL thumbnail((max_w, max_h), LANCZOS) of N same-size H x W x 3 uint8 images
        (N x H x W x 3 array / tensor) in one llfe_thumbnail_pil_batch call."""
        torch = _torch()
        x = images if _is_torch(images) else torch.from_numpy(np.ascontiguousarray(images, np.uint8))
        x = x.to(f"cuda:{self.device}").contiguous()
        n, h, w, ch = x.shape
        plan = thumbnail_size(w, h, max_w, max_h)
        ow, oh = plan if plan else (w, h)
        out = torch.empty((n, oh, ow, ch), dtype=torch.uint8, device=x.device)
        ro, co = C.c_int32(0), C.c_int32(0)
        self._call("llfe_thumbnail_pil_batch", x.data_ptr(), n, h, w, ch, max_w, max_h, out.data_ptr(),
                                                     out.numel(), C.byref(ro), C.byref(co), self._stream(x))
        assert (ro.value, co.value) == (oh, ow)
        return out


# "gpu_force_fallback": diagnostic GPU mode whose chunks all take the host fallback
CONTOUR_MODES = {"host": 0, "gpu": 1, "gpu_force_fallback": 2}
CV_INTER = {"linear": 1, "cubic": 2, "area": 3, "lanczos4": 4}
PRE_MODES = {"none": 0, "auto": 1, "high_quality": 2, "performance": 3}
_INTER_NAME = {1: "INTER_LINEAR", 3: "INTER_AREA", 4: "INTER_LANCZOS4"}


def preprocess_size(w, h, mode):
    """validate_and_preprocess_image's size rule (utils.py:118-143) through the ABI:
    -> (new_w, new_h, interpolation code) or None when the mode does not resize."""
    if mode not in PRE_MODES:
        return None
    ow, oh, it = C.c_int32(0), C.c_int32(0), C.c_int32(0)
    rc = L.lib().llfe_preprocess_size(w, h, PRE_MODES[mode], C.byref(ow), C.byref(oh), C.byref(it))
    if rc < 0:
        raise L.LlfeError(rc, "invalid preprocessing geometry")
    return (ow.value, oh.value, it.value) if rc == 1 else None


def thumbnail_size(w, h, max_w=1920, max_h=1080):
    """-> (new_w, new_h) or None when PIL's thumbnail would not resize."""
    ow, oh = C.c_int32(0), C.c_int32(0)
    rc = L.lib().llfe_thumbnail_size(w, h, max_w, max_h, C.byref(ow), C.byref(oh))
    if rc < 0:
        raise L.LlfeError(rc, "invalid thumbnail geometry")
    return (ow.value, oh.value) if rc == 1 else None


# ---------------------------------------------------------------------- host-only geometry
def find_contours(mask: np.ndarray) -> list:
    """findContours(mask, RETR_EXTERNAL, CHAIN_APPROX_SIMPLE) -> list of (n,2) int32."""
    lib = L.lib()
    m = np.ascontiguousarray(mask, np.uint8)
    h, w = m.shape
    cap = 1 << 16
    while True:
        pts = np.empty((cap, 2), np.int32)
        offs = np.empty(cap + 1, np.int32)
        need = C.c_int64(0)
        nc = lib.llfe_find_contours(m.ctypes.data, h, w, pts.ctypes.data, cap, offs.ctypes.data, cap + 1,
                                    C.byref(need))
        if nc == L.LLFE_ERR_CAPACITY:
            cap = max(int(need.value), cap * 2)
            continue
        if nc < 0:
            raise L.LlfeError(nc, "llfe_find_contours failed")
        return [pts[offs[i]:offs[i + 1]].copy() for i in range(nc)]


def _contour_xy(contour) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(contour).reshape(-1, 2), np.int32)


def border_radius(contour, epsilon_factor=0.02) -> float:
    p = _contour_xy(contour)
    return float(L.lib().llfe_border_radius(p.ctypes.data, len(p), epsilon_factor))


def classify_contour(contour):
    p = _contour_xy(contour)
    s = L.LlfeShape()
    rc = L.lib().llfe_classify_contour(p.ctypes.data, len(p), C.byref(s))
    if rc < 0:
        raise L.LlfeError(rc, "llfe_classify_contour failed")
    if rc == 0:
        return None
    return {"type": L.SHAPE_TYPES[s.type], "x": int(s.x), "y": int(s.y), "width": int(s.width),
            "height": int(s.height), "border_radius": float(s.border_radius), "area": float(s.area)}


def shapes_from_mask(mask: np.ndarray) -> list:
    lib = L.lib()
    m = np.ascontiguousarray(mask, np.uint8)
    h, w = m.shape
    cap = 1024
    while True:
        arr = (L.LlfeShape * cap)()
        nc = C.c_int32(0)
        n = lib.llfe_shapes_from_mask(m.ctypes.data, h, w, arr, cap, C.byref(nc))
        if n == L.LLFE_ERR_CAPACITY:
            cap *= 4
            continue
        if n < 0:
            raise L.LlfeError(n, "llfe_shapes_from_mask failed")
        return [{"type": L.SHAPE_TYPES[s.type], "x": int(s.x), "y": int(s.y), "width": int(s.width),
                 "height": int(s.height), "border_radius": float(s.border_radius), "area": float(s.area)}
                for s in arr[:n]]
