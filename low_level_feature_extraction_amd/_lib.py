"""ctypes binding of libllfe.so (the C ABI declared in include/llfe.h).

This is the same binding a non-Python caller would write.  Importing
it never falls back to a CPU implementation: if the shared library is missing or cannot
be loaded, ``lib()`` raises.

One HIP runtime per process.  PyTorch-ROCm ships its own ``libamdhip64.so`` (SONAME
``libamdhip64.so.7``, the name libllfe's DT_NEEDED asks for).  When torch is importable
it is imported *before* libllfe is loaded, so the dynamic linker binds libllfe to the
runtime torch already mapped: torch's device pointers and ``cuda_stream`` handles are
then objects of libllfe's own runtime.  ``lib()`` verifies that exactly one
libamdhip64 is mapped and raises otherwise.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libllfe.so")

LLFE_OK = 0
LLFE_ERR_INVALID = -1
LLFE_ERR_HIP = -2
LLFE_ERR_CAPACITY = -3
LLFE_ERR_OOM = -4
LLFE_ERR_UNSUPPORTED = -5

FEATURE_COLORS = 1
FEATURE_SHAPES = 2
FEATURE_SHADOWS = 4

SHAPE_TYPES = {0: "unknown", 1: "triangle", 2: "rectangle", 3: "circle", 4: "polygon"}


MAX_COLORS = 32  # LLFE_MAX_COLORS (include/llfe.h)


class LlfeBatch(C.Structure):
    _fields_ = [
        ("data", C.c_void_p),
        ("n", C.c_int32),
        ("height", C.c_int32),
        ("width", C.c_int32),
        ("on_device", C.c_int32),
        ("noise", C.c_void_p),
        ("noise_on_device", C.c_int32),
        ("n_colors", C.c_int32),
        ("index_base", C.c_int64),
        ("indices", C.c_void_p),
    ]


class LlfeImageResult(C.Structure):
    _fields_ = [
        ("n_colors", C.c_int32),
        ("counts", C.c_int32 * MAX_COLORS),
        ("centers_rgb", (C.c_uint8 * 3) * MAX_COLORS),
        ("pad_", C.c_uint8 * 4),
        ("n_unique", C.c_int64),
        ("compactness", C.c_double),
        ("shadow_sum", C.c_uint64),
        ("shadow_count", C.c_uint64),
        ("shape_offset", C.c_int64),
        ("n_shapes", C.c_int32),
        ("n_contours", C.c_int32),
        ("primary", C.c_char * 8),
        ("background", C.c_char * 8),
        ("accent", (C.c_char * 8) * 3),
        ("shadow_level", C.c_int32),
        ("pad2_", C.c_int32),
    ]


class LlfeImageDesc(C.Structure):
    _fields_ = [
        ("data", C.c_void_p),
        ("height", C.c_int32),
        ("width", C.c_int32),
        ("row_stride", C.c_int64),
        ("on_device", C.c_int32),
        ("noise_on_device", C.c_int32),
        ("noise", C.c_void_p),
    ]


class LlfeShape(C.Structure):
    _fields_ = [
        ("type", C.c_int32),
        ("x", C.c_int32),
        ("y", C.c_int32),
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("pad_", C.c_int32),
        ("border_radius", C.c_double),
        ("area", C.c_double),
    ]


class LlfeKernelStat(C.Structure):
    _fields_ = [
        ("name", C.c_char * 32),
        ("launches", C.c_int64),
        ("total_ms", C.c_double),
        ("bytes", C.c_double),
    ]


class LlfeKmeansAttempt(C.Structure):
    _fields_ = [
        ("pp_centers", (C.c_float * 3) * 5),
        ("centers", (C.c_float * 3) * 5),
        ("counts", C.c_int32 * 5),
        ("iters", C.c_int32),
        ("compactness", C.c_double),
    ]


# every symbol declared in include/llfe.h, with its ctypes signature
_vp, _i32, _i64, _u32, _u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64
SIGNATURES = {
    "llfe_init": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "llfe_destroy": (C.c_int, [_vp]),
    "llfe_last_error": (C.c_char_p, [_vp]),
    "llfe_abi_version": (C.c_int, []),
    "llfe_hip_runtime": (C.c_char_p, []),
    "llfe_default_host_threads": (C.c_int, []),
    "llfe_set_profiling": (C.c_int, [_vp, C.c_int]),
    "llfe_set_concurrency": (C.c_int, [_vp, C.c_int]),
    "llfe_set_contour_mode": (C.c_int, [_vp, C.c_int]),
    "llfe_get_contour_mode": (C.c_int, [_vp]),
    "llfe_set_inflight": (C.c_int, [_vp, _i32]),
    "llfe_get_inflight": (C.c_int, [_vp]),
    "llfe_submit_batch": (C.c_int, [_vp, C.POINTER(LlfeBatch), _u32, _u64, _vp, C.POINTER(C.c_int64)]),
    "llfe_collect_batch": (C.c_int, [_vp, C.c_int64, _vp, _vp, C.c_int64, C.POINTER(C.c_int64)]),
    "llfe_submit_images": (C.c_int, [_vp, _vp, _i32, _u32, _i32, _u64, _vp, _vp, C.POINTER(C.c_int64)]),
    "llfe_batch_capacity": (C.c_int, [_i32, _i32]),
    "llfe_kernel_stats": (C.c_int, [_vp, C.POINTER(LlfeKernelStat), _i32]),
    "llfe_host_contour_stats": (C.c_int, [_vp, C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_int32), _i32]),
    "llfe_process_batch": (C.c_int, [_vp, C.POINTER(LlfeBatch), _u32, _u64, _vp, _vp, _i64, C.POINTER(C.c_int64), _vp]),
    "llfe_process_images": (C.c_int, [_vp, _vp, _i32, _u32, _i32, _i32, _u64, _i64, _vp, _vp, _i64,
                                      C.POINTER(C.c_int64), _vp]),
    "llfe_gray_blur5": (C.c_int, [_vp, _vp, _vp, _i32, _i32, _i32, _vp]),
    "llfe_shape_mask": (C.c_int, [_vp, _vp, _vp, _i32, _i32, _i32, _vp]),
    "llfe_edge_classes": (C.c_int, [_vp, _vp, _vp, _i32, _i32, _i32, _vp]),
    "llfe_canny": (C.c_int, [_vp, _vp, _vp, _i32, _i32, _i32, _vp]),
    "llfe_dilate3": (C.c_int, [_vp, _vp, _vp, _i32, _i32, _i32, _vp]),
    "llfe_font_binary": (C.c_int, [_vp, _vp, _vp, _i32, _i32, _i32, _vp]),
    "llfe_text_binary": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, C.POINTER(_i32), _vp]),
    "llfe_text_size": (C.c_int, [_i32, _i32, C.POINTER(_i32), C.POINTER(_i32)]),
    "llfe_shadow_stats": (C.c_int, [_vp, _vp, _vp, _vp, _i32, _i32, _i32, _vp]),
    "llfe_color_unique": (C.c_int, [_vp, C.POINTER(LlfeBatch), _u64, _vp, _vp, _vp]),
    "llfe_kmeans": (C.c_int, [_vp, _vp, _i64, _vp, _i32, _i32, _u64, _i64, _vp, _vp]),
    "llfe_kmeans_attempts": (C.c_int, [_vp, _i32, _vp]),
    "llfe_palette_rules": (C.c_int, [_vp, _vp, _i32, _vp]),
    "llfe_resize_lanczos_pil": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _i32, _i32, _vp, _vp]),
    "llfe_reduce_pil": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp]),
    "llfe_thumbnail_size": (C.c_int, [_i32, _i32, _i32, _i32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "llfe_resize_cv": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _i32, _i32, _i32, _vp]),
    "llfe_preprocess_size": (C.c_int, [_i32, _i32, _i32, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                       C.POINTER(C.c_int32)]),
    "llfe_thumbnail_pil": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _i64, C.POINTER(C.c_int32),
                                     C.POINTER(C.c_int32), _vp]),
    "llfe_thumbnail_pil_batch": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i64,
                                           C.POINTER(C.c_int32), C.POINTER(C.c_int32), _vp]),
    "llfe_find_contours":(C.c_int, [_vp, _i32, _i32, _vp, _i64, _vp, _i32, C.POINTER(C.c_int64)]),
    "llfe_border_radius": (C.c_double, [_vp, _i32, C.c_double]),
    "llfe_classify_contour": (C.c_int, [_vp, _i32, C.POINTER(LlfeShape)]),
    "llfe_shapes_from_mask": (C.c_int, [_vp, _i32, _i32, _vp, _i32, C.POINTER(C.c_int32)]),
    "llfe_find_contours_gpu": (C.c_int, [_vp, _vp, _i32, _i32, _vp, _i64, _vp, _i32, C.POINTER(C.c_int64)]),
    "llfe_shapes_from_masks_gpu": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _i64, _vp, _vp,
                                             C.POINTER(C.c_int64)]),
    "llfe_png_info": (C.c_int, [_vp, C.c_uint64, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "llfe_decode_png_batch": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _i32]),
    "llfe_image_info": (C.c_int, [_vp, C.c_uint64, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "llfe_decode_batch": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _i32]),
    "llfe_decoder_info": (C.c_int, [C.c_char_p, _i32]),
}

_lib = None
_lock = threading.Lock()


class LlfeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"llfe error {code}: {msg}")
        self.code = code


def hip_runtimes_mapped() -> list:
    """Distinct libamdhip64 files mapped into this process (from /proc/self/maps)."""
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1] if line.strip() else ""
                if "libamdhip64" in os.path.basename(p):
                    paths.add(os.path.realpath(p))
    except OSError:  # pragma: no cover - non-Linux
        pass
    return sorted(paths)


def lib():
    """Load libllfe.so (building it from source if it is absent or stale), bound to the
    same HIP runtime as PyTorch when torch is importable."""
    global _lib
    with _lock:
        if _lib is None:
            from . import _build

            try:  # torch first: its libamdhip64 becomes the one libllfe binds to
                import torch  # noqa: F401
            except ImportError:  # pragma: no cover - C-only deployments
                pass
            if _build._stale():
                try:
                    _build.build()
                except Exception as e:  # pragma: no cover - surfaced to caller
                    if not os.path.exists(LIB_PATH):
                        raise RuntimeError(f"libllfe.so is missing and could not be built: {e}") from e
            L = C.CDLL(os.environ.get("LLFE_LIB_PATH", LIB_PATH))
            # (tools/debug/identity.sh runs older builds, which lack later entry points)
            old_ok = os.environ.get("LLFE_LIB_PATH") is not None
            for name, (res, args) in SIGNATURES.items():
                if old_ok and not hasattr(L, name):
                    continue
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            rts = hip_runtimes_mapped()
            if len(rts) > 1:
                raise RuntimeError("two HIP runtimes are mapped into this process (%s); libllfe is bound to %s. "
                                   "Import torch before loading libllfe so both share one runtime."
                                   % (", ".join(rts), L.llfe_hip_runtime().decode()))
            _lib = L
    return _lib


def check(ctx, rc):
    if rc < 0:
        msg = lib().llfe_last_error(ctx)
        raise LlfeError(rc, msg.decode() if msg else "")
    return rc
