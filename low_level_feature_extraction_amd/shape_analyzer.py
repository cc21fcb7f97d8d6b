"""Drop-in ShapeAnalyzer (app/services/__pycache__/shape_analyzer.cpython-312.pyc, whose
behaviour is restated in SURVEY.md Appendix A) on the MI355X backend.

* ``preprocess_image`` (@L6-30): gray -> GaussianBlur 5x5 -> Canny(50,150) -> dilate 3x3
  computed by libllfe's HIP kernels; returns the 0/255 uint8 mask.
* ``detect_border_radius`` (@L32-61) and the ``analyze_shapes`` loop (@L144-181) run in
  libllfe's host C++ (findContours RETR_EXTERNAL / CHAIN_APPROX_SIMPLE, contourArea,
  arcLength, approxPolyDP, convexHull) on the mask copied back bit-packed.
* ``analyze_shapes`` (@L125-189) returns the reference's dict.  cv2 exceptions in the
  reference propagate; here invalid inputs raise ValueError.
"""
from __future__ import annotations

from typing import Any, Dict, List

import numpy as np


def _bgr(image) -> np.ndarray:
    """H x W x 3 BGR uint8 view of the analyzers' input.  cvtColor(BGR2GRAY) (shape pyc
    @L18, shadow pyc @L8) takes 3- or 4-channel input and ignores alpha (a BGRA pixel
    gives the gray value of its B, G, R), so a BGRA image drops its alpha plane here;
    any other shape or dtype raises as cvtColor does."""
    a = np.asarray(image)
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] not in (3, 4):
        raise ValueError(f"ShapeAnalyzer expects an H x W x 3 (BGR) or x 4 (BGRA) uint8 image, got {a.shape} {a.dtype}")
    if a.shape[2] == 4:
        a = a[:, :, :3]
    return np.ascontiguousarray(a)


class ShapeAnalyzer:
    @staticmethod
    def preprocess_image(image) -> np.ndarray:
        from .backend import Backend

        return Backend.get().shape_mask(_bgr(image)[None]).cpu().numpy()[0]

    @staticmethod
    def detect_border_radius(contour, epsilon_factor: float = 0.02) -> float:
        from .backend import border_radius

        return border_radius(contour, epsilon_factor)

    @staticmethod
    def analyze_shapes(image) -> Dict[str, Any]:
        from .pipeline import run_batch

        return run_batch([_bgr(image)], ("shapes",))[0]["shapes"]

    @staticmethod
    def analyze_shapes_batch(images) -> List[Dict[str, Any]]:
        from .pipeline import run_batch

        return [r["shapes"] for r in run_batch(images, ("shapes",))]
