"""Drop-in ShadowAnalyzer (app/services/__pycache__/shadow_analyzer.cpython-312.pyc,
SURVEY.md Appendix A) on the MI355X backend.

* ``preprocess_image`` (@L5-10): gray + GaussianBlur 5x5 on the GPU.
* ``analyze_shadow_level`` (@L12-31): adaptiveThreshold(GAUSSIAN_C, 11, 2, INV) and the
  masked sum / count are fused into the stencil kernel; the Low / Moderate / High
  decision on 255 - mean is made on the host exactly as in the reference.
"""
from __future__ import annotations

from typing import List

import numpy as np

from .shape_analyzer import _bgr


class ShadowAnalyzer:
    @staticmethod
    def preprocess_image(image) -> np.ndarray:
        from .backend import Backend

        return Backend.get().gray_blur5(_bgr(image)[None]).cpu().numpy()[0]

    @staticmethod
    def analyze_shadow_level(image) -> str:
        from .pipeline import run_batch

        return run_batch([_bgr(image)], ("shadows",))[0]["shadows"]["shadow_level"]

    @staticmethod
    def analyze_shadow_level_batch(images) -> List[str]:
        from .pipeline import run_batch

        return [r["shadows"]["shadow_level"] for r in run_batch(images, ("shadows",))]
