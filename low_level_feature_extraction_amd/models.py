"""Result schemas used by the drop-in services.

When this package runs inside the reference application, the reference's own
schemas (app/api/v1/models/analyze.py) are used unchanged -- they are the output
contract.  Standalone, equivalent pydantic models with the same fields and the same
hex-colour validation are defined here (FeatureType gains the shapes / shadows members
that the reference's analyzers need).
"""
from __future__ import annotations

import re
from enum import Enum
from typing import Any, Dict, List, Optional

from pydantic import BaseModel, Field, field_validator

_HEX = r"^#(?:[0-9a-fA-F]{3}){1,2}$"

try:  # inside the reference app: use its contract directly
    from app.api.v1.models.analyze import ColorFeatures  # type: ignore  # noqa: F401
except Exception:  # standalone

    class ColorFeatures(BaseModel):
        """Colour palette (same fields / validation as the reference's ColorFeatures,
        app/api/v1/models/analyze.py:157-204)."""

        primary: Optional[str] = Field(None, pattern=_HEX)
        background: Optional[str] = Field(None, pattern=_HEX)
        accent: List[str] = Field(default_factory=list)
        metadata: Dict[str, Any] = Field(default_factory=dict)

        @field_validator("accent")
        @classmethod
        def _accent_hex(cls, v):
            for c in v:
                if not re.match(_HEX, c):
                    raise ValueError(f"Invalid hex color code: {c}")
            return v

        @classmethod
        def from_dict(cls, data: Dict[str, Any]) -> "ColorFeatures":
            md = data.get("metadata", {})
            return cls(primary=data.get("primary"), background=data.get("background"),
                       accent=data.get("accent", []),
                       metadata={"success": md.get("success", True), "timestamp": md.get("timestamp", 0.0),
                                 "processing_time": md.get("processing_time", 0.0)})


try:  # inside the reference app: use its contract directly
    from app.api.v1.models.analyze import FontFeatures  # type: ignore  # noqa: F401
except Exception:  # standalone

    class FontFeatures(BaseModel):
        """Font analysis result (same fields as the reference's FontFeatures,
        app/api/v1/models/analyze.py:207-241)."""

        font_family: Optional[str] = None
        font_size: Optional[float] = None
        font_style: Optional[str] = None
        confidence: Optional[float] = None

        @classmethod
        def from_dict(cls, data: Dict[str, Any]) -> "FontFeatures":
            return cls(font_family=data.get("font_family"), font_size=data.get("font_size"),
                       font_style=data.get("font_style"), confidence=data.get("confidence"))


class FeatureType(str, Enum):
    """FeatureType of app/api/v1/models/analyze.py:6-10 plus the two analyzers that
    exist in the reference only as bytecode (shape / shadow)."""

    COLORS = "colors"
    TEXT = "text"
    FONTS = "fonts"
    SHAPES = "shapes"
    SHADOWS = "shadows"


HOT_PATH_FEATURES = (FeatureType.COLORS, FeatureType.SHAPES, FeatureType.SHADOWS)
