"""Glue for the reference endpoint: one result per requested feature, in order.

``process_feature_results`` (app/services/analyze/utils.py:155-214) zips the requested
features with the results *by position* (:177).  The reference endpoint
(app/api/v1/endpoints/analyze.py:94-111) iterates ``list(FeatureType)`` and ``continue``s
past features it has no extractor for, which would shift every later result onto the
wrong name once shapes / shadows join ``FeatureType``.  ``feature_results`` always
returns exactly one entry per requested feature -- the batched hot-path result, an
extra extractor's result, or the exception that feature raised -- so positional
alignment holds for any feature list.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Mapping, Optional, Sequence, Union

HOT_PATH = ("colors", "shapes", "shadows")


def _name(f) -> str:
    return getattr(f, "value", f)


def feature_results(features: Sequence, batched: Union[Mapping, BaseException, None],
                    extra: Optional[Dict[str, Callable[[], object]]] = None) -> List[object]:
    """``batched``: the dict ``MicroBatcher.analyze`` / ``run_batch`` returned for this
    image (or the exception it raised); ``extra``: zero-argument callables for features
    outside the hot path (e.g. ``{"text": lambda: TextExtractor.extract_text(image)}``).
    Returns one result or exception per feature, in ``features`` order."""
    out: List[object] = []
    for f in features:
        name = _name(f)
        if name in HOT_PATH and isinstance(batched, BaseException):
            out.append(batched)
        elif name in HOT_PATH and batched is not None and name in batched:
            out.append(batched[name])
        elif extra and name in extra:
            try:
                out.append(extra[name]())
            except Exception as e:  # per-feature error, as analyze.py:109-111
                out.append(e)
        else:
            out.append(ValueError(f"feature {name!r} was not computed"))
    return out


async def analyze_features(image, features: Sequence, batcher,
                           extra: Optional[Dict[str, Callable[[], object]]] = None) -> List[object]:
    """The endpoint's feature loop: hot-path features through the micro-batcher (one
    shared GPU launch), the others through ``extra``; positionally aligned."""
    want = [_name(f) for f in features]
    batched: Union[Mapping, BaseException, None] = None
    if any(n in HOT_PATH for n in want):
        try:
            batched = await batcher.analyze(image)
        except Exception as e:
            batched = e
    return feature_results(features, batched, extra)
