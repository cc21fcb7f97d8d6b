"""The reference-side binding of INTEGRATION.md: every requested feature appears once,
under its own name, in the response built by the reference's positional
``process_feature_results`` (app/services/analyze/utils.py:155-214, restated below;
the reference module itself needs cv2 and is not imported)."""
import asyncio

import numpy as np
import pytest

from low_level_feature_extraction_amd.integration import analyze_features, feature_results
from low_level_feature_extraction_amd.models import FeatureType


def process_feature_results(features_requested, results):
    """utils.py:174-195: zip(features, results) -> features / errors dicts + status."""
    features, errors = {}, {}
    for feature, result in zip(features_requested, results):
        name = feature.value
        if isinstance(result, Exception):
            errors[name] = {"code": type(result).__name__, "message": str(result)}
        else:
            features[name] = result
    status = "success" if not errors else ("failure" if len(errors) == len(features_requested) else "partial")
    return {"status": status, "features": features, "errors": errors}


BATCHED = {"colors": {"primary": "#112233"}, "shapes": {"shapes": [], "total_shapes": 0},
           "shadows": {"shadow_level": "Low"}}


@pytest.mark.parametrize("order", [list(FeatureType), list(reversed(list(FeatureType))),
                                   [FeatureType.SHADOWS, FeatureType.COLORS], [FeatureType.TEXT]])
def test_each_feature_once_under_its_own_name(order):
    extra = {"text": lambda: {"lines": ["hi"]}, "fonts": lambda: {"font_family": "Arial"}}
    res = process_feature_results(order, feature_results(order, BATCHED, extra))
    assert set(res["features"]) == {f.value for f in order} and not res["errors"]
    for f in order:
        if f.value in BATCHED:
            assert res["features"][f.value] is BATCHED[f.value]
    assert res["features"].get("text", {"lines": ["hi"]}) == {"lines": ["hi"]}


def test_errors_stay_on_their_feature():
    order = list(FeatureType)
    boom = RuntimeError("gpu batch failed")

    def bad_text():
        raise ValueError("no tesseract")

    res = process_feature_results(order, feature_results(order, boom, {"text": bad_text,
                                                                       "fonts": lambda: None}))
    assert set(res["errors"]) == {"colors", "shapes", "shadows", "text"}
    assert res["errors"]["colors"]["message"] == "gpu batch failed"
    assert res["errors"]["text"]["code"] == "ValueError"
    assert res["features"] == {"fonts": None} and res["status"] == "partial"
    # a feature nobody computes is an error under its own name, not a silent shift
    res = process_feature_results(order, feature_results(order, BATCHED, None))
    assert set(res["errors"]) == {"text", "fonts"} and set(res["features"]) == {"colors", "shapes", "shadows"}


def test_analyze_features_with_a_stand_in_batcher():
    class Fake:
        async def analyze(self, image):
            return dict(BATCHED)

    order = list(FeatureType)
    out = asyncio.run(analyze_features(np.zeros((4, 4, 3), np.uint8), order, Fake(),
                                       {"text": lambda: {}, "fonts": lambda: None}))
    assert len(out) == len(order)
    res = process_feature_results(order, out)
    assert res["status"] == "success" and res["features"]["shadows"] == {"shadow_level": "Low"}


@pytest.mark.gpu
def test_real_batch_through_the_positional_response(orc):
    from low_level_feature_extraction_amd import synth
    from low_level_feature_extraction_amd.batcher import MicroBatcher
    from low_level_feature_extraction_amd.pipeline import run_batch

    imgs = [synth.synth_numpy(i, 120, 200, seed=12) for i in range(3)]
    order = [FeatureType.TEXT, FeatureType.SHADOWS, FeatureType.FONTS, FeatureType.SHAPES, FeatureType.COLORS]
    with MicroBatcher(max_batch=8, max_wait_ms=20) as mb:
        for im in imgs:
            out = asyncio.run(analyze_features(im, order, mb, {"text": lambda: {"lines": []}}))
            res = process_feature_results(order, out)
            assert set(res["features"]) == {"text", "shadows", "shapes", "colors"}
            assert set(res["errors"]) == {"fonts"}
            assert res["features"]["shapes"]["shapes"] == orc.analyze_shapes(im)["shapes"]
            assert res["features"]["shadows"] == {"shadow_level": orc.analyze_shadow_level(im)}
            assert res["features"]["colors"].metadata["success"] is True
    direct = run_batch(imgs, ("shapes",))
    assert [d["shapes"]["shapes"] for d in direct] == [orc.analyze_shapes(im)["shapes"] for im in imgs]
