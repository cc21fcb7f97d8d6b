"""GPU tests for the round-3 hardening items (VERDICT r2 "next" #6).

* 64-bit row offsets in the row-streaming stencil: a 4 GiB+ image (h*w*3 > 2^32) whose
  rows repeat with period 64 gives, past the 2^31- and 2^32-byte marks, the class rows
  the oracle computes for the same pattern (Canny classes are a function of a 9-row
  window, so interior rows repeat too).
* BGRA input to ShapeAnalyzer / ShadowAnalyzer equals the BGR result, as
  cvtColor(BGR2GRAY) ignores alpha (shape pyc @L18, shadow pyc @L8).
* process_images with a stride-0 (broadcast) torch tensor reads each row once.
* Backend stage calls from a second thread beside batches keep their results (the
  context lock).
"""
import threading

import numpy as np
import pytest

from low_level_feature_extraction_amd import synth

pytestmark = pytest.mark.gpu

PERIOD = 64


def test_stencil_rows_past_4gib(backend, orc):
    import torch

    w = 4096
    reps = -(-(1 << 32) // (3 * w * PERIOD)) + 1  # h * w * 3 > 2^32 with a period to spare
    h = reps * PERIOD
    assert h * w * 3 > (1 << 32) and h * w < (1 << 31)
    pat = synth.synth_numpy(0, PERIOD, w, seed=17)
    exp3 = orc.canny_nms(orc.blur5(orc.bgr2gray(np.concatenate([pat] * 3, 0))))
    mid = exp3[PERIOD:2 * PERIOD]  # interior rows of the periodic image
    assert np.any(mid != 1), "pattern has no Canny candidates"
    big = torch.from_numpy(pat).cuda().repeat(reps, 1, 1)[None]
    got = backend.edge_classes(big)
    del big
    for byte_mark in (1 << 31, 1 << 32):
        y0 = (byte_mark // (3 * w)) // PERIOD * PERIOD  # the period holding the mark
        rows = got[0, y0:y0 + PERIOD].cpu().numpy()
        assert np.array_equal(rows, mid), f"rows {y0}..{y0 + PERIOD} differ past byte {byte_mark}"
    top = got[0, :PERIOD].cpu().numpy()
    assert np.array_equal(top[8:], exp3[8:PERIOD])  # the first period away from the top border
    del got
    torch.cuda.empty_cache()


def test_analyzers_accept_bgra(orc):
    from low_level_feature_extraction_amd import ShadowAnalyzer, ShapeAnalyzer

    bgr = synth.synth_numpy(0, 240, 320, seed=21)
    alpha = np.random.default_rng(3).integers(0, 256, (240, 320, 1), dtype=np.uint8)
    bgra = np.concatenate([bgr, alpha], axis=2)
    assert ShapeAnalyzer.analyze_shapes(bgra) == ShapeAnalyzer.analyze_shapes(bgr) == orc.analyze_shapes(bgr)
    assert ShadowAnalyzer.analyze_shadow_level(bgra) == ShadowAnalyzer.analyze_shadow_level(bgr)
    assert np.array_equal(ShapeAnalyzer.preprocess_image(bgra), orc.shape_mask(bgr))
    assert np.array_equal(ShadowAnalyzer.preprocess_image(bgra), orc.blur5(orc.bgr2gray(bgr)))
    for bad in (bgr[:, :, 0], np.zeros((8, 8, 2), np.uint8), bgr.astype(np.float32)):
        with pytest.raises(ValueError):
            ShapeAnalyzer.analyze_shapes(bad)


@pytest.mark.parametrize("device", ["cpu", "cuda"])
def test_process_images_broadcast_rows(backend, orc, device):
    import torch

    row = torch.from_numpy(synth.synth_numpy(1, 1, 300, seed=4)).to(device)  # 1 x W x 3
    bcast = row.expand(50, 300, 3)
    assert bcast.stride(0) == 0
    got = backend.process_images([bcast], ("shapes", "shadows"), seed=1)[0]
    ref_img = np.ascontiguousarray(bcast.cpu().numpy())
    assert (got.shadow_sum, got.shadow_count) == orc.shadow_stats(ref_img)
    assert got.shapes == orc.analyze_shapes(ref_img)["shapes"]


def test_stage_calls_beside_batches(backend, orc):
    """text_binary / gray_blur5 from a second thread while the main thread runs batches
    on the same context: every result equals its serial value."""
    imgs = np.stack([synth.synth_numpy(i, 180, 240, seed=9) for i in range(6)])
    small = synth.synth_numpy(2, 20, 60, seed=9)  # upscaled by text_binary (shares d_rsz_*)
    ref_batch = backend.process(imgs, ("shapes", "shadows"), seed=2)
    ref_text = backend.text_binary(small)[0].cpu().numpy()
    ref_blur = backend.gray_blur5(imgs[:2]).cpu().numpy()
    errors = []
    stop = threading.Event()

    def side():
        try:
            while not stop.is_set():
                t = backend.text_binary(small)[0].cpu().numpy()
                b = backend.gray_blur5(imgs[:2]).cpu().numpy()
                if not (np.array_equal(t, ref_text) and np.array_equal(b, ref_blur)):
                    errors.append("stage result changed")
                    return
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    th = threading.Thread(target=side)
    th.start()
    try:
        for _ in range(6):
            res = backend.process(imgs, ("shapes", "shadows"), seed=2)
            for r, e in zip(res, ref_batch):
                assert r.shapes == e.shapes and (r.shadow_sum, r.shadow_count) == (e.shadow_sum, e.shadow_count)
    finally:
        stop.set()
        th.join(timeout=60)
    assert not errors, errors
