"""Request micro-batching (batcher.py) and the host decode pool (decode.py): CPU tests
with a stand-in batch runner; one GPU test through the real backend."""
import asyncio
import io
import threading

import numpy as np
import pytest
from PIL import Image

from low_level_feature_extraction_amd import decode
from low_level_feature_extraction_amd.batcher import MicroBatcher


def _fake_run(calls):
    def run(images, features):
        calls.append(len(images))
        return [{"sum": int(im.sum()), "shape": im.shape, "features": features} for im in images]

    return run


def test_batcher_groups_concurrent_requests_and_keeps_order():
    calls = []
    imgs = [np.full((4 + i % 3, 5, 3), i, np.uint8) for i in range(40)]
    with MicroBatcher(features=("colors",), max_batch=16, max_wait_ms=50, run=_fake_run(calls)) as b:
        futs = [b.submit(im) for im in imgs]
        res = [f.result(timeout=10) for f in futs]
    assert [r["sum"] for r in res] == [int(im.sum()) for im in imgs]
    assert [r["shape"] for r in res] == [im.shape for im in imgs]
    assert sum(calls) == 40 and max(calls) <= 16 and len(calls) < 40


def test_batcher_from_threads_and_asyncio():
    calls = []
    b = MicroBatcher(max_batch=8, max_wait_ms=20, run=_fake_run(calls))
    out = {}

    def worker(i):
        out[i] = b.submit(np.full((3, 3, 3), i, np.uint8)).result(timeout=10)["sum"]

    th = [threading.Thread(target=worker, args=(i,)) for i in range(12)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert out == {i: 27 * i for i in range(12)}

    async def main():
        rs = await asyncio.gather(*[b.analyze(np.full((2, 2, 3), i, np.uint8)) for i in range(5)])
        return [r["sum"] for r in rs]

    assert asyncio.run(main()) == [12 * i for i in range(5)]
    b.close()
    with pytest.raises(RuntimeError):
        b.submit(np.zeros((2, 2, 3), np.uint8))


def test_batcher_propagates_errors_to_every_request():
    def boom(images, features):
        raise ValueError("backend failed")

    with MicroBatcher(max_batch=4, max_wait_ms=20, run=boom) as b:
        futs = [b.submit(np.zeros((2, 2, 3), np.uint8)) for _ in range(3)]
        for f in futs:
            with pytest.raises(ValueError, match="backend failed"):
                f.result(timeout=10)


def test_batcher_rejects_bad_inputs():
    with MicroBatcher(run=_fake_run([])) as b:
        with pytest.raises(ValueError):
            b.submit(np.zeros((4, 4), np.uint8))
    with pytest.raises(ValueError):
        MicroBatcher(max_batch=0, run=_fake_run([]))


def _png(a):
    b = io.BytesIO()
    Image.fromarray(a).save(b, "PNG")
    return b.getvalue()


def test_decode_batch_and_many():
    rng = np.random.default_rng(3)
    rgb = [rng.integers(0, 256, (17, 23, 3), dtype=np.uint8) for _ in range(6)]
    blobs = [_png(a) for a in rgb]
    out = decode.decode_batch(blobs, workers=3)
    assert out.shape == (6, 17, 23, 3)
    for i in range(6):
        np.testing.assert_array_equal(out[i], rgb[i][:, :, ::-1])
    buf = np.zeros((6, 17, 23, 3), np.uint8)
    assert decode.decode_batch(blobs, out=buf, workers=2) is buf
    many = decode.decode_many(blobs + [b"junk"], workers=4)
    assert isinstance(many[-1], decode.DecodeError)
    np.testing.assert_array_equal(many[2], rgb[2][:, :, ::-1])


def test_decode_batch_errors():
    a = np.zeros((8, 8, 3), np.uint8)
    with pytest.raises(decode.DecodeError, match="image 1"):
        decode.decode_batch([_png(a), b"not an image"], workers=2)
    with pytest.raises(decode.DecodeError, match="differs"):
        decode.decode_batch([_png(a), _png(np.zeros((9, 8, 3), np.uint8))], workers=2)
    with pytest.raises(decode.DecodeError):
        decode.decode_batch([])


@pytest.mark.gpu
def test_batcher_on_gpu_matches_run_batch():
    from low_level_feature_extraction_amd import synth
    from low_level_feature_extraction_amd.pipeline import run_batch

    imgs = [synth.synth_numpy(i, 120 + 8 * (i % 2), 200, seed=5) for i in range(10)]
    ref = run_batch(imgs, ("shapes", "shadows"))
    with MicroBatcher(features=("colors", "shapes", "shadows"), max_batch=8, max_wait_ms=20) as b:
        got = [f.result(timeout=60) for f in [b.submit(im) for im in imgs]]
    for r, g in zip(ref, got):
        assert g["shapes"] == r["shapes"] and g["shadows"] == r["shadows"]
        assert g["colors"].primary is not None and g["colors"].metadata.get("success", True)
    assert max(b.batch_sizes) > 1


def test_decode_ignores_pillow_bomb_limit(monkeypatch):
    """Pillow-decoded formats follow cv2.imdecode's CV_IO_MAX_IMAGE_PIXELS (2^30), not
    Pillow's decompression-bomb limit: a GIF above a lowered
    PIL.Image.MAX_IMAGE_PIXELS still decodes -- and the process-global Pillow limit is left
    as it was for other Pillow users."""
    import io

    from PIL import Image

    from low_level_feature_extraction_amd import decode

    rgb = np.random.default_rng(1).integers(0, 256, (60, 70, 3), dtype=np.uint8)
    buf = io.BytesIO()
    Image.fromarray(rgb).convert("P").save(buf, "GIF")
    monkeypatch.setattr(Image, "MAX_IMAGE_PIXELS", 1000)  # 2 * 1000 < 60 * 70: a bomb to Pillow
    out = decode.decode_bgr(buf.getvalue())
    assert out.shape == (60, 70, 3)
    assert Image.MAX_IMAGE_PIXELS == 1000
    # between Pillow's warning and error thresholds: decodes, and no warning escapes
    import warnings

    monkeypatch.setattr(Image, "MAX_IMAGE_PIXELS", 3000)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert decode.decode_bgr(buf.getvalue()).shape == (60, 70, 3)
    assert Image.MAX_IMAGE_PIXELS == 3000


def test_pillow_bomb_guard_untouched_by_concurrent_decodes():
    """decode_many over bomb-sized images (Pillow fallback path: GIF headers of
    100 MP, between Pillow's warning and error limits, and 225 MP, above its error limit but
    below cv2's 2^30) on the decode pool leaves Image.MAX_IMAGE_PIXELS and the process's
    warning filters exactly as they were."""
    import struct
    import warnings

    from PIL import Image

    from low_level_feature_extraction_amd import decode

    def gif(w, h):  # header + one truncated frame: open() parses it, load() fails
        b = b"GIF89a" + struct.pack("<HHBBB", w, h, 0x80, 0, 0) + b"\x00\x00\x00\xff\xff\xff"
        return b + b"," + struct.pack("<HHHHB", 0, 0, w, h, 0) + b"\x02\x02\x44\x01\x00;"

    filters0 = list(warnings.filters)
    limit0 = Image.MAX_IMAGE_PIXELS
    blobs = [gif(10000, 10000), gif(15000, 15000)] * 4
    out = decode.decode_many(blobs, workers=4)
    assert all(isinstance(o, decode.DecodeError) for o in out)  # truncated frames
    assert Image.MAX_IMAGE_PIXELS == limit0
    assert warnings.filters == filters0


class _Rec:
    def __init__(self, level):
        self.shadow_level = level


class _FakePipelinedBackend:
    """submit_images / collect stand-in: records what a launch held and how many were in
    flight (the pipelined worker path without a GPU)."""

    def __init__(self, cap=4):
        self.inflight = 1
        self.cap = cap
        self.launches = {}
        self.next = 0
        self.open = 0
        self.max_open = 0

    def batch_capacity(self, h, w):
        return self.cap

    def submit_images(self, images, features, seed=0, indices=None, n_colors=5):
        assert len(images) <= self.cap and len({tuple(im.shape) for im in images}) == 1
        t = self.next
        self.next += 1
        self.open += 1
        assert self.open <= self.inflight, "more launches in flight than the depth"
        self.max_open = max(self.max_open, self.open)
        self.launches[t] = [f"{int(np.asarray(im).sum())}:{i}" for im, i in zip(images, indices)]
        return t

    def collect(self, t):
        import time

        time.sleep(0.01)  # the launch's device time
        self.open -= 1
        return [_Rec(x) for x in self.launches.pop(t)]


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_batcher_pipelined_keeps_launches_in_flight(depth):
    fake = _FakePipelinedBackend(cap=4)
    imgs = [np.full((3 + i % 2, 4, 3), i, np.uint8) for i in range(40)]
    with MicroBatcher(features=("shadows",), max_batch=8, max_wait_ms=30, inflight=depth, backend=fake,
                      freeze_gc=False) as b:
        futs = [b.submit(im, index=1000 + i) for i, im in enumerate(imgs)]
        res = [f.result(timeout=20)["shadows"]["shadow_level"] for f in futs]
    # each request's own result and global index, whatever it was batched with
    assert res == [f"{int(im.sum())}:{1000 + i}" for i, im in enumerate(imgs)]
    assert sum(b.batch_sizes) == 40 and max(b.batch_sizes) <= 4
    assert fake.max_open == b.max_in_flight == min(depth, len(b.batch_sizes))
    if depth > 1:  # launch k + 1 submitted before launch k's collect returned
        log = b.launch_log
        assert any(log[k + 1][0] < log[k][2] for k in range(len(log) - 1))


def test_batcher_pipelined_isolates_a_refused_launch(monkeypatch):
    fake = _FakePipelinedBackend(cap=8)
    fake.inflight = 2

    def refuse(images, *a, **k):
        raise RuntimeError("launch refused")

    monkeypatch.setattr(fake, "submit_images", refuse)
    from low_level_feature_extraction_amd import pipeline

    def one(images, feats, **kw):
        if int(images[0].sum()) == 0:
            raise ValueError("bad image")
        return [{"ok": kw["index_base"]}]

    monkeypatch.setattr(pipeline, "run_batch", one)
    with MicroBatcher(features=("shadows",), max_batch=8, max_wait_ms=30, inflight=2, backend=fake,
                      freeze_gc=False) as b:
        futs = [b.submit(np.full((2, 2, 3), v, np.uint8), index=7 + i) for i, v in enumerate([1, 0, 2])]
        assert futs[0].result(timeout=10) == {"ok": 7}
        with pytest.raises(ValueError, match="bad image"):
            futs[1].result(timeout=10)
        assert futs[2].result(timeout=10) == {"ok": 9}


@pytest.mark.gpu
def test_batcher_pipelined_on_gpu_device_images_equal_run_batch():
    """The request path on the headline's serving loop: single device images from
    concurrent requests, two launches in flight through llfe_submit_images, every result
    equal to run_batch's for the same image and global index."""
    import torch

    from low_level_feature_extraction_amd import synth
    from low_level_feature_extraction_amd.pipeline import run_batch

    feats = ("colors", "shapes", "shadows")
    imgs = [synth.synth_numpy(i, 270, 480, seed=11) for i in range(24)]
    dev = [torch.from_numpy(im).to("cuda:0") for im in imgs]  # separately allocated
    # images 16..23 start 3 bytes into their allocation: not 16-B aligned, so their launch
    # gathers them (k_gather_images) instead of reading them in place through the table
    for i in range(16, 24):
        flat = torch.empty(imgs[i].size + 3, dtype=torch.uint8, device="cuda:0")
        dev[i] = flat[3:].view(270, 480, 3)
        dev[i].copy_(torch.from_numpy(imgs[i]))
    ref = run_batch(imgs, feats, seed=77, index_base=4000)
    with MicroBatcher(features=feats, max_batch=8, max_wait_ms=50, inflight=2, seed=77) as b:
        futs = [b.submit(t, index=4000 + i) for i, t in enumerate(dev)]
        got = [f.result(timeout=120) for f in futs]
    for i, (r, g) in enumerate(zip(ref, got)):
        assert g["shapes"] == r["shapes"], i
        assert g["shadows"] == r["shadows"], i
        assert g["colors"] == r["colors"], i
    assert b.max_in_flight == 2 and len(b.batch_sizes) >= 3
    log = b.launch_log
    assert any(log[k + 1][0] < log[k][2] for k in range(len(log) - 1)), "no two launches overlapped"
