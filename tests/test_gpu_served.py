"""GPU parity at the SERVED launch shapes: the bench's own serving loop, checked image by
image against the oracle.

bench.py times ``llfe_submit_batch`` / ``llfe_collect_batch`` with two batches in
flight over 512 x 1080p resident images (BASELINE configs[3] per GPU), production
noise (no caller noise: the device's seeded stream, unique.hip / DESIGN.md §6).  These
tests run exactly that launch -- the same synthetic batch (synth_batch on the device,
seed 2025, 50/50 ui/photo), the same feature set, three submissions so a workspace slot
is reused at full size -- and check the collected records against the CPU oracle:

* shapes (ShapeAnalyzer.analyze_shapes, shape pyc @L125-189) and the shadow sum /
  count (ShadowAnalyzer, shadow pyc @L12-24): bit-exact for EVERY image;
* n_unique (len(np.unique(pixels, axis=0)) after the noise, color_extractor.py:177,
  223-225): exact for every image, through the oracle's restatement of the device noise
  (orc_device_noise) -- the production keys themselves are pinned bit-exactly on one
  image per class;
* palettes (cv2.kmeans, color_extractor.py:189-197, and the palette rules :231-284) on
  the k-means bar (tests/kmeans_bar.py) for a spread of images that includes indices
  >= 256, whose key-buffer offsets pass 2^32 bytes.

Also at 256 x 1080p (configs[1] colours, configs[2] colours + shapes: results must
equal the 512 launch's for the same seed and index) and 128 x 4K high_quality
(configs[4] per GPU).  The oracle runs on a thread pool (ctypes releases the GIL).
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from low_level_feature_extraction_amd import synth
from tests import kmeans_bar

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

FULL = ("colors", "shapes", "shadows")
SEED = 2025  # bench.py's default --seed (and its synth seed)


def _log(msg):
    """progress on stderr (a GPU run is taken to be hung after minutes without output)"""
    import sys
    import time

    print(f"[served {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _threads():
    from low_level_feature_extraction_amd.decode import usable_cores

    return max(1, min(16, usable_cores()))


def _pmap(fn, items):
    with ThreadPoolExecutor(max_workers=_threads()) as ex:
        return list(ex.map(fn, items))


def _serve(backend, imgs, feats, seeds, index_base=0):
    """bench.py run_steps(pipelined=True): submit, keep `inflight` batches in flight,
    collect in order."""
    pending, out = [], []
    for s in seeds:
        pending.append(backend.submit(imgs, feats, seed=s, index_base=index_base))
        if len(pending) == backend.inflight:
            out.append(backend.collect(pending.pop(0)))
    while pending:
        out.append(backend.collect(pending.pop(0)))
    return out


class _Served:
    """One device batch, its host copy and a cache of per-image oracle results."""

    def __init__(self, n, h, w):
        import torch

        self.h, self.w = h, w
        _log(f"synthesising {n} x {w}x{h}")
        self.dev = synth.synth_batch(n, h, w, seed=SEED, device="cuda:0", index_base=0)
        torch.cuda.synchronize()
        self.host = self.dev.cpu().numpy()
        self._shape = {}

    def shapes_shadows(self, orc, idx):
        todo = [i for i in idx if i not in self._shape]

        def one(i):
            img = self.host[i]
            return i, orc.analyze_shapes(img)["shapes"], orc.shadow_stats(img)

        for i, sh, sd in _pmap(one, todo):
            self._shape[i] = (sh, sd)
        return {i: self._shape[i] for i in idx}

    def n_unique(self, orc, seed, idx):
        P = self.h * self.w

        def one(i):
            return len(orc.color_unique(self.host[i], orc.device_noise(P, seed, i)))

        return dict(zip(idx, _pmap(one, list(idx))))

    def colours(self, orc, seed, idx):
        P = self.h * self.w

        def one(i):
            return orc.dominant_colors(self.host[i], orc.device_noise(P, seed, i), 5, orc.image_rng_state(seed, i))

        return dict(zip(idx, _pmap(one, list(idx))))


@pytest.fixture(scope="module")
def served1080():
    return _Served(512, 1080, 1920)


def _check_shapes(orc, served, res, idx):
    _log(f"oracle shapes / shadows of {len(idx)} images")
    want = served.shapes_shadows(orc, idx)
    bad = [i for i in idx if res[i].shapes != want[i][0] or (res[i].shadow_sum, res[i].shadow_count) != want[i][1]]
    assert not bad, f"shape / shadow mismatch at images {bad[:10]} (of {len(bad)})"


def _check_n_unique(orc, served, res, seed, idx):
    _log(f"oracle n_unique of {len(idx)} images (seed {seed})")
    want = served.n_unique(orc, seed, idx)
    bad = [(i, res[i].n_unique, want[i]) for i in idx if res[i].n_unique != want[i]]
    assert not bad, f"n_unique mismatch (image, got, want): {bad[:10]} (of {len(bad)})"


def _check_colours(orc, served, res, seed, idx, tag):
    from low_level_feature_extraction_amd.color_extractor import ColorExtractor

    _log(f"oracle k-means of {len(idx)} images (seed {seed})")
    want = served.colours(orc, seed, idx)
    for i in idx:
        centers, counts, nu, comp = want[i]
        r = res[i]
        assert r.n_unique == nu, (i, r.n_unique, nu)
        assert int(r.counts.sum()) == nu
        kmeans_bar.check(r.centers_rgb, r.counts, r.compactness, centers, counts, comp, nu, tag=f"{tag}-img{i}")
        # the palette rules (color_extractor.py:231-284) on the served record: equal to the
        # oracle's whenever the clusters are the same (equal-count clusters form a set)
        if sorted(map(tuple, r.centers_rgb.tolist())) == sorted(map(tuple, centers.tolist())) and \
                sorted(r.counts.tolist()) == sorted(counts.tolist()):
            got = ColorExtractor._palette(r.centers_rgb, r.counts)
            exp = orc.color_palette(centers, counts)
            if len(set(counts.tolist())) == len(counts):  # no count ties: order is defined
                assert (got.primary, got.background, got.accent) == (exp["primary"], exp["background"],
                                                                        exp["accent"]), i


def _spread(n, per_class):
    """Images spread over the batch, both classes (even = ui, odd = photo), incl. the top half."""
    step = max(2, (n // per_class) // 2 * 2)
    return sorted(list(range(0, n, step))[:per_class] + list(range(1, n, step))[:per_class])


def test_production_keys_bit_exact(backend, orc, served1080):
    """The production noise + np.unique keys of one ui and one photo image at 1080p equal
    the oracle's restatement key for key (llfe_color_unique, no caller noise)."""
    for i in (0, 1, 300, 301):
        keys, nu = backend.color_unique(served1080.dev[i:i + 1], seed=SEED, index_base=i)
        exp = orc.color_unique(served1080.host[i], orc.device_noise(1080 * 1920, SEED, i))
        assert int(nu[0]) == len(exp)
        assert np.array_equal(keys[0, : nu[0]].cpu().numpy().view(np.uint32), exp), i


def test_headline_512_two_in_flight(backend, orc, served1080):
    """configs[3] per GPU: 512 x 1080p, colors + shapes + shadows, the bench's serving loop
    (three submissions, two in flight: the third reuses the first one's workspace)."""
    assert backend.inflight == 2
    seeds = [SEED, SEED + 1, SEED + 2]
    runs = _serve(backend, served1080.dev, FULL, seeds)
    assert [len(r) for r in runs] == [512] * 3
    every = list(range(512))
    # shapes / shadows do not depend on the seed: all three submissions agree, and agree
    # with the oracle on every image
    for k in (1, 2):
        assert all(a.shapes == b.shapes and (a.shadow_sum, a.shadow_count) == (b.shadow_sum, b.shadow_count)
                   for a, b in zip(runs[0], runs[k]))
    _check_shapes(orc, served1080, runs[0], every)
    # n_unique of every image, first and reused slot
    _check_n_unique(orc, served1080, runs[0], seeds[0], every)
    _check_n_unique(orc, served1080, runs[2], seeds[2], every)
    # palettes on the bar: 64 images (32 ui, 32 photo) over the whole batch, from the
    # submission that reused slot 0
    sel = _spread(512, 32)
    assert len(sel) == 64 and sum(i >= 256 for i in sel) >= 32
    _check_colours(orc, served1080, runs[2], seeds[2], sel, "served512")
    served1080.runs512 = runs  # (compared by the 256-image configs below)


@pytest.mark.parametrize("feats", [("colors",), ("colors", "shapes")], ids=["configs1", "configs2"])
def test_256_configs(backend, orc, served1080, feats):
    """configs[1] / configs[2] per GPU: 256 x 1080p, three batches in flight as bench.py
    keeps them at this size (--inflight auto), four submissions so the first slot is reused.
    Results equal the 512 launch's for the same seed and global index (seeds follow the
    image, not the batch), and the oracle."""
    sub = served1080.dev[:256]
    seeds = [SEED, SEED + 7, SEED + 3, SEED]
    assert backend.inflight == 2
    backend.inflight = 3
    try:
        runs = _serve(backend, sub, feats, seeds)
    finally:
        backend.inflight = 2
    for a, b in zip(runs[0], runs[3]):  # slot 0 reused by the fourth batch, same seed
        assert np.array_equal(a.centers_rgb, b.centers_rgb) and np.array_equal(a.counts, b.counts)
        assert a.n_unique == b.n_unique and a.shapes == b.shapes
    every = list(range(256))
    _check_n_unique(orc, served1080, runs[0], seeds[0], every)
    ref = getattr(served1080, "runs512", None)
    if ref is not None:
        for a, b in zip(runs[0], ref[0][:256]):
            assert np.array_equal(a.centers_rgb, b.centers_rgb) and np.array_equal(a.counts, b.counts)
            assert a.n_unique == b.n_unique and a.compactness == b.compactness
            if "shapes" in feats:
                assert a.shapes == b.shapes
    if "shapes" in feats:
        bad = [i for i in every if runs[1][i].shapes != served1080.shapes_shadows(orc, [i])[i][0]]
        assert not bad, bad[:10]
        assert all(r.shadow_count == 0 and r.shadow_sum == 0 for r in runs[1])  # shadows not requested
    else:
        assert all(r.shapes == [] for r in runs[1])
    _check_colours(orc, served1080, runs[1], seeds[1], _spread(256, 8), f"served256-{'+'.join(feats)}")


def test_4k_high_quality_128(backend, orc):
    """configs[4] per GPU: 128 x 3840x2160, high_quality (no resize below 4000 px), full
    feature set, two in flight."""
    from low_level_feature_extraction_amd.backend import preprocess_size

    assert preprocess_size(3840, 2160, "high_quality") is None
    served = _Served(128, 2160, 3840)
    seeds = [SEED, SEED + 1, SEED + 2]
    runs = _serve(backend, served.dev, FULL, seeds)
    every = list(range(128))
    for a, b in zip(runs[0], runs[2]):
        assert a.shapes == b.shapes and (a.shadow_sum, a.shadow_count) == (b.shadow_sum, b.shadow_count)
    _check_shapes(orc, served, runs[0], every)
    _check_n_unique(orc, served, runs[2], seeds[2], every)
    _check_colours(orc, served, runs[2], seeds[2], _spread(128, 6), "served4k")
    del served
