"""Ragged batches through llfe_process_images: per-image sizes, row
strides, host / device memory and validate_and_preprocess_image's GPU resize, each image
with its own global index -- so every result equals that image run alone."""
import numpy as np
import pytest

from low_level_feature_extraction_amd import synth

pytestmark = pytest.mark.gpu

FEATS = ("colors", "shapes", "shadows")


def _same(a, b, tag):
    assert (a.width, a.height, a.n_unique) == (b.width, b.height, b.n_unique), tag
    assert np.array_equal(a.centers_rgb, b.centers_rgb) and np.array_equal(a.counts, b.counts), tag
    assert a.compactness == b.compactness, tag
    assert (a.shadow_sum, a.shadow_count) == (b.shadow_sum, b.shadow_count), tag
    assert a.shapes == b.shapes and a.n_contours == b.n_contours, tag


def test_alternating_sizes_equal_single_images(backend):
    imgs = [synth.synth_numpy(i, (90, 150)[i % 2], (160, 96)[i % 2], seed=21) for i in range(7)]
    got = backend.process_images(imgs, FEATS, seed=5, index_base=100)
    for i, im in enumerate(imgs):
        one = backend.process(im[None], FEATS, seed=5, index_base=100 + i)[0]
        _same(got[i], one, f"image {i}")


def test_strided_host_and_device_views(backend):
    import torch

    big = synth.synth_numpy(1, 300, 400, seed=4)
    views = [big[10:210, 20:300], big[::1, 50:51], big[150:300, :]]  # row stride 1200 B, 1-column, packed
    dev = torch.from_numpy(big).cuda()
    tviews = [dev[10:210, 20:300], dev[150:300, :]]
    got = backend.process_images(views + tviews, FEATS, seed=3, index_base=7)
    ref = [np.ascontiguousarray(v) for v in views] + [np.ascontiguousarray(big[10:210, 20:300]),
                                                      np.ascontiguousarray(big[150:300, :])]
    for i, im in enumerate(ref):
        one = backend.process(im[None], FEATS, seed=3, index_base=7 + i)[0]
        _same(got[i], one, f"view {i}")


def test_caller_indices_in_batch(backend):
    """llfe_batch.indices: the same images with scattered global indices in one batch."""
    import ctypes as C

    from low_level_feature_extraction_amd import _lib as L

    x = np.stack([synth.synth_numpy(i, 64, 80, seed=2) for i in range(4)])
    idx = np.array([40, 3, 977, 12], np.int64)
    b = L.LlfeBatch(C.c_void_p(x.ctypes.data), 4, 64, 80, 0, None, 0, 5, 0, C.c_void_p(idx.ctypes.data))
    res = (L.LlfeImageResult * 4)()
    shapes = (L.LlfeShape * 4096)()
    need = C.c_int64(0)
    assert backend._lib.llfe_process_batch(backend.ctx, C.byref(b), L.FEATURE_COLORS, C.c_uint64(8), res, shapes, 4096,
                                           C.byref(need), None) == 0
    for i in range(4):
        one = backend.process(x[i:i + 1], ("colors",), seed=8, index_base=int(idx[i]))[0]
        assert res[i].n_unique == one.n_unique and res[i].compactness == one.compactness


@pytest.mark.parametrize("mode,h,w", [("auto", 1400, 2600), ("performance", 900, 1500), ("high_quality", 300, 500),
                                      ("none", 1400, 2600)])
def test_preprocessing_on_gpu(backend, orc, mode, h, w):
    """The resize of validate_and_preprocess_image inside the call equals resize-then-process."""
    from low_level_feature_extraction_amd.utils import preprocess_decoded

    img = synth.synth_numpy(1, h, w, seed=6)
    small = synth.synth_numpy(0, 120, 200, seed=6)
    got = backend.process_images([img, small], FEATS, seed=2, index_base=50, preprocessing=mode)
    pre = preprocess_decoded(img, mode)
    one = backend.process(np.ascontiguousarray(pre)[None], FEATS, seed=2, index_base=50)[0]
    _same(got[0], one, mode)
    assert (got[0].height, got[0].width) == pre.shape[:2]
    _same(got[1], backend.process(small[None], FEATS, seed=2, index_base=51)[0], "small")


def test_parity_noise_mixed_sizes_vs_oracle(backend, orc):
    from tests import kmeans_bar

    imgs = [synth.synth_numpy(i, (70, 110)[i % 2], (90, 60)[i % 2], seed=9) for i in range(4)]
    noise = [orc.numpy_noise(im.shape[0] * im.shape[1], 60 + i) for i, im in enumerate(imgs)]
    got = backend.process_images(imgs, FEATS, seed=4, index_base=0, noise=noise)
    for i, im in enumerate(imgs):
        centers, counts, nu, comp = orc.dominant_colors(im, noise[i], 5, orc.image_rng_state(4, i))
        assert got[i].n_unique == nu
        kmeans_bar.check(got[i].centers_rgb, got[i].counts, got[i].compactness, centers, counts, comp, nu,
                         tag=f"ragged-{i}")
        assert got[i].shapes == orc.analyze_shapes(im)["shapes"]
        assert (got[i].shadow_sum, got[i].shadow_count) == orc.shadow_stats(im)


def test_invalid_descriptors(backend):
    from low_level_feature_extraction_amd import _lib as L

    with pytest.raises(L.LlfeError):
        backend.process_images([synth.synth_numpy(0, 40, 40, seed=1), synth.synth_numpy(1, 40, 40, seed=1)],
                               FEATS, noise=[np.zeros(40 * 40 * 3, np.int8), None])
    assert backend.process_images([], FEATS) == []
