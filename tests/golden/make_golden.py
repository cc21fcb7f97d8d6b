"""Generates the golden fixtures in tests/golden/ from the libraries the reference
itself calls (Pillow, NumPy), as importable in this container.

    python tests/golden/make_golden.py

Fixtures (all small, inputs regenerated from the stored seeds):
  pil_lanczos.npz  Image.resize(size, LANCZOS[, box]) / thumbnail outputs (Pillow)
  pil_reduce.npz   Image.reduce((fx, fy)) outputs (Pillow)
  numpy_noise.npz  RandomState(seed).normal(0, 0.5, (P, 3)).astype(int8) streams
  unique_order.npz np.unique(pixels, axis=0) rows for noised random images
  meta.json        library versions used
"""
from __future__ import annotations

import json
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))

LANCZOS_CASES = [  # (h, w, ch, out_h, out_w, box or None)
    (48, 64, 3, 18, 32, None),
    (300, 400, 3, 90, 120, None),
    (37, 53, 3, 11, 29, None),
    (100, 100, 3, 100, 50, None),
    (50, 80, 3, 120, 160, None),
    (64, 96, 1, 20, 30, None),
    (120, 200, 3, 40, 70, (10.5, 3.25, 190.0, 117.75)),
    (90, 160, 3, 45, 80, (0.0, 0.0, 80.0, 45.0)),
]
THUMB_CASES = [(3840, 2160), (2000, 1125), (3000, 2001), (1000, 4000), (1920, 1080), (7680, 4320), (5, 10000),
               (10000, 3), (1919, 1081), (2048, 1536), (1080, 1920), (4000, 4000)]
REDUCE_CASES = [(11, 16, 2, 2), (16, 23, 3, 3), (16, 16, 2, 3), (21, 30, 4, 4), (11, 37, 5, 2), (36, 51, 7, 7),
                (13, 9, 1, 3), (9, 13, 3, 1)]


def lanczos():
    out = {}
    for k, (h, w, ch, oh, ow, box) in enumerate(LANCZOS_CASES):
        rng = np.random.default_rng(1000 + k)
        a = rng.integers(0, 256, (h, w, ch) if ch > 1 else (h, w), dtype=np.uint8)
        im = Image.fromarray(a)
        r = np.array(im.resize((ow, oh), Image.Resampling.LANCZOS, box=box))
        out[f"case{k}"] = r
    sizes = []
    for w, h in THUMB_CASES:
        im = Image.new("L", (w, h))
        im.thumbnail((1920, 1080), Image.Resampling.LANCZOS)
        sizes.append([w, h, im.size[0], im.size[1]])
    out["thumb_sizes"] = np.array(sizes, np.int64)
    # a full thumbnail with the reducing_gap reduce() pre-pass (>= 4x the target)
    rng = np.random.default_rng(77)
    a = rng.integers(0, 256, (90, 200, 3), dtype=np.uint8)
    im = Image.fromarray(a)
    im.thumbnail((40, 20), Image.Resampling.LANCZOS)
    out["thumb_reduce"] = np.array(im)
    np.savez_compressed(os.path.join(HERE, "pil_lanczos.npz"), **out)


def reduce_():
    out = {}
    for k, (h, w, fx, fy) in enumerate(REDUCE_CASES):
        rng = np.random.default_rng(2000 + k)
        a = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        out[f"case{k}"] = np.array(Image.fromarray(a).reduce((fx, fy)))
    np.savez_compressed(os.path.join(HERE, "pil_reduce.npz"), **out)


def noise():
    out = {}
    for seed in (0, 1, 7, 12345):
        rs = np.random.RandomState(seed)
        out[f"seed{seed}"] = rs.normal(0, 0.5, (4096, 3)).astype(np.int8)
    np.savez_compressed(os.path.join(HERE, "numpy_noise.npz"), **out)


def unique_order():
    out = {}
    for k, (h, w) in enumerate([(16, 16), (40, 30), (64, 64)]):
        rng = np.random.default_rng(3000 + k)
        bgr = (rng.integers(0, 8, (h, w, 3)) * 32 + 100).astype(np.uint8)  # few colours, many repeats
        rgb = bgr[:, :, ::-1].reshape(-1, 3)
        nz = np.random.RandomState(k).normal(0, 0.5, rgb.shape).astype(np.int8)
        px = np.clip(rgb.astype(np.int32) + nz, 0, 255).astype(np.uint8)
        out[f"case{k}"] = np.unique(px, axis=0)
    np.savez_compressed(os.path.join(HERE, "unique_order.npz"), **out)


def main():
    lanczos()
    reduce_()
    noise()
    unique_order()
    import PIL

    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump({"pillow": PIL.__version__, "numpy": np.__version__}, f, indent=1)


if __name__ == "__main__":
    main()
