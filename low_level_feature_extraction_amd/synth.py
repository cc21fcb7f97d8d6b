"""Synthetic BGR images for benchmarks and parity tests.

* "ui" class (even index): a linear two-colour gradient background, 20-60 filled
  shapes (rectangles, rounded rectangles, circles, triangles) with uniform random BGR
  colours and sizes of 2-25 % of min(H, W), plus N(0, 2) sensor noise.  After the
  reference's own N(0, 0.5) noise this gives U ~ 6e4 unique colours at 1080p and
  non-trivial contours.
* "photo" class (odd index): a full-frame gradient with an independent direction per
  channel plus N(0, 8) noise -> U ~ 1.4e6 at 1080p (the k-means worst case).

The generator is torch-based so the same code fills a batch directly in GPU memory for
the benchmark; on CPU it is deterministic for a given seed.
"""
from __future__ import annotations

import math

import numpy as np


def _draw_ui(torch, gen, img, h, w, dev):
    # background gradient
    c0 = torch.randint(0, 256, (3,), generator=gen, device="cpu").float()
    c1 = torch.randint(0, 256, (3,), generator=gen, device="cpu").float()
    vertical = bool(torch.randint(0, 2, (1,), generator=gen).item())
    n = h if vertical else w
    t = torch.linspace(0, 1, n, device=dev)
    grad = c0.to(dev)[None, :] * (1 - t[:, None]) + c1.to(dev)[None, :] * t[:, None]  # n x 3
    if vertical:
        img[:] = grad[:, None, :]
    else:
        img[:] = grad[None, :, :]
    n_shapes = int(torch.randint(20, 61, (1,), generator=gen).item())
    m = min(h, w)
    params = torch.rand((n_shapes, 8), generator=gen)
    colors = torch.randint(0, 256, (n_shapes, 3), generator=gen).float()
    for k in range(n_shapes):
        p = params[k].tolist()
        kind = int(p[0] * 4)
        size = (0.02 + 0.23 * p[1]) * m
        sw = max(2, int(size * (0.6 + 0.8 * p[2])))
        sh = max(2, int(size * (0.6 + 0.8 * p[3])))
        x0 = int(p[4] * max(1, w - sw))
        y0 = int(p[5] * max(1, h - sh))
        x1, y1 = min(w, x0 + sw), min(h, y0 + sh)
        if x1 <= x0 or y1 <= y0:
            continue
        yy = torch.arange(y0, y1, device=dev, dtype=torch.float32)[:, None] + 0.5
        xx = torch.arange(x0, x1, device=dev, dtype=torch.float32)[None, :] + 0.5
        if kind == 0:  # rectangle
            mask = torch.ones((y1 - y0, x1 - x0), dtype=torch.bool, device=dev)
        elif kind == 1:  # rounded rectangle
            r = max(1.0, min(sw, sh) * (0.1 + 0.3 * p[6]))
            cx = torch.clamp(xx, x0 + r, x1 - r)
            cy = torch.clamp(yy, y0 + r, y1 - r)
            mask = (xx - cx) ** 2 + (yy - cy) ** 2 <= r * r
        elif kind == 2:  # circle / ellipse
            cx, cy = (x0 + x1) / 2, (y0 + y1) / 2
            rx, ry = (x1 - x0) / 2, (y1 - y0) / 2
            mask = ((xx - cx) / rx) ** 2 + ((yy - cy) / ry) ** 2 <= 1.0
        else:  # triangle
            ax, ay = x0 + p[6] * (x1 - x0), float(y0)
            bx, by = float(x0), float(y1)
            cx_, cy_ = float(x1), float(y1)

            def edge(px, py, qx, qy):
                return (qx - px) * (yy - py) - (qy - py) * (xx - px)

            e0, e1, e2 = edge(ax, ay, bx, by), edge(bx, by, cx_, cy_), edge(cx_, cy_, ax, ay)
            mask = ((e0 >= 0) & (e1 >= 0) & (e2 >= 0)) | ((e0 <= 0) & (e1 <= 0) & (e2 <= 0))
        region = img[y0:y1, x0:x1]
        region[mask] = colors[k].to(dev)
    return 2.0


def _draw_photo(torch, gen, img, h, w, dev):
    yy = torch.linspace(0, 1, h, device=dev)[:, None]
    xx = torch.linspace(0, 1, w, device=dev)[None, :]
    for c in range(3):
        ang = float(torch.rand(1, generator=gen).item()) * 2 * math.pi
        lo = float(torch.randint(0, 96, (1,), generator=gen).item())
        hi = float(torch.randint(160, 256, (1,), generator=gen).item())
        t = (xx * math.cos(ang) + yy * math.sin(ang))
        t = (t - t.min()) / max(float((t.max() - t.min()).item()), 1e-6)
        img[:, :, c] = lo + (hi - lo) * t
    return 8.0


def synth_image(i: int, h: int, w: int, seed: int = 1234, device="cpu", kind: str | None = None):
    """One synthetic BGR uint8 image (torch tensor on ``device``)."""
    import torch

    gen = torch.Generator(device="cpu")
    gen.manual_seed(seed + i)
    dev = torch.device(device)
    img = torch.zeros((h, w, 3), dtype=torch.float32, device=dev)
    kind = kind or ("ui" if i % 2 == 0 else "photo")
    sigma = _draw_ui(torch, gen, img, h, w, dev) if kind == "ui" else _draw_photo(torch, gen, img, h, w, dev)
    if dev.type == "cpu":
        noise = torch.randn((h, w, 3), generator=gen) * sigma
    else:
        g2 = torch.Generator(device=dev)
        g2.manual_seed(seed * 7919 + i)
        noise = torch.randn((h, w, 3), generator=g2, device=dev) * sigma
    img += noise
    return img.round_().clamp_(0, 255).to(torch.uint8)


def synth_batch(n: int, h: int, w: int, seed: int = 1234, device="cpu", index_base: int = 0, kind=None):
    import torch

    out = torch.empty((n, h, w, 3), dtype=torch.uint8, device=device)
    for j in range(n):
        out[j] = synth_image(index_base + j, h, w, seed=seed, device=device, kind=kind)
    return out


def synth_numpy(i: int, h: int, w: int, seed: int = 1234, kind=None) -> np.ndarray:
    return synth_image(i, h, w, seed=seed, device="cpu", kind=kind).numpy()


def encode_png(bgr: np.ndarray) -> bytes:
    import io

    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(bgr[:, :, ::-1])).save(buf, format="PNG")
    return buf.getvalue()
