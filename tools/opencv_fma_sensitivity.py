#!/usr/bin/env python3
"""OpenCV-parity risk without OpenCV: how much do the oracle's outputs depend on the one
host-build detail the restatement had to assume -- fused multiply-add (OpenCV's
AVX2/FMA3 dispatch, what oracle and device reproduce) versus separate multiply and add
(OpenCV's SSE2 baseline build) -- in the two float paths of the hot path:

* adaptiveThreshold's CV_32F 11x11 Gaussian mean (shadow pyc @L17-18): mask pixels that
  flip, and whether the shadow level changes;
* cv2.kmeans' normL2Sqr (color_extractor.py:194-196): centres (ΔE76 after Hungarian
  matching), per-centre counts and compactness, same noise and RNG stream.

Integer stages (gray, blur5, Canny, dilate, contours) have no such freedom.

    python tools/opencv_fma_sensitivity.py [--n 4] [--out profiles/r2/opencv_fma_sensitivity.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from low_level_feature_extraction_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests import kmeans_bar  # noqa: E402


def one(img, i, seed):
    h, w = img.shape[:2]
    gray = O.blur5(O.bgr2gray(img))
    out = {}
    means, stats, km = {}, {}, {}
    noise = O.numpy_noise(h * w, 1000 + i)
    for mode in (True, False):
        O.set_fma(mode)
        means[mode] = O.gauss_float_mean(gray)
        stats[mode] = O.shadow_stats(img)
        km[mode] = O.dominant_colors(img, noise, 5, O.image_rng_state(seed, i))
    O.set_fma(True)
    thr = {m: (gray.astype(int) - means[m].astype(int)) <= -2 for m in (True, False)}
    out["pixels"] = int(h * w)
    out["mean_pixels_differ"] = int((means[True] != means[False]).sum())
    out["mask_pixels_differ"] = int((thr[True] != thr[False]).sum())
    out["shadow_level_fma"] = O.shadow_level_from_stats(*stats[True])
    out["shadow_level_no_fma"] = O.shadow_level_from_stats(*stats[False])
    (c1, n1, u1, k1), (c2, n2, u2, k2) = km[True], km[False]
    out["n_unique"] = int(u1)
    r, c, de = kmeans_bar.match(c1, c2)
    out["kmeans_centres_equal"] = bool(np.array_equal(np.sort(c1, 0), np.sort(c2, 0)))
    out["kmeans_max_de76"] = float(de.max()) if len(de) else 0.0
    out["kmeans_max_channel_diff"] = int(np.abs(c1[r].astype(int) - c2[c].astype(int)).max()) if len(r) else 0
    out["kmeans_max_count_diff"] = int(np.abs(n1[r] - n2[c]).max()) if len(r) else 0
    out["kmeans_compactness_rel_diff"] = abs(k1 - k2) / max(1.0, abs(k1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4, help="images per size (half ui, half photo)")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r2", "opencv_fma_sensitivity.json"))
    args = ap.parse_args()
    res = {"what": __doc__.strip().splitlines()[0], "sizes": {}}
    for (h, w) in [(1080, 1920), (2160, 3840)]:
        rows = []
        for i in range(args.n):
            t = time.time()
            img = synth.synth_numpy(i, h, w, seed=2025)
            r = one(img, i, seed=7)
            r["kind"] = "ui" if i % 2 == 0 else "photo"
            r["seconds"] = round(time.time() - t, 1)
            rows.append(r)
            print(h, w, r, flush=True)
        tot = sum(r["pixels"] for r in rows)
        res["sizes"][f"{w}x{h}"] = {
            "images": rows,
            "mask_pixels_differ_total": sum(r["mask_pixels_differ"] for r in rows),
            "mask_pixels_differ_fraction": sum(r["mask_pixels_differ"] for r in rows) / tot,
            "shadow_levels_differ": sum(r["shadow_level_fma"] != r["shadow_level_no_fma"] for r in rows),
            "kmeans_images_with_different_centres": sum(not r["kmeans_centres_equal"] for r in rows),
            "kmeans_max_de76": max(r["kmeans_max_de76"] for r in rows),
        }
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "images"} for k, v in res["sizes"].items()}))


if __name__ == "__main__":
    main()
