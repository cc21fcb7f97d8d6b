#!/usr/bin/env python3
"""CPU simulation (round 6): how much of a Lloyd sweep's one-by-one labelling could per-cube
label reuse across iterations save?  On the bench's synthetic photos (1080p, noise as the
reference's trunc(N(0, 0.5))), runs Lloyd in float64 from k-means++-like random centres with
OpenCV's criteria (eps 0.2, 200 iterations) and, per iteration, takes the cubes the device
labels one by one (those failing the box margin test) and asks:

* ideal: of the colours labelled one by one in iteration t, how many sit in a cube that was
  also labelled in t - 1 and whose colours' labels are all unchanged (an upper bound for any
  reuse rule);
* bounded: how many of those a conservative rule could prove unchanged before labelling:
  per cube, the smallest margin d_second - d_best over its colours at t - 1 must exceed the
  largest change the centre moves can make to any colour's margin in the cube (the exact
  change at the cube centre q plus 2 |p - q|_1 max |delta_j - delta_k|), plus 1.

    python tools/km_reuse_sim.py [images] [seed]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def photo_colours(i, seed):
    from low_level_feature_extraction_amd import synth

    bgr = synth.synth_numpy(i, 1080, 1920, seed=seed, kind="photo")
    rng = np.random.default_rng(seed + i)
    rgb = bgr[..., ::-1].reshape(-1, 3).astype(np.int16)
    noise = np.trunc(rng.normal(0, 0.5, rgb.shape)).astype(np.int16)
    rgb = np.clip(rgb + noise, 0, 255).astype(np.int64)
    keys = np.unique((rgb[:, 0] << 16) | (rgb[:, 1] << 8) | rgb[:, 2])
    return np.stack([(keys >> 16) & 255, (keys >> 8) & 255, keys & 255], 1).astype(np.float64)


def run(p, K=5, seed=0):
    rng = np.random.default_rng(seed)
    c = p[rng.choice(len(p), K, replace=False)].copy()
    cube = (p // 4).astype(np.int64)
    cid = (cube[:, 0] << 12) | (cube[:, 1] << 6) | cube[:, 2]
    uc, inv = np.unique(cid, return_inverse=True)
    q = np.stack([(uc >> 12) & 63, (uc >> 6) & 63, uc & 63], 1) * 4.0 + 1.5  # cube centres
    prev = None
    tot = dict(labelled=0, ideal=0, bounded=0, iters=0)
    for it in range(200):
        d = ((p[:, None, :] - c[None, :, :]) ** 2).sum(-1)
        lab = d.argmin(1)
        ds = np.sort(d, 1)
        marg = ds[:, 1] - ds[:, 0]
        # the box test at each cube centre: owner k = argmin at q, pass when every other j
        # is farther by more than 3 L1(c_j - c_k) + 1
        dq = ((q[:, None, :] - c[None, :, :]) ** 2).sum(-1)
        k = dq.argmin(1)
        thr = 3.0 * np.abs(c[None, :, :] - c[k][:, None, :]).sum(-1) + 1.0
        ok = (dq - dq[np.arange(len(q)), k][:, None] > thr)
        ok[np.arange(len(q)), k] = True
        fail_cube = ~ok.all(1)
        fail_pt = fail_cube[inv]
        n_lab = int(fail_pt.sum())
        if prev is not None:
            plab, pfail_cube, pmarg, pc = prev
            same = np.ones(len(uc), bool)
            np.logical_and.at(same, inv, lab == plab)
            cand = fail_cube & pfail_cube
            ideal = cand & same
            # bounded rule: the cube's smallest margin at t - 1 against the largest change
            delta = c - pc
            dd = np.abs(delta[:, None, :] - delta[None, :, :]).max(-1).max()  # max_jk |delta_j - delta_k|_inf
            cmin = np.full(len(uc), np.inf)
            np.minimum.at(cmin, inv, pmarg)
            # exact change of d_j - d_k at q over all pairs, bounded by its largest magnitude
            dq_prev = ((q[:, None, :] - pc[None, :, :]) ** 2).sum(-1)
            chg = np.abs((dq - dq_prev)[:, :, None] - (dq - dq_prev)[:, None, :]).max((1, 2))
            bounded = cand & (cmin > chg + 2 * 4.5 * dd + 1.0)
            tot["ideal"] += int(np.bincount(inv, minlength=len(uc))[ideal].sum())
            tot["bounded"] += int(np.bincount(inv, minlength=len(uc))[bounded].sum())
            tot["labelled"] += n_lab
            tot["iters"] += 1
        prev = (lab, fail_cube, marg, c.copy())
        new = np.stack([np.bincount(lab, p[:, a], K) for a in range(3)], 1) / np.maximum(np.bincount(lab, None, K), 1)[:, None]
        shift = np.sqrt(((new - c) ** 2).sum(1)).max()
        c = new
        if shift < 0.2:
            break
    return tot


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 2025
    agg = dict(labelled=0, ideal=0, bounded=0, iters=0)
    for i in range(n):
        p = photo_colours(2 * i + 1, seed)
        for a in range(2):
            t = run(p, seed=seed + 10 * i + a)
            for key in agg:
                agg[key] += t[key]
            print(f"image {i} attempt {a}: U={len(p)} iters={t['iters'] + 1} labelled/iter={t['labelled'] / max(t['iters'], 1):.0f} "
                  f"ideal {t['ideal'] / max(t['labelled'], 1):.3f} bounded {t['bounded'] / max(t['labelled'], 1):.3f}", flush=True)
    print(f"all: of the colours labelled one by one (iterations >= 2), reusable ideal "
          f"{agg['ideal'] / max(agg['labelled'], 1):.3f}, provable {agg['bounded'] / max(agg['labelled'], 1):.3f}")


if __name__ == "__main__":
    main()
