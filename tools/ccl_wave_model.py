#!/usr/bin/env python3
"""Round 6 (verdict item 1): a wave-level model of the COMPILED control flow of round 5's
first k_ccl_runs, run over the class maps of test_gpu_parity's shape-mask inputs.

The source loop (tools/debug/ccl_probe.hip, k_runs_perwave, the form DESIGN.md describes)::

    for (;;) {
        int it = 0;
        if (lane == 0) it = atomicAdd(&ftcount[1], 1);
        it = __shfl(it, 0);                       // ds_bpermute from lane 0
        if (it >= nft) break;
        ... if (__ballot(C != 0) == 0) { if (lane == 0) nroots[t] = 0; continue; }
        ccl_runs_tile(...);                       // lane 0: *cnt = 0 ... nroots[t] = *cnt
        if (lane == 0) tlist2[atomicAdd(tcount2, 1)] = tt;
    }

What hipcc (ROCm 7.2, -O3, gfx950) makes of it (``--cuda-device-only -S``, kept in
profiles/r6/ccl_root_cause/): the latch's ``lane != 0`` path is threaded straight back to
the ``ds_bpermute`` of the tile index -- a second loop (``Loop Header: Depth=2``) whose
back-edge sets the index register to 0 (``int it = 0``) and skips the header's
``if (lane == 0)`` atomic.  Lane 0 leaves that loop (it has the ``tlist2`` append and the
atomic to run), lanes 1-63 go round it: they execute the shuffle with lane 0 inactive
(ds_bpermute returns 0 for a disabled source lane) and run list entry 0's tile again with
lane 0 masked off.  Only lane 0 resets the tile's root counter ``*cnt``, so every such trip
appends that tile's row >= 1 roots at ``roots[gbase + atomicAdd(cnt, 1)]`` with ``cnt``
growing without bound, and the trips end only when entry 0's tile has no candidate in rows
1-63 (the threaded lanes then take the ``continue`` path, whose exit rejoins lane 0).

This script applies exactly those semantics to the class maps (oracle Canny classes of the
test's images) and prints, per size, whether the wave terminates and, if not, after how
many threaded trips ``roots`` leaves its buffer (hysteresis_ids(n, h, w) u16 entries).
Model of the threaded read: 0 (disabled source lane) or the stale index (``--stale``).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TW = TH = 64


def test_images(h, w, n=2, seed=0):
    """tests/test_gpu_parity.py::_imgs"""
    from low_level_feature_extraction_amd import synth

    rng = np.random.default_rng(seed + h * 1000 + w)
    out = []
    for i in range(n):
        if h >= 32 and w >= 32:
            out.append(synth.synth_numpy(i, h, w, seed=seed))
        else:
            out.append(rng.integers(0, 256, (h, w, 3), dtype=np.uint8))
    return np.stack(out)


def tile_rows(cls, tx, ty):
    """64 candidate-row masks (class != 1) of one tile, as row_masks() forms them."""
    H, W = cls.shape
    rows = []
    for r in range(TH):
        y = ty * TH + r
        m = 0
        if y < H:
            seg = cls[y, tx * TW:min(W, tx * TW + TW)]
            for x, v in enumerate(seg):
                if v != 1:
                    m |= 1 << x
        rows.append(m)
    return rows


def runs(m):
    out, x = [], 0
    while m >> x:
        if (m >> x) & 1:
            a = x
            while (m >> x) & 1:
                x += 1
            out.append((a, x - 1))
        else:
            x += 1
    return out


def roots_by_row(rows):
    """Union-find over the rows' runs (8-connected to the row above), node = row * 32 +
    rank, root = the component's smallest node (atomicMin unions): roots per row."""
    parent = {}

    def find(a):
        while parent[a] != a:
            a = parent[a]
        return a

    prev = []
    for r, m in enumerate(rows):
        cur = []
        for j, (a, b) in enumerate(runs(m)):
            node = r * 32 + j
            parent[node] = node
            for ju, (ua, ub) in enumerate(prev):
                if ua <= b + 1 and ub >= a - 1:
                    x, y = find(node), find((r - 1) * 32 + ju)
                    if x != y:
                        lo, hi = min(x, y), max(x, y)
                        parent[hi] = lo
            cur.append((a, b))
        prev = cur
    per_row = [0] * len(rows)
    for node in parent:
        if find(node) == node:
            per_row[node // 32] += 1
    return per_row


def model(h, w, stale=False, n=2, trip_cap=10 ** 7):
    from oracle import oracle as O

    imgs = test_images(h, w, n)
    ntx, nty = (w + TW - 1) // TW, (h + TH - 1) // TH
    ntiles = ntx * nty
    tiles = []  # per global tile: rows
    for i in range(n):
        cls = O.canny_nms(O.blur5(O.bgr2gray(imgs[i])))
        for t in range(ntiles):
            tiles.append(tile_rows(cls, t % ntx, t // ntx))
    # the stencil's tile flags: tiles with a candidate
    ftlist = [tt for tt, rows in enumerate(tiles) if any(rows)]
    nft = len(ftlist)
    cap_entries = n * ntiles * TH * TW  # hysteresis_ids(n, h, w): the roots buffer, u16 entries
    report = {"size": f"{h}x{w}", "listed_tiles": nft, "roots_buffer_entries": cap_entries}
    ctr = 0
    waves = []
    # one wave per list entry suffices: every other wave reads it >= nft and exits
    for _ in range(nft):
        it = ctr
        ctr += 1
        tt = ftlist[it]
        rows = tiles[tt]
        # (lane 0 present) the body runs; the counter ends at the tile's root count
        per_row = roots_by_row(rows)
        cnt = sum(per_row)
        # lanes 1..63 threaded back to the shuffle with lane 0 inactive
        trips = 0
        it2 = it if stale else 0
        gbase = ftlist[it2] * TH * TW
        while True:
            if it2 >= nft:
                break
            rows2 = tiles[ftlist[it2]]
            if not any(rows2[1:]):  # no candidate in rows 1-63: the `continue` path, exit
                break
            trips += 1
            cnt += sum(roots_by_row(rows2)[1:])  # appends past the tile's real roots
            if gbase + cnt >= cap_entries:
                waves.append({"entry": it, "threaded_tile": ftlist[it2], "runaway": True,
                              "trips_to_overflow": trips, "cnt": cnt})
                break
            if trips >= trip_cap:
                waves.append({"entry": it, "runaway": True, "trips": trips, "cnt": cnt})
                break
        else:  # pragma: no cover
            pass
        if not waves or waves[-1]["entry"] != it:
            waves.append({"entry": it, "threaded_tile": ftlist[it2] if it2 < nft else None, "runaway": False,
                          "extra_trips": trips})
    report["waves"] = waves
    report["outcome"] = ("roots[] written past its buffer (illegal address / hang)"
                         if any(wv["runaway"] for wv in waves) else "terminates")
    return report


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stale", action="store_true", help="threaded shuffle reads the stale index instead of 0")
    ap.add_argument("sizes", nargs="*", default=["1x1", "2x3", "5x7"])
    a = ap.parse_args()
    import json

    for s in a.sizes:
        h, w = map(int, s.split("x"))
        print(json.dumps(model(h, w, stale=a.stale)))


if __name__ == "__main__":
    main()
