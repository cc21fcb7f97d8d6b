#!/usr/bin/env python3
"""Summarise an LLFE_KM_TRACE file (one line per k-means attempt, see llfe_api.cpp):
per-phase times for the "photo" (U > 300k) and "ui" classes, Lloyd time per iteration,
Lloyd bytes per iteration relative to a plain sweep, and the kernel span / CU balance.

    python tools/km_trace_summary.py gpurun_out/km_trace.txt [launch_index] [attempts_per_launch]
"""
import sys

import numpy as np


def main():
    path = sys.argv[1]
    launch = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    a = np.loadtxt(path, dtype=np.int64)
    n_att = int(sys.argv[3]) if len(sys.argv) > 3 else 5120  # attempts per launch (10 x images per pass)
    n_att = n_att if len(a) >= n_att else len(a)
    nl = len(a) // n_att
    a = a[(launch % nl) * n_att:(launch % nl + 1) * n_att]
    img, att, U, it, t0, t1, hw, xcc, tpp, tll, by = a.T[:11]
    z = np.zeros_like(U)
    pp_pts, ncub = (a.T[11], a.T[12]) if a.shape[1] >= 13 else (z, z)
    pp_sel = a.T[13] if a.shape[1] >= 14 else z
    t_sel = a.T[14] / 100.0 if a.shape[1] >= 15 else z
    ll_pts = a.T[15] if a.shape[1] >= 16 else z
    t_sw = a.T[16] / 100.0 if a.shape[1] >= 17 else z
    dh = a.T[19].astype(np.uint64) if a.shape[1] >= 20 else z.astype(np.uint64)
    ok = it > 1
    pp = (tpp - t0) / 100.0
    # Lloyd start stamp: its own launch's in a split build (a one-launch kernel stamps t_start)
    split = a.shape[1] >= 23 and ((a.T[20] > 0) & (a.T[20] != t0)).any()
    tl0 = a.T[20] if split else tpp
    ll = (tll - tl0) / 100.0
    cp = (t1 - tll) / 100.0
    ph = U > 300000
    for name, m in [("photo", ph & ok), ("ui", ~ph & ok)]:
        if not m.any():
            continue
        print(f"{name:5s} n={m.sum():4d} U={U[m].mean():9.0f} iters={it[m].mean():5.1f}  PP {pp[m].mean()/1e3:6.3f} ms"
              f"  Lloyd {ll[m].mean()/1e3:6.3f} ms ({(ll[m] / (it[m] - 1)).mean():6.1f} us/iter,"
              f" {np.mean(ll_pts[m] / (it[m] - 1) / U[m]):.3f} of the colours labelled one by one)  compact {cp[m].mean()/1e3:6.3f} ms")
        if ncub[m].any():
            print(f"      cubes/U {np.mean(ncub[m] / U[m]):.3f}  k-means++ colours read one by one / U"
                  f" {np.mean(pp_pts[m] / U[m]):.3f} (undecided cubes) + {np.mean(pp_sel[m] / U[m]):.3f} (selection);"
                  f" selection time {t_sel[m].mean() / 1e3:.3f} ms; Lloyd sweeps {t_sw[m].mean() / 1e3:.3f} ms")
        if dh[m].any():
            bins = np.stack([((dh[m] >> np.uint64(8 * b)) & np.uint64(255)).astype(np.int64) for b in range(8)], 1)
            print("      iterations by largest centre move [<.25 <.5 <1 <2 <4 <8 <16 >=16]:",
                  np.round(bins.mean(0), 2).tolist(), f"; iters max {it[m].max()}")
    # slot gaps per phase: one interval per attempt and CU; the gap after an attempt ends
    # is the wait until the next attempt starts on the same CU (two workgroup slots per
    # CU), and the idle share is the slot time not covered by attempts over the phase's span
    def cu_of(h, x):
        return x * 1000 + ((h >> 13) & 7) * 100 + ((h >> 12) & 1) * 16 + ((h >> 8) & 15)

    phases = [("k-means++", t0, tpp, cu_of(hw, xcc))]
    if split:
        tls, hw2, xcc2 = a.T[20], a.T[21], a.T[22]
        phases.append(("Lloyd", tls, t1, cu_of(hw2, xcc2)))
    else:
        phases = [("attempt", t0, t1, cu_of(hw, xcc))]
    for name, s0, s1, cus in phases:
        m = it > 1 if name != "attempt" else np.ones_like(it, bool)
        gaps = []
        for c in np.unique(cus[m]):
            sel = m & (cus == c)
            st, en = np.sort(s0[sel]), s1[sel]
            for e in en:
                k = np.searchsorted(st, e)
                if k < len(st):
                    gaps.append((st[k] - e) / 100.0)
        span = (s1[m].max() - s0[m].min()) / 100.0
        slots = 2 * len(np.unique(cus[m]))
        idle = 1 - ((s1[m] - s0[m]) / 100.0).sum() / (slots * span)
        g = np.array(gaps) if gaps else np.zeros(1)
        print(f"{name:9s} span {span / 1e3:.2f} ms over {slots} slots: idle share {idle:.3f}; gap after an attempt"
              f" median {np.median(g):.1f} us, mean {g.mean():.1f}, p90 {np.percentile(g, 90):.1f}")
    dur = (t1 - t0) / 100.0
    cu = xcc * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 15)
    busy = {}
    for k, d in zip(cu, dur):
        busy[k] = busy.get(k, 0.0) + d
    b = np.array(list(busy.values())) / 1e3
    print(f"span {(t1.max() - t0.min()) / 1e5:.2f} ms; per-CU busy min/mean/max {b.min():.2f}/{b.mean():.2f}/{b.max():.2f} ms;"
          f" longest attempts (ms): {np.round(np.sort(dur)[-4:] / 1e3, 2)}")


if __name__ == "__main__":
    main()
