"""GPU box: where an all-ui pipelined step goes (host side): submit / collect wall time,
the C collect vs the Python conversion, host contour pool busy, GPU-only step."""
import sys
import time

import torch

sys.path.insert(0, ".")
from low_level_feature_extraction_amd import synth  # noqa: E402
from low_level_feature_extraction_amd.backend import Backend  # noqa: E402

be = Backend.get(0)
kind = sys.argv[1] if len(sys.argv) > 1 else "ui"
B = 512
imgs = synth.synth_batch(B, 1080, 1920, seed=1234, device="cuda:0", kind=kind)
feats = ("colors", "shapes", "shadows")
conv_t = [0.0]
orig = be._convert


def timed_convert(*a, **k):
    t = time.perf_counter()
    r = orig(*a, **k)
    conv_t[0] += time.perf_counter() - t
    return r


be._convert = timed_convert
for mode in ("host", "gpu"):
    be.set_contour_mode(mode)
    for rep in range(2):
        pending, ts, tc = [], 0.0, 0.0
        conv_t[0] = 0.0
        be.host_contour_stats(reset=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(6):
            a = time.perf_counter()
            pending.append(be.submit(imgs, feats, seed=k))
            ts += time.perf_counter() - a
            if len(pending) == 2:
                a = time.perf_counter()
                be.collect(pending.pop(0))
                tc += time.perf_counter() - a
        while pending:
            a = time.perf_counter()
            be.collect(pending.pop(0))
            tc += time.perf_counter() - a
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        hc = be.host_contour_stats(reset=True)
        print(f"{kind} contours={mode}: {dt / 6 * 1e3:.2f} ms/step ({B * 6 / dt:.0f} img/s) | submit {ts / 6 * 1e3:.2f} "
              f"collect {tc / 6 * 1e3:.2f} (python convert {conv_t[0] / 6 * 1e3:.2f}) | host pool busy "
              f"{hc['busy_ms'] / 6:.2f} ms/step", flush=True)
be.set_contour_mode("host")
# GPU-only: colours + shadows (no contours at all)
for rep in range(2):
    pending = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(6):
        pending.append(be.submit(imgs, ("colors", "shadows"), seed=k))
        if len(pending) == 2:
            be.collect(pending.pop(0))
    while pending:
        be.collect(pending.pop(0))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{kind} colors+shadows only: {dt / 6 * 1e3:.2f} ms/step", flush=True)
