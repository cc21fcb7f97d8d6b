"""GPU box: where a pipelined step's time goes.  Runs the bench's serving loop (two batches in
flight, the result assembly on a worker thread) with libllfe's profiler on and LLFE_TIMELINE
set, so every kernel's start / end (hipEvents on its stream, ms after a base event) lands in
a file beside the serving thread's submit / collect times on the same clock (the base event
is synchronised right before the host clock starts).  Prints, per step, the batch's colour
front, stencil, k-means and the host calls.

    python tools/debug/pipe_timeline.py OUT.txt [steps] [inflight]
"""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

out = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
if len(sys.argv) > 3:
    os.environ["LLFE_INFLIGHT"] = sys.argv[3]
kt = out + ".kernels"
if os.path.exists(kt):
    os.remove(kt)
os.environ["LLFE_TIMELINE"] = kt

import torch  # noqa: E402

from low_level_feature_extraction_amd import synth  # noqa: E402
from low_level_feature_extraction_amd.backend import Backend  # noqa: E402
from low_level_feature_extraction_amd.pipeline import assemble_batch  # noqa: E402

feats = ("colors", "shapes", "shadows")
be = Backend.get(0)
x = synth.synth_batch(512, 1080, 1920, seed=2025, device="cuda:0")
torch.cuda.synchronize()
pool = ThreadPoolExecutor(max_workers=1)


def loop(n, seed0, log):
    pending, futs = [], []
    for k in range(n):
        a = time.perf_counter()
        pending.append(be.submit(x, feats, seed=seed0 + k))
        b = time.perf_counter()
        log.append(("submit", k, a, b))
        if len(pending) == be.inflight:
            c = time.perf_counter()
            recs = be.collect(pending.pop(0))
            d = time.perf_counter()
            log.append(("collect", k - be.inflight + 1, c, d))
            futs.append(pool.submit(assemble_batch, recs, feats))
    while pending:
        c = time.perf_counter()
        recs = be.collect(pending.pop(0))
        d = time.perf_counter()
        log.append(("collect", n - len(pending) - 1, c, d))
        futs.append(pool.submit(assemble_batch, recs, feats))
    for f in futs:
        f.result()


loop(3, 100, [])  # warm-up
if os.environ.get("PIPE_FREEZE") == "1":  # as bench.py: the startup heap out of the collector's passes
    import gc

    gc.collect()
    gc.freeze()
be.set_profiling(True)
t0 = time.perf_counter()
log = []
loop(steps, 0, log)
torch.cuda.synchronize()
t1 = time.perf_counter()
be.set_profiling(False)
print("freeze", os.environ.get("PIPE_FREEZE", "0"), "inflight", be.inflight, "steps", steps, "ms/step %.2f" % ((t1 - t0) / steps * 1e3), "images/s %.0f" % (512 * steps / (t1 - t0)))
ker = []
for line in open(kt):
    if line.startswith("#"):
        continue
    name, slot, a, b = line.split()
    ker.append((float(a), float(b), name, int(slot)))
ker.sort()
with open(out, "w") as f:
    for kind, k, a, b in log:
        f.write("host %s %d %.3f %.3f\n" % (kind, k, (a - t0) * 1e3, (b - t0) * 1e3))
    for a, b, name, slot in ker:
        f.write("gpu %s %d %.3f %.3f\n" % (name, slot, a, b))
# per batch: the kernels in submission order (k-th launch of each name = batch k)
seen = {}
rows = {}
for a, b, name, slot in ker:
    i = seen.get(name, 0)
    seen[name] = i + 1
    rows.setdefault(i, []).append((name, a, b))
sub = {k: (a - t0) * 1e3 for kind, k, a, b in log if kind == "submit"}
col = {k: ((a - t0) * 1e3, (b - t0) * 1e3) for kind, k, a, b in log if kind == "collect"}
for i in sorted(rows):
    r = {n: (a, b) for n, a, b in rows[i]}
    def g(n, j):
        return "%8.2f" % r[n][j] if n in r else "       -"
    print("batch %d: submit %8.2f | scatter %s-%s part -%s kmeans %s-%s | stencil %s-%s hyst-end %s | collect %s-%s" % (
        i, sub.get(i, -1), g("k_uq_scatter", 0), g("k_uq_scatter", 1), g("k_uq_part", 1), g("k_kmeans", 0),
        g("k_kmeans", 1), g("k_stencil", 0), g("k_stencil", 1), g("k_hysteresis_dilate", 1),
        "%8.2f" % col[i][0] if i in col else "-", "%8.2f" % col[i][1] if i in col else "-"))
