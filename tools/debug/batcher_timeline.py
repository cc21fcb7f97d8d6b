"""GPU box (round 6): where the served_batcher leg loses to `value`.  Runs, in one process,
the bench's serving loop on a resident 512 x 1080p batch and then the MicroBatcher leg
(asyncio producers, single device images, depth 3), each for N launches with libllfe's
profiler on and LLFE_TIMELINE set, and prints per mode: wall ms per launch, the GPU's busy
share (union of kernel intervals), the mean duration of the big kernels, and the gaps in
which no kernel ran.

    python tools/debug/batcher_timeline.py OUT_PREFIX [launches]
"""
import asyncio
import itertools
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

out = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
kt = out + ".kernels"
if os.path.exists(kt):
    os.remove(kt)
os.environ["LLFE_TIMELINE"] = kt

import torch  # noqa: E402

from low_level_feature_extraction_amd import synth  # noqa: E402
from low_level_feature_extraction_amd.backend import Backend  # noqa: E402
from low_level_feature_extraction_amd.batcher import MicroBatcher  # noqa: E402
from low_level_feature_extraction_amd.pipeline import assemble_batch  # noqa: E402

feats = ("colors", "shapes", "shadows")
B = 512
x = synth.synth_batch(B, 1080, 1920, seed=2025, device="cuda:0")
torch.cuda.synchronize()


def read_kernels():
    ker = []
    if not os.path.exists(kt):
        return ker
    for line in open(kt):
        if line.startswith("#"):
            ker.append(None)
            continue
        name, slot, a, b = line.split()
        ker.append((float(a), float(b), name))
    return ker


def summarize(tag, ker, wall_ms):
    ker = sorted(k for k in ker if k)
    if not ker:
        print(tag, "no kernels")
        return
    t0, t1 = ker[0][0], max(k[1] for k in ker)
    busy, cur_a, cur_b, gaps = 0.0, ker[0][0], ker[0][1], []
    for a, b, _ in ker[1:]:
        if a > cur_b:
            busy += cur_b - cur_a
            gaps.append(a - cur_b)
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    busy += cur_b - cur_a
    by = {}
    for a, b, name in ker:
        by.setdefault(name, []).append(b - a)
    big = {k: round(sum(v) / len(v), 3) for k, v in by.items() if k in ("k_kmeans", "k_uq_part", "k_uq_scatter", "k_stencil", "k_hysteresis_dilate")}
    gaps.sort(reverse=True)
    print("%s: wall %.2f ms/launch, GPU span %.1f ms busy %.3f, gaps > 0.1 ms: %d (sum %.1f ms, largest %s), kernels %s"
          % (tag, wall_ms, t1 - t0, busy / (t1 - t0), sum(1 for g in gaps if g > 0.1), sum(g for g in gaps if g > 0.1),
             [round(g, 2) for g in gaps[:5]], big))


# --- the bench's serving loop (value)
be = Backend.get(0)


def loop(k_steps, seed0):
    pending, res = [], []
    for k in range(k_steps):
        pending.append(be.submit(x, feats, seed=seed0 + k))
        if len(pending) == be.inflight:
            res.append(assemble_batch(be.collect(pending.pop(0)), feats))
    while pending:
        res.append(assemble_batch(be.collect(pending.pop(0)), feats))


loop(3, 100)
import gc  # noqa: E402

gc.collect()
gc.freeze()
be.set_profiling(True)
t = time.perf_counter()
loop(n, 0)
torch.cuda.synchronize()
wall = (time.perf_counter() - t) * 1e3 / n
be.set_profiling(False)
summarize("value (depth %d)" % be.inflight, read_kernels(), wall)
os.remove(kt)

# --- the MicroBatcher leg (as bench.served_batcher), its worker on a context made here
depth = int(os.environ.get("BT_DEPTH", "3"))
producers = (depth + 1) * B
dev = [x[i % B].clone() for i in range(producers)]
torch.cuda.synchronize()
bbe = Backend(0)
bt = MicroBatcher(features=feats, max_batch=B, max_wait_ms=2.0, inflight=depth, seed=7, backend=bbe)


async def drive(n_requests):
    counter = itertools.count()

    async def producer(img):
        while next(counter) < n_requests:
            await bt.analyze(img)

    await asyncio.gather(*(producer(t) for t in dev))


asyncio.run(drive(2 * B))
torch.cuda.synchronize()
n0 = len(bt.batch_sizes)
bbe.set_profiling(True)
t = time.perf_counter()
asyncio.run(drive(n * B))
torch.cuda.synchronize()
wall = (time.perf_counter() - t) * 1e3 / n
bbe.set_profiling(False)
bt.close()
log = [e for e in bt.launch_log[n0:] if e[2] is not None]
wait = [e[2] - e[1] for e in log]
summarize("batcher (depth %d, launches %s)" % (depth, bt.batch_sizes[n0:]), read_kernels(), wall)
print("batcher worker: collect wait %.2f ms/launch" % (1e3 * sum(wait) / max(len(wait), 1)))
