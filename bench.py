#!/usr/bin/env python3
"""Benchmark: images/sec on the full colors+shapes+shadows hot path, 1080p batches.

One step = one pass of the hot path over one batch of synthetic 1920x1080 BGR images
already resident in HBM: colour palette (noise -> unique colours -> 10-attempt k-means),
shapes (gray/blur/Canny/dilate on the GPU, contours + geometry on the host thread pool)
and shadows (adaptive-threshold statistics), ending with every per-image result on the
host.  Per-GPU batch is fixed (weak scaling): BASELINE.json config 4 is 4096 images over
8 GPUs = 512 per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

--gpus is authoritative: without a launcher (no WORLD_SIZE) and N > 1 the script starts N
ranks itself under torch.distributed.run (child processes, before any GPU call); under a
launcher WORLD_SIZE must equal N.

Rank 0 prints ONE JSON line.  Kernel durations come from hipEvents recorded by
libllfe on the launch stream during the timed steps (llfe_set_profiling); the
`cpu_baseline` leg runs the CPU oracle (C restatement of the reference's
OpenCV/NumPy path) on a bounded sample on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec, 1080p batch, full colors+shapes+shadows pipeline @1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# HBM bytes per launch measured with rocprofv3 PMC counters (tools/profile.sh ->
# profiles/traffic_latest.json); None when unmeasured.
def _load_traffic():
    try:
        with open(os.path.join(ROOT, "profiles", "traffic_latest.json")) as f:
            k = json.load(f)["kernels"]
        return ({n: round(v["bytes"]) for n, v in k.items()},
                {n: v["valu_insts"] for n, v in k.items() if "valu_insts" in v})
    except (OSError, KeyError, ValueError):
        return {}, {}


# VALU issue capacity, measured here (tools/debug/valu_rate.hip ->
# profiles/r2/r2b/valu_rate.txt, 8 waves per SIMD, shader clock 2.21 GHz under load):
# only plain VOP2 add / sub / logic / mov / lshr / f32 add-mul / u16 ops issue every 2
# cycles; FMA, mad, min/max u32, compares, converts, bfe / perm / alignbit, DPP, SDWA,
# SGPR operands and every packed (pk_) op take 4.  The stencil and k-means streams are
# ~90 % the 4-cycle kind, so capacity = 256 CUs x 4 SIMDs / 4 cycles x 2.21 GHz.
VALU_SLOTS_PER_S = 256 * 4 / 4 * 2.21e9
TRAFFIC, VALU_INSTS = _load_traffic()


def _cpu_worker(args):
    i, h, w, feats, png = args
    import numpy as np

    from low_level_feature_extraction_amd import synth
    from oracle import oracle as O

    img = synth.synth_numpy(i, h, w, seed=4321)
    blob = synth.encode_png(img) if png else None
    t = time.perf_counter()
    if png:  # cv2.imdecode stand-in (no cv2 on the box): Pillow's PNG decoder, BGR out
        import io

        from PIL import Image

        img = np.ascontiguousarray(np.asarray(Image.open(io.BytesIO(blob)).convert("RGB"))[:, :, ::-1])
    nu = 0
    if "colors" in feats:
        noise = O.numpy_noise(h * w, i)                              # color_extractor.py:224
        centers, counts, nu, _ = O.dominant_colors(img, noise, 5, O.image_rng_state(0, i))
        O.color_palette(centers, counts)                             # :231-284
    if "shapes" in feats:
        O.analyze_shapes(img)                                        # shape pyc @L125-189
    if "shadows" in feats:
        O.analyze_shadow_level(img)                                  # shadow pyc @L12-31
    return time.perf_counter() - t, int(nu)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def cpu_baseline(n_images, h, w, workers, feats=("colors", "shapes", "shadows"), png=False):
    """a process pool of single-threaded workers, one image per task,
    N = the cores this process may use (affinity / cgroup quota: on the GPU box
    os.cpu_count() reports the whole machine, of which one GPU's share is a slice).
    png=True: every task starts from PNG bytes (decode timed; Pillow stands in for
    cv2.imdecode, utils.py:108-109)."""
    import multiprocessing as mp

    from oracle import oracle as O

    O.lib()
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(i, h, w, tuple(feats), png) for i in range(n_images)], chunksize=1)
    wall = time.perf_counter() - t0
    mean = sum(r[0] for r in res) / len(res)
    return {
        # steady-state rate of the pool: every core busy on one image at a time
        "value": round(workers / mean, 3),
        "value_wall": round(n_images / wall, 3),  # incl. pool start and image synthesis
        "unit": "images/s",
        "cores": workers,
        "kind": "port",
        "input": "png bytes (Pillow decode timed)" if png else "decoded arrays",
        "cpu_model": cpu_model(),
        "os_cpu_count": os.cpu_count(),
        "sample": f"{n_images} synthetic {w}x{h} images ({(n_images + 1) // 2} ui / {n_images // 2} photo), "
                  f"{'+'.join(feats)} via the C oracle (oracle/llfe_oracle.c), {workers} single-threaded worker "
                  f"processes (one per usable core), {wall:.1f}s wall (incl. pool start and the images' "
                  f"synthesis, outside the per-image timer); mean per-image time {mean:.2f}s; value = cores / "
                  f"mean per-image time",
    }


def _encode(args):
    i, h, w, seed, fmt = args
    import io

    from PIL import Image

    from low_level_feature_extraction_amd import synth

    b = io.BytesIO()
    im = Image.fromarray(synth.synth_numpy(i, h, w, seed=seed)[:, :, ::-1])
    if fmt == "JPEG":
        im.save(b, "JPEG", quality=85)
    else:
        im.save(b, fmt)
    return b.getvalue()


def e2e_host(be, imgs_dev, feats, steps, seed, index_base):
    """End-to-end from decoded host arrays: the batch sits in pinned host
    memory and every step pays its H2D inside libllfe (llfe_submit_batch copies host
    inputs into the workspace on its own stream); two batches in flight, so batch k+1's
    H2D overlaps batch k's kernels.  Reported beside `value`, never as it."""
    import torch

    host = [torch.empty(imgs_dev.shape, dtype=torch.uint8).pin_memory() for _ in range(2)]
    for hb in host:
        hb.copy_(imgs_dev.cpu())
    arrs = [hb.numpy() for hb in host]
    be.process(arrs[0][:2], feats, seed=seed)  # warm the host-input path
    # the PCIe ceiling of this path: one plain pinned H2D copy of a batch (best of 3)
    scratch = torch.empty_like(imgs_dev)
    peak = 0.0
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        scratch.copy_(host[0], non_blocking=True)
        torch.cuda.synchronize()
        peak = max(peak, host[0].numel() / (time.perf_counter() - t) / 1e9)
    del scratch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pending = []
    for k in range(steps):
        pending.append(be.submit(arrs[k % 2], feats, seed=seed + k, index_base=index_base))
        if len(pending) == 2:
            be.collect(pending.pop(0))
    while pending:
        be.collect(pending.pop(0))
    dt = time.perf_counter() - t0
    n, h, w = imgs_dev.shape[0], imgs_dev.shape[1], imgs_dev.shape[2]
    gb = n * h * w * 3 * steps / 1e9
    return {"value": round(n * steps / dt, 2), "unit": "images/s", "h2d_gbs": round(gb / dt, 2),
            "pcie_h2d_peak_gbs": round(peak, 2), "frac_of_pcie": round(gb / dt / peak, 3),
            "bound": "PCIe H2D (the batch's bytes at pcie_h2d_peak_gbs take longer than its kernels)",
            "sample": f"{steps} x {n} decoded {w}x{h} BGR arrays in pinned host memory (two alternating buffers), "
                      f"H2D + full GPU path per batch, two batches in flight (llfe_submit_batch / llfe_collect_batch)"}


def served_batcher(imgs_dev, feats, batches, seed, inflight, device, backend=None):
    """The product request path at load (the reference serves one
    image per /analyze call, app/api/v1/endpoints/analyze.py:94-111): P concurrent asyncio
    producers each await ``MicroBatcher.analyze`` on its own single 1080p device image
    (separately allocated, resident in HBM like `value`'s batch), back to back, until
    ``batches`` x B requests have completed.  The batcher forms launches of up to B
    (max_batch) and keeps ``inflight`` of them in flight through llfe_submit_images /
    llfe_collect_batch; every request's reference-shaped result dict is resolved inside
    the timed region.  Timed like `value` (synchronised clock around the requests)."""
    import asyncio
    import itertools

    import torch

    from low_level_feature_extraction_amd.batcher import MicroBatcher

    B = int(imgs_dev.shape[0])
    producers = (inflight + 1) * B  # enough outstanding requests to keep every slot full
    dev = [imgs_dev[i % B].clone() for i in range(producers)]  # one allocation per request image
    torch.cuda.synchronize()
    # the worker drives the rank's own context (`backend`; the main thread only waits on the
    # event loop meanwhile), so the leg adds no second set of device workspaces
    depth0 = backend.inflight if backend is not None else None
    bt = MicroBatcher(features=feats, max_batch=B, max_wait_ms=2.0, inflight=inflight, seed=seed, device=device,
                      backend=backend)

    async def drive(n_requests):
        counter = itertools.count()

        async def producer(img):
            while next(counter) < n_requests:
                await bt.analyze(img)

        await asyncio.gather(*(producer(t) for t in dev))

    try:
        asyncio.run(drive(2 * B))  # warm-up: the worker's context, workspaces, gc.freeze
        n0 = len(bt.batch_sizes)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        asyncio.run(drive(batches * B))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    finally:
        bt.close()
        if backend is not None:
            backend.inflight = depth0  # (the batcher set its own depth on the context)
    del dev
    torch.cuda.empty_cache()  # the request images' memory back to the device for the next legs
    sizes = bt.batch_sizes[n0:]
    log = [e for e in bt.launch_log[n0:] if e[2] is not None]
    # the worker's clock per launch: blocked in collect (the GPU still on it), and from one
    # collect's return to the next submit (gather + descriptors + llfe_submit_images)
    wait = [e[2] - e[1] for e in log]
    gap = [log[k + 1][0] - log[k][2] for k in range(len(log) - 1) if log[k + 1][0] > log[k][2]]
    worker = {"collect_wait_ms": round(1e3 * sum(wait) / max(len(wait), 1), 3),
              "collect_to_next_submit_ms": round(1e3 * sum(gap) / max(len(gap), 1), 3)}
    return {"value": round(batches * B / dt, 2), "unit": "images/s", "requests": batches * B, "worker": worker,
            "producers": producers, "max_batch": B, "inflight": inflight,
            "launches": len(sizes), "mean_launch": round(sum(sizes) / max(len(sizes), 1), 1),
            "max_in_flight": bt.max_in_flight,
            "sample": f"{batches * B} single {imgs_dev.shape[2]}x{imgs_dev.shape[1]} device images from {producers} "
                      f"concurrent asyncio producers through MicroBatcher.analyze (llfe_submit_images, images read in place + "
                      f"the full GPU path, {inflight} launches in flight, results assembled per request)"}


def e2e_png(be, B, H, W, feats, steps, distinct, seed, fmt="PNG", decode_steps=2, contours=None):
    """End-to-end from encoded bytes (PNG, or JPEG quality 85):
    host decode on the decode thread pool into pinned host batches, driven through the
    same serving loop as `value` (llfe_submit_batch / llfe_collect_batch, two batches in
    flight), so decoding batch k + 1 overlaps batch k's H2D and kernels.  Beside it, the
    warm decode-only rate of the same threads: the e2e value is decode-bound when it is
    within 10 % of that rate.  `split` times the leg's phases on the serving thread (waiting
    for the decode of the next batch, submit, collect) and the decode producer itself, and
    the host contour pool's busy share.  contours: the contour mode for the leg ("gpu": the
    host cores all go to decoding; None: the context's).  Reported beside `value`, never
    as it."""
    from concurrent.futures import ThreadPoolExecutor

    import torch

    from low_level_feature_extraction_amd import decode

    with ThreadPoolExecutor(max_workers=min(distinct, decode.default_decode_threads())) as ex:
        blobs_d = list(ex.map(_encode, [(i, H, W, seed, fmt) for i in range(distinct)]))
    blobs = [blobs_d[i % distinct] for i in range(B)]
    threads = decode.default_decode_threads()
    # three pinned batches: decoding batch k + 1 may not reuse the buffer of a batch still in flight
    pinned = [torch.empty((B, H, W, 3), dtype=torch.uint8).pin_memory() for _ in range(3)]
    bufs = [p.numpy() for p in pinned]
    # warm, steady-state decode-only rate over all decode threads
    decode.decode_batch(blobs, bufs[0], threads)
    t = time.perf_counter()
    for k in range(decode_steps):
        decode.decode_batch(blobs, bufs[k % 3], threads)
    dec_rate = B * decode_steps / (time.perf_counter() - t)
    mode0 = be.contour_mode()
    if contours:
        be.set_contour_mode(contours)
    be.process(bufs[0][:2], feats, seed=seed)  # warm the host-input path
    dec_s = []

    def produce(buf):
        t = time.perf_counter()
        out = decode.decode_batch(blobs, buf, threads)
        dec_s.append(time.perf_counter() - t)
        return out

    wait = sub = col = 0.0
    be.host_contour_stats(reset=True)
    with ThreadPoolExecutor(max_workers=1) as prod:
        t0 = time.perf_counter()
        fut = prod.submit(produce, bufs[0])
        pending = []
        for k in range(steps):
            ta = time.perf_counter()
            batch = fut.result()
            tb = time.perf_counter()
            # decode batch k + 1 (started before batch k is submitted, so the decode threads
            # never wait on the submission) while batch k - 1 is collected: buffer
            # (k + 1) % 3 last held batch k - 2, collected one step earlier
            if k + 1 < steps:
                fut = prod.submit(produce, bufs[(k + 1) % 3])
            pending.append(be.submit(batch, feats, seed=seed + k))
            tc = time.perf_counter()
            if len(pending) == 2:
                be.collect(pending.pop(0))
            wait, sub, col = wait + tb - ta, sub + tc - tb, col + time.perf_counter() - tc
        tc = time.perf_counter()
        while pending:
            be.collect(pending.pop(0))
        col += time.perf_counter() - tc
        dt = time.perf_counter() - t0
    hc = be.host_contour_stats(reset=True)
    if contours:
        be.set_contour_mode(mode0)
    value = B * steps / dt
    mb = sum(len(p) for p in blobs_d) / distinct / 2**20
    # what the leg's time went to: its decodes (the producer runs them back to back while
    # the serving thread submits / collects), the pipeline's fill and drain (the first
    # batch's decode before any GPU work, the last batches' GPU path and collects after the
    # last decode), and decode slowed by sharing the cores (host contour pool, driver threads)
    dec_leg = sum(dec_s) / len(dec_s)
    decodes_share = steps * dec_leg / dt
    fill_drain_ms = (dt - steps * dec_leg) * 1e3
    slow = dec_leg / (B / dec_rate) - 1
    if decodes_share >= 0.85:
        bound = (f"host decode: the {threads} decode threads were busy {decodes_share:.2f} of the leg (back to back; "
                 f"the rest is the pipeline fill / drain, {fill_drain_ms:.0f} ms per {steps}-batch leg); a decode took "
                 f"{100 * slow:+.0f} % against decode alone (cores shared with the host contour pool and driver "
                 f"threads); e2e is {value / dec_rate:.2f} of the decode-only rate")
    else:
        bound = (f"not decode alone: decodes fill {decodes_share:.2f} of the leg; e2e is {value / dec_rate:.2f} of the "
                 f"decode-only rate (GPU path / host contour pool)")
    split = {"ms_per_step": round(dt / steps * 1e3, 2),
             "decode_ms_per_batch_in_leg": round(sum(dec_s) / len(dec_s) * 1e3, 2),
             "decode_ms_per_batch_alone": round(B / dec_rate * 1e3, 2),
             "decodes_share_of_leg": round(decodes_share, 3), "fill_drain_ms_per_leg": round(fill_drain_ms, 1),
             "serving_thread_ms_per_step": {"wait_for_decode": round(wait / steps * 1e3, 2),
                                            "submit": round(sub / steps * 1e3, 2),
                                            "collect": round(col / steps * 1e3, 2)},
             "host_contour_busy": round(hc["busy_ms"] / 1e3 / dt, 3)}
    return {"value": round(value, 2), "unit": "images/s", "decode_threads": threads,
            "decode_only": round(dec_rate, 2), "decode_ms_per_image_per_thread": round(threads / dec_rate * 1e3, 2),
            "codecs": decode.decoder_info(), "contours": contours or mode0, "bound": bound, "split": split,
            "sample": f"{steps} x {B} {fmt}-encoded {W}x{H} synthetic images ({distinct} distinct, {mb:.2f} MiB each), "
                      f"decoded on the host (libllfe {fmt} decoder, cv2.imdecode IMREAD_COLOR semantics) into pinned "
                      f"host batches, then the full GPU path incl. H2D, two batches in flight; decode-only: "
                      f"{decode_steps} warm batches on the same threads"}


def _config_name(B, H, W, feats, pre):
    full = set(feats) == {"colors", "shapes", "shadows"}
    if (H, W) == (1080, 1920) and full and pre == "auto":
        return "BASELINE configs[3]: 4096 x 1080p over 8 GPUs = 512 per GPU"
    if (H, W) == (2160, 3840) and full and pre == "high_quality":
        return "BASELINE configs[4]: 1024 x 4K high_quality over 8 GPUs = 128 per GPU"
    if (H, W) == (1080, 1920) and set(feats) == {"colors"}:
        return "BASELINE configs[1]: 256 x 1080p colours"
    if (H, W) == (1080, 1920) and set(feats) == {"colors", "shapes"}:
        return "BASELINE configs[2]: 256 x 1080p colours + shapes"
    return "custom"


def launch_ranks(n: int, argv: list[str]) -> list[str]:
    """The command that runs this script as `n` ranks of one node (one process per GPU,
    Dockerfile:26's process-per-worker model): torch.distributed.run on 127.0.0.1 with a
    free port, the same arguments."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def visible_gpus(env=os.environ, sysfs="/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPUs a rank could be given, counted without starting a HIP runtime (the launching
    parent must not touch the GPU): the kfd topology nodes with SIMDs (CPU nodes have
    none), or the length of a *_VISIBLE_DEVICES list when one is set."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() not in ("", "-1")])
    n = 0
    try:
        nodes = os.listdir(sysfs)
    except OSError:
        return 0
    for node in nodes:
        try:
            with open(os.path.join(sysfs, node, "properties")) as f:
                props = dict(line.split(None, 1) for line in f if len(line.split(None, 1)) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0").strip() or 0) > 0:
            n += 1
    return n


def check_world(gpus: int, env=os.environ) -> str:
    """--gpus is authoritative.  'launch': no launcher ran us and N > 1, so start N ranks
    (before anything touches the GPU); 'run': this process is one rank of the N asked for
    (or the single rank of N = 1).  A launcher whose WORLD_SIZE disagrees with --gpus is
    an error: the line would report a GPU count that did not run."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {gpus}")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "launch" if gpus > 1 else "run"
    if int(ws) != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} from the launcher but --gpus {gpus}; they must agree")
    return "run"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512, help="images per GPU per step")
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--features", default="colors,shapes,shadows")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-images", type=int, default=0, help="0: two images per worker")
    ap.add_argument("--cpu-workers", type=int, default=0, help="0: the usable cores (affinity / cgroup)")
    ap.add_argument("--cpu-input", choices=["decoded", "png", "both"], default="decoded",
                    help="CPU baseline input: decoded arrays, PNG bytes (decode timed), or both (cpu_baseline_png)")
    ap.add_argument("--preprocessing", default="auto", choices=["none", "auto", "high_quality", "performance"],
                    help="validate_and_preprocess_image mode the workload is quoted under (the bench checks that "
                         "it does not resize this size: BASELINE configs [3] auto at 1080p, [4] high_quality at 4K)")
    ap.add_argument("--e2e-host-steps", type=int, default=8, help="0 disables the decoded-host-array line")
    ap.add_argument("--seed", type=int, default=2025)
    ap.add_argument("--e2e-png-steps", type=int, default=8, help="0 disables the PNG end-to-end line")
    ap.add_argument("--e2e-jpeg-steps", type=int, default=10, help="0 disables the JPEG end-to-end line")
    ap.add_argument("--e2e-alt-contours", type=int, default=1,
                    help="1: also run the JPEG leg with the other contour mode (host <-> gpu)")
    ap.add_argument("--e2e-at-scale", nargs="?", const="on", default="on", choices=["on", "off"],
                    help="the e2e lines also at WORLD_SIZE > 1 (default on: every rank decodes its own shard "
                         "on its NUMA node's core share at the same time, which is the 8-rank node's host-side "
                         "contention -- decode cores, PCIe, pinned memory placement; each line then carries a "
                         "per-rank breakdown)")
    ap.add_argument("--per-class-steps", type=int, default=12,
                    help="steps of an all-ui and an all-photo batch (SURVEY.md 8d per-class throughput; 4 steps "
                         "left the pipeline's fill and drain in a third of the timed region: ui 21-30k across "
                         "round-5 runs); 0 disables")
    ap.add_argument("--batcher-inflight", type=int, default=2,
                    help="launches the batcher keeps in flight (MicroBatcher's default, 2 like `value`'s loop; "
                         "with four 256-thread k-means workgroups per CU a third launch in flight costs more "
                         "than it hides: 0.935 vs 0.99 of `value`, profiles/r6/batcher/depth_ab_kt256.txt)")
    ap.add_argument("--batcher-steps", type=int, default=None,
                    help="launches of B requests the served_batcher line times (default: 2 x --steps: its "
                         "fill and drain -- producers ramping up, the last launches' futures -- are longer "
                         "than `value`'s; at 20 launches the ratio spread 0.88-0.97 between runs); 0 disables the line "
                         "(single-image requests through MicroBatcher)")
    ap.add_argument("--contours", choices=["auto", "host", "gpu"], default="auto",
                    help="where findContours + the shape loop run: the host pool from the copied-back mask "
                         "(overlaps k-means), the GPU (contours_gpu.hip), or auto (the library's choice: "
                         "host unless the rank has < 4 host cores)")
    ap.add_argument("--pipeline", choices=["on", "off"], default="on",
                    help="on: a serving loop with two batches in flight (llfe_submit_batch / "
                         "llfe_collect_batch: batch k+1's front kernels fill the tail of batch k's k-means; "
                         "kernel timings then come from the same steps run one batch at a time); "
                         "off: one llfe_process_batch per step")
    ap.add_argument("--inflight", choices=["auto", "2", "3"], default="auto",
                    help="batches the pipelined loop keeps in flight: auto = 3 for batches of at most 102 "
                         "images (k-means' attempts all resident at once, its 512-thread build; 64 x 512^2: "
                         "41.6k vs 32.5k), else 2 (the 256-thread k-means packs beside the next batch's "
                         "kernels and a third batch only contends: 256 x 1080p colours+shapes 26.8k vs 22.1k, "
                         "512 x 1080p 27.3k vs 25.4k; profiles/r6/kmeans_wg/depth_small.txt)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch the ranks, initialise the process group and run the control-plane collectives "
                         "(barrier, MAX over ranks), print the line's identity fields with value null; no workload")
    args = ap.parse_args()

    if check_world(args.gpus) == "launch":
        # no GPU call has happened in this process: the ranks are children, and this
        # process only waits for them and exits with their status
        # (the parent never touches the GPU -- counting devices through torch would start a
        # HIP runtime here -- it reads the kfd topology; each rank then checks that its
        # LOCAL_RANK names a GPU its own runtime sees)
        import subprocess

        if os.environ.get("LLFE_BENCH_SHARE_GPU") != "1":
            have = visible_gpus()
            # (0: no kfd topology readable here -- leave the check to the ranks' own runtimes)
            if 0 < have < args.gpus:
                raise SystemExit(f"bench.py: --gpus {args.gpus} but {have} GPUs are visible")

        sys.exit(subprocess.call(launch_ranks(args.gpus, sys.argv[1:])))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and args.e2e_at_scale == "off":
        args.e2e_host_steps = args.e2e_png_steps = args.e2e_jpeg_steps = 0
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N-rank path on a one-GPU box: every rank on cuda:0, gloo for the
    # control-plane collectives (RCCL refuses two ranks on one device)
    share_gpu = os.environ.get("LLFE_BENCH_SHARE_GPU") == "1"
    if share_gpu:
        local = 0
    # host placement before any thread pool or pinned buffer exists: this rank's threads
    # (decode, contour pool, the serving loop) on its GPU's NUMA node, that node's cores
    # split among the ranks whose GPUs sit on it (placement.py; LLFE_NUMA_BIND=0: off)
    from low_level_feature_extraction_amd import placement

    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    placed = placement.bind(int(os.environ.get("LOCAL_RANK", "0")), local_world,
                            [0] * local_world if share_gpu else None)

    import torch

    # --dry-run on a host without a GPU: the rank / collective plumbing only (CPU tests)
    no_gpu = args.dry_run and not torch.cuda.is_available()
    if no_gpu:
        share_gpu = True
    else:
        if local >= torch.cuda.device_count():
            raise SystemExit(f"bench.py: rank {rank} needs GPU {local} but {torch.cuda.device_count()} are visible "
                             f"(--gpus {args.gpus}; LLFE_BENCH_SHARE_GPU=1 rehearses N ranks on one GPU)")
        torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if share_gpu:
            dist.init_process_group("gloo")  # (host tensors for its collectives: coll_dev)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if args.dry_run:
        from low_level_feature_extraction_amd import shard

        base, stop = shard.shard_bounds(args.batch * world, rank, world)
        shard.barrier(device=None if no_gpu else local)
        t = shard.max_over_ranks(float(rank), device=None if share_gpu else f"cuda:{local}")
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "dry_run": True, "n_gpus": world,
                              "max_over_ranks_probe": t,
                              "config": {"global_batch": args.batch * world, "batch_per_gpu": args.batch,
                                         "parallelism": f"replicas x{world} (host-side shard, no collective)"}}))
        if dist is not None:
            dist.destroy_process_group()
        return

    from low_level_feature_extraction_amd import shard, synth
    from low_level_feature_extraction_amd.backend import Backend

    be = Backend.get(local)
    depth = (3 if args.batch * 10 <= 1024 else 2) if args.inflight == "auto" else int(args.inflight)
    if args.pipeline == "on":
        be.inflight = depth
    if args.contours != "auto":
        be.set_contour_mode(args.contours)
    feats = tuple(f for f in args.features.split(",") if f)
    B, H, W = args.batch, args.height, args.width
    from low_level_feature_extraction_amd.backend import preprocess_size

    if preprocess_size(W, H, args.preprocessing) is not None:
        raise SystemExit(f"preprocessing={args.preprocessing!r} would resize {W}x{H}; bench the resized size instead")
    base, _ = shard.shard_bounds(B * world, rank, world)  # weak scaling: B images per rank
    imgs = synth.synth_batch(B, H, W, seed=args.seed, device=f"cuda:{local}", index_base=base)
    torch.cuda.synchronize()

    coll_dev = None if share_gpu else f"cuda:{local}"  # device of the MAX-over-ranks tensor

    def barrier():
        shard.barrier(device=local)

    from concurrent.futures import ThreadPoolExecutor

    from low_level_feature_extraction_amd.pipeline import assemble_batch

    asm_pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="llfe-assemble")
    asm_log = []  # (CPU ms of one batch's assembly)

    def assemble_step(recs):
        """The reference-shaped results of one collected batch:
        ColorFeatures by the palette rules (color_extractor.py:231-284), the analyze_shapes
        dict (shape pyc @L184-189) and {"shadow_level": ...} (shadow pyc @L21-31), as
        process_feature_results receives them (utils.py:155-214)."""
        t = time.thread_time()
        out = assemble_batch(recs, feats)
        asm_log.append((time.thread_time() - t) * 1e3)
        return sum(len(o["shapes"]["shapes"]) for o in out) if "shapes" in feats else 0

    def run_steps(k_steps, seed0, pipelined, batch=None):
        """k_steps full passes over the batch (``imgs`` unless given), each ending with every
        image's reference-shaped result objects on the host (assembled on a worker thread
        while the GPU runs the next batches; the caller's timed region waits for them).
        Pipelined: a serving loop that keeps be.inflight batches in flight (llfe_submit_batch /
        llfe_collect_batch), so batch k + 1's front kernels start in the tail of batch k's
        k-means."""
        batch = imgs if batch is None else batch
        futs = []
        if not pipelined:
            for k in range(k_steps):
                futs.append(asm_pool.submit(assemble_step, be.process(batch, feats, seed=seed0 + k, index_base=base)))
        else:
            pending = []
            ts = tc = 0.0  # serving thread: wall time in submit / collect
            for k in range(k_steps):
                t_a = time.perf_counter()
                pending.append(be.submit(batch, feats, seed=seed0 + k, index_base=base))
                t_b = time.perf_counter()
                ts += t_b - t_a
                if len(pending) == be.inflight:
                    recs = be.collect(pending.pop(0))
                    tc += time.perf_counter() - t_b
                    futs.append(asm_pool.submit(assemble_step, recs))
            while pending:
                t_b = time.perf_counter()
                recs = be.collect(pending.pop(0))
                tc += time.perf_counter() - t_b
                futs.append(asm_pool.submit(assemble_step, recs))
            run_steps.serving = {"submit_ms_per_step": round(ts / k_steps * 1e3, 3),
                                 "collect_ms_per_step": round(tc / k_steps * 1e3, 3)}
        t_last = time.perf_counter()
        shapes = sum(f.result() for f in futs)
        run_steps.tail_ms = (time.perf_counter() - t_last) * 1e3  # assembly left after the last collect
        return shapes

    pipelined = args.pipeline == "on"
    run_steps(args.warmup, args.seed + 1000, pipelined)
    # A serving process's startup heap (torch, numpy, this package: ~180k objects) never
    # becomes garbage; left in the collector's oldest generation, every full collection
    # walks it -- a 45-90 ms stop of the serving thread (holding the GIL inside collect's
    # result conversion) every few steps, long enough to drain both in-flight batches and
    # idle the GPU (round 5, tools/debug/pipe_timeline.py).  gc.freeze() moves it out of
    # the collector's passes (what long-running Python servers do after start-up); every
    # object the steps allocate is still collected.
    import gc

    gc.collect()
    gc.freeze()
    barrier()
    # hipEvent kernel timings: in the one-batch-at-a-time steps only (two batches in flight
    # overlap, so an event-timed span would include the other batch's kernels)
    be.set_profiling(not pipelined)
    be.host_contour_stats(reset=True)
    asm_log.clear()
    t0 = time.perf_counter()
    n_shapes = run_steps(args.steps, args.seed, pipelined)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    host_ct = be.host_contour_stats(reset=True)
    asm_ms, asm_tail = list(asm_log), run_steps.tail_ms
    serving = getattr(run_steps, "serving", None) if pipelined else None
    barrier()
    dt = shard.max_over_ranks(t1 - t0, device=coll_dev)
    stats = be.kernel_stats()
    # the same steps one batch at a time (llfe_process_batch): the reference rate and,
    # when pipelined, the kernel timings
    dt_sync = None
    if pipelined:
        be.set_profiling(True)
        barrier()
        ts0 = time.perf_counter()
        run_steps(args.steps, args.seed, False)
        torch.cuda.synchronize()
        ts1 = time.perf_counter()
        barrier()
        dt_sync = shard.max_over_ranks(ts1 - ts0, device=coll_dev)
        stats = be.kernel_stats()
        be.set_profiling(False)
    dt_kernels = dt_sync if pipelined else dt  # the steps the kernel timings come from
    # one extra, untimed step with every kernel in order on one stream: isolated kernel
    # durations for the secondary rooflines (in the timed steps the shapes kernels share
    # the GPU with the colour front, which stretches their event-timed spans)
    be.set_concurrency(False)
    be.set_profiling(True)
    be.process(imgs, feats, seed=args.seed, index_base=base)
    torch.cuda.synchronize()
    iso = be.kernel_stats()
    be.set_concurrency(True)
    be.set_profiling(False)

    # the product request path at the same load: single-image requests through the
    # MicroBatcher, beside `value`
    served = None
    if args.batcher_steps is None:
        args.batcher_steps = 2 * args.steps
    if args.batcher_steps > 0 and pipelined:
        barrier()
        served = served_batcher(imgs, feats, args.batcher_steps, args.seed, args.batcher_inflight, local, backend=be)
        barrier()

    # per-class throughput: the same step on an all-"ui" and an all-"photo"
    # batch of the same size (k-means cost scales with the unique-colour count U)
    per_class = None
    if args.per_class_steps > 0:
        per_class = {}
        for kind in ("ui", "photo"):
            cb = synth.synth_batch(B, H, W, seed=args.seed, device=f"cuda:{local}", index_base=base, kind=kind)
            run_steps(2, args.seed + 2000, pipelined, cb)  # warm-up
            torch.cuda.synchronize()
            barrier()
            # the headline's serving loop (two batches in flight when pipelined): a class
            # bound by the host contour pool shows it here, not the serial tail of one batch
            be.host_contour_stats(reset=True)
            tc0 = time.perf_counter()
            run_steps(args.per_class_steps, args.seed + 3000, pipelined, cb)
            torch.cuda.synchronize()
            tc1 = time.perf_counter()
            hc = be.host_contour_stats(reset=True)
            barrier()
            dtc = shard.max_over_ranks(tc1 - tc0, device=coll_dev)
            per_class[kind] = {"value": round(B * world * args.per_class_steps / dtc, 2), "unit": "images/s",
                               "ms_per_step": round(dtc / args.per_class_steps * 1e3, 3), "pipelined": pipelined,
                               # wall share of the timed steps the host contour pool was tracing
                               "host_contour_busy": round(hc["busy_ms"] / 1e3 / (tc1 - tc0), 3),
                               "host_contour_ms_per_image": round(hc["busy_ms"] * hc["threads"] / max(hc["images"], 1), 3)}
            del cb

    # (the e2e lines run on every rank before rank 0 reports: each rank pays its own
    # host-side work, as a serving node would)

    total_images = B * world * args.steps
    # the committed PMC profile (tools/profile.sh) is of the default workload: its per-launch
    # traffic and VALU counts only describe launches of that shape
    profiled = (B, args.height, args.width, args.features, args.preprocessing) == \
        (512, 1080, 1920, "colors,shapes,shadows", "auto")
    traffic, valu_insts = (TRAFFIC, VALU_INSTS) if profiled else ({}, {})

    def roof(name, src=None):
        """HBM roofline of one kernel: algorithmic bytes per launch
        / its average hipEvent-timed launch duration."""
        st = (src or stats)[name]
        avg_ms = st["total_ms"] / max(st["launches"], 1)
        bpl = st["bytes"] / max(st["launches"], 1)
        achieved = bpl / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        r = {"kernel": name, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic.get(name),
             "bytes_per_launch": bpl, "avg_launch_ms": round(avg_ms, 4)}
        if name in valu_insts and avg_ms > 0:
            # PMC SQ_INSTS_VALU per launch (profiles/traffic_latest.json) over the launch's
            # VALU issue capacity (VALU_SLOTS_PER_S): how close the kernel is to its compute bound
            r["valu_busy"] = round(valu_insts[name] / (VALU_SLOTS_PER_S * avg_ms * 1e-3), 3)
        if traffic.get(name) and avg_ms > 0:  # what the counters saw, beside the algorithmic rate
            r["hbm_gbs_pmc"] = round(traffic[name] / (avg_ms * 1e-3) / 1e9, 1)
        if "valu_busy" in r:
            # the limiter the counters show: the busier of VALU issue and the HBM bytes the
            # counters saw (without a traffic count, VALU when it is > 70 % busy); frac stays
            # the HBM fraction of the algorithmic bytes, against HBM peak
            hbm_util = r["hbm_gbs_pmc"] / HBM_PEAK_GBS if "hbm_gbs_pmc" in r else 0.7
            if r["valu_busy"] > hbm_util:
                r["bound"] = "valu"
        return r

    kernels = {}
    for name, st in stats.items():
        r = roof(name)
        alg = r["achieved"] if st["bytes"] else None
        pmc = (round(traffic[name] / (r["avg_launch_ms"] * 1e-3) / 1e9, 1)
               if traffic.get(name) and r["avg_launch_ms"] > 0 else None)
        kernels[name] = {"launches": st["launches"], "avg_ms": r["avg_launch_ms"],
                         "share_of_step": round(st["total_ms"] / (dt_kernels * 1e3), 4),
                         # gbs: the HBM bytes the PMC counters saw per launch (the committed
                         # profile of this workload, profiles/traffic_latest.json) over the same
                         # average duration -- what the kernel moved; without a profile, the
                         # algorithmic rate.  algorithmic_gbs / frac: SURVEY.md 8d's bytes, the
                         # roofline's definition; a kernel that moves less than its algorithmic
                         # bytes (k_kmeans: the cube tables stand in for its repeated key passes)
                         # shows a higher algorithmic than measured rate
                         "gbs": pmc if pmc is not None else alg,
                         "gbs_source": "pmc" if pmc is not None else ("algorithmic" if alg is not None else None),
                         "algorithmic_gbs": alg, "frac": r["frac"] if st["bytes"] else None}
    # `roofline` is the dominant kernel's (largest total time); k_kmeans' algorithmic
    # bytes are SURVEY.md 8d's 4U per fused multi-attempt pass x (K k-means++ passes + the
    # longest attempt's Lloyd sweeps), k_kmeans_finalize.
    dominant = max(stats, key=lambda k: stats[k]["total_ms"]) if stats else None
    roofline = roof(dominant) if dominant else None
    roofline_stencil = None
    if "k_stencil" in iso:
        roofline_stencil = roof("k_stencil", iso)
        roofline_stencil["measured"] = "isolated step (all kernels on one stream), after the timed region"
    for name, st in iso.items():
        if name in kernels:
            kernels[name]["isolated_ms"] = round(st["total_ms"] / max(st["launches"], 1), 4)

    cpu = cpu_png = None
    if args.cpu_baseline == "auto" and world == 1:
        from low_level_feature_extraction_amd.decode import usable_cores

        workers = args.cpu_workers or usable_cores()
        n_cpu = args.cpu_images or 2 * workers
        if args.cpu_input in ("decoded", "both"):
            cpu = cpu_baseline(n_cpu, H, W, workers, feats)
        if args.cpu_input in ("png", "both"):
            cpu_png = cpu_baseline(n_cpu, H, W, workers, feats, png=True)
            if cpu is None:
                cpu = cpu_png

    def all_ranks(line, steps):
        """Whole-job rate of an e2e line every rank ran at once (`steps` batches of B per
        rank): images of all ranks over the slowest rank's time."""
        if line is None or world == 1:
            return line
        t = B * steps / line["value"]
        line = dict(line)
        line["value"] = round(B * world * steps / shard.max_over_ranks(t, device=coll_dev), 2)
        # each rank's own rate and host placement (its GPU's NUMA node and CPU share)
        line["per_rank"] = shard.all_gather({"rank": rank, "value": round(B * steps / t, 2),
                                             "numa_node": (placed or {}).get("numa_node"),
                                             "cpus": (placed or {}).get("cpus")})
        return line

    served = all_ranks(served, args.batcher_steps)
    barrier()
    e2e_h = None
    if args.e2e_host_steps > 0:
        e2e_h = all_ranks(e2e_host(be, imgs, feats, args.e2e_host_steps, args.seed, base), args.e2e_host_steps)
    barrier()
    e2e = e2e_j = None
    if args.e2e_png_steps > 0:  # every rank decodes its own shard with its core share
        e2e = all_ranks(e2e_png(be, B, H, W, feats, args.e2e_png_steps, 8, args.seed), args.e2e_png_steps)
    barrier()
    if args.e2e_jpeg_steps > 0:
        e2e_j = all_ranks(e2e_png(be, B, H, W, feats, args.e2e_jpeg_steps, 8, args.seed, fmt="JPEG"), args.e2e_jpeg_steps)
    e2e_j_alt = None
    if args.e2e_jpeg_steps > 0 and args.e2e_alt_contours and "shapes" in feats:
        # the same JPEG leg with the other contour mode: whether the host contour pool's
        # share of the cores is what keeps the leg below its decode-only rate
        alt = "gpu" if be.contour_mode() == "host" else "host"
        e2e_j_alt = all_ranks(e2e_png(be, B, H, W, feats, args.e2e_jpeg_steps, 8, args.seed, fmt="JPEG",
                                      contours=alt), args.e2e_jpeg_steps)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    out = {
        "metric": METRIC,
        "value": round(total_images / dt, 2),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "pipelined": pipelined,
        "inflight": be.inflight if pipelined else 1,
        "value_one_batch_at_a_time": round(total_images / dt_sync, 2) if dt_sync else None,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": f"{B} x {W}x{H} BGR images per GPU per step, features={list(feats)}, "
                        f"preprocessing={args.preprocessing!r} (no resize at this size), 50% ui / 50% photo "
                        f"synthetic mix ({_config_name(B, H, W, feats, args.preprocessing)})",
            "preprocessing": args.preprocessing,
            "global_batch": B * world,
            "batch_per_gpu": B,
            "height": H,
            "width": W,
            "features": list(feats),
            "parallelism": f"replicas x{world} (host-side shard, no collective)",
            "contours": be.contour_mode(),
        },
        "roofline": roofline,
        "roofline_stencil": roofline_stencil,
        "dominant_kernel": dominant,
        "kernels": kernels,
        "shapes_per_image": round(n_shapes / (B * args.steps), 2),
        # rows a6 / a10 inside the timed steps: every image's ColorFeatures / shapes dict /
        # {"shadow_level"} built on a worker thread beside the serving loop
        "serving_thread": serving,
        "result_assembly": {"host_cpu_ms_per_step": round(sum(asm_ms) / max(len(asm_ms), 1), 3),
                            "us_per_image": round(sum(asm_ms) / max(len(asm_ms), 1) / B * 1e3, 2),
                            "tail_ms_after_last_collect": round(asm_tail, 3),
                            "in_timed_region": True},
        "per_class": per_class,
        "served_batcher": served,
        # this rank's host placement (placement.py): GPU -> NUMA node -> its share of that
        # node's cores, the threads its pools take; every rank's in the e2e lines' per_rank
        "placement": placed,
        # wall share of the timed steps the host contour pool spent tracing (host mode)
        "host_contour_busy": round(host_ct["busy_ms"] / 1e3 / max(t1 - t0, 1e-9), 3),
        "cpu_baseline": cpu,
        "cpu_baseline_png": cpu_png if args.cpu_input == "both" else None,
        "e2e_host": e2e_h,
        "e2e_png": e2e,
        "e2e_jpeg": e2e_j,
        "e2e_jpeg_other_contour_mode": e2e_j_alt,
    }
    if served is not None:
        served["ratio_to_value"] = round(served["value"] / out["value"], 3)
    print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
