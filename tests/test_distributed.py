"""N>1 path on CPU: world_size-2 gloo process groups exercising the sharding,
timing reduction and result gather that bench.py and run_sharded use on RCCL."""
import os

import numpy as np
import socket

import pytest
import torch.multiprocessing as mp

from low_level_feature_extraction_amd.shard import shard_bounds


def test_shard_bounds_partition():
    for n in range(0, 40):
        for world in range(1, 9):
            spans = [shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(4, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from low_level_feature_extraction_amd import shard

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # stand-in per-image work: a record derived only from the global index, as the
        # real pipeline's results are (seeds are per global image index)
        def process(a, b):
            return [{"index": i, "rank": rank, "value": (i * 2654435761) % 1000} for i in range(a, b)]

        got = shard.run_sharded(n_total, process, gather_to=0)
        local = shard.run_sharded(n_total, process, gather_to=None)
        t = shard.max_over_ranks(1.5 if rank == 1 else 0.25)
        shard.barrier()
        q.put((rank, got, [r["index"] for r in local], t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [7, 64])
def test_gloo_world2_sharded_run(n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(2):
        rank, got, local, t = q.get(timeout=120)
        out[rank] = (got, local, t)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got0 = out[0][0]
    assert out[1][0] is None
    assert [r["index"] for r in got0] == list(range(n_total))
    assert [r["value"] for r in got0] == [(i * 2654435761) % 1000 for i in range(n_total)]
    a0, b0 = shard_bounds(n_total, 0, 2)
    assert out[0][1] == list(range(a0, b0)) and out[1][1] == list(range(b0, n_total))
    assert {r["rank"] for r in got0[:b0]} == {0} and {r["rank"] for r in got0[b0:]} == {1}
    assert out[0][2] == out[1][2] == 1.5  # MAX over ranks


def test_single_process_fallthrough():
    from low_level_feature_extraction_amd import shard

    assert shard.run_sharded(5, lambda a, b: list(range(a, b))) == [0, 1, 2, 3, 4]
    assert shard.max_over_ranks(3.0) == 3.0


def _cpu_records(a, b):
    """Per-image ImageFeatures records of the images [a, b) computed on the host only:
    shapes through libllfe's host contour path (llfe_shapes_from_mask, the code the
    batch runs on the host pool) over the oracle's dilated Canny mask, shadows from the
    oracle's statistics -- what a rank contributes, minus the GPU stages."""
    from low_level_feature_extraction_amd import backend, synth
    from low_level_feature_extraction_amd.backend import ImageFeatures
    from oracle import oracle as O

    out = []
    for i in range(a, b):
        img = synth.synth_numpy(i, 96, 160, seed=31)
        s, c = O.shadow_stats(img)
        shapes = backend.shapes_from_mask(O.shape_mask(img))
        out.append(ImageFeatures(np.zeros((0, 3), np.uint8), np.zeros(0, np.int64), 0, 0.0, s, c, shapes, 0, 160, 96))
    return out


def _worker_records(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
    import torch.distributed as dist

    from low_level_feature_extraction_amd import _lib, decode, shard

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        got = shard.run_sharded(n_total, _cpu_records, gather_to=0)
        # per-rank host thread budgets: the rank's share of the usable cores
        threads = (_lib.lib().llfe_default_host_threads(), decode.default_decode_threads(), decode.usable_cores())
        q.put((rank, got, threads))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gathers_real_records():
    import numpy as np  # noqa: F401

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n_total = 6
    procs = [ctx.Process(target=_worker_records, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(2):
        rank, got, threads = q.get(timeout=240)
        out[rank] = (got, threads)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = out[0][0]
    assert out[1][0] is None and len(got) == n_total
    want = _cpu_records(0, n_total)
    assert [r.shapes for r in got] == [r.shapes for r in want]
    assert [(r.shadow_sum, r.shadow_count) for r in got] == [(r.shadow_sum, r.shadow_count) for r in want]
    assert any(r.shapes for r in got)
    for rank in (0, 1):
        host, dec, usable = out[rank][1]
        assert host == max(1, min(usable // 2, 16))
        assert dec == max(1, min(usable // 2, 64))


def test_gloo_world8_local8_budgets_and_ordered_records():
    """8 ranks on one node (LOCAL_WORLD_SIZE=8, as torchrun --nproc-per-node 8 sets it):
    every rank's host contour pool and decode pool get usable cores / 8, and the real
    per-image records gather to rank 0 in global order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world, n_total = 8, 19  # ragged shards: 3 ranks hold 3 images, 5 hold 2
    procs = [ctx.Process(target=_worker_records, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, got, threads = q.get(timeout=300)
        out[rank] = (got, threads)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = out[0][0]
    assert all(out[r][0] is None for r in range(1, world)) and len(got) == n_total
    want = _cpu_records(0, n_total)
    assert [r.shapes for r in got] == [r.shapes for r in want]
    assert [(r.shadow_sum, r.shadow_count) for r in got] == [(r.shadow_sum, r.shadow_count) for r in want]
    for rank in range(world):
        host, dec, usable = out[rank][1]
        assert host == max(1, min(usable // world, 16))
        assert dec == max(1, min(usable // world, 64))
