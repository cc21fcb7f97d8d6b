"""Request micro-batching in front of the batched backend.

The reference's ``/analyze`` endpoint (app/api/v1/endpoints/analyze.py:63-129) runs
every request through the per-image extractors on the event-loop thread, one image per
call.  ``MicroBatcher`` lets concurrent requests share launches: requests queue up and a
single worker thread (with its own device context) drains up to ``max_batch`` images, or
whatever arrived within ``max_wait_ms`` of the first one, into one launch.

The worker runs the serving loop the headline measures (bench.py): it keeps ``inflight``
(default 2, like the bench's loop: with four 256-thread k-means workgroups per CU a third
launch in flight slows the GPU more than it hides host work) launches in flight through
``Backend.submit_images`` / ``Backend.collect``
(llfe_submit_images reads the requests' separately allocated device images in place through
an address table, or gathers other layouts on the device; batch k + 1's kernels start in
the tail of batch k's k-means), and a resolver thread
turns each collected batch into the reference-shaped results (``pipeline.assemble_batch``)
and resolves the requests' futures while the worker submits the next batch.  After its
first batch the worker calls ``gc.collect(); gc.freeze()`` (``freeze_gc``): the serving
process's start-up heap then stays out of the collector's full passes, which otherwise
stop the worker for 45-90 ms every few batches -- long enough to drain the in-flight
launches and idle the GPU.

    batcher = MicroBatcher(features=("colors", "shapes", "shadows"))
    result = await batcher.analyze(image_bgr)          # inside an async endpoint
    fut = batcher.submit(image_bgr); fut.result()      # from any thread

Images are H x W x 3 BGR uint8 numpy arrays or torch tensors (host or device).  Every
request takes a global index when it is submitted (or the one it passes), which fixes its
noise stream and k-means seeds: its result equals ``run_batch([image],
index_base=index)``'s whatever it was batched with.  ``run=`` replaces the backend with a
synchronous batch function ``run(images, features) -> list`` (one launch at a time; CPU
tests).
"""
from __future__ import annotations

import asyncio
import collections
import threading
import time
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Callable, Optional, Sequence

import numpy as np

_STOP = object()


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch") and hasattr(x, "data_ptr")


def _settle(fut, r, e):
    if not fut.done():
        if e is not None:
            fut.set_exception(e)
        else:
            fut.set_result(r)


def _settle_many(items):
    for fut, r in items:
        if not fut.done():
            fut.set_result(r)


class _LoopFuture:
    """The request side of ``analyze``: an asyncio future of the caller's loop, resolved
    from the batcher's threads.  A batch's results reach each loop in ONE
    call_soon_threadsafe (``_resolve``), not one wake-up and one wrapped concurrent future
    per request -- at ~20k requests/s that per-request overhead is what holds the event
    loop's GIL."""

    __slots__ = ("loop", "fut")

    def __init__(self, loop, fut):
        self.loop, self.fut = loop, fut

    def set_running_or_notify_cancel(self) -> bool:
        return not self.fut.cancelled()  # (a cancel racing this read only loses its result)

    def done(self) -> bool:
        return self.fut.done()

    def set_result(self, r):
        self._post(_settle, self.fut, r, None)

    def set_exception(self, e):
        self._post(_settle, self.fut, None, e)

    def _post(self, fn, *args):
        try:
            self.loop.call_soon_threadsafe(fn, *args)
        except RuntimeError:  # the caller's loop is closed: nobody waits for this request
            pass


def _resolve(futs, results):
    """set_result over a batch: concurrent futures directly, asyncio ones per loop in one
    call."""
    by_loop: dict = {}
    for f, r in zip(futs, results):
        if isinstance(f, _LoopFuture):
            by_loop.setdefault(f.loop, []).append((f.fut, r))
        else:
            f.set_result(r)
    for loop, items in by_loop.items():
        try:
            loop.call_soon_threadsafe(_settle_many, items)
        except RuntimeError:
            pass


class MicroBatcher:
    # max_batch: requests per launch at most (split further per image size by the device pass
    # capacity, llfe_batch_capacity: 512 for 1080p); at light load launches stay small anyway
    # (max_wait_ms), at high load a full pass amortises the k-means launch's tail
    def __init__(self, features: Sequence[str] = ("colors", "shapes", "shadows"), max_batch: int = 512,
                 max_wait_ms: float = 2.0, run: Optional[Callable] = None, inflight: int = 2,
                 seed: Optional[int] = None, n_colors: int = 5, freeze_gc: bool = True, backend=None,
                 device: Optional[int] = None, fill_wait_ms: float = 8.0):
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        if inflight not in (1, 2, 3):
            raise ValueError("inflight must be 1, 2 or 3")
        self.features = tuple(getattr(f, "value", f) for f in features)
        self.max_batch = int(max_batch)
        self.max_wait = max(0.0, float(max_wait_ms)) / 1e3
        # while launches are in flight (the GPU is busy for a step anyway) a partial batch
        # waits up to fill_wait_ms for more requests: fuller launches, the same latency bound
        self.fill_wait = max(self.max_wait, float(fill_wait_ms) / 1e3)
        self.inflight = int(inflight)
        self.n_colors = int(n_colors)
        self.freeze_gc = bool(freeze_gc)
        self._seed = seed
        self._run = run
        self._backend = backend  # (tests: a stand-in with submit_images / collect / inflight)
        self._device = device  # GPU of the worker's context (default: LLFE_DEVICE / LOCAL_RANK)
        # request queue: a deque the producers append to without a lock (at ~20k requests/s
        # queue.Queue's lock and condition cost ~12 us per put under contention); the worker
        # sleeps on _wake only when it found the deque empty (_sleeping)
        self._q: "collections.deque" = collections.deque()
        self._wake = threading.Event()
        self._sleeping = False
        self._want = 1  # (a sleeping worker wants this many queued items before it wakes)
        self.batch_sizes: list = []  # sizes of the launches so far (diagnostics)
        # (submit time, collect-start time, collect-end time) per launch, worker clock
        # (perf_counter): launches overlap when one is submitted before the previous one's
        # collect returned
        self.launch_log: list = []
        self.max_in_flight = 0
        self._closed = False
        self._thread = threading.Thread(target=self._loop, name="llfe-batcher", daemon=True)
        self._thread.start()

    # ---------------------------------------------------------------- submission
    def submit(self, image, index: Optional[int] = None) -> Future:
        """Queue one H x W x 3 BGR uint8 image (numpy array or torch tensor, host or
        device); the future yields its result dict.  ``index``: its global index (default:
        the next one of the process counter)."""
        fut: Future = Future()
        self._enqueue(image, fut, index)
        return fut

    _U8 = None  # torch.uint8, once torch is seen

    def _enqueue(self, image, fut, index):
        if self._closed:
            raise RuntimeError("MicroBatcher is closed")
        if _is_torch(image):
            img = image
            if MicroBatcher._U8 is None:
                import torch

                MicroBatcher._U8 = torch.uint8
            sh = img.shape
            if len(sh) != 3 or sh[2] != 3 or img.dtype is not MicroBatcher._U8:
                raise ValueError(f"expected H x W x 3 BGR uint8 image, got {tuple(sh)} {img.dtype}")
        else:
            img = np.ascontiguousarray(np.asarray(image, np.uint8))
            if img.ndim != 3 or img.shape[2] != 3:
                raise ValueError(f"expected H x W x 3 BGR uint8 image, got {img.shape}")
        # (index None: the worker hands out the next global indices in arrival order, one
        # counter call per launch)
        q = self._q
        q.append((img, fut, None if index is None else int(index)))
        if self._sleeping and len(q) >= self._want:
            self._wake.set()

    def submit_bytes(self, image_bytes: bytes, preprocessing: str = "auto") -> Future:
        """Decode + preprocess (validate_and_preprocess_image semantics) on the calling
        thread, then queue the image."""
        from .utils import preprocess_decoded
        from .decode import decode_bgr

        return self.submit(preprocess_decoded(decode_bgr(image_bytes), preprocessing))

    async def analyze(self, image, index: Optional[int] = None) -> dict:
        """``submit`` for an async endpoint: awaits the image's result dict."""
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._enqueue(image, _LoopFuture(loop, fut), index)
        return await fut

    def close(self, timeout: Optional[float] = None):
        if not self._closed:
            self._closed = True
            self._q.append(_STOP)
            self._wake.set()
            self._thread.join(timeout)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---------------------------------------------------------------- worker
    def _pop_wait(self, timeout: Optional[float], want: int = 1):
        """The next queued item, waiting up to ``timeout`` (None: forever) -- woken early
        only once ``want`` items are queued (or at close); None if none."""
        q = self._q
        while True:
            if q:
                return q.popleft()
            if timeout is not None and timeout <= 0:
                return None
            self._wake.clear()
            self._want = max(1, want)
            self._sleeping = True
            try:
                if not q:  # (re-checked after announcing the sleep: no lost wake-up)
                    t0 = time.monotonic()
                    self._wake.wait(timeout)
                    if timeout is not None:
                        timeout -= time.monotonic() - t0
            finally:
                self._sleeping = False

    def _gather(self, block: bool, wait: Optional[float] = None):
        """Up to max_batch queued requests: the first one (waiting for it when ``block``,
        else at most ``wait``), then whatever arrives within ``wait`` (default max_wait) of
        it.  Returns (items, stop)."""
        wait = self.max_wait if wait is None else wait
        first = self._pop_wait(None if block else wait)
        if first is None:
            return [], False
        if first is _STOP:
            return [], True
        items = [first]
        deadline = time.monotonic() + wait
        stop = False
        q = self._q
        while len(items) < self.max_batch:
            while q and len(items) < self.max_batch:  # (drain what is there without waiting)
                nxt = q.popleft()
                if nxt is _STOP:
                    stop = True
                    break
                items.append(nxt)
            if stop or len(items) >= self.max_batch:
                break
            nxt = self._pop_wait(deadline - time.monotonic(), self.max_batch - len(items))
            if nxt is None:
                break
            if nxt is _STOP:
                stop = True
                break
            items.append(nxt)
        live = [x for x in items if x[1].set_running_or_notify_cancel()]
        need = sum(1 for x in live if x[2] is None)
        if need:  # global indices for the requests that did not bring one, in arrival order
            from .color_extractor import _next_index

            nxt_i = _next_index(need)
            for k, x in enumerate(live):
                if x[2] is None:
                    live[k] = (x[0], x[1], nxt_i)
                    nxt_i += 1
        return live, stop

    def _loop(self):
        if self._run is not None:
            self._loop_sync()
        else:
            self._loop_pipelined()
        # fail whatever is still queued after close()
        while self._q:
            item = self._q.popleft()
            if item is not _STOP:
                item[1].set_exception(RuntimeError("MicroBatcher is closed"))

    def _loop_sync(self):
        """``run=`` given: one synchronous launch at a time."""
        stop = False
        while not stop:
            live, stop = self._gather(block=True)
            if not live:
                continue
            self.batch_sizes.append(len(live))
            try:
                res = self._run([im for im, _, _ in live], self.features)
                _resolve([f for _, f, _ in live], res)
            except Exception as e:
                if len(live) == 1:
                    live[0][1].set_exception(e)
                    continue
                # one bad image must not fail the requests it was batched with (the
                # reference isolates every request): rerun them one by one
                for im, f, _ in live:
                    try:
                        f.set_result(self._run([im], self.features)[0])
                    except Exception as e1:
                        f.set_exception(e1)
            except BaseException as e:  # interpreter shutdown etc.: fail the batch
                for _, f, _ in live:
                    f.set_exception(e)

    def _loop_pipelined(self):
        from .pipeline import assemble_batch

        try:
            if self._backend is not None:
                be = self._backend
            else:
                from .backend import Backend

                be = Backend.get(self._device)  # this thread's own context
            if self.inflight > 1:
                be.inflight = self.inflight
            depth = self.inflight
            seed = self._seed
            if seed is None:
                from .color_extractor import _SEED as seed
        except BaseException as e:  # no device: every request fails loudly (no CPU fallback)
            while True:
                live, stop = self._gather(block=True)
                for _, f, _ in live:
                    f.set_exception(e)
                if stop:
                    return
        resolver = ThreadPoolExecutor(max_workers=1, thread_name_prefix="llfe-batcher-resolve")
        pending: "collections.deque" = collections.deque()  # (ticket, live, log entry)
        feats = self.features
        froze = not self.freeze_gc

        def resolve(recs, live):
            try:
                out = assemble_batch(recs, feats)
            except BaseException as e:
                for _, f, _ in live:
                    f.set_exception(e)
                return
            _resolve([f for _, f, _ in live], out)

        def finish_oldest():
            nonlocal froze
            ticket, live, log = pending.popleft()
            log[1] = time.perf_counter()
            try:
                recs = be.collect(ticket)
            except Exception as e:
                log[2] = time.perf_counter()
                for _, f, _ in live:
                    f.set_exception(e)
                return
            log[2] = time.perf_counter()
            resolver.submit(resolve, recs, live)
            if not froze:
                # the start-up heap out of the collector's full passes (module docstring)
                import gc

                gc.collect()
                gc.freeze()
                froze = True

        def run_one_by_one(live):
            # a launch the backend refused (e.g. one malformed image): the requests run
            # alone, synchronously, so each gets its own result or error
            from .pipeline import run_batch

            while pending:
                finish_oldest()
            for im, f, idx in live:
                try:
                    f.set_result(run_batch([im], feats, seed=seed, index_base=idx, n_colors=self.n_colors,
                                           backend=be)[0])
                except Exception as e:
                    f.set_exception(e)

        stop = False
        try:
            while not stop or pending:
                live = []
                if not stop:
                    live, stop = self._gather(block=not pending, wait=self.fill_wait if pending else None)
                if not live:
                    if pending:
                        finish_oldest()
                    continue
                # one launch per image size (the launch packs one size), at most one device
                # pass each
                groups: dict = {}
                for it in live:
                    groups.setdefault((tuple(it[0].shape), _is_torch(it[0]) and it[0].is_cuda), []).append(it)
                for (shape, _), grp in groups.items():
                    cap = max(1, self._capacity(be, shape[0], shape[1]))
                    for a in range(0, len(grp), cap):
                        part = grp[a:a + cap]
                        if len(pending) >= depth:
                            finish_oldest()
                        log = [time.perf_counter(), None, None]
                        try:
                            ticket = be.submit_images([im for im, _, _ in part], feats, seed=seed,
                                                      indices=[idx for _, _, idx in part], n_colors=self.n_colors)
                        except Exception:
                            run_one_by_one(part)
                            continue
                        self.batch_sizes.append(len(part))
                        self.launch_log.append(log)
                        pending.append((ticket, part, log))
                        self.max_in_flight = max(self.max_in_flight, len(pending))
        except BaseException as e:  # interpreter shutdown etc.: fail what is in flight
            for _, live, _ in pending:
                for _, f, _ in live:
                    if not f.done():
                        f.set_exception(e)
            raise
        finally:
            resolver.shutdown(wait=True)
            if self._backend is None:  # the worker's own context: its workspaces go with it
                from .backend import Backend

                Backend.release(be)

    @staticmethod
    def _capacity(be, h, w) -> int:
        """Images of h x w one launch takes (llfe_batch_capacity)."""
        cap = getattr(be, "batch_capacity", None)
        return int(cap(h, w)) if cap else 1 << 30
