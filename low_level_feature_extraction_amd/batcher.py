"""Request micro-batching in front of the batched backend.

The reference's ``/analyze`` endpoint (app/api/v1/endpoints/analyze.py:63-129) runs
every request through the per-image extractors on the event-loop thread, one image per
call.  ``MicroBatcher`` lets concurrent requests share one ``llfe_process_batch``
launch: requests queue up, a single worker thread (with its own device context) drains
up to ``max_batch`` images or whatever arrived within ``max_wait_ms`` of the first one,
runs them through ``pipeline.run_batch`` (which groups them by size) and resolves each
request's future with exactly the dict ``run_batch`` returns for that image.

    batcher = MicroBatcher(features=("colors", "shapes", "shadows"))
    result = await batcher.analyze(image_bgr)          # inside an async endpoint
    fut = batcher.submit(image_bgr); fut.result()      # from any thread

Results do not depend on how requests were grouped: every image carries its own global
index for the noise stream and the k-means seeds.
"""
from __future__ import annotations

import asyncio
import queue
import threading
import time
from concurrent.futures import Future
from typing import Callable, Optional, Sequence

import numpy as np

_STOP = object()


class MicroBatcher:
    def __init__(self, features: Sequence[str] = ("colors", "shapes", "shadows"), max_batch: int = 64,
                 max_wait_ms: float = 2.0, run: Optional[Callable] = None):
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self.features = tuple(getattr(f, "value", f) for f in features)
        self.max_batch = int(max_batch)
        self.max_wait = max(0.0, float(max_wait_ms)) / 1e3
        self._run = run
        self._q: "queue.Queue" = queue.Queue()
        self.batch_sizes: list = []  # sizes of the batches launched so far (diagnostics)
        self._closed = False
        self._thread = threading.Thread(target=self._loop, name="llfe-batcher", daemon=True)
        self._thread.start()

    # ---------------------------------------------------------------- submission
    def submit(self, image) -> Future:
        """Queue one H x W x 3 BGR uint8 image; the future yields its result dict."""
        if self._closed:
            raise RuntimeError("MicroBatcher is closed")
        img = np.ascontiguousarray(np.asarray(image, np.uint8))
        if img.ndim != 3 or img.shape[2] != 3:
            raise ValueError(f"expected H x W x 3 BGR uint8 image, got {img.shape}")
        fut: Future = Future()
        self._q.put((img, fut))
        return fut

    def submit_bytes(self, image_bytes: bytes, preprocessing: str = "auto") -> Future:
        """Decode + preprocess (validate_and_preprocess_image semantics) on the calling
        thread, then queue the image."""
        from .utils import preprocess_decoded
        from .decode import decode_bgr

        return self.submit(preprocess_decoded(decode_bgr(image_bytes), preprocessing))

    async def analyze(self, image) -> dict:
        return await asyncio.wrap_future(self.submit(image))

    def close(self, timeout: Optional[float] = None):
        if not self._closed:
            self._closed = True
            self._q.put(_STOP)
            self._thread.join(timeout)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---------------------------------------------------------------- worker
    def _run_batch(self, images):
        if self._run is not None:
            return self._run(images, self.features)
        from .pipeline import run_batch

        return run_batch(images, self.features)

    def _loop(self):
        stop = False
        while not stop:
            item = self._q.get()
            if item is _STOP:
                break
            items = [item]
            deadline = time.monotonic() + self.max_wait
            while len(items) < self.max_batch:
                left = deadline - time.monotonic()
                try:
                    nxt = self._q.get(timeout=left) if left > 0 else self._q.get_nowait()
                except queue.Empty:
                    break
                if nxt is _STOP:
                    stop = True
                    break
                items.append(nxt)
            live = [(im, f) for im, f in items if f.set_running_or_notify_cancel()]
            if not live:
                continue
            self.batch_sizes.append(len(live))
            try:
                res = self._run_batch([im for im, _ in live])
                for (_, f), r in zip(live, res):
                    f.set_result(r)
            except Exception as e:
                if len(live) == 1:
                    live[0][1].set_exception(e)
                    continue
                # one bad image must not fail the requests it was batched with (the
                # reference isolates every request): rerun them one by one
                for im, f in live:
                    try:
                        f.set_result(self._run_batch([im])[0])
                    except Exception as e1:
                        f.set_exception(e1)
            except BaseException as e:  # interpreter shutdown etc.: fail the batch
                for _, f in live:
                    f.set_exception(e)
        # fail whatever is still queued after close()
        while True:
            try:
                item = self._q.get_nowait()
            except queue.Empty:
                break
            if item is not _STOP:
                item[1].set_exception(RuntimeError("MicroBatcher is closed"))
