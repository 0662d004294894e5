"""Linger-bounded publish batcher (the host side of the dirty-NIF integration).

Publishing in the reference is one ``emqx_router:match_routes/1`` call per
message in the publisher's process (apps/emqx/src/emqx_broker.erl:208).  A
GPU batch only pays off for many topics at once, so callers push single
topics here and wait on a future; a flusher thread commits a batch when
``batch_size`` topics are queued or ``linger_ms`` has passed since the first
one — the policy of ``emqx_batch`` (apps/emqx/src/emqx_batch.erl:50-81: size
limit + linger timer, ``commit`` callback).
"""
from __future__ import annotations

import threading
import time
from concurrent.futures import Future
from typing import Callable, List, Sequence


class Batcher:
    def __init__(self, commit: Callable[[Sequence], List], batch_size: int = 4096, linger_ms: float = 1.0):
        if batch_size < 1 or linger_ms < 0:
            raise ValueError("batch_size >= 1, linger_ms >= 0")
        self._commit = commit
        self.batch_size = batch_size
        self.linger = linger_ms / 1000.0
        self._items: List = []
        self._futs: List[Future] = []
        self._first = 0.0
        self._cv = threading.Condition()
        self._stop = False
        self.batches = 0
        self._t = threading.Thread(target=self._run, name="egm-batcher", daemon=True)
        self._t.start()

    def push(self, item) -> Future:
        f: Future = Future()
        with self._cv:
            if self._stop:
                raise RuntimeError("batcher closed")
            if not self._items:
                self._first = time.monotonic()
            self._items.append(item)
            self._futs.append(f)
            if len(self._items) >= self.batch_size:
                self._cv.notify()
            elif len(self._items) == 1:
                self._cv.notify()
        return f

    def _take(self):
        items, futs = self._items, self._futs
        self._items, self._futs = [], []
        return items, futs

    def _run(self):
        while True:
            with self._cv:
                while not self._stop and not self._items:
                    self._cv.wait()
                if self._stop and not self._items:
                    return
                while not self._stop and len(self._items) < self.batch_size:
                    left = self._first + self.linger - time.monotonic()
                    if left <= 0:
                        break
                    self._cv.wait(left)
                items, futs = self._take()
            try:
                res = self._commit(items)
                if len(res) != len(items):
                    raise RuntimeError("commit returned a result list of the wrong length")
                for f, r in zip(futs, res):
                    f.set_result(r)
            except BaseException as e:  # noqa: BLE001 - propagate to every waiter
                for f in futs:
                    f.set_exception(e)
            self.batches += 1

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._t.join()
