"""Python mirror of the Erlang integration processes (erl/*.erl).

The Erlang side cannot be compiled here (no ERTS), so its logic is restated
call for call on the Python host and tested (tests/test_gpu_batch_mirror.py):

* ``RouteTable``  — ``emqx_route``: a bag of (topic, dest) with the add/delete
  rules of ``emqx_router:do_add_route/2`` / ``do_delete_route/2``
  (apps/emqx/src/emqx_router.erl:114-125,164-170) and the post-commit table
  events mnesia delivers to subscribers.
* ``GpuFilters``  — ``emqx_gpu_match``'s id map + ``build/1`` / ``sync/2`` /
  ``filters_of/1`` over a NIF-shaped matcher (``GpuMatcher``: apply / commit /
  submit / wait / cancel).
* ``RouteSync``   — ``emqx_gpu_routes``: collects the wildcard topics touched
  by route events and publishes them as ONE delta + commit per linger, a
  topic being in the table iff it has routes at flush time — never inside a
  route transaction.
* ``BatchServer`` — ``emqx_gpu_batch``: per-message ``match_routes/1`` calls
  batched (size + linger), matched in TRIE mode (``emqx_trie:match/1``) and
  expanded as ``lookup_routes/1`` of ``[Topic | Matched]``, which is
  ``emqx_router:match_routes/1`` exactly (emqx_router.erl:129-134); every
  failure falls back to the reference ``match_routes``.
"""
from __future__ import annotations

import threading
import time
from collections import namedtuple
from typing import Callable, Dict, List, Optional, Sequence

from . import _lib as L
from .batcher import Batcher
from .engine import pack_strings
from .topic import wildcard

Route = namedtuple("Route", "topic dest")


class RouteTable:
    """emqx_route (a bag) with post-commit events: ('write', topic) and
    ('delete_object', topic), as mnesia:subscribe({table, emqx_route, simple})
    delivers them."""

    def __init__(self):
        self._routes: Dict[bytes, List[object]] = {}
        self._subs: List[Callable[[str, bytes], None]] = []
        self._mu = threading.Lock()

    def subscribe(self, fn: Callable[[str, bytes], None]):
        self._subs.append(fn)

    def _event(self, kind: str, topic: bytes):
        for fn in self._subs:
            fn(kind, topic)

    def add_route(self, topic: bytes, dest="local"):     # do_add_route/2 :114-125
        with self._mu:
            cur = self._routes.setdefault(topic, [])
            if dest in cur:
                return "ok"
            cur.append(dest)
        self._event("write", topic)                      # after the commit
        return "ok"

    def delete_route(self, topic: bytes, dest="local"):  # do_delete_route/2 :164-170
        with self._mu:
            cur = self._routes.get(topic)
            if not cur or dest not in cur:
                return "ok"
            cur.remove(dest)
            if not cur:
                del self._routes[topic]
        self._event("delete_object", topic)
        return "ok"

    def lookup_routes(self, topic: bytes) -> List[Route]:   # :144-145
        with self._mu:
            return [Route(topic, d) for d in self._routes.get(topic, [])]

    def has_routes(self, topic: bytes) -> bool:             # :148-150
        with self._mu:
            return topic in self._routes

    def topics(self) -> List[bytes]:                        # :173-175
        with self._mu:
            return list(self._routes)


class GpuFilters:
    """emqx_gpu_match's filter-id map over one matcher context."""

    def __init__(self, nif):
        self.nif = nif
        self.ids: Dict[bytes, int] = {}
        self.names: Dict[int, bytes] = {}
        self.next_id = 0
        self._mu = threading.Lock()

    def build(self, filters: Sequence[bytes]):
        with self._mu:
            self.ids = {f: i for i, f in enumerate(filters)}
            self.names = {i: f for i, f in enumerate(filters)}
            self.next_id = len(filters)
            blob, off = pack_strings(list(filters))
            self.nif.build(blob, off)

    def sync(self, inserts: Sequence[bytes], deletes: Sequence[bytes]):
        with self._mu:
            new = [f for f in inserts if f not in self.ids]
            gone = [(f, self.ids[f]) for f in deletes if f in self.ids]
            if not new and not gone:
                return
            ins = []
            for f in new:
                ins.append((f, self.next_id))
                self.ids[f] = self.next_id
                self.names[self.next_id] = f
                self.next_id += 1
            self.nif.apply(inserts=[f for f, _ in ins] or None, deletes=[f for f, _ in gone] or None,
                           insert_ids=[i for _, i in ins] or None)
            self.nif.commit()
            for f, i in gone:   # ids leave the map after the epoch without them is published
                del self.ids[f]
                del self.names[i]

    def filters_of(self, ids) -> List[bytes]:
        with self._mu:
            return [self.names[i] for i in ids if i in self.names]


class RouteSync:
    """emqx_gpu_routes: post-commit route events -> one GPU epoch per linger."""

    def __init__(self, routes: RouteTable, filters: GpuFilters, batch_size: int = 65536, linger_ms: float = 5.0):
        self.routes, self.filters = routes, filters
        self.size, self.linger = batch_size, linger_ms / 1000.0
        self._touched: Dict[bytes, bool] = {}
        self._first = 0.0
        self._mu = threading.Lock()
        self.epochs = 0
        filters.build([t for t in routes.topics() if wildcard(t)])
        routes.subscribe(self.on_event)

    def on_event(self, kind: str, topic: bytes):
        if not wildcard(topic):     # exact filters never enter the trie (emqx_router.erl:120-124)
            return
        with self._mu:
            if topic in self._touched:
                return
            if not self._touched:
                self._first = time.monotonic()
            self._touched[topic] = True
            full = len(self._touched) >= self.size
        if full:
            self.publish()

    def due(self) -> bool:
        with self._mu:
            return bool(self._touched) and time.monotonic() - self._first >= self.linger

    def publish(self):
        with self._mu:
            touched, self._touched = list(self._touched), {}
        if not touched:
            return
        ins = [t for t in touched if self.routes.has_routes(t)]
        dels = [t for t in touched if t not in set(ins)]
        self.filters.sync(ins, dels)
        self.epochs += 1


class BatchServer:
    """emqx_gpu_batch: batched match_routes/1 with the reference as fallback."""

    def __init__(self, routes: RouteTable, filters: GpuFilters, fallback: Callable[[bytes], List[Route]],
                 batch_size: int = 4096, linger_ms: float = 1.0):
        self.routes, self.filters, self.fallback = routes, filters, fallback
        self._b: Optional[Batcher] = Batcher(self._commit, batch_size=batch_size, linger_ms=linger_ms)
        self.fallbacks = 0

    def _commit(self, topics: Sequence[bytes]):
        """One committed batch: submit (TRIE mode) + wait -> id rows, or the
        error for every caller (handle_info/submit/answer of the Erlang side)."""
        nif = self.filters.nif
        try:
            blob, off = pack_strings(list(topics))
            t = nif.submit(blob, off, L.EGM_MODE_TRIE)
            res = nif.wait(t)
            return [("ok", res.row(k).tolist()) for k in range(len(topics))]
        except Exception as e:  # noqa: BLE001 - an error is an answer: the caller falls back
            return [("error", repr(e))] * len(topics)

    def match_routes(self, topic: bytes, timeout: float = 5.0) -> List[Route]:
        if not isinstance(topic, (bytes, bytearray)):
            raise TypeError("function_clause: topic must be a binary")
        topic = bytes(topic)
        try:
            if self._b is None:
                raise RuntimeError("noproc")
            tag, val = self._b.push(topic).result(timeout=timeout)
        except Exception:   # noqa: BLE001 - noproc / timeout / server down
            tag, val = "error", "unavailable"
        if tag != "ok":
            self.fallbacks += 1
            return self.fallback(topic)
        matched = self.filters.filters_of(val)
        out: List[Route] = []
        for to in [topic] + matched:
            out.extend(self.routes.lookup_routes(to))
        return out

    def stop(self):
        if self._b is not None:
            self._b.close()
            self._b = None
