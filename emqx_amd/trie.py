"""Host mirror of ``emqx_trie`` (apps/emqx/src/emqx_trie.erl) on the GPU table.

Same API and semantics: ``insert/1`` is idempotent (:82-87), ``delete/1`` is a
no-op for an absent filter (:91-96), ``match/1`` returns the matching filters
of the trie and ``[]`` for a wildcard topic (:100-114), ``empty/0`` (:118).
Mutations are staged on the host table and published as a new table epoch on
the next match (or explicitly with :meth:`commit`) — the counterpart of the
mnesia transaction boundary around the reference's trie updates
(apps/emqx/src/emqx_router.erl:252-303).  Matching always runs the HIP path;
there is no CPU fallback.
"""
from __future__ import annotations

from contextlib import contextmanager
from typing import Dict, List, Optional, Sequence

from . import _lib as L
from .engine import GpuMatcher


def _check_bin(x):
    if not isinstance(x, (bytes, bytearray)):
        raise TypeError("function_clause: topic must be a binary")  # the reference's is_binary guard
    return bytes(x)


class Trie:
    """``emqx_trie`` over one GPU matcher (EGM_MODE_TRIE semantics)."""

    def __init__(self, matcher: Optional[GpuMatcher] = None, device: int = 0, compact: bool = True):
        self.m = matcher or GpuMatcher(device, compact=compact)
        self._compact = compact
        self._ids: Dict[bytes, int] = {}
        self._names: Dict[int, bytes] = {}
        self._next = 0
        self._dirty = False
        self._in_txn = 0

    # -- emqx_trie API --------------------------------------------------------
    def insert(self, topic: bytes) -> str:
        topic = _check_bin(topic)
        if topic in self._ids:
            return "ok"
        fid = self._next
        self._next += 1
        self.m.apply(inserts=[topic], insert_ids=[fid])
        self._ids[topic] = fid
        self._names[fid] = topic
        self._dirty = True
        return "ok"

    def delete(self, topic: bytes) -> str:
        topic = _check_bin(topic)
        fid = self._ids.pop(topic, None)
        if fid is None:
            return "ok"
        self.m.apply(deletes=[topic])
        del self._names[fid]
        self._dirty = True
        return "ok"

    def match(self, topic: bytes) -> List[bytes]:
        return self.match_batch([_check_bin(topic)])[0]

    def match_batch(self, topics: Sequence[bytes]) -> List[List[bytes]]:
        """One GPU batch for many publish topics (the batched NIF call)."""
        topics = [_check_bin(t) for t in topics]
        self.commit()
        res = self.m.match_strings(topics, L.EGM_MODE_TRIE)
        names = self._names
        return [[names[int(i)] for i in res.row(k)] for k in range(len(topics))]

    def empty(self) -> bool:
        return not self._ids

    def lock_tables(self) -> str:
        return "ok"

    def is_compact(self) -> bool:
        return self._compact

    def set_compact(self, flag: bool) -> None:
        # broker.perf.trie_compaction: changes the reference's key layout and
        # walk order only; the match *set* is identical, and the GPU
        # graph has no compaction.
        self._compact = bool(flag)

    # -- epochs ---------------------------------------------------------------
    def commit(self) -> None:
        if self._dirty and not self._in_txn:
            self.m.commit()
            self._dirty = False

    @contextmanager
    def transaction(self):
        """Batch several inserts/deletes into one published epoch."""
        self._in_txn += 1
        try:
            yield self
        finally:
            self._in_txn -= 1
            self.commit()

    def filter_id(self, topic: bytes) -> Optional[int]:
        return self._ids.get(topic)

    def filter_of(self, fid: int) -> bytes:
        return self._names[fid]
