"""Host mirror of ``emqx_router`` (apps/emqx/src/emqx_router.erl) on the GPU table.

The route table is a bag of ``Route(topic, dest)`` (apps/emqx/include/emqx.hrl:90-93).
``match_routes/1`` (:129-134) = the exact routes of the topic itself plus the
routes of every trie-matched wildcard filter.  Here one GPU table holds every
filter with at least one route, exact and wildcard alike, and the
EGM_MODE_ROUTES walk returns exactly that union in one pass; the host then
expands each matched filter to its destinations.

Route add/delete keep the reference's rules: a route is added once
(:116-117); a filter enters the table with its first route and leaves with its
last (:230-248).
"""
from __future__ import annotations

from collections import namedtuple
from typing import Dict, List, Optional, Sequence

from . import _lib as L
from .engine import GpuMatcher
from .topic import wildcard

Route = namedtuple("Route", "topic dest")


def _check_bin(x):
    if not isinstance(x, (bytes, bytearray)):
        raise TypeError("function_clause: topic must be a binary")
    return bytes(x)


class Router:
    def __init__(self, matcher: Optional[GpuMatcher] = None, device: int = 0, node: str = "local"):
        self.m = matcher or GpuMatcher(device)
        self.node = node
        self.routes: Dict[bytes, List[object]] = {}
        self._ids: Dict[bytes, int] = {}
        self._names: Dict[int, bytes] = {}
        self._next = 0
        self._dirty = False

    # -- table maintenance (emqx_router.erl:114-125,164-170,227-248) ----------
    def add_route(self, topic: bytes, dest=None) -> str:
        return self.do_add_route(topic, dest)

    def do_add_route(self, topic: bytes, dest=None) -> str:
        topic = _check_bin(topic)
        dest = self.node if dest is None else dest
        cur = self.routes.setdefault(topic, [])
        if dest in cur:
            return "ok"
        if not cur:
            fid = self._next
            self._next += 1
            self.m.apply(inserts=[topic], insert_ids=[fid])
            self._ids[topic] = fid
            self._names[fid] = topic
            self._dirty = True
        cur.append(dest)
        return "ok"

    def delete_route(self, topic: bytes, dest=None) -> str:
        return self.do_delete_route(topic, dest)

    def do_delete_route(self, topic: bytes, dest=None) -> str:
        topic = _check_bin(topic)
        dest = self.node if dest is None else dest
        cur = self.routes.get(topic)
        if not cur or dest not in cur:
            return "ok"
        cur.remove(dest)
        if not cur:
            del self.routes[topic]
            fid = self._ids.pop(topic)
            del self._names[fid]
            self.m.apply(deletes=[topic])
            self._dirty = True
        return "ok"

    def commit(self):
        if self._dirty:
            self.m.commit()
            self._dirty = False

    # -- lookups ----------------------------------------------------------------
    def lookup_routes(self, topic: bytes) -> List[Route]:
        return [Route(topic, d) for d in self.routes.get(topic, [])]

    def has_routes(self, topic: bytes) -> bool:
        return topic in self.routes

    def topics(self) -> List[bytes]:
        return list(self.routes)

    def match_filters_batch(self, topics: Sequence[bytes]):
        """GPU batch -> per topic the list of matched filter ids."""
        topics = [_check_bin(t) for t in topics]
        self.commit()
        res = self.m.match_strings(topics, L.EGM_MODE_ROUTES)
        return res

    def match_routes(self, topic: bytes) -> List[Route]:
        return self.match_routes_batch([_check_bin(topic)])[0]

    def match_routes_batch(self, topics: Sequence[bytes]) -> List[List[Route]]:
        res = self.match_filters_batch(topics)
        out = []
        for k in range(len(topics)):
            rs = []
            for fid in res.row(k).tolist():
                f = self._names[fid]
                rs.extend(Route(f, d) for d in self.routes[f])
            out.append(rs)
        return out

    def print_routes(self, topic: bytes) -> None:
        for r in self.match_routes(topic):
            print(f"{r.topic.decode(errors='replace')} -> {r.dest}")

    def filter_id(self, topic: bytes) -> Optional[int]:
        return self._ids.get(topic)

    def filter_of(self, fid: int) -> bytes:
        return self._names[fid]

    @staticmethod
    def is_wildcard(topic: bytes) -> bool:
        return wildcard(topic)
