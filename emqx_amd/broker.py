"""Host mirror of the publish side of ``emqx_broker`` + ``emqx_shared_sub``.

``publish_batch`` is the batched ``emqx_broker:publish/1`` (apps/emqx/src/emqx_broker.erl:200-209)
for many messages: ``emqx_router:match_routes/1`` on the GPU, then the
``dispatch/2`` subscriber expansion (:283-308) on the GPU fan-out kernel from
a filter -> subscriber CSR, then per shared group one member picked by the
configured strategy (emqx_shared_sub.erl:239-290) and remote node routes
turned into forwards (:242-245).

Delivery entries:
  ("sub", filter, sub_id)                    local subscriber of filter
  ("group", filter, group, member)           $share group, one member picked
  ("node", filter, node)                     route to another node (forward)

``publish_result`` / ``publish_result_batch`` return what ``publish/1``
returns (``emqx_types:publish_result()``): one entry per aggregated route
(``aggre/1``, :249-260) — ``(node, filter, {ok, N} | {error, no_subscribers})``
for this node (``dispatch/2``, :283-295: N alive subscribers), ``(node,
filter, "forward")`` for another node (async ``forward/4``, :265-271), and
``("share", filter, {ok, 1} | {error, no_subscribers})`` per $share group
(emqx_shared_sub.erl:120-127) — and keep the reference's metrics: a message
with no route, or a local route none of whose subscribers is alive, counts
``messages.dropped`` and ``messages.dropped.no_subscribers`` (not for a
system message, ``inc_dropped_cnt/1`` :311-316, emqx_message.erl:173-177).

Subscriber sharding ({shard, Topic, I} bags beyond 1024 subscribers,
emqx_broker.erl:149-157, emqx_broker_helper.erl:82-86) changes only the layout
of the reference's ETS bags, never the delivery set; the fan-out CSR is the
flattened union.
"""
from __future__ import annotations

import random
import zlib
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .router import Router
from .topic import parse

GROUP_BIT = 0x80000000
SHARD_THRESHOLD = 1024        # ?SHARD, emqx_broker_helper.erl:54
STRATEGIES = ("random", "round_robin", "sticky", "hash", "hash_clientid", "hash_topic")


class SharedSub:
    """``emqx_shared_sub``'s member pick and its ack/nack redispatch
    (apps/emqx/src/emqx_shared_sub.erl:120-134 ``dispatch/4``, :150-194
    ``dispatch_per_qos``/``dispatch_with_ack``, :239-290 ``pick``/``do_pick``,
    :390-397 ``is_active_sub``) over a group's member list; no GPU involved.

    phash2 (ERTS) is replaced by crc32 and ``rand`` by a seeded
    ``random.Random``: the member a hash or random pick chooses is not the
    reference's (parity-unpinned); the retry chain is: a fresh pick
    excludes the members that failed this delivery, a member that nacks (its
    queue was full), is down or times out is added to them, and once every
    member has failed one is picked from all of them and sent without an ack
    (``retry``).  ``{error, no_subscribers}`` only for a group with no member.
    """

    def __init__(self, strategy: str = "random", seed: int = 0):
        if strategy not in STRATEGIES:
            raise ValueError(strategy)
        self.strategy = strategy
        self._rng = random.Random(seed)
        self._rr: Dict[Tuple[bytes, bytes], int] = {}
        self._sticky: Dict[Tuple[bytes, bytes], int] = {}

    def _nth(self, key, strategy: str, source_topic: bytes, clientid: bytes, subs: List[int]) -> int:
        """pick_subscriber/6 + do_pick_subscriber/6 (:268-290)."""
        n = len(subs)
        if n == 1:
            return subs[0]
        if strategy == "random":
            return subs[self._rng.randrange(n)]
        if strategy == "round_robin":
            i = self._rr.get(key)
            i = self._rng.randrange(n) if i is None else (i + 1) % n
            self._rr[key] = i
            return subs[i]
        if strategy in ("hash", "hash_clientid"):
            return subs[zlib.crc32(clientid) % n]
        return subs[zlib.crc32(source_topic) % n]   # hash_topic

    def _do_pick(self, key, strategy, source_topic, clientid, members, failed):
        """do_pick/6 (:255-266): None = no subscriber; (type, member)."""
        if not members:
            return None
        rest = [m for m in members if m not in failed]
        if not rest:   # all of them failed: pick one anyway, sent without an ack
            return "retry", self._nth(key, strategy, source_topic, clientid, members)
        return "fresh", self._nth(key, strategy, source_topic, clientid, rest)

    def pick(self, group: bytes, topic: bytes, members: List[int], source_topic: bytes = b"",
             clientid: bytes = b"", failed: Sequence[int] = (), alive=lambda m: True):
        """pick/6 (:239-253): (type, member) or None."""
        key = (group, topic)
        if self.strategy == "sticky":
            cur = self._sticky.get(key)
            if cur is not None and alive(cur) and cur not in failed:   # is_active_sub/2 (:390-391)
                return "fresh", cur
            got = self._do_pick(key, "random", source_topic, clientid, members,
                                list(failed) + ([cur] if cur is not None else []))
            if got is not None:
                self._sticky[key] = got[1]
            return got
        return self._do_pick(key, self.strategy, source_topic, clientid, members, failed)

    def dispatch(self, group: bytes, topic: bytes, members: List[int], source_topic: bytes = b"",
                 clientid: bytes = b"", qos: int = 0, ack_enabled: bool = False,
                 respond=lambda m: "ack", alive=lambda m: True):
        """dispatch/4 (:123-134): -> (("ok", 1) | ("error", "no_subscribers"),
        the member delivered to or None, the members that failed on the way).
        ``respond(member)`` is the member session's answer to a delivery that
        needs an ack (QoS 1/2 with ``shared_dispatch_ack_enabled``): "ack", or
        "nack" / "down" / "timeout" (:173-190)."""
        failed: List[int] = []
        while True:
            got = self.pick(group, topic, members, source_topic, clientid, failed, alive)
            if got is None:
                return ("error", "no_subscribers"), None, failed
            typ, m = got
            if qos == 0 or typ == "retry" or not ack_enabled or respond(m) == "ack":   # dispatch_per_qos/4
                return ("ok", 1), m, failed
            failed.append(m)   # "Failed to dispatch to this sub, try next"


class Broker:
    def __init__(self, router: Optional[Router] = None, device: int = 0, node: str = "local",
                 shared_strategy: str = "random", seed: int = 0, shards: int = 32):
        if shared_strategy not in STRATEGIES:
            raise ValueError(shared_strategy)
        self.router = router or Router(device=device, node=node)
        self.node = node
        self.strategy = shared_strategy
        self.subscribers: Dict[bytes, List[int]] = {}            # filter -> local sub ids
        self.shard_of: Dict[Tuple[bytes, int], int] = {}         # (filter, sub) -> shard (layout only)
        self.shared: Dict[Tuple[bytes, bytes], List[int]] = {}   # (group, filter) -> members
        self.group_ids: Dict[bytes, int] = {}
        self.group_names: List[bytes] = []
        self.clientid: Dict[int, bytes] = {}
        self.share = SharedSub(shared_strategy, seed)
        self._shards = shards
        # the GPU subscriber table (egm_subs_*): built once, then kept by deltas
        self._built = False
        self._d_add: List[Tuple[int, int]] = []   # (filter id, subscriber entry) since the last commit
        self._d_del: List[Tuple[bytes, int]] = []
        self.subscriptions: Dict[int, set] = {}     # ?SUBSCRIPTION: sub -> {(filter, group or None)}
        self._fid_flt: Dict[int, bytes] = {}         # filter ids seen in subscriber events
        self.dead: set = set()   # subscribers whose process is gone (is_process_alive/1 false)
        self.metrics = {"messages.publish": 0, "messages.dropped": 0, "messages.dropped.no_subscribers": 0,
                        "messages.forward": 0}

    def kill(self, sub_id: int):
        """The subscriber's process exits without unsubscribing: dispatch/3
        skips it (emqx_broker.erl:297-302) until it unsubscribes."""
        self.dead.add(sub_id)

    # -- subscribe side (emqx_broker.erl:116-162, emqx_shared_sub.erl:108-109) --
    def subscribe(self, topic: bytes, sub_id: int, opts: Optional[dict] = None, clientid: Optional[bytes] = None):
        flt, o = parse(topic, opts)
        if clientid is not None:
            self.clientid[sub_id] = clientid
        group = o.get("share")
        if group is None:
            subs = self.subscribers.setdefault(flt, [])
            if sub_id in subs:
                return "ok"
            subs.append(sub_id)
            if len(subs) > SHARD_THRESHOLD:
                self.shard_of[(flt, sub_id)] = zlib.crc32(str(sub_id).encode()) % self._shards + 1
            self.router.do_add_route(flt, self.node)
            self._note(self._d_add, flt, sub_id)
        else:
            mem = self.shared.setdefault((group, flt), [])
            if sub_id in mem:
                return "ok"
            mem.append(sub_id)
            if group not in self.group_ids:
                self.group_ids[group] = len(self.group_names)
                self.group_names.append(group)
            self.router.do_add_route(flt, ("group", group))
            if len(mem) == 1:   # the (filter, group) entry: one per group, whatever its members
                self._note(self._d_add, flt, GROUP_BIT | self.group_ids[group])
        self.subscriptions.setdefault(sub_id, set()).add((flt, group))
        return "ok"

    def unsubscribe(self, topic: bytes, sub_id: int, opts: Optional[dict] = None):
        flt, o = parse(topic, opts)
        group = o.get("share")
        self._unsubscribe(flt, group, sub_id)
        return "ok"

    def _unsubscribe(self, flt: bytes, group, sub_id: int):
        if group is None:
            subs = self.subscribers.get(flt, [])
            if sub_id in subs:
                subs.remove(sub_id)
                self.shard_of.pop((flt, sub_id), None)
                self._note(self._d_del, flt, sub_id)   # (its filter id, before the route may go)
                if not subs:
                    del self.subscribers[flt]
                    self.router.do_delete_route(flt, self.node)
        else:
            mem = self.shared.get((group, flt), [])
            if sub_id in mem:
                mem.remove(sub_id)
                if not mem:
                    del self.shared[(group, flt)]
                    self._note(self._d_del, flt, GROUP_BIT | self.group_ids[group])
                    self.router.do_delete_route(flt, ("group", group))
        s = self.subscriptions.get(sub_id)
        if s is not None:
            s.discard((flt, group))
            if not s:
                del self.subscriptions[sub_id]

    def subscriber_down(self, sub_id: int):
        """emqx_broker:subscriber_down/1 (emqx_broker.erl:331-345, driven by
        emqx_broker_helper's monitor, emqx_broker_helper.erl:133-163; a $share
        member by emqx_shared_sub's): every subscription of the dead subscriber
        is removed, and a filter left without subscribers loses its route."""
        for flt, group in sorted(self.subscriptions.get(sub_id, ()), key=lambda x: (x[0], x[1] or b"")):
            self._unsubscribe(flt, group, sub_id)
        self.dead.discard(sub_id)

    # -- fan-out table ------------------------------------------------------------
    def _upload_csr(self):
        """The GPU subscriber table before a publish: built once (egm_subs_build),
        then every subscribe / unsubscribe / subscriber_down since the last
        publish goes in as one delta and one epoch (egm_subs_apply_delta +
        egm_subs_commit) instead of a rebuild."""
        r = self.router
        r.commit()
        if self._built:
            if self._d_add or self._d_del:
                self._apply_ordered(self._d_add, self._d_del)
                r.m.subs_commit()
                self._d_add.clear()
                self._d_del.clear()
            return
        self._d_add.clear()
        self._d_del.clear()
        n = r._next
        lists: List[List[int]] = [[] for _ in range(n)]
        for flt, subs in self.subscribers.items():
            lists[r.filter_id(flt)].extend(subs)
        for (group, flt) in self.shared:
            lists[r.filter_id(flt)].append(GROUP_BIT | self.group_ids[group])
        row = np.zeros(n + 1, dtype=np.uint64)
        row[1:] = np.cumsum([len(x) for x in lists]) if n else []
        flat = np.fromiter((s for x in lists for s in x), dtype=np.uint32, count=int(row[-1]) if n else 0)
        r.m.subs_build(row, flat)
        self._built = True

    def _apply_ordered(self, add, dele):
        """One delta for the pairs touched since the last publish: each pair's
        net effect, read from the host lists (a pair deleted and added again
        is present; the C-ABI applies a call's adds before its deletes, so the
        raw event log could not be replayed in one call).  Sets, not order,
        are what dispatch/2 parity is about."""
        touched = dict.fromkeys(list(add) + list(dele))
        a2 = [p for p in touched if self._present(*p)]
        d2 = [p for p in touched if not self._present(*p)]
        self.router.m.subs_apply_delta(add=a2, delete=d2)

    def _note(self, log: list, flt: bytes, entry: int):
        """A subscriber-table event as (filter id, entry), the id taken now: a
        filter whose last route goes loses its id, and its row must still be
        emptied on the GPU."""
        fid = self.router.filter_id(flt)
        if fid is not None:
            self._fid_flt[fid] = flt
            log.append((fid, entry))

    def _present(self, fid: int, entry: int) -> bool:
        flt = self._fid_flt[fid]
        if self.router.filter_id(flt) != fid:   # the filter left the table (its id is not reused)
            return False
        if entry & GROUP_BIT:
            g = self.group_names[entry & ~GROUP_BIT]
            return bool(self.shared.get((g, flt)))
        return entry in self.subscribers.get(flt, [])

    # -- publish side -------------------------------------------------------------------
    def publish(self, topic: bytes, clientid: bytes = b"") -> List[tuple]:
        return self.publish_batch([topic], [clientid])[0]

    def publish_batch(self, topics: Sequence[bytes], clientids: Optional[Sequence[bytes]] = None) -> List[List[tuple]]:
        self._upload_csr()
        r = self.router
        res = r.match_filters_batch(topics)
        drow, dfid, dsub = r.m.fanout(res)
        out = []
        for k, t in enumerate(topics):
            dl: List[tuple] = []
            for j in range(int(drow[k]), int(drow[k + 1])):
                f = r.filter_of(int(dfid[j]))
                s = int(dsub[j])
                if s & GROUP_BIT:
                    g = self.group_names[s & ~GROUP_BIT]
                    m = self._pick(g, f, t, clientids[k] if clientids else b"")
                    if m is not None:
                        dl.append(("group", f, g, m))
                else:
                    dl.append(("sub", f, s))
            # routes to other nodes are forwarded, not expanded here
            for fid in res.row(k).tolist():
                f = r.filter_of(fid)
                for d in r.routes[f]:
                    if d != self.node and not (isinstance(d, tuple) and d[0] == "group"):
                        dl.append(("node", f, d))
            out.append(dl)
        return out

    @staticmethod
    def _is_sys(topic: bytes, sys_flag: bool) -> bool:
        return sys_flag or topic.startswith(b"$SYS/")

    def _dropped(self, topic: bytes, sys_flag: bool):
        if not self._is_sys(topic, sys_flag):
            self.metrics["messages.dropped"] += 1
            self.metrics["messages.dropped.no_subscribers"] += 1

    def publish_result(self, topic: bytes, clientid: bytes = b"", sys: bool = False) -> List[tuple]:
        return self.publish_result_batch([topic], [clientid], [sys])[0]

    def publish_result_batch(self, topics: Sequence[bytes], clientids: Optional[Sequence[bytes]] = None,
                             sys_flags: Optional[Sequence[bool]] = None) -> List[List[tuple]]:
        """``publish/1`` results for a batch (see the module docstring)."""
        self._upload_csr()
        r = self.router
        res = r.match_filters_batch(topics)
        drow, dfid, dsub = r.m.fanout(res)
        out = []
        for k, t in enumerate(topics):
            sysf = bool(sys_flags[k]) if sys_flags else False
            if not self._is_sys(t, sysf):
                self.metrics["messages.publish"] += 1
            alive: Dict[int, int] = {}
            for j in range(int(drow[k]), int(drow[k + 1])):
                s = int(dsub[j])
                if not s & GROUP_BIT and s not in self.dead:
                    f = int(dfid[j])
                    alive[f] = alive.get(f, 0) + 1
            entries: List[tuple] = []
            groups = set()
            for fid in res.row(k).tolist():
                f = r.filter_of(fid)
                for d in r.routes[f]:
                    if isinstance(d, tuple) and d[0] == "group":
                        groups.add((f, d[1]))
                    elif d == self.node:
                        n = alive.get(fid, 0)
                        if n:
                            entries.append((d, f, ("ok", n)))
                        else:
                            self._dropped(t, sysf)
                            entries.append((d, f, ("error", "no_subscribers")))
                    else:
                        self.metrics["messages.forward"] += 1
                        entries.append((d, f, "forward"))
            for f, g in sorted(groups):   # aggre/1 usorts the {Topic, Group} entries
                live = [m for m in self.shared.get((g, f), []) if m not in self.dead]
                m = self._pick(g, f, t, clientids[k] if clientids else b"", live)
                entries.append(("share", f, ("ok", 1) if m is not None else ("error", "no_subscribers")))
            if not entries:   # route([], Delivery)
                self._dropped(t, sysf)
            out.append(entries)
        return out

    def _pick(self, group: bytes, flt: bytes, source_topic: bytes, clientid: bytes,
              members: Optional[List[int]] = None) -> Optional[int]:
        """One member of a group for a delivery without an ack (SharedSub.pick,
        emqx_shared_sub.erl:239-290): ``publish_result`` passes the group's
        live members (the DOWNs of dead ones already processed)."""
        mem = self.shared.get((group, flt)) if members is None else members
        got = self.share.pick(group, flt, mem or [], source_topic, clientid, (), lambda m: m not in self.dead)
        return None if got is None else got[1]

    def dispatch_shared(self, group: bytes, flt: bytes, source_topic: bytes, clientid: bytes = b"", qos: int = 0,
                        ack_enabled: bool = False, respond=None):
        """``emqx_shared_sub:dispatch/3`` for one (filter, group) entry of the
        fan-out, with the ack/nack redispatch (SharedSub.dispatch) over the
        group's members as ?TAB holds them — a member whose process is gone
        but not yet cleaned up answers an ack-requiring delivery with DOWN.
        ``respond(member)`` overrides the live members' answers (default: ack)."""
        members = self.shared.get((group, flt), [])

        def answer(m):
            if m in self.dead:
                return "down"
            return respond(m) if respond is not None else "ack"

        return self.share.dispatch(group, flt, members, source_topic, clientid, qos, ack_enabled, answer,
                                   lambda m: m not in self.dead)
