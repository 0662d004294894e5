"""Multi-GPU route lookup on one node, one process per GPU.

Two layouts, both over ``torch.distributed`` (backend "nccl" = RCCL on ROCm,
"gloo" for the CPU tests):

* **replicate** (default for throughput): every rank holds the whole filter
  table (10M filters is ~2 GB of a 288 GB HBM3E card) and matches its own
  slice of the topic stream.  Topics are independent units, so there is no
  data-path collective — weak scaling.
* **prefix** (tables too large for one GPU, the layout that scales): filters
  are partitioned by their first two words (``egm_prefix_assign``: keys hash
  into virtual partitions mapped to ranks by filter count; a filter with '+' or
  '#' in its first two levels is replicated), every rank routes its OWN topic
  batch to the key owners (``egm_prefix_route``, HIP) and ONE
  ``all_to_all_single`` exchanges the fixed-size slots; each rank matches the
  slots it received against its partition (``egm_match_device_counted``, the
  topic count read on the device).  No broadcast, no gather; results stay on
  the owner rank (where, in a broker, the owner's subscribers are
  dispatched).  ``PrefixExchange.run`` adds one 24-byte all-reduce per step so
  that a slot overflowed by key skew is redone with grown slots.
* **shard** (round 3, kept for comparison): filters are split by
  ``word_hash(filter) mod G`` (egm_common.h filter_shard) with global filter
  ids; rank 0's topic batch is broadcast, every rank matches it against its
  shard, per-topic counts are all-gathered and the id lists gathered to rank 0
  (point-to-point over xGMI), where the shard rows are merged.  The match set
  over F is the disjoint union of the match sets over the shards, so the
  merge needs no dedup.

The reference replicates its route tables to every node with mnesia/ekka and
matches locally (apps/emqx/src/emqx_trie.erl:53, emqx_router.erl:71); this is
the intra-node, GPU-native counterpart.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, List, Optional, Tuple

import numpy as np

from . import _lib as L


def shard_of(strings, n_shards: int) -> np.ndarray:
    """Shard index per filter (u32), computed by the library's filter_shard."""
    lib = L.load()
    off = np.ascontiguousarray(strings.off, dtype=np.uint32)
    out = np.zeros(len(off) - 1, dtype=np.uint32)
    rc = lib.egm_shard_assign(C.c_void_p(strings.blob.ctypes.data), C.c_void_p(off.ctypes.data), len(off) - 1,
                              n_shards, C.c_void_p(out.ctypes.data))
    if rc != 0:
        raise L.EgmError(rc, "egm_shard_assign")
    return out


LocalMatch = Callable[["object", "object", int], Tuple["object", "object", int, bool]]
Merge = Callable[["object", list, int, int], Tuple["object", "object"]]


class ShardExchange:
    """Collective steps of the filter-sharded layout (torch.distributed).

    ``local_match(blob, off, n) -> (row int64[n+1], ids int32, total, overflow)``
    is this rank's matcher on its filter shard (the GPU path in production,
    ``total``/``overflow`` already known on the host); ``merge(counts, ids_list,
    total, n) -> (row, ids)`` combines the gathered shard CSRs on rank 0 (the
    HIP kernel behind ``egm_shard_merge``, see ``gpu_merge``).  The CPU tests
    inject both to run the collectives over gloo.

    One step:
      1. broadcast the topic batch (blob, offsets) from rank 0      [RCCL]
      2. every rank matches it against its shard
      3. all-gather (total, overflow) per rank: 2 x int64          [RCCL]
      4. gather per-topic counts and ids to rank 0, point to point [RCCL]
      5. rank 0 merges: per topic, shard 0's ids, then shard 1's ...
    A rank whose id buffer overflowed is reported to every rank in 3, and the
    step returns ``None`` everywhere with the true totals (``last_totals``) so
    the caller can grow its buffers — no rank ever sends a short buffer.
    """

    def __init__(self, rank: int, world: int, device, local_match: LocalMatch, merge: Optional[Merge] = None,
                 group=None):
        if rank == 0 and merge is None:
            raise ValueError("rank 0 needs a merge function (emqx_amd.dist.gpu_merge)")
        self.rank, self.world, self.device = rank, world, device
        self.local_match = local_match
        self.merge = merge
        self.group = group
        self.last_totals: List[int] = []
        self.last_overflow = False
        self._bufs = {}

    def _buf(self, key, numel, dtype):
        import torch
        b = self._bufs.get(key)
        if b is None or b.numel() < numel or b.dtype != dtype:
            b = torch.empty(max(numel, 1), dtype=dtype, device=self.device)
            self._bufs[key] = b
        return b[:numel]

    def step(self, blob=None, off=None, sizes: Optional[Tuple[int, int]] = None):
        """Rank 0 passes (blob u8, off int32).  ``sizes`` = (n, blob bytes) when
        every rank knows them already (skips a broadcast and a sync).
        Returns (row int64[n+1], ids int32[total]) on rank 0, None elsewhere."""
        import torch
        import torch.distributed as dist
        dev, G, g = self.device, self.world, self.group
        if sizes is None:
            meta = torch.zeros(2, dtype=torch.int64, device=dev)
            if self.rank == 0:
                meta[0] = off.numel() - 1
                meta[1] = blob.numel()
            dist.broadcast(meta, 0, group=g)                                    # sizes
            sizes = (int(meta[0].item()), int(meta[1].item()))
        n, nb = sizes
        if self.rank != 0:
            blob = self._buf("blob", nb, torch.uint8)
            off = self._buf("off", n + 1, torch.int32)
        dist.broadcast(blob, 0, group=g)                                        # 1. topic batch
        dist.broadcast(off, 0, group=g)
        row, ids, total, ovf = self.local_match(blob, off, n)                   # 2. this shard
        info = torch.tensor([total, 1 if ovf else 0], dtype=torch.int64, device=dev)
        allinfo = [torch.empty_like(info) for _ in range(G)]
        dist.all_gather(allinfo, info, group=g)                                 # 3. totals + overflow
        allinfo = torch.stack(allinfo).cpu().tolist()
        self.last_totals = [int(x[0]) for x in allinfo]
        self.last_overflow = any(x[1] for x in allinfo)
        if self.last_overflow:
            return None
        cnt = (row[1 : n + 1] - row[:n]).to(torch.int32)
        if self.rank != 0:                                                      # 4. counts + ids -> rank 0
            ops = [dist.P2POp(dist.isend, cnt.contiguous(), 0, group=g)]
            if total:
                ops.append(dist.P2POp(dist.isend, ids[:total].contiguous(), 0, group=g))
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            return None
        counts = self._buf("counts", G * n, torch.int32)
        counts[:n].copy_(cnt)
        parts = [ids[:total]]
        ops = []
        for r in range(1, G):
            ops.append(dist.P2POp(dist.irecv, counts[r * n:(r + 1) * n], r, group=g))
            b = self._buf(("ids", r), self.last_totals[r], torch.int32)
            parts.append(b)
            if self.last_totals[r]:
                ops.append(dist.P2POp(dist.irecv, b, r, group=g))
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()
        return self.merge(counts, parts, sum(self.last_totals), n)              # 5. merge


class ShardFanout:
    """The filter-sharded layout with subscriber fan-out (SURVEY §8e:
    "Subscriber CSR rows live with their filter's shard").

    One step:
      1. broadcast the topic batch from rank 0                      [RCCL]
      2. every rank matches it against its filter shard and expands the
         matches through ITS subscriber rows (emqx_broker:dispatch/2,
         apps/emqx/src/emqx_broker.erl:283-308): the deliveries of a topic are
         the disjoint union over the ranks, and each rank keeps its part where
         its subscribers' connections are
      3. reduce the per-topic delivery totals to rank 0 (SUM)       [RCCL]
         — the N of {ok, N} per topic (emqx_broker.erl:283-295)

    ``local(blob, off, n) -> (delivery_row int64[n+1], overflow)`` is this
    rank's match + fan-out.  No id or delivery list crosses xGMI: a C4 batch
    has ~4.6 G deliveries (36 GB), gathering them would be the whole cost.
    Returns (per-topic delivery totals int64[n]) on rank 0, None elsewhere;
    ``last_overflow`` is set on every rank when any rank overflowed."""

    def __init__(self, rank: int, world: int, device, local, group=None):
        self.rank, self.world, self.device, self.local, self.group = rank, world, device, local, group
        self.last_overflow = False
        self._bufs = {}

    def step(self, blob=None, off=None, sizes: Optional[Tuple[int, int]] = None):
        import torch
        import torch.distributed as dist
        dev, g = self.device, self.group
        n, nb = sizes
        if self.rank != 0:
            blob = self._bufs.get("blob")
            if blob is None or blob.numel() < nb:
                blob = self._bufs["blob"] = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
            off = self._bufs.get("off")
            if off is None or off.numel() < n + 1:
                off = self._bufs["off"] = torch.empty(n + 1, dtype=torch.int32, device=dev)
            blob, off = blob[:nb], off[: n + 1]
        dist.broadcast(blob, 0, group=g)                                        # 1. topic batch
        dist.broadcast(off, 0, group=g)
        drow, ovf = self.local(blob, off, n)                                    # 2. match + own fan-out
        flag = torch.tensor([1 if ovf else 0], dtype=torch.int64, device=dev)
        dist.all_reduce(flag, group=g)
        self.last_overflow = bool(flag.item())
        if self.last_overflow:
            return None
        per = (drow[1 : n + 1] - drow[:n]).contiguous()
        dist.reduce(per, 0, op=dist.ReduceOp.SUM, group=g)                       # 3. totals -> rank 0
        return per if self.rank == 0 else None


def gpu_merge(gm, stream: int, out_row, out_ids):
    """The merge of ShardExchange on rank 0: egm_shard_merge (HIP kernel) into
    caller-owned device buffers out_row int64[n+1] and out_ids int32[cap]."""

    def merge(counts, parts, total, n):
        if total > out_ids.numel():
            raise ValueError(f"merged ids {total} exceed the output buffer {out_ids.numel()}")
        gm.shard_merge(len(parts), n, counts.data_ptr(), [p.data_ptr() for p in parts], total, stream,
                       out_row.data_ptr(), out_ids.data_ptr(), out_ids.numel())
        return out_row[: n + 1], out_ids[:total]

    return merge


# ---------------------------------------------------------------- prefix ----
N_VPARTS = 4096


def prefix_assign(strings, n_ranks: int, n_vparts: int = N_VPARTS) -> Tuple[np.ndarray, np.ndarray]:
    """(vpart_rank u8[n_vparts], filter_rank u32[n]) — egm_prefix_assign; a
    filter_rank of L.EGM_PREFIX_ALL means the filter lives on every rank."""
    lib = L.load()
    off = np.ascontiguousarray(strings.off, dtype=np.uint32)
    n = len(off) - 1
    vr = np.zeros(n_vparts, dtype=np.uint8)
    fr = np.zeros(n, dtype=np.uint32)
    rc = lib.egm_prefix_assign(C.c_void_p(strings.blob.ctypes.data), C.c_void_p(off.ctypes.data), n, n_vparts,
                               n_ranks, C.c_void_p(vr.ctypes.data), C.c_void_p(fr.ctypes.data))
    if rc != 0:
        raise L.EgmError(rc, "egm_prefix_assign")
    return vr, fr


class PrefixSlots:
    """The send/receive slot layout of egm_prefix_route (include/emqx_gpu_match.h)."""

    def __init__(self, n_ranks: int, cap_topics: int, cap_bytes: int):
        self.n_ranks, self.cap_topics, self.cap_bytes = n_ranks, cap_topics, cap_bytes
        self.off_tids = 16
        self.off_offsets = 16 + 4 * cap_topics
        self.off_bytes = (self.off_offsets + 4 * (cap_topics + 1) + 15) & ~15
        self.slot_bytes = (self.off_bytes + cap_bytes + 15) & ~15
        assert self.slot_bytes == int(L.load().egm_prefix_slot_bytes(n_ranks, cap_topics, cap_bytes))

    @classmethod
    def for_batch(cls, n_ranks: int, n_topics: int, n_bytes: int, slack: float = 1.25):
        """Capacities for batches of up to n_topics / n_bytes per rank, spread
        over n_ranks owners with `slack` for imbalance (C2 at 8 ranks: the
        busiest owner gets 1.03x the mean)."""
        ct = int(n_topics * slack / n_ranks) + 1024
        cb = int(n_bytes * slack / n_ranks) + 65536
        return cls(n_ranks, ct, cb)

    def parse(self, buf: np.ndarray, r: int):
        """Slot r of a host copy of a send/receive buffer: (count, bytes,
        overflow, source topic indices, offsets[count+1], topic bytes)."""
        s = buf[r * self.slot_bytes:(r + 1) * self.slot_bytes]
        h = s[:16].view(np.uint32)
        cnt, nb, ovf = int(h[0]), int(h[1]), int(h[2])
        tids = s[self.off_tids:self.off_tids + 4 * cnt].view(np.uint32)
        offs = s[self.off_offsets:self.off_offsets + 4 * (cnt + 1)].view(np.uint32)
        return cnt, nb, ovf, tids, offs, s[self.off_bytes:self.off_bytes + nb]


def prefix_key(topic: bytes) -> bytes:
    """The partition key: the bytes before the second '/' (egm_common.h prefix_key_len)."""
    i = topic.find(b"/")
    if i < 0:
        return topic
    j = topic.find(b"/", i + 1)
    return topic if j < 0 else topic[:j]


def prefix_route_reference(blob: np.ndarray, off: np.ndarray, vpart_rank: np.ndarray, ps: PrefixSlots) -> np.ndarray:
    """Host restatement of egm_prefix_route (the gloo path and the GPU test's
    checker): the same slots, topics in input order within a slot (the kernel
    may order them differently: per-topic content is what is compared).  A
    slot past its capacity keeps the topics placed before the capacity ran out
    (a topic is placed iff its position < cap_topics and its bytes end within
    cap_bytes — in slot order that is a prefix) and flags overflow."""
    lib = L.load()
    G, V = ps.n_ranks, len(vpart_rank)
    out = np.zeros(G * ps.slot_bytes, dtype=np.uint8)
    b = blob.tobytes()
    per = [[] for _ in range(G)]
    for t in range(len(off) - 1):
        tp = b[int(off[t]):int(off[t + 1])]
        k = prefix_key(tp)
        r = int(vpart_rank[int(lib.egm_word_hash(k, len(k))) % V])
        per[r].append((t, tp))
    for r in range(G):
        base = r * ps.slot_bytes
        items = per[r]
        placed, nbytes = 0, 0
        for _, x in items:
            if placed >= ps.cap_topics or nbytes + len(x) > ps.cap_bytes:
                break
            placed += 1
            nbytes += len(x)
        ovf = placed < len(items)
        items = items[:placed]
        tids = np.array([t for t, _ in items], dtype=np.uint32)
        lens = np.array([len(x) for _, x in items], dtype=np.uint64)
        offs = np.full(ps.cap_topics + 1, nbytes, dtype=np.uint32)
        offs[:len(items)] = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint32) if len(items) else []
        out[base:base + 16] = np.array([len(items), nbytes, int(ovf), 0], dtype=np.uint32).view(np.uint8)
        out[base + ps.off_tids:base + ps.off_tids + 4 * len(items)] = tids.view(np.uint8)
        out[base + ps.off_offsets:base + ps.off_offsets + 4 * (ps.cap_topics + 1)] = offs.view(np.uint8)
        data = b"".join(x for _, x in items)
        out[base + ps.off_bytes:base + ps.off_bytes + len(data)] = np.frombuffer(data, dtype=np.uint8)
    return out


SlotMatch = Callable[["object", int], object]


class TorchComm:
    """The prefix exchange's two collectives over torch.distributed (RCCL
    over xGMI on the GPU, gloo on the CPU)."""

    def __init__(self, group=None):
        self.group = group

    def all_to_all(self, recv, send):
        import torch.distributed as dist
        dist.all_to_all_single(recv, send, group=self.group)

    def all_max(self, t):
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t


class PrefixExchange:
    """One step of the prefix-partition layout on every rank (torch.distributed):

      1. route this rank's own topic batch into n_ranks slots    [HIP egm_prefix_route]
      2. all_to_all_single of the equal-size slots               [RCCL over xGMI]
      3. match each received slot against this rank's partition [egm_match_device_counted]

    ``make(ps) -> (route, match_slot)`` builds the two injected stages for a
    slot layout: ``route(blob, off, n) -> send`` (uint8 tensor of n_ranks *
    slot_bytes) and ``match_slot(recv, g) -> result`` — the GPU path in
    production (``gpu_route`` / ``gpu_match_slot``), numpy + the oracle in the
    gloo tests.  ``comm`` carries the collectives (``TorchComm`` by default).

    ``step`` never syncs the host: a slot's topic count is read from its
    header on the device, an overflowed slot (header flag) is matched as empty,
    and ``overflow_flag`` accumulates the received flags on the device for the
    caller to check where it syncs anyway.  ``run`` is the step that always
    completes: one small all-reduce decides whether any rank received an
    overflowed slot, and if so every rank regrows its slots to hold the
    largest rank's whole batch — which no key skew can overflow, even every
    topic sharing one prefix — and redoes the step.  The grown layout is kept
    (a skewed workload stays skewed).  The reference has no such step: it
    replicates its tables (apps/emqx/src/emqx_trie.erl:53, emqx_router.erl:71)."""

    def __init__(self, rank: int, world: int, device, ps: PrefixSlots, make, comm=None):
        import torch
        self.rank, self.world, self.device = rank, world, device
        self.make = make
        self.comm = comm if comm is not None else TorchComm()
        self.overflow_flag = torch.zeros(1, dtype=torch.int64, device=device)
        self.last_flag = torch.zeros(1, dtype=torch.int64, device=device)
        self.reruns = 0
        self._layout(ps)

    def _layout(self, ps: PrefixSlots):
        import torch
        self.ps = ps
        self.route, self.match_slot = self.make(ps)
        self.recv = torch.empty(self.world * ps.slot_bytes, dtype=torch.uint8, device=self.device)

    def exchange(self, send):
        if self.world > 1:
            self.comm.all_to_all(self.recv, send)                                # 2. exchange
            return self.recv
        return send

    def step(self, blob, off, n: int):
        import torch
        recv = self.exchange(self.route(blob, off, n))                           # 1. route, 2.
        hdr = recv.view(self.world, self.ps.slot_bytes)[:, :16].view(torch.int32)
        self.last_flag = hdr[:, 2].to(torch.int64).sum().reshape(1)             # stays on the device
        self.overflow_flag += self.last_flag
        return [self.match_slot(recv, g) for g in range(self.world)]             # 3. match

    def run(self, blob, off, n: int, n_bytes: int):
        """step(), redone with grown slots if any rank's received slot
        overflowed (one all-reduce of 3 int64 per step: a host sync)."""
        import torch
        out = self.step(blob, off, n)
        info = torch.cat([self.last_flag, torch.tensor([n, n_bytes], dtype=torch.int64, device=self.device)])
        if self.world > 1:
            info = self.comm.all_max(info)
        flag, mn, mb = (int(x) for x in info.tolist())
        if flag == 0:
            return out
        self.overflow_flag -= self.last_flag                                    # handled here
        self.reruns += 1
        self._layout(PrefixSlots(self.world, max(mn, 1), max(mb, 16)))
        out = self.step(blob, off, n)
        return out

    def overflowed(self) -> bool:
        """Any overflow in a step not redone by run() (a host sync: call it
        where the caller syncs anyway)."""
        return bool(self.overflow_flag.item())


def gpu_route(gm, ps: PrefixSlots, d_vpart_rank, stream: int, send):
    """route() of PrefixExchange on the GPU: egm_prefix_route into `send` (a
    device uint8 tensor of ps.n_ranks * ps.slot_bytes)."""

    def route(blob, off, n):
        gm.prefix_route(blob.data_ptr(), off.data_ptr(), n, d_vpart_rank.data_ptr(), d_vpart_rank.numel(), ps.n_ranks,
                        ps.cap_topics, ps.cap_bytes, stream, send.data_ptr())
        return send

    return route


def _require_torch_stream(stream: int):
    """The GPU stages launch on `stream` and then read their results (the
    topic gather below) and drop old buffers on torch's CURRENT stream: the
    two must be one stream, or the gather could read d_topic before the
    compaction wrote it and the caching allocator could hand a buffer the
    kernels still write to someone else.  Checked, not assumed."""
    import torch
    cur = torch.cuda.current_stream().cuda_stream
    if int(stream or 0) != int(cur or 0):
        raise ValueError(f"prefix stages: stream {stream:#x} is not torch's current stream {cur:#x}")


def gpu_match_slot(gm, ps: PrefixSlots, mode: int, stream: int, rows: list, ids: list, topic: Optional[list] = None):
    """match_slot() of PrefixExchange on the GPU: slot g of the received buffer
    matched in place (no copy) with its count read on the device; rows[g]
    (int64[cap_topics + 1]) and ids[g] (int32) are the caller's output buffers.
    Returns (row, ids, source topic indices) views of slot g: row k holds the
    matches of source topic tids[k].  With `topic` (int32[cap_topics] buffers)
    the rows come in the walk's order (egm_match_device_counted_ordered) and
    the returned indices are gathered through the row -> slot topic map."""
    import torch
    _require_torch_stream(stream)

    def match_slot(recv, g):
        base = recv.data_ptr() + g * ps.slot_bytes
        tids = recv[g * ps.slot_bytes + ps.off_tids:g * ps.slot_bytes + ps.off_offsets].view(torch.int32)
        if topic is None:
            gm.match_device_counted(base + ps.off_bytes, ps.cap_bytes, base + ps.off_offsets, ps.cap_topics, base,
                                    mode, stream, rows[g].data_ptr(), ids[g].data_ptr(), ids[g].numel())
            return rows[g], ids[g], tids
        gm.match_device_counted_ordered(base + ps.off_bytes, ps.cap_bytes, base + ps.off_offsets, ps.cap_topics, base,
                                        mode, stream, rows[g].data_ptr(), topic[g].data_ptr(), ids[g].data_ptr(),
                                        ids[g].numel())
        return rows[g], ids[g], tids[topic[g].long()]

    return match_slot


def gpu_prefix_stages(gm, d_vpart_rank, mode: int, stream: int, ids_per_topic: int = 64, ordered: bool = False):
    """make(ps) for PrefixExchange on the GPU: a send buffer, per-slot row and
    id buffers sized for ps (ids_per_topic per slot topic + 4096), and the
    route / match stages over them.  The buffers stay reachable as attributes
    of the returned route function (`route.send`, `match.rows`, `match.ids`).
    ordered: the slots' rows in the walk's order (gpu_match_slot)."""
    import torch

    def make(ps: PrefixSlots):
        _require_torch_stream(stream)
        dev = d_vpart_rank.device
        send = torch.zeros(ps.n_ranks * ps.slot_bytes, dtype=torch.uint8, device=dev)
        rows = [torch.zeros(ps.cap_topics + 1, dtype=torch.int64, device=dev) for _ in range(ps.n_ranks)]
        ids = [torch.zeros(ids_per_topic * ps.cap_topics + 4096, dtype=torch.int32, device=dev)
               for _ in range(ps.n_ranks)]
        topic = ([torch.zeros(ps.cap_topics, dtype=torch.int32, device=dev) for _ in range(ps.n_ranks)]
                 if ordered else None)
        route = gpu_route(gm, ps, d_vpart_rank, stream, send)
        match = gpu_match_slot(gm, ps, mode, stream, rows, ids, topic)
        route.send, match.rows, match.ids = send, rows, ids
        return route, match

    return make


def topic_slice(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Replicate layout: the [lo, hi) slice of a topic batch this rank matches."""
    return n * rank // world, n * (rank + 1) // world
