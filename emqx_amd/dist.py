"""Multi-GPU route lookup on one node, one process per GPU.

Two layouts, both over ``torch.distributed`` (backend "nccl" = RCCL on ROCm,
"gloo" for the CPU tests):

* **replicate** (default for throughput): every rank holds the whole filter
  table (10M filters is ~2 GB of a 288 GB HBM3E card) and matches its own
  slice of the topic stream.  Topics are independent units, so there is no
  data-path collective — weak scaling.
* **shard** (tables too large or too slow for one GPU): filters are split by
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


def topic_slice(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Replicate layout: the [lo, hi) slice of a topic batch this rank matches."""
    return n * rank // world, n * (rank + 1) // world
