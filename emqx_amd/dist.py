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
from typing import Callable, List, Sequence, Tuple

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


def merge_shard_results(parts: Sequence[Tuple[np.ndarray, np.ndarray]]) -> Tuple[np.ndarray, np.ndarray]:
    """Per topic, concatenate the shard rows in shard order (host, numpy)."""
    rows = [np.asarray(r, dtype=np.uint64) for r, _ in parts]
    n = len(rows[0]) - 1
    cnts = np.stack([np.diff(r).astype(np.int64) for r in rows])          # [G, n]
    tot = cnts.sum(axis=0)
    row = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(tot, out=row[1:])
    before = np.cumsum(cnts, axis=0) - cnts                                 # ids of earlier shards per topic
    ids = np.zeros(int(row[-1]), dtype=np.uint32)
    for g, (r, gi) in enumerate(parts):
        c = cnts[g]
        if c.sum() == 0:
            continue
        tpos = np.repeat(np.arange(n, dtype=np.int64), c)
        k = np.arange(len(gi), dtype=np.int64) - np.repeat(rows[g][:-1].astype(np.int64), c)
        ids[row[:-1].astype(np.int64)[tpos] + before[g][tpos] + k] = gi
    return row, ids


def merge_shard_results_torch(counts, ids_list):
    """Device merge on rank 0: counts [G, n] (int64), ids_list[g] (int32).

    Returns (row int64 [n+1], ids int32) — the same layout as the single-GPU
    CSR (shard g's ids of topic t follow those of shards < g).
    """
    import torch
    G, n = counts.shape
    dev = counts.device
    tot = counts.sum(0)
    row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(tot, 0, out=row[1:])
    before = torch.cumsum(counts, 0) - counts
    out = torch.empty(int(row[-1].item()), dtype=torch.int32, device=dev)
    for g in range(G):
        c = counts[g]
        m = int(c.sum().item())
        if m == 0:
            continue
        t = torch.repeat_interleave(torch.arange(n, device=dev), c)
        srow = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(c, 0, out=srow[1:])
        k = torch.arange(m, device=dev) - srow[:-1][t]
        out[row[:-1][t] + before[g][t] + k] = ids_list[g][:m]
    return row, out


LocalMatch = Callable[["object", "object", int], Tuple["object", "object"]]


class ShardExchange:
    """Collective steps of the filter-sharded layout (torch.distributed).

    ``local_match(blob, off, n) -> (row int64[n+1], ids int32[m])`` is this
    rank's matcher (the GPU path in production; tests inject a CPU matcher to
    exercise the collectives over gloo).
    """

    def __init__(self, rank: int, world: int, device, local_match: LocalMatch, group=None):
        self.rank, self.world, self.device = rank, world, device
        self.local_match = local_match
        self.group = group

    def step(self, blob=None, off=None):
        """Rank 0 passes (blob u8, off int32); returns merged (row, ids) on rank 0."""
        import torch
        import torch.distributed as dist
        dev = self.device
        meta = torch.zeros(2, dtype=torch.int64, device=dev)
        if self.rank == 0:
            meta[0] = off.numel() - 1
            meta[1] = blob.numel()
        dist.broadcast(meta, 0, group=self.group)                              # 1. sizes
        n, nb = int(meta[0].item()), int(meta[1].item())
        if self.rank != 0:
            blob = torch.empty(nb, dtype=torch.uint8, device=dev)
            off = torch.empty(n + 1, dtype=torch.int32, device=dev)
        dist.broadcast(blob, 0, group=self.group)                              # 2. topic batch
        dist.broadcast(off, 0, group=self.group)
        row, ids = self.local_match(blob, off, n)                              # 3. local shard
        cnt = (row[1:] - row[:-1]).to(torch.int64)
        allc = [torch.empty_like(cnt) for _ in range(self.world)]
        dist.all_gather(allc, cnt, group=self.group)                           # 4. counts
        totals = [int(c.sum().item()) for c in allc]
        if self.rank == 0:                                                     # 5. gatherv ids
            bufs = [ids[: totals[0]].to(torch.int32)]
            ops = []
            for g in range(1, self.world):
                b = torch.empty(max(totals[g], 1), dtype=torch.int32, device=dev)
                bufs.append(b)
                if totals[g]:
                    ops.append(dist.P2POp(dist.irecv, b[: totals[g]], g, group=self.group))
            for w in (dist.batch_isend_irecv(ops) if ops else []):
                w.wait()
            return merge_shard_results_torch(torch.stack(allc), bufs)
        if totals[self.rank]:
            w = dist.batch_isend_irecv([dist.P2POp(dist.isend, ids[: totals[self.rank]].to(torch.int32).contiguous(),
                                                   0, group=self.group)])
            for x in w:
                x.wait()
        return None


def topic_slice(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Replicate layout: the [lo, hi) slice of a topic batch this rank matches."""
    return n * rank // world, n * (rank + 1) // world
