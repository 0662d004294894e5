#!/usr/bin/env python3
"""bench.py — publish-time route lookup throughput on MI355X.

Metric (BASELINE.json): topics matched/sec (node) at 10M filters, 1/2/4/8
GPUs, with the HBM-roofline fraction of the dominant kernel.

A *step* is one pass of the hot path — tokenise + NFA walk (+ heavy path) +
CSR finalisation, i.e. emqx_router:match_routes/1's filter sets for a whole
batch — over one batch of synthetic topics already resident in HBM.
The steps run one batch at a time on one HIP stream, so the walk's HIP-event
time is its own (the roofline's kernel time); the same steps with two batches
in flight (two streams with their own workspaces: one batch's sort, scan and
compaction beside the next one's walk) are timed after them and reported as
the line's `pipelined` (`--streams 2` makes that the timed mode instead).

Layouts (emqx_amd/dist.py), named in the line's config.workload:
  replicate (default)  every GPU holds the 10M-filter table and matches its own
                       10M-topic batch; no data-path collective -> "weak".
  prefix               filters partitioned by their first two words (a filter
                       with '+'/'#' there on every rank); every GPU routes its
                       OWN 10M-topic batch to the prefix owners with one RCCL
                       all_to_all and matches what it receives against its
                       partition -> "weak"; no broadcast, no gather, no host
                       sync per step (SURVEY §8e "partition by root word").
  shard                (round 3) filters split by hash, rank 0's batch
                       broadcast, counts and ids gathered to rank 0 over RCCL
                       and merged by the HIP merge kernel -> "strong".

At N>1 the replicate `value` is followed by the prefix layout timed on the
same node (the line's `sharded`; --sharded-layout shard for the round-3 one).

    python bench.py [--gpus N --steps K --warmup W] [--config c2] [--mode replicate|prefix|shard]

Rank 0 prints ONE JSON line on stdout; progress goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "topics matched/sec (node) at 10M filters, 1/2/4/8 GPUs; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

WORKLOADS = {
    "c1": "C1: 1M filters (depth 4-8, 20% wildcard) x 10M-topic batch per GPU",
    "c2": "C2: 10M wildcard filters (depth 4-8, '+' p=.15, '#' p=.5) x 10M-topic batch per GPU",
    "c3": "C3: 10M wildcard filters, depth-16 topics, '+' p=.35, '#' p=.7, match + subscriber fan-out "
          "(1+Poisson(1) subscribers, 0.1% of filters with 2000, 10% $share/g0..g63 groups of 2-16 members)",
    "c4": "C4: 100M filters (depth 4-8, 20% wildcard) x 10M-topic batch per GPU, match + subscriber fan-out "
          "(1+Poisson(1) subscribers, 0.1% of filters with 2000, 10% $share groups)",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def kernel_src_sha() -> str:
    """Hash of the kernel sources: a PMC traffic record is only used for the
    build it was collected on (tools/pmc_traffic.py stores the same hash)."""
    import hashlib
    h = hashlib.sha256()
    for name in ("egm_kernels.hip", "egm_kernels.h", "egm_common.h"):
        with open(os.path.join(ROOT, "emqx_amd", "csrc", name), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def levels_sum(blob: np.ndarray, off: np.ndarray) -> int:
    nbytes = int(off[-1])
    return int(np.count_nonzero(blob[:nbytes] == ord("/"))) + (len(off) - 1)


def walk_traffic(config: str, filters: int, topics: int):
    """HBM bytes per k_walk launch from the committed PMC record of this exact
    workload (tools/pmc_traffic.py over rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes), or None.  bench.py cannot collect counters itself: PMC passes
    need their own rocprofv3 runs."""
    import glob
    found = []
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_walk_pmc.json"))):
        try:
            with open(p) as fh:
                r = json.load(fh)
        except (OSError, ValueError):
            continue
        if (r.get("workload") == config and r.get("filters") == filters and r.get("topics") == topics
                and r.get("kernel_src_sha") == kernel_src_sha()):
            found.append((r, os.path.relpath(p, ROOT)))
    if not found:
        return None
    # several records of one source must agree (the last one in glob
    # order won silently); disagreeing records give no traffic at all
    tr = [r["traffic_bytes_per_launch"] for r, _ in found]
    if max(tr) > 1.03 * min(tr):
        log(f"PMC records of this kernel source disagree ({[p for _, p in found]}): traffic not reported")
        return None
    return found[-1]


def cpu_baseline(f, t, match_mode: int, seconds: float) -> dict:
    """C++ restatement of emqx_trie (compact) + route lookup, timed on host cores."""
    from emqx_amd import hostinfo
    from oracle.cpp import OracleTrie
    threads = hostinfo.usable_cpus()   # every CPU this process may run on (affinity and cgroup quota)
    o = OracleTrie(True, match_mode)
    t0 = time.time()
    o.add(f.blob, f.off)
    build_s = time.time() - t0
    probe = min(t.n, 2_000 * threads)
    sub = t.subset(np.arange(probe))
    t0 = time.time()
    o.match_count(sub.blob, sub.off, threads)
    dt = max(time.time() - t0, 1e-3)
    n = int(min(t.n, max(probe, probe * seconds / dt)))
    sub = t.subset(np.arange(n))
    t0 = time.time()
    m = o.match_count(sub.blob, sub.off, threads)
    dt = time.time() - t0
    # one thread on a short prefix of the same sample (1 and N threads)
    n1 = max(1, min(n, int(n / threads / 4)))
    sub1 = t.subset(np.arange(n1))
    t1 = time.time()
    o.match_count(sub1.blob, sub1.off, 1)
    dt1 = max(time.time() - t1, 1e-3)
    return {"value": n / dt, "unit": "topics/s", "cores": threads, "kind": "port",
            "value_1thread": n1 / dt1, "sample_1thread": f"first {n1} topics, 1 thread",
            "sample": f"first {n} topics of the same batch, {threads} threads, static partition; "
                      f"C++ restatement of emqx_trie compact DFS + lookup_routes (oracle/trie_oracle.cpp), "
                      f"not BEAM; {m} matches; table build {build_s:.1f}s untimed",
            "host": hostinfo.describe()}


def host_e2e(gm, t, mode, batch: int = 1_000_000, batches: int = 24, depth: int = 3) -> dict:
    """The PCIe-inclusive rate the NIF sees: topics/s from
    a host topic blob to a host CSR through egm_match_submit / egm_match_wait
    (pinned staging, H2D on a copy stream, match, D2H on the SDMA engines),
    `depth` batches in flight (a broker's dirty schedulers submit
    concurrently).  Never `value` (which is measured with the batch in HBM).
    The NIF submits with EGM_RESULT_PACKED (u32 rows, 3-byte ids; round 6,
    VERDICT r5 item 7): that form is this leg's value, the plain one beside it."""
    from emqx_amd import _lib as L
    # each form once untimed first: the pipeline slots' id room grows on their
    # first batches (an overflowed batch is rerun), which must not land in either timing
    host_e2e_form(gm, t, mode | L.EGM_RESULT_PACKED, batch, 2 * depth, depth)
    host_e2e_form(gm, t, mode, batch, 2 * depth, depth)
    packed = host_e2e_form(gm, t, mode | L.EGM_RESULT_PACKED, batch, batches, depth)
    plain = host_e2e_form(gm, t, mode, batch, batches, depth)
    packed["result_form"] = "packed: u32 row starts + 3-byte ids (EGM_RESULT_PACKED, the NIF's submit/3)"
    packed["plain_form"] = {k: plain[k] for k in ("value", "ms_per_batch", "submit_ms_per_batch", "wait_ms_per_batch",
                                                  "host_bytes_per_batch")}
    return packed


def host_e2e_form(gm, t, mode, batch: int, batches: int, depth: int) -> dict:
    from emqx_amd import _lib as L
    batch = min(batch, t.n)
    parts = [t.subset(np.arange(i * batch, (i + 1) * batch)) for i in range(max(1, min(2, t.n // batch)))]
    # create and size the pipeline slots `depth` batches in flight use (untimed)
    tk = [gm.submit(parts[k % len(parts)].blob, parts[k % len(parts)].off, mode) for k in range(depth)]
    for x in tk:
        gm.wait(x, copy=False)
    ids = 0
    t_sub = t_wait = 0.0
    t0 = time.perf_counter()
    inflight = []
    for k in range(batches + 1):
        if k < batches:
            p = parts[k % len(parts)]
            a = time.perf_counter()
            inflight.append(gm.submit(p.blob, p.off, mode))
            t_sub += time.perf_counter() - a
        if len(inflight) == depth or (k == batches and inflight):
            a = time.perf_counter()
            gm.wait(inflight.pop(0), copy=False)
            t_wait += time.perf_counter() - a
            ids += gm.last_stats()["n_ids"]
    while inflight:
        gm.wait(inflight.pop(0), copy=False)
        ids += gm.last_stats()["n_ids"]
    dt = time.perf_counter() - t0
    packed_form = bool(mode & L.EGM_RESULT_PACKED) and gm.wait(gm.submit(parts[0].blob, parts[0].off, mode)).id_bytes == 3
    return {"value": batch * batches / dt, "unit": "topics/s", "batch_topics": batch, "batches": batches,
            "in_flight": depth, "ms_per_batch": dt / batches * 1e3,
            "submit_ms_per_batch": t_sub / batches * 1e3, "wait_ms_per_batch": t_wait / batches * 1e3,
            "host_bytes_per_batch": {"in": int(parts[0].off[-1]) + 4 * (batch + 1),
                                     "out": (int(ids / batches) * 3 + 5 * batch + 4) if packed_form else
                                            (int(ids / batches) * 4 + 9 * batch + 8)},
            "path": "host blob -> pinned staging -> H2D -> match -> SDMA D2H into pinned CSR (egm_match_submit/wait)"}


def host_batcher_curve(gm, t, mode, sizes=(1024, 4096, 16384, 65536), depth: int = 2, seconds: float = 0.3,
                       default_size: int = 4096) -> dict:
    """The drop-in's own operating point: the Erlang
    batcher (erl/emqx_gpu_batch.erl: batch_size 4096, depth 2, linger 1 ms;
    emqx_batch.erl:50-81's size + linger policy) commits a batch of topics to
    submit/3 and answers its callers when wait/2 returns, with at most `depth`
    tickets in flight.  Saturated (every batch full, the next one committed as
    soon as a ticket slot frees), per batch size: topics/s and the latency of
    each batch from its submit to its wait-return (p50 / p99) — what a
    publisher's match_routes/1 call waits on top of the linger
    (emqx_broker.erl:200-209, the PUBACK after it, emqx_channel.erl:601-609).
    Host blob in, host CSR out, through egm_match_submit / egm_match_wait."""
    out = []
    pool = min(t.n, 1 << 20)
    for b in sizes:
        b = min(b, pool)
        k = max(2, min(16, pool // b))
        parts = [t.subset(np.arange(i * b, (i + 1) * b)) for i in range(k)]
        tk = [gm.submit(parts[i % k].blob, parts[i % k].off, mode) for i in range(depth + 1)]   # slots sized, untimed
        for x in tk:
            gm.wait(x, copy=False)
        lat = []
        inflight = []
        done = i = 0
        t0 = time.perf_counter()
        while True:
            running = time.perf_counter() - t0 < seconds or i < 4 * depth
            if running:   # the next full batch, committed as soon as a ticket slot is free
                p = parts[i % k]
                inflight.append((time.perf_counter(), gm.submit(p.blob, p.off, mode)))
                i += 1
            if inflight and (len(inflight) == depth or not running):
                ts, tick = inflight.pop(0)
                gm.wait(tick, copy=False)
                lat.append(time.perf_counter() - ts)
                done += 1
            if not running and not inflight:
                break
        dt = time.perf_counter() - t0
        lat_ms = np.array(lat) * 1e3
        out.append({"batch_topics": b, "in_flight": depth, "batches": done, "topics_per_s": b * done / dt,
                    "latency_ms_p50": float(np.percentile(lat_ms, 50)), "latency_ms_p99": float(np.percentile(lat_ms, 99)),
                    "latency_ms_max": float(lat_ms.max())})
    dflt = next((r for r in out if r["batch_topics"] == default_size), None)
    return {"defaults": {"batch_size": default_size, "depth": depth, "linger_ms": 1}, "at_defaults": dflt,
            "sweep": out,
            "what": "saturated batcher: full batches, `depth` tickets in flight; latency = submit -> wait-return "
                    "of one batch (a caller also waits up to linger_ms for its batch to fill)"}


def _heartbeat(period: float = 30.0):
    """Progress on stderr while long host steps (100M-filter generation and
    table build) run inside ctypes calls, so a watchdog sees a live process."""
    import threading
    t0 = time.time()

    def beat():
        while True:
            time.sleep(period)
            log(f"[heartbeat] {time.time() - t0:.0f}s")

    threading.Thread(target=beat, daemon=True).start()


LAYOUTS = {
    "replicate": "replicated table: every GPU holds all filters and matches its own topic batch "
                 "(no data-path collective)",
    "prefix": "prefix-partitioned: filters split by their first two words (those with '+'/'#' there on every "
              "rank), every GPU routes its own topic batch to the prefix owners with one RCCL all_to_all and "
              "matches what it receives; results stay on the owner (no broadcast, no gather)",
    "shard": "filter-sharded: filters split over the GPUs by word_hash(filter) mod N, rank 0's topic batch "
             "broadcast, per-topic counts and ids gathered to rank 0 and merged by the HIP merge kernel "
             "(RCCL over xGMI; at N=1 the collectives are no-ops)",
}


class ShardLeg:
    """The filter-sharded layout (BASELINE C2 as worded: "10M
    filters sharded across 8xMI355X, topic batch broadcast, RCCL gather of
    match IDs over xGMI") on this rank: its shard of the filters
    (word_hash(filter) mod N, global ids), rank 0's batch broadcast every step.
    Without fan-out each step gathers counts and ids to rank 0 and merges them
    on the GPU (dist.ShardExchange); with fan-out every rank expands its own
    matches through the subscriber rows of its own filters and only the
    per-topic delivery totals are reduced to rank 0 (dist.ShardFanout)."""

    def __init__(self, gm, f, t, rank, world, dev, stream, mode, fanout, seed, sizes=None):
        import torch
        from emqx_amd import synth
        from emqx_amd.dist import ShardExchange, ShardFanout, gpu_merge, shard_of
        self.gm, self.rank, self.world, self.dev, self.sp, self.mode = gm, rank, world, dev, stream, mode
        idx = np.nonzero(shard_of(f, world) == rank)[0].astype(np.uint32)
        sub = f.subset(idx)
        gm.build(sub.blob, sub.off, idx)
        self.n_filters = len(idx)
        del sub
        self.sizes = sizes if sizes is not None else (t.n, len(t.blob))   # (topics, blob bytes) of rank 0's batch
        n = self.n = self.sizes[0]
        self.d_blob = torch.from_numpy(t.blob).to(dev) if rank == 0 else None
        self.d_off = torch.from_numpy(t.off.view(np.int32)).to(dev) if rank == 0 else None
        self.cap = max(4 * n // max(1, world) + 4096, 1 << 20)
        self.row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        self.ids = torch.zeros(self.cap, dtype=torch.int32, device=dev)
        self.fanout = fanout
        self.sub_entries = 0
        if fanout:
            # the subscriber rows of this shard's filters only (empty rows elsewhere)
            srow, ssubs = synth.subscribers(f.n, lam=1.0, p_big=0.001, n_big=2000, p_share=0.1, groups=64, seed=seed)
            per = np.diff(srow)
            mine = np.zeros(f.n, bool)
            mine[idx] = True
            lrow = np.zeros(f.n + 1, np.uint64)
            np.cumsum(np.where(mine, per, 0), out=lrow[1:])
            keep = np.repeat(mine, per.astype(np.int64))
            lsubs = ssubs[keep]
            del srow, ssubs, per, keep
            gm.subs_build(lrow, lsubs)
            self.sub_entries = len(lsubs)
            del lrow, lsubs
            self.fcap = max(8 * n // max(1, world), 1 << 20)
            self.drow = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            self.dpos = torch.zeros(self.cap + 1, dtype=torch.int64, device=dev)   # compact delivery form
            self.dsub = torch.zeros(self.fcap, dtype=torch.int32, device=dev)
            self.ex = ShardFanout(rank, world, dev, self._local_fanout)
        else:
            self.mcap = max(4 * n, 1 << 20) if rank == 0 else 0
            self.mrow = torch.zeros(n + 1, dtype=torch.int64, device=dev) if rank == 0 else None
            self.mids = torch.zeros(max(1, self.mcap), dtype=torch.int32, device=dev) if rank == 0 else None
            self.ex = self._exchange()

    def _exchange(self):
        from emqx_amd.dist import ShardExchange, gpu_merge
        mg = gpu_merge(self.gm, self.sp, self.mrow, self.mids) if self.rank == 0 else None
        return ShardExchange(self.rank, self.world, self.dev, self._local_match, mg)

    def _local_match(self, tb, to, nn):
        self.gm.match_device(tb.data_ptr(), tb.numel(), to.data_ptr(), nn, self.mode, self.sp, self.row.data_ptr(),
                             self.ids.data_ptr(), self.cap)
        st = self.gm.last_stats()   # syncs: the id count is needed on the host for the gather
        return self.row, self.ids, int(st["n_ids"]), bool(st["overflow"])

    def _local_fanout(self, tb, to, nn):
        self.gm.match_device(tb.data_ptr(), tb.numel(), to.data_ptr(), nn, self.mode, self.sp, self.row.data_ptr(),
                             self.ids.data_ptr(), self.cap)
        st = self.gm.last_stats()
        self.last_ids = int(st["n_ids"])
        if st["overflow"]:
            return self.row, True
        self.gm.fanout_device_compact(self.row.data_ptr(), self.ids.data_ptr(), self.cap, nn, self.sp,
                                      self.drow.data_ptr(), self.dpos.data_ptr(), self.dsub.data_ptr(), self.fcap)
        fo = self.gm.last_fanout()
        self.last_deliveries = int(fo["deliveries"])
        return self.drow, bool(fo["overflow"])

    def step(self):
        if self.rank == 0:
            return self.ex.step(self.d_blob, self.d_off, sizes=self.sizes)
        return self.ex.step(sizes=self.sizes)

    def size(self):
        """Untimed steps until no rank overflows (buffers grown from the totals)."""
        import torch
        import torch.distributed as dist
        for _ in range(6):
            self.step()
            torch.cuda.synchronize(self.dev)
            if not self.ex.last_overflow:
                return
            if self.fanout:
                # grow both local buffers from this rank's own counts
                if self.last_ids > self.cap:
                    self.cap = int(self.last_ids * 1.25) + 1024
                    self.ids = torch.zeros(self.cap, dtype=torch.int32, device=self.dev)
                    self.dpos = torch.zeros(self.cap + 1, dtype=torch.int64, device=self.dev)
                d = getattr(self, "last_deliveries", 0)
                if d > self.fcap:
                    self.fcap = int(d * 1.1) + 1024
                    self.dsub = torch.zeros(self.fcap, dtype=torch.int32, device=self.dev)
                continue
            tots = self.ex.last_totals
            if tots[self.rank] > self.cap:
                self.cap = int(tots[self.rank] * 1.25) + 1024
                self.ids = torch.zeros(self.cap, dtype=torch.int32, device=self.dev)
            if self.rank == 0 and sum(tots) > self.mcap:
                self.mcap = int(sum(tots) * 1.25) + 1024
                self.mids = torch.zeros(self.mcap, dtype=torch.int32, device=self.dev)
            self.ex = self._exchange()
        raise RuntimeError("shard leg: buffers did not settle")

    def merged_ids(self):
        return None if self.fanout else sum(self.ex.last_totals)


class PrefixLeg:
    """The prefix-partition layout on this rank (dist.PrefixExchange):
    this rank's partition of the filters (egm_prefix_assign: replicated filters
    + its prefixes, global ids) in `gm`, its own topic batch in HBM; a step
    routes the batch (egm_prefix_route), exchanges the slots with one
    all_to_all_single and matches each received slot in place
    (egm_match_device_counted_ordered: the slot's count is read on the device,
    rows in the walk's order as the replicate leg's)."""

    def __init__(self, gm, f, t, rank, world, dev, stream, mode, have_pg, slack=1.25):
        import torch
        import torch.distributed as dist
        from emqx_amd import _lib as L
        from emqx_amd.dist import PrefixSlots, prefix_assign
        self.gm, self.rank, self.world, self.dev, self.sp, self.mode = gm, rank, world, dev, stream, mode
        vr, fr = prefix_assign(f, world)
        idx = np.nonzero((fr == rank) | (fr == L.EGM_PREFIX_ALL))[0].astype(np.uint32)
        self.replicated = int(np.count_nonzero(fr == L.EGM_PREFIX_ALL))
        sub = f.subset(idx)
        gm.build(sub.blob, sub.off, idx)
        self.n_filters = len(idx)
        del sub, fr
        self.n, self.nbytes = t.n, len(t.blob)
        # the slots are the layout's (equal all_to_all splits): sized from the largest batch of any rank
        mx = torch.tensor([t.n, len(t.blob)], dtype=torch.int64, device=dev)
        if have_pg:
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        ps = PrefixSlots.for_batch(world, int(mx[0].item()), int(mx[1].item()), slack)
        self.d_blob = torch.from_numpy(t.blob).to(dev)
        self.d_off = torch.from_numpy(t.off.view(np.int32)).to(dev)
        self.d_vr = torch.from_numpy(vr).to(dev)
        self.ids_per_topic = 64
        self.settled = False
        self._make(ps)

    def _make(self, ps):
        from emqx_amd.dist import PrefixExchange, gpu_prefix_stages
        self.ex = PrefixExchange(self.rank, self.world, self.dev, ps,
                                 gpu_prefix_stages(self.gm, self.d_vr, self.mode, self.sp, self.ids_per_topic,
                                                   ordered=True))

    @property
    def ps(self):
        return self.ex.ps

    @property
    def rows(self):
        return self.ex.match_slot.rows

    @property
    def cap(self):
        return self.ex.match_slot.ids[0].numel()

    def step(self):
        """One step.  Until size() has settled the layout it is
        PrefixExchange.run (an overflowed slot is redone with grown slots: one
        24-byte all-reduce and a host readback per step).  After that the batch
        and the slot layout are fixed, so a step is PrefixExchange.step with no
        host sync — consecutive steps queue back to back at N > 1 — and the
        received slots' overflow flags accumulate on the device for check(),
        which fails loudly on any (run() serialised the steps)."""
        if self.settled:
            return self.ex.step(self.d_blob, self.d_off, self.n)
        return self.ex.run(self.d_blob, self.d_off, self.n, self.nbytes)

    def size(self):
        """Untimed steps until every received slot's ids fit (grown from the
        device totals) and the slot layout has settled."""
        import torch
        for _ in range(4):
            self.step()
            torch.cuda.synchronize(self.dev)
            need = max(int(r[self.ps.cap_topics].item()) for r in self.rows)
            if need <= self.cap:
                self.settled = True
                return
            self.ids_per_topic = int(need * 1.25 / max(self.ps.cap_topics, 1)) + 1
            self._make(self.ps)
        raise RuntimeError("prefix leg: buffers did not settle")

    def merged_ids(self):
        return None

    def check(self):
        """After the timed steps (the caller has synced): no slot overflow left
        unredone on any rank, ids fit."""
        flag = self.ex.overflow_flag.clone()
        if self.world > 1:
            flag = self.ex.comm.all_max(flag)
        assert int(flag.item()) == 0, "prefix slot overflow"
        ids = [int(r[self.ps.cap_topics].item()) for r in self.rows]
        assert max(ids) <= self.cap, (ids, self.cap)
        return sum(ids)

    def census(self):
        """One untimed step with a sync after every slot's match: the step's
        totals (levels, states created, ids, topics received) for the byte model."""
        import torch
        st = {"levels": 0, "visited": 0, "ids": 0, "topics": 0}
        recv = self.ex.exchange(self.ex.route(self.d_blob, self.d_off, self.n))
        torch.cuda.synchronize(self.dev)
        host = recv.cpu().numpy()
        for g in range(self.world):
            cnt, nb, ovf, tids, offs, data = self.ps.parse(host, g)
            assert not ovf
            self.ex.match_slot(recv, g)
            ls = self.gm.last_stats()
            st["levels"] += int(np.count_nonzero(data == ord("/"))) + cnt
            st["visited"] += ls["visited"]
            st["ids"] += ls["n_ids"]
            st["topics"] += cnt
        return st


def prefix_cost_model(n, blob_bytes, world, ps):
    """Bytes one prefix-partition step moves: each rank sends
    (N-1)/N of its slots over xGMI in one all_to_all; the route kernel reads
    the batch and writes the slots."""
    slots = world * ps.slot_bytes
    return {"all_to_all_bytes_per_rank": int(slots * (world - 1) / world), "slot_bytes": ps.slot_bytes,
            "cap_topics_per_slot": ps.cap_topics, "route_bytes": blob_bytes + 4 * (n + 1) + 8 * n + slots}


def shard_cost_model(n, blob_bytes, world, merged_ids):
    """Bytes one sharded step moves over xGMI: the broadcast
    of the batch to N-1 ranks, the gather of N-1 shards' counts and ids to
    rank 0 (ids: (N-1)/N of the merged total on average)."""
    bcast = blob_bytes + 4 * (n + 1)
    gather_ids = int(4 * merged_ids * (world - 1) / world) if merged_ids is not None else 0
    return {"broadcast_bytes": bcast, "gather_bytes": 4 * n * (world - 1) + gather_ids,
            "merge_bytes_on_rank0": (8 * merged_ids + 4 * n * world + 16 * n) if merged_ids is not None else 0}


def _init_dist(args, rank, world, dev):
    """A process group whenever the layout exchanges data (shard mode runs its
    collectives at every world size, world 1 included)."""
    import torch.distributed as dist
    if world > 1 or args.mode == "shard" or args.sharded_leg == "on":
        if "MASTER_ADDR" not in os.environ:   # plain `python bench.py --mode shard`: a world of one
            import socket
            so = socket.socket()
            so.bind(("127.0.0.1", 0))
            os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(so.getsockname()[1])
            so.close()
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        return True
    return False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--filters", type=int, default=None, help="override filter count")
    ap.add_argument("--topics", type=int, default=None, help="override topics per batch")
    ap.add_argument("--mode", default="replicate", choices=sorted(LAYOUTS))
    ap.add_argument("--match", default="routes", choices=["routes", "trie"])
    ap.add_argument("--fanout", default="auto", choices=["auto", "on", "off"],
                    help="add emqx_broker:dispatch/2 subscriber fan-out to each step (auto: on for c3, c4)")
    ap.add_argument("--streams", type=int, default=0,
                    help="replicate mode: consecutive batches alternate over this many HIP streams (each with its "
                         "own match workspace), so one batch's compaction overlaps the next one's walk "
                         "(0 = 1; the other setting is timed beside it)")
    ap.add_argument("--x-presort", type=int, default=-1,
                    help="experiment: sort the batch's topics on the host (untimed) by their first K levels "
                         "(0: whole topic) to measure how much trie-path locality between neighbouring topics "
                         "would save the walk")
    ap.add_argument("--x-orders", default="",
                    help="experiment: after the timed steps, time the same steps under each walk order "
                         "'shape[/flush],...' (EGM_WALK_KEY: key bits per level as hex nibbles, level 0 lowest, 0 = "
                         "input order; EGM_FLUSH_AT: staged emits per flush record) and check "
                         "that every order gives the same rows (stderr)")
    ap.add_argument("--rows", default="walk", choices=["walk", "input"],
                    help="result rows in the walk's order with the row -> topic map (egm_match_device_ordered, "
                         "the default) or in input order (egm_match_device); the other form is timed beside it "
                         "(`rows_other`)")
    ap.add_argument("--pipelined", default="on", choices=["on", "off"],
                    help="after the timed steps, time them again in the other stream setting: one stream "
                         "(`serial`) after two, two streams (`pipelined`) after --streams 1 (replicate mode, "
                         "no fan-out)")
    ap.add_argument("--host-e2e", default="on", choices=["on", "off"],
                    help="also time the host-visible path (pinned staging, H2D, match, D2H) at N=1")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--fanout-form", default="compact", choices=["compact", "pairs"],
                    help="delivery lists as subscriber ids + each match entry's first delivery "
                         "(egm_fanout_device_compact), or as (filter, subscriber) pairs (egm_fanout_device)")
    ap.add_argument("--sharded-timeout", type=float, default=300.0,
                    help="seconds the sharded leg may take before the line is printed without it")
    ap.add_argument("--sharded-layout", default="prefix", choices=["prefix", "shard"],
                    help="the layout of the sharded leg: prefix partition (one all_to_all, weak) or the round-3 "
                         "filter shards (broadcast + gather + merge, strong); with fan-out always shard")
    ap.add_argument("--sharded-leg", default="auto", choices=["auto", "on", "off"],
                    help="replicate mode at N>1 (auto) or any N (on): also time the filter-sharded layout "
                         "(BASELINE C2 as worded: broadcast + RCCL gather + GPU merge; with fan-out, fan-out on "
                         "the owner shard + a reduce of per-topic delivery totals), reported as the line's "
                         "`sharded`")
    args = ap.parse_args()
    fanout = args.fanout == "on" or (args.fanout == "auto" and args.config in ("c3", "c4"))
    _heartbeat()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")

    from emqx_amd import build as B
    if not os.path.exists(B.LIB):
        B.build_all()
    import torch
    import torch.distributed as dist
    from emqx_amd import _lib as L
    from emqx_amd import synth
    from emqx_amd.engine import GpuMatcher

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    have_pg = _init_dist(args, rank, world, dev)
    shard = args.mode == "shard"
    prefix = args.mode == "prefix"
    mode = L.EGM_MODE_ROUTES if args.match == "routes" else L.EGM_MODE_TRIE

    c = synth.CONFIGS[args.config]
    seed = synth.SEED_BASE + synth.CONFIG_INDEX[args.config]
    nf = args.filters or c["n_filters"]
    nt = args.topics or c["n_topics"]
    t0 = time.time()
    f = synth.filters(nf, c["dmin"], c["dmax"], c["wc"], c["p_plus"], c["p_hash"], seed=seed)
    tseed = seed + (0 if shard else 7919 * rank)   # shard: rank 0's batch is the one broadcast
    t = synth.topics(nt, f, c["dmin"], c["dmax"], seed=tseed)
    log(f"[rank {rank}] generated {f.n} filters, {t.n} topics in {time.time() - t0:.1f}s")
    if args.x_presort >= 0:
        tl = t.to_list()
        K = args.x_presort
        keys = tl if K == 0 else [b"/".join(x.split(b"/", K)[:K]) for x in tl]
        order = sorted(range(len(tl)), key=keys.__getitem__)
        del keys
        t = t.subset(np.asarray(order, dtype=np.int64))
        del tl, order
        log(f"[rank {rank}] topics presorted (experiment)")

    gm = GpuMatcher(local, max_batch=nt)
    t0 = time.time()
    nstreams = 1 if (shard or prefix or fanout) else max(1, args.streams)
    piped = args.pipelined == "on" and args.mode == "replicate" and not fanout and nstreams == 1
    serial_leg = args.pipelined == "on" and args.mode == "replicate" and not fanout and nstreams > 1
    nbuf = 2 if piped else nstreams
    streams = [torch.cuda.Stream(dev) for _ in range(nbuf)]
    stream = streams[0]
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    leg = None
    if shard:
        leg = ShardLeg(gm, f, t, rank, world, dev, sp, mode, fanout, seed)
    elif prefix:
        if fanout:
            raise SystemExit("--mode prefix: match only (the fan-out would run on the owner rank; not timed here)")
        leg = PrefixLeg(gm, f, t, rank, world, dev, sp, mode, have_pg)
    else:
        gm.build(f.blob, f.off)
    tstats = gm.stats()
    log(f"[rank {rank}] table built in {time.time() - t0:.1f}s: {tstats}")
    sub_entries = getattr(leg, "sub_entries", 0)   # the shard leg's subscriber table; none for prefix
    if fanout and not shard:
        # filter id -> subscriber CSR (emqx_subscriber bag, shards flattened)
        t0 = time.time()
        srow, ssubs = synth.subscribers(f.n, lam=1.0, p_big=0.001, n_big=2000, p_share=0.1, groups=64, seed=seed)
        gm.subs_build(srow, ssubs)
        sub_entries = len(ssubs)
        del srow, ssubs
        log(f"[rank {rank}] subscriber table: {sub_entries} entries in {time.time() - t0:.1f}s")

    # one explicit stream for every kernel and copy of the step (the library
    # and torch share one HIP runtime: emqx_amd._lib loads torch first);
    # the pipelined leg (after the timed steps): consecutive batches over two streams
    n = t.n
    nbytes = int(t.off[-1])
    d_blob = torch.from_numpy(t.blob).to(dev)
    d_off = torch.from_numpy(t.off.view(np.int32)).to(dev)
    torch.cuda.synchronize(dev)
    bufs = {"cap": max(4 * n, 1 << 20), "k": 0, "ns": nstreams}
    bufs["rows"] = [torch.zeros(n + 1, dtype=torch.int64, device=dev) for _ in range(nbuf)]
    bufs["idss"] = [torch.zeros(bufs["cap"], dtype=torch.int32, device=dev) for _ in range(nbuf)]
    bufs["row"], bufs["ids"] = bufs["rows"][0], bufs["idss"][0]
    bufs["walk_rows"] = args.rows == "walk" and leg is None
    bufs["tops"] = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(nbuf)]

    compact = args.fanout_form == "compact"
    fcap = max(8 * n, 1 << 20) if fanout else 0
    d_drow = torch.zeros(n + 1, dtype=torch.int64, device=dev) if fanout else None
    # compact: each match entry's first delivery (the filter of a delivery), else a filter id per delivery
    d_fid = (torch.zeros(bufs["cap"] + 1, dtype=torch.int64, device=dev) if compact
             else torch.zeros(fcap, dtype=torch.int32, device=dev)) if fanout else None
    d_sub = torch.zeros(fcap, dtype=torch.int32, device=dev) if fanout else None
    fan_on = False   # enabled once the id buffer holds a whole match batch

    def run_local():
        # batch k on stream k mod ns, with that stream's output buffers
        i = bufs["k"] % bufs["ns"]
        bufs["k"] += 1
        s_i = streams[i].cuda_stream
        row, ids = bufs["rows"][i], bufs["idss"][i]
        if bufs["walk_rows"]:   # rows in walk order + the row -> topic map
            gm.match_device_ordered(d_blob.data_ptr(), nbytes, d_off.data_ptr(), n, mode, s_i, row.data_ptr(),
                                    bufs["tops"][i].data_ptr(), ids.data_ptr(), bufs["cap"])
        else:
            gm.match_device(d_blob.data_ptr(), nbytes, d_off.data_ptr(), n, mode, s_i, row.data_ptr(),
                            ids.data_ptr(), bufs["cap"])
        if fan_on:
            fan = gm.fanout_device_compact if compact else gm.fanout_device
            fan(row.data_ptr(), ids.data_ptr(), bufs["cap"], n, s_i, d_drow.data_ptr(), d_fid.data_ptr(),
                d_sub.data_ptr(), fcap)

    def step():
        if leg is None:
            run_local()
        else:
            leg.step()

    # size the id buffers (untimed), then warm up
    if leg is not None:
        leg.size()
    else:
        for _ in range(4):
            step()
            torch.cuda.synchronize(dev)
            st = gm.last_stats()
            if not st["overflow"]:
                break
            bufs["cap"] = int(st["n_ids"] * 1.25) + 1024
            bufs["idss"] = [torch.zeros(bufs["cap"], dtype=torch.int32, device=dev) for _ in range(nbuf)]
            bufs["ids"] = bufs["idss"][0]
            bufs["k"] = 0
            log(f"[rank {rank}] grew id buffers to {bufs['cap']}")
    if fanout and leg is None:
        if compact:   # the entry offsets follow the (grown) id buffer
            d_fid = torch.zeros(bufs["cap"] + 1, dtype=torch.int64, device=dev)
        fan_on = True
        bufs["k"] = 0
        step()
        torch.cuda.synchronize(dev)
        need = int(d_drow[n].item())
        if need > fcap:   # k_fan_fill wrote nothing: size the delivery buffers and run again
            fcap = int(need * 1.1) + 1024
            del d_sub
            if not compact:
                del d_fid
                d_fid = torch.zeros(fcap, dtype=torch.int32, device=dev)
            d_sub = torch.zeros(fcap, dtype=torch.int32, device=dev)
            log(f"[rank {rank}] grew delivery buffers to {fcap}")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    st = gm.last_stats()
    assert st["overflow"] == 0 and st["errors"] == 0, st
    if prefix:
        leg.check()
    elif leg is not None:
        assert not leg.ex.last_overflow

    gm.set_timing(True)
    if have_pg:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if have_pg:
        dist.barrier()
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    tim = gm.get_timing()
    st = gm.last_stats()
    if prefix:
        leg.check()
    deliveries = int(d_drow[n].item()) if (fanout and leg is None) else None
    if fanout and leg is not None:   # every rank's own part of the batch's deliveries, summed
        dt = torch.tensor([leg.last_deliveries], dtype=torch.int64, device=dev)
        if have_pg:
            dist.all_reduce(dt)
        deliveries = int(dt.item())
    if fanout and leg is None:
        assert deliveries <= fcap, (deliveries, fcap)
    wc = gm.walk_counters()
    gm.set_timing(False)
    iso_ms = None
    if nstreams > 1:
        # the walk alone (one stream, nothing overlapping it), untimed: the
        # kernel's own speed next to its time inside the overlapped steps
        gm.set_timing(True)
        for _ in range(3):
            bufs["k"] = 0
            run_local()
        torch.cuda.synchronize(dev)
        ti = gm.get_timing()
        iso_ms = ti["walk_ms"] / max(1, ti["walk_launches"])
        gm.set_timing(False)
    pipelined = serial = None
    if serial_leg:
        # the same steps one batch at a time on one stream (nothing overlaps):
        # reported beside `value`
        bufs["ns"], bufs["k"] = 1, 0
        for _ in range(2):
            run_local()
        if have_pg:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run_local()
        torch.cuda.synchronize(dev)
        pe = time.perf_counter() - t0
        if have_pg:
            dist.barrier()
            e = torch.tensor([pe], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            pe = float(e.item())
        serial = {"streams": 1, "value": n * world * args.steps / pe, "ms_per_step": pe / args.steps * 1e3,
                  "note": "same steps, one batch at a time on one HIP stream"}
        bufs["ns"], bufs["k"] = nstreams, 0
    if piped:
        # the same steps with consecutive batches alternating over two streams,
        # so one batch's bandwidth-bound kernels (sort, scan, compaction) run
        # beside the next one's latency-bound walk; reported beside `value`
        bufs["ns"], bufs["k"] = 2, 0
        for _ in range(2):
            run_local()
        if have_pg:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run_local()
        torch.cuda.synchronize(dev)
        pe = time.perf_counter() - t0
        if have_pg:
            dist.barrier()
            e = torch.tensor([pe], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            pe = float(e.item())
        st2 = gm.last_stats()
        assert st2["overflow"] == 0 and st2["errors"] == 0, st2
        pipelined = {"streams": 2, "value": n * world * args.steps / pe, "ms_per_step": pe / args.steps * 1e3,
                     "note": "same steps, consecutive batches alternating over two HIP streams (separate "
                             "workspaces and output buffers)"}
        bufs["ns"], bufs["k"] = nstreams, 0
    rows_other = None
    if leg is None and not fanout:
        # the same steps with the other row form (input order <-> walk order), reported beside `value`
        bufs["walk_rows"], bufs["k"] = not bufs["walk_rows"], 0
        for _ in range(2):
            run_local()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run_local()
        torch.cuda.synchronize(dev)
        pe = time.perf_counter() - t0
        if have_pg:
            e = torch.tensor([pe], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            pe = float(e.item())
        st2 = gm.last_stats()
        assert st2["overflow"] == 0 and st2["errors"] == 0, st2
        rows_other = {"rows": "walk" if bufs["walk_rows"] else "input", "streams": bufs["ns"],
                      "value": n * world * args.steps / pe, "ms_per_step": pe / args.steps * 1e3,
                      "api": "egm_match_device_ordered" if bufs["walk_rows"] else "egm_match_device"}
        bufs["walk_rows"], bufs["k"] = not bufs["walk_rows"], 0
    merged_ids = leg.merged_ids() if leg is not None else None
    if args.x_orders and leg is None:
        order_experiment(args, gm, run_local, bufs, dev, n)
    run_sharded = leg is None and (args.sharded_leg == "on" or (args.sharded_leg == "auto" and world > 1))

    units_per_step = n if shard else n * world
    value = units_per_step * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # ---- roofline (dominant kernel = k_walk), SURVEY §8d byte model ----
    walk_ms = tim["walk_ms"] / max(1, tim["walk_launches"])
    if prefix:
        # one walk launch per received slot: the byte model over the step's
        # totals (an untimed census step), the kernel time over its launches
        cz = leg.census()
        sum_d, n_ids, visited, n_walked = cz["levels"], cz["ids"], cz["visited"], cz["topics"]
        walk_ms *= world
    else:
        sum_d = levels_sum(t.blob, t.off)
        n_ids, visited, n_walked = st["n_ids"], st["visited"], n
    walk_bytes = 8 * sum_d + 32 * visited + 4 * (n_ids + n_walked)
    achieved = walk_bytes / (walk_ms * 1e-3) / 1e9
    path_bytes = (nbytes + 4 * n) + 16 * sum_d + 32 * visited + 4 * (n_ids + n)

    traffic = walk_traffic(args.config, f.n, n) if (args.mode == "replicate" and world == 1) else None
    host = None
    if _host_leg(args, world, shard):
        log("[rank 0] timing the host-visible path ...")
        host = host_e2e(gm, t, mode)
        log("[rank 0] timing the batcher's operating points ...")
        host["batcher"] = host_batcher_curve(gm, t, mode)
    if rank == 0:
        cpu = None
        if args.cpu_baseline == "auto" and world == 1 and f.n > 20_000_000:
            log("[rank 0] CPU baseline skipped: the string-keyed oracle table does not fit this host at "
                f"{f.n} filters")
        elif args.cpu_baseline == "auto" and world == 1:
            log("[rank 0] timing the CPU baseline ...")
            cpu = cpu_baseline(f, t, mode, args.cpu_seconds)
        line = {
            "metric": METRIC, "value": value, "unit": "topics/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "strong" if shard else "weak",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": f"{WORKLOADS[args.config]}; layout: {LAYOUTS[args.mode]}", "filters": f.n,
                       "topics_per_step": units_per_step, "topics_per_gpu": n,
                       "filters_on_rank0": tstats["filters"],
                       "match": "emqx_router:match_routes" if args.match == "routes" else "emqx_trie:match",
                       "parallelism": f"{args.mode}{world}", "streams": nstreams, "table": tstats,
                       "rows": ("walk order + row -> topic map (egm_match_device_ordered)" if bufs["walk_rows"]
                                else "input order (egm_match_device)")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic[0]["traffic_bytes_per_launch"] if traffic else None,
                         "traffic_source": traffic[1] if traffic else None,
                         # the counters' bytes over the same time (beside, not instead of,
                         # the algorithmic `frac` the contract prescribes)
                         "frac_measured": (traffic[0]["traffic_bytes_per_launch"] / (walk_ms * 1e-3) / 1e9 /
                                           HBM_PEAK_GBS) if traffic else None,
                         "kernel": "k_walk", "kernel_ms": walk_ms, "bytes_per_launch": walk_bytes,
                         "kernel_src_sha": kernel_src_sha(),
                         "kernel_ms_isolated": iso_ms,
                         "frac_isolated": (walk_bytes / (iso_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if iso_ms else None,
                         "path_frac": path_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS},
            "stats": {"ids_per_step": n_ids, "visited_per_step": visited, "levels_per_step": sum_d,
                      "merged_ids_per_step": merged_ids,
                      "deferred_chunks": st["deferred_chunks"], "walk_iters": wc["iters"],
                      "walk_popped": wc["popped"], "walk_bounded_pops": wc["bounded"],
                      "walk_lane_occupancy": wc["lane_occupancy"], "walk_bucket_reads": wc["lit_probes"],
                      "walk_plus_record_reads": wc["plus_reads"],
                      "walk_second_bucket_reads": wc.get("slow_probes"),
                      "walk_iters_with_second_read": wc.get("slow_iters")},
            "fanout": ({"deliveries_per_step": deliveries, "subscriber_entries": sub_entries,
                        "fanout_ms": tim["fanout_ms"] / max(1, tim["fanout_launches"]),
                        "deliveries_per_s": deliveries * (1 if shard else world) * args.steps / elapsed,
                        "form": args.fanout_form,
                        # compact: subscriber id read + written, entry offsets; pairs: + a filter id written
                        "bytes_per_launch": ((8 * deliveries + 28 * n_ids if args.fanout_form == "compact"
                                              else 12 * deliveries + 20 * n_ids) + 8 * (n + 1))}
                       if fanout else None),
            "pipelined": pipelined,
            "serial": serial,
            "rows_other": rows_other,
            "sharded": None,
            "xgmi_model": (shard_cost_model(n, nbytes, world, merged_ids) if shard else
                           prefix_cost_model(n, nbytes, world, leg.ps) if prefix else None),
            "partition": ({"filters_on_rank": leg.n_filters, "replicated_filters": leg.replicated,
                           "topics_matched_on_rank0": n_walked, "slot_reruns": leg.ex.reruns} if prefix else None),
            "host_e2e": host,
            "cpu_baseline": cpu,
        }
    if run_sharded:
        # the filter-sharded layout beside the value, after it is measured: a
        # leg that fails or hangs (a collective that never completes) must not
        # cost the line, so each rank runs it under a watchdog that prints the
        # line without it and ends the process — with a non-zero status, so the
        # failure still shows in the return code
        def give_up(why):
            if rank == 0:
                line["sharded"] = {"error": why}
                print(json.dumps(line), flush=True)
            sys.stderr.write(f"[rank {rank}] {why}\n")
            sys.stderr.flush()
            os._exit(SHARDED_LEG_FAILED)

        sharded = guarded(lambda: sharded_leg(args, f, t, rank, world, dev, mode, fanout, seed, have_pg),
                          args.sharded_timeout, give_up, "sharded leg")
        if rank == 0:
            line["sharded"] = sharded
    if rank == 0:
        print(json.dumps(line), flush=True)
    gm.close()
    if have_pg:
        dist.destroy_process_group()


SHARDED_LEG_FAILED = 3   # exit status after a line printed without its failed sharded leg


def guarded(fn, seconds, give_up, what):
    """fn() under a watchdog: if it raises, or has not returned after `seconds`
    (a collective that never completes), give_up(reason) is called — from a
    timer thread in the second case, so it must end the process itself.
    Exactly one of {fn's result, the timer's give_up, the error's give_up}
    wins (a timer firing as fn returns must not print a second
    line): the first to take `decided` does; a loser that is the main thread
    waits for the timer thread to end the process."""
    import threading
    decided = threading.Lock()

    def fire():
        if decided.acquire(blocking=False):
            give_up(f"{what} did not finish within {seconds:.0f} s")

    wd = threading.Timer(seconds, fire)
    wd.daemon = True
    wd.start()
    try:
        out = fn()
    except Exception as e:   # noqa: BLE001 - reported, the caller's result stands
        out, err = None, e
    else:
        err = None
    if not decided.acquire(blocking=False):
        while True:          # the timer fired first: it prints the line and exits
            time.sleep(3600)
    wd.cancel()
    if err is not None:
        return give_up(f"{what} failed: {err!r}"[:300])
    return out


def sharded_leg(args, f, t, rank, world, dev, mode, fanout, seed, have_pg):
    """The filter-sharded layout timed beside the replicate `value` (VERDICT
    r2 item 5): a second context per rank holds this rank's filter shard, rank
    0's batch (its own replicate batch) is broadcast each step.  value =
    topics of the broadcast batch per second for the whole node."""
    import torch
    import torch.distributed as dist
    from emqx_amd.engine import GpuMatcher
    if args.sharded_layout == "prefix" and not fanout:
        return prefix_leg(args, f, t, rank, world, dev, mode, have_pg)
    meta = torch.tensor([t.n, len(t.blob)] if rank == 0 else [0, 0], dtype=torch.int64, device=dev)
    if have_pg:
        dist.broadcast(meta, 0)
    sizes = (int(meta[0].item()), int(meta[1].item()))
    gm2 = GpuMatcher(dev.index, max_batch=sizes[0])
    s = torch.cuda.Stream(dev)
    try:
        t0 = time.time()
        leg = ShardLeg(gm2, f, t if rank == 0 else None, rank, world, dev, s.cuda_stream, mode, fanout, seed, sizes)
        log(f"[rank {rank}] sharded leg: {leg.n_filters} filters on this rank, built in {time.time() - t0:.1f}s")
        with torch.cuda.stream(s):
            leg.size()
            for _ in range(args.warmup):
                leg.step()
            torch.cuda.synchronize(dev)
            if have_pg:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                leg.step()
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - t0
        if have_pg:
            dist.barrier()
            e = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = float(e.item())
        merged = leg.merged_ids()
        out = {"value": sizes[0] * args.steps / el, "unit": "topics/s", "ms_per_step": el / args.steps * 1e3,
               "scaling": "strong", "filters_per_rank": leg.n_filters,
               "layout": LAYOUTS["shard"] + (" — fan-out on the owner shard, per-topic delivery totals reduced to "
                                             "rank 0" if fanout else ""),
               "merged_ids_per_step": merged,
               "xgmi_model": shard_cost_model(sizes[0], sizes[1], world, merged)}
        if fanout:
            dtot = torch.tensor([leg.last_deliveries], dtype=torch.int64, device=dev)
            if have_pg:
                dist.all_reduce(dtot)
            out["deliveries_per_step"] = int(dtot.item())
        return out
    finally:
        gm2.close()


def prefix_leg(args, f, t, rank, world, dev, mode, have_pg):
    """The prefix-partition layout timed beside the replicate `value` (VERDICT
    r3 item 5): a second context per rank holds this rank's partition, each
    rank's own batch is routed to the prefix owners every step.  value = the
    topics of all ranks' batches per second for the whole node (weak)."""
    import torch
    import torch.distributed as dist
    from emqx_amd.engine import GpuMatcher
    gm2 = GpuMatcher(dev.index, max_batch=t.n)
    s = torch.cuda.Stream(dev)
    try:
        t0 = time.time()
        with torch.cuda.stream(s):
            leg = PrefixLeg(gm2, f, t, rank, world, dev, s.cuda_stream, mode, have_pg)
            log(f"[rank {rank}] prefix leg: {leg.n_filters} filters on this rank ({leg.replicated} replicated), "
                f"built in {time.time() - t0:.1f}s")
            leg.size()
            for _ in range(args.warmup):
                leg.step()
            torch.cuda.synchronize(dev)
            if have_pg:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                leg.step()
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - t0
            ids = leg.check()
        if have_pg:
            dist.barrier()
            e = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = float(e.item())
            fr = torch.tensor([leg.n_filters], dtype=torch.int64, device=dev)
            dist.all_reduce(fr, op=dist.ReduceOp.MAX)
            max_filters = int(fr.item())
        else:
            max_filters = leg.n_filters
        return {"value": t.n * world * args.steps / el, "unit": "topics/s", "ms_per_step": el / args.steps * 1e3,
                "scaling": "weak", "layout": LAYOUTS["prefix"], "filters_per_rank_max": max_filters,
                "replicated_filters": leg.replicated, "filters_total": f.n, "ids_on_rank0": ids,
                "slot_reruns": leg.ex.reruns,
                "xgmi_model": prefix_cost_model(t.n, len(t.blob), world, leg.ps)}
    finally:
        gm2.close()


def order_experiment(args, gm, run_local, bufs, dev, n):
    """Walk-order A/B inside one process (the table is built once): steps
    timed per order, rows checked against the default order's (row_ptr equal,
    per-row id sums equal)."""
    import torch

    def rows_sig():
        # per input topic: (ids, sum of ids) — walk-order rows mapped through the topic map
        row, ids = bufs["rows"][0], bufs["idss"][0]
        tot = int(row[n].item())
        cs = torch.cumsum(ids[:tot].to(torch.int64), 0)
        cs = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), cs])
        cnt, sm = row[1:] - row[:-1], cs[row[1:]] - cs[row[:-1]]
        if bufs["walk_rows"]:
            top = bufs["tops"][0].to(torch.int64)
            cnt = torch.zeros_like(cnt).scatter_(0, top, cnt)
            sm = torch.zeros_like(sm).scatter_(0, top, sm)
        return cnt, sm

    saved = {k: os.environ.get(k) for k in ("EGM_WALK_KEY", "EGM_FLUSH_AT")}
    bufs["k"] = 0
    run_local()
    torch.cuda.synchronize(dev)
    ref_row, ref_sig = rows_sig()
    for spec in args.x_orders.split(","):
        shape, _, fl = spec.partition("/")
        os.environ["EGM_WALK_KEY"] = shape
        if fl:
            os.environ["EGM_FLUSH_AT"] = fl
        else:
            os.environ.pop("EGM_FLUSH_AT", None)
        for _ in range(2):
            bufs["k"] = 0
            run_local()
        torch.cuda.synchronize(dev)
        gm.set_timing(True)
        bufs["k"] = 0
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run_local()   # consecutive batches alternate over the bench's streams
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / args.steps
        tim = gm.get_timing()
        gm.set_timing(False)
        wc = gm.walk_counters()
        bufs["k"] = 0
        run_local()
        torch.cuda.synchronize(dev)
        row, sig = rows_sig()
        same = bool(torch.equal(row, ref_row) and torch.equal(sig, ref_sig))
        log(json.dumps({"order": spec, "ms_per_step": dt * 1e3,
                        "walk_ms": tim["walk_ms"] / max(1, tim["walk_launches"]),
                        "topics_per_s": n / dt, "lane_occupancy": wc["lane_occupancy"], "rows_equal": same}))
        if not same:
            raise RuntimeError(f"walk order {spec} changed the result rows")
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _host_leg(args, world, shard):
    return args.host_e2e == "on" and world == 1 and args.mode == "replicate"


if __name__ == "__main__":
    try:
        main()
    except BaseException:
        # leave at once: after a device fault the runtime's teardown can hang
        import traceback
        traceback.print_exc()
        sys.stderr.flush()
        os._exit(1)
