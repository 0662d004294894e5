"""N>1 path on CPU: world_size-2 gloo run of the filter-sharded exchange
(broadcast topics, all-gather counts, gatherv ids, merge on rank 0).  The
per-rank matcher is injected: here the C++ oracle over the rank's shard
(stand-in for the GPU matcher, which needs a device).  The merged result must
equal the whole-table oracle result."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from emqx_amd import synth
from emqx_amd.dist import ShardExchange, shard_of, topic_slice
from emqx_amd.engine import pack_strings
from oracle.cpp import OracleTrie, canonical
from tests.shard_ref import merge_shard_results


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    f, t = synth.config("c0", n_filters=3000, n_topics=4000)
    sh = shard_of(f, world)
    fl = f.to_list()
    idx = np.nonzero(sh == rank)[0]
    o = OracleTrie(True, 0)
    blob, off = pack_strings([fl[i] for i in idx])
    o.add(blob, off, idx.astype(np.uint32))

    def local_match(tb, to, n):
        row, ids = o.match(tb.numpy(), to.numpy().view(np.uint32), threads=1)
        return torch.from_numpy(row.astype(np.int64)), torch.from_numpy(ids.astype(np.int32)), len(ids), False

    def merge(counts, parts, total, n):   # test-side numpy merge (the product merge is the HIP kernel)
        G = len(parts)
        cs = counts.numpy().reshape(G, n).astype(np.int64)
        rows = [np.concatenate([[0], np.cumsum(c)]).astype(np.uint64) for c in cs]
        row, ids = merge_shard_results([(rows[k], parts[k].numpy().view(np.uint32)) for k in range(G)])
        assert int(row[-1]) == total
        return torch.from_numpy(row.astype(np.int64)), torch.from_numpy(ids.astype(np.int32))

    ex = ShardExchange(rank, world, torch.device("cpu"), local_match, merge if rank == 0 else None)
    if rank == 0:
        out = ex.step(torch.from_numpy(t.blob.copy()), torch.from_numpy(t.off.view(np.int32).copy()))
        q.put((out[0].numpy(), out[1].numpy()))
    else:
        ex.step()
    dist.barrier()
    dist.destroy_process_group()


def test_shard_exchange_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    row, ids = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    f, t = synth.config("c0", n_filters=3000, n_topics=4000)
    o = OracleTrie(True, 0)
    o.add(f.blob, f.off)
    wrow, wids = o.match(t.blob, t.off)
    assert np.array_equal(row.astype(np.uint64), wrow)
    assert np.array_equal(canonical(wrow, ids.astype(np.uint32)), canonical(wrow, wids))


def test_topic_slices_cover():
    for n in (0, 1, 7, 1000):
        for w in (1, 2, 3, 8):
            s = [topic_slice(n, r, w) for r in range(w)]
            assert s[0][0] == 0 and s[-1][1] == n
            assert all(s[i][1] == s[i + 1][0] for i in range(w - 1))


def _fanout_worker(rank, world, port, q):
    """ShardFanout over gloo: each rank matches its filter shard (oracle
    stand-in for the GPU matcher) and expands through the subscriber rows of
    ITS filters; only the per-topic delivery totals reach rank 0."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from emqx_amd.dist import ShardFanout
    f, t = synth.config("c0", n_filters=3000, n_topics=4000)
    srow, subs = synth.subscribers(f.n, lam=1.0, p_big=0.01, n_big=50, p_share=0.1, seed=5)
    sh = shard_of(f, world)
    fl = f.to_list()
    idx = np.nonzero(sh == rank)[0]
    o = OracleTrie(True, 1)
    blob, off = pack_strings([fl[i] for i in idx])
    o.add(blob, off, idx.astype(np.uint32))
    per_sub = np.diff(srow).astype(np.int64)

    def local(tb, to, n):
        row, ids = o.match(tb.numpy(), to.numpy().view(np.uint32), threads=1)
        dcount = np.zeros(n, np.int64)
        rid = np.repeat(np.arange(n), np.diff(row).astype(np.int64))
        np.add.at(dcount, rid, per_sub[ids.astype(np.int64)])
        drow = np.concatenate([[0], np.cumsum(dcount)])
        return torch.from_numpy(drow.astype(np.int64)), False

    ex = ShardFanout(rank, world, torch.device("cpu"), local)
    sizes = (t.n, len(t.blob))
    if rank == 0:
        out = ex.step(torch.from_numpy(t.blob.copy()), torch.from_numpy(t.off.view(np.int32).copy()), sizes)
        q.put(out.numpy())
    else:
        assert ex.step(sizes=sizes) is None
    dist.barrier()
    dist.destroy_process_group()


def test_shard_fanout_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fanout_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    per = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    f, t = synth.config("c0", n_filters=3000, n_topics=4000)
    srow, subs = synth.subscribers(f.n, lam=1.0, p_big=0.01, n_big=50, p_share=0.1, seed=5)
    o = OracleTrie(True, 1)
    o.add(f.blob, f.off)
    row, ids = o.match(t.blob, t.off)
    want = np.zeros(t.n, np.int64)
    np.add.at(want, np.repeat(np.arange(t.n), np.diff(row).astype(np.int64)),
              np.diff(srow).astype(np.int64)[ids.astype(np.int64)])
    assert np.array_equal(per, want) and want.sum() > t.n


# ---- prefix partition (SURVEY §8e "partition by root word")
def _prefix_case(skew: bool):
    """The C0 sets; with skew, every topic's first two words are replaced by
    the most common literal two-word prefix of the filters, so every topic
    routes to one rank (the typical tenant/site/... MQTT tree)."""
    f, t = synth.config("c0", n_filters=3000, n_topics=4000)
    if not skew:
        return f, t
    from collections import Counter
    pre = Counter(tuple(x.split(b"/")[:2]) for x in f.to_list()
                  if x.count(b"/") >= 2 and b"+" not in x.split(b"/")[:2] and b"#" not in x.split(b"/")[:2])
    (w0, w1), _ = pre.most_common(1)[0]
    topics = []
    for x in t.to_list():
        w = x.split(b"/")
        topics.append(b"/".join([w0, w1] + w[2:]))
    blob, off = pack_strings(topics)
    return f, synth.StringSet(blob, off)


def _prefix_worker(rank, world, port, q, skew):
    """PrefixExchange.run over gloo: every rank routes ITS OWN batch (host
    restatement of egm_prefix_route), one all_to_all exchanges the slots, and
    each rank matches what it received against its partition (replicated
    filters + its own keys; the C++ oracle stands in for the GPU matcher, and
    like egm_match_device_counted it matches an overflowed slot as empty).
    With skew every topic goes to one rank: the first step overflows that
    slot and run() redoes it with grown slots.  The (source rank, topic, ids)
    triples are gathered to rank 0 only to be checked."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from emqx_amd.dist import PrefixExchange, PrefixSlots, prefix_assign, prefix_route_reference
    from emqx_amd import _lib as L
    f, t = _prefix_case(skew)
    vr, fr = prefix_assign(f, world, n_vparts=256)
    idx = np.nonzero((fr == rank) | (fr == L.EGM_PREFIX_ALL))[0]
    fl = f.to_list()
    o = OracleTrie(True, 0)
    blob, off = pack_strings([fl[i] for i in idx])
    o.add(blob, off, idx.astype(np.uint32))
    lo, hi = topic_slice(t.n, rank, world)
    mine = t.subset(np.arange(lo, hi))
    # the slot capacities are the layout's, the same on every rank (equal all_to_all splits)
    # (skew: the layout's default slack without for_batch's additive margin,
    # which one rank's whole load overflows at this small size)
    if skew:
        ps = PrefixSlots(world, int(1.25 * t.n / world / world) + 16, int(1.25 * int(t.off[-1]) / world / world) + 1024)
    else:
        ps = PrefixSlots.for_batch(world, -(-t.n // world), int(t.off[-1]) // world + 4096, slack=2.0)

    def make(ps):
        def route(tb, to, n):
            return torch.from_numpy(prefix_route_reference(tb.numpy(), to.numpy().view(np.uint32), vr, ps))

        def match_slot(recv, g):
            cnt, nb, ovf, tids, offs, data = ps.parse(recv.numpy(), g)
            if ovf:
                return []
            row, ids = o.match(np.ascontiguousarray(data), np.ascontiguousarray(offs), threads=1)
            return [(g, int(tids[k]), sorted(ids[row[k]:row[k + 1]].tolist())) for k in range(cnt)]

        return route, match_slot

    ex = PrefixExchange(rank, world, torch.device("cpu"), ps, make)
    out = ex.run(torch.from_numpy(mine.blob.copy()), torch.from_numpy(mine.off.view(np.int32).copy()), mine.n,
                 len(mine.blob))
    assert not ex.overflowed()
    got = [x for part in out for x in part]
    allg = [None] * world if rank == 0 else None
    dist.gather_object((rank, len(idx), ex.reruns, got), allg, dst=0)
    if rank == 0:
        q.put(allg)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,skew", [(2, False), (3, False), (2, True), (3, True)])
def test_prefix_exchange_gloo(world, skew):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_prefix_worker, args=(r, world, port, q, skew)) for r in range(world)]
    for p in procs:
        p.start()
    allg = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    f, t = _prefix_case(skew)
    o = OracleTrie(True, 0)
    o.add(f.blob, f.off)
    wrow, wids = o.match(t.blob, t.off)
    seen, owners = {}, set()
    for rank, n_filters, reruns, got in allg:
        assert n_filters < f.n          # a partition, not the whole table
        assert reruns == (1 if skew else 0)
        for src, tid, ids in got:
            lo, _ = topic_slice(t.n, src, world)
            assert (lo + tid) not in seen   # every topic matched on exactly one rank
            seen[lo + tid] = ids
            owners.add(rank)
    assert len(seen) == t.n
    if skew:
        assert len(owners) == 1         # every topic went to one rank
    assert sum(1 for i in range(t.n) if wrow[i + 1] > wrow[i]) > t.n // 10
    for i in range(t.n):
        assert seen[i] == sorted(wids[wrow[i]:wrow[i + 1]].tolist()), i
