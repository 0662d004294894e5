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
from emqx_amd.dist import merge_shard_results, merge_shard_results_torch, shard_of, topic_slice, ShardExchange
from emqx_amd.engine import pack_strings
from oracle.cpp import OracleTrie, canonical


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
        return torch.from_numpy(row.astype(np.int64)), torch.from_numpy(ids.astype(np.int32))

    ex = ShardExchange(rank, world, torch.device("cpu"), local_match)
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


def test_merge_numpy_equals_torch():
    rng = np.random.default_rng(0)
    n, G = 500, 3
    parts = []
    for g in range(G):
        c = rng.integers(0, 4, n)
        row = np.zeros(n + 1, np.uint64)
        row[1:] = np.cumsum(c)
        parts.append((row, rng.integers(0, 1 << 30, int(row[-1])).astype(np.uint32)))
    r1, i1 = merge_shard_results(parts)
    cnt = torch.stack([torch.from_numpy(np.diff(p[0]).astype(np.int64)) for p in parts])
    r2, i2 = merge_shard_results_torch(cnt, [torch.from_numpy(p[1].astype(np.int32)) for p in parts])
    assert np.array_equal(r1, r2.numpy().astype(np.uint64))
    assert np.array_equal(i1, i2.numpy().astype(np.uint32))


def test_topic_slices_cover():
    for n in (0, 1, 7, 1000):
        for w in (1, 2, 3, 8):
            s = [topic_slice(n, r, w) for r in range(w)]
            assert s[0][0] == 0 and s[-1][1] == n
            assert all(s[i][1] == s[i + 1][0] for i in range(w - 1))
