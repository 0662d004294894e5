"""Filter-sharded layout on the GPU: the HIP merge kernel
(egm_shard_merge) against the numpy reference merge, G logical shards on one
MI355X merged on the device against the whole table, and ShardExchange over
RCCL ("nccl") at world size 1 — the bench's shard step end to end."""
import os
import socket

import numpy as np
import pytest

from emqx_amd import _lib as L
from emqx_amd import synth
from emqx_amd.dist import ShardExchange, gpu_merge, shard_of
from emqx_amd.engine import GpuMatcher, pack_strings
from oracle.cpp import canonical
from tests.shard_ref import merge_shard_results

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gm():
    m = GpuMatcher(0)
    yield m
    m.close()


def test_shard_merge_kernel_vs_numpy(gm):
    import torch
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(7)
    for G, n in ((1, 1), (3, 5_001), (8, 70_000), (16, 640)):
        parts = []
        for g in range(G):
            c = rng.integers(0, 6, n) * (rng.random(n) < 0.7)
            c[rng.random(n) < 0.001] = 3000          # a few long rows (several copy rounds per window)
            row = np.zeros(n + 1, np.uint64)
            row[1:] = np.cumsum(c)
            parts.append((row, rng.integers(0, 1 << 31, int(row[-1]), dtype=np.uint32)))
        want_row, want_ids = merge_shard_results(parts)
        counts = torch.from_numpy(np.concatenate([np.diff(p[0]).astype(np.int32) for p in parts])).to(dev)
        dids = [torch.from_numpy(p[1].view(np.int32)).to(dev) for p in parts]
        total = int(want_row[-1])
        out_row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        out_ids = torch.zeros(total + 16, dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        gm.shard_merge(G, n, counts.data_ptr(), [d.data_ptr() for d in dids], total, s, out_row.data_ptr(),
                       out_ids.data_ptr(), out_ids.numel())
        torch.cuda.synchronize()
        assert np.array_equal(out_row.cpu().numpy().view(np.uint64), want_row), (G, n)
        assert np.array_equal(out_ids[:total].cpu().numpy().view(np.uint32), want_ids), (G, n)
    with pytest.raises(L.EgmError):   # too small an output buffer is refused, nothing written
        gm.shard_merge(1, 1, counts.data_ptr(), [dids[0].data_ptr()], 100, 0, out_row.data_ptr(),
                       out_ids.data_ptr(), 10)


def test_logical_shards_merged_on_device(gm):
    """G filter shards on one GPU (each its own context and table), the same
    batch matched by each, merged by the HIP kernel == the whole table."""
    import torch
    dev = torch.device("cuda:0")
    f, t = synth.config("c0", n_topics=40_000)
    fl = f.to_list()
    G = 4
    sh = shard_of(f, G)
    d_blob = torch.from_numpy(t.blob).to(dev)
    d_off = torch.from_numpy(t.off.view(np.int32)).to(dev)
    n = t.n
    s = torch.cuda.current_stream().cuda_stream
    mats, rows, idss = [], [], []
    for g in range(G):
        idx = np.nonzero(sh == g)[0]
        m = GpuMatcher(0)
        m.build(*pack_strings([fl[i] for i in idx]), idx.astype(np.uint32))
        r = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        ids = torch.zeros(20 * n, dtype=torch.int32, device=dev)
        m.match_device(d_blob.data_ptr(), int(t.off[-1]), d_off.data_ptr(), n, L.EGM_MODE_ROUTES, s,
                       r.data_ptr(), ids.data_ptr(), ids.numel())
        torch.cuda.synchronize()
        assert m.last_stats()["overflow"] == 0
        mats.append(m)
        rows.append(r)
        idss.append(ids)
    counts = torch.cat([(r[1:] - r[:-1]).to(torch.int32) for r in rows])
    total = int(sum(int(r[-1].item()) for r in rows))
    out_row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    out_ids = torch.zeros(total + 1, dtype=torch.int32, device=dev)
    gm.shard_merge(G, n, counts.data_ptr(), [x.data_ptr() for x in idss], total, s, out_row.data_ptr(),
                   out_ids.data_ptr(), out_ids.numel())
    torch.cuda.synchronize()
    for m in mats:
        m.close()
    gm.build(f.blob, f.off)
    whole = gm.match(t.blob, t.off, L.EGM_MODE_ROUTES)
    row = out_row.cpu().numpy().view(np.uint64)
    ids = out_ids[:total].cpu().numpy().view(np.uint32)
    assert np.array_equal(row, whole.row_ptr)
    assert np.array_equal(canonical(row, ids), canonical(whole.row_ptr, whole.ids))


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def test_shard_exchange_rccl_world1(gm):
    """ShardExchange over RCCL at world size 1 with the GPU matcher on the
    shard-built table and the HIP merge: the bench's --mode shard step."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda:0")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        f, t = synth.config("c0", n_topics=50_000)
        sh = shard_of(f, 1)
        idx = np.nonzero(sh == 0)[0]
        fl = f.to_list()
        gm.build(*pack_strings([fl[i] for i in idx]), idx.astype(np.uint32))
        n = t.n
        s = torch.cuda.current_stream().cuda_stream
        d_blob = torch.from_numpy(t.blob).to(dev)
        d_off = torch.from_numpy(t.off.view(np.int32)).to(dev)
        d_row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        d_ids = torch.zeros(4 * n, dtype=torch.int32, device=dev)

        def local_match(tb, to, nn):
            gm.match_device(tb.data_ptr(), tb.numel(), to.data_ptr(), nn, L.EGM_MODE_ROUTES, s,
                            d_row.data_ptr(), d_ids.data_ptr(), d_ids.numel())
            st = gm.last_stats()
            return d_row, d_ids, int(st["n_ids"]), bool(st["overflow"])

        m_row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        m_ids = torch.zeros(40 * n, dtype=torch.int32, device=dev)
        ex = ShardExchange(0, 1, dev, local_match, gpu_merge(gm, s, m_row, m_ids))
        out = ex.step(d_blob, d_off)
        if out is None:   # first step sized the id buffer
            d_ids = torch.zeros(ex.last_totals[0] + 1024, dtype=torch.int32, device=dev)
            out = ex.step(d_blob, d_off, sizes=(n, d_blob.numel()))
        assert out is not None
        torch.cuda.synchronize()
        row = out[0].cpu().numpy().view(np.uint64)
        ids = out[1].cpu().numpy().view(np.uint32)
        gm.build(f.blob, f.off)
        whole = gm.match(t.blob, t.off, L.EGM_MODE_ROUTES)
        assert np.array_equal(row, whole.row_ptr)
        assert np.array_equal(canonical(row, ids), canonical(whole.row_ptr, whole.ids))
    finally:
        dist.destroy_process_group()


# ---- prefix partition ------------------------------------
def _prefix_setup(f, world, n_vparts=4096):
    from emqx_amd.dist import prefix_assign
    vr, fr = prefix_assign(f, world, n_vparts)
    return vr, fr


def test_prefix_route_kernel_vs_reference(gm):
    """egm_prefix_route (HIP) against its host restatement: per destination
    slot the same header, and the same source topic -> bytes pairs (the kernel
    orders a slot's topics by block arrival, so pairs are compared as sets);
    offsets consistent with the bytes; an undersized slot reports overflow."""
    import torch
    from emqx_amd.dist import PrefixSlots, prefix_route_reference
    dev = torch.device("cuda:0")
    f, t = synth.config("c2", n_filters=50_000, n_topics=60_000)
    for world in (1, 3, 8):
        vr, _ = _prefix_setup(f, world)
        ps = PrefixSlots.for_batch(world, t.n, len(t.blob))
        want = prefix_route_reference(t.blob, t.off, vr, ps)
        blob = torch.from_numpy(t.blob.copy()).to(dev)
        off = torch.from_numpy(t.off.view(np.int32).copy()).to(dev)
        dvr = torch.from_numpy(vr).to(dev)
        send = torch.zeros(world * ps.slot_bytes, dtype=torch.uint8, device=dev)
        gm.prefix_route(blob.data_ptr(), off.data_ptr(), t.n, dvr.data_ptr(), len(vr), world, ps.cap_topics,
                        ps.cap_bytes, torch.cuda.current_stream().cuda_stream, send.data_ptr())
        torch.cuda.synchronize()
        got = send.cpu().numpy()
        tl = t.to_list()
        total = 0
        for r in range(world):
            gc, gb, go, gt, goff, gdata = ps.parse(got, r)
            wc, wb, wo, wt, woff, wdata = ps.parse(want, r)
            assert (gc, gb, go) == (wc, wb, wo) == (wc, wb, 0), (world, r)
            full = got[r * ps.slot_bytes + ps.off_offsets:][:4 * (ps.cap_topics + 1)].view(np.uint32)
            assert np.all(full[gc:] == gb)   # padding topics: empty, at the end
            pairs = {int(gt[k]): bytes(gdata[int(goff[k]):int(goff[k + 1])]) for k in range(gc)}
            assert len(pairs) == gc and all(pairs[k] == tl[k] for k in pairs)
            assert set(pairs) == set(int(x) for x in wt)
            total += gc
        assert total == t.n
    # capacities too small: overflow flagged in the header, and the slot holds
    # a consistent prefix of its topics (count, bytes and offsets describe
    # exactly the topics placed) that egm_match_device_counted matches as
    # empty, without a fault (a byte overflow with topic room left
    # used to leave unwritten offsets below the header count)
    vr, _ = _prefix_setup(f, 2)
    dvr = torch.from_numpy(vr).to(dev)
    gm.build(f.blob, f.off)
    for small in (PrefixSlots(2, 100, 1 << 16), PrefixSlots(2, t.n, 1 << 16), PrefixSlots(2, t.n, 40_000)):
        send = torch.full((2 * small.slot_bytes,), 0xAB, dtype=torch.uint8, device=dev)   # stale bytes
        gm.prefix_route(blob.data_ptr(), off.data_ptr(), t.n, dvr.data_ptr(), len(vr), 2,
                        small.cap_topics, small.cap_bytes, 0, send.data_ptr())
        torch.cuda.synchronize()
        host = send.cpu().numpy()
        for r in range(2):
            gc, gb, go, gt, goff, gdata = small.parse(host, r)
            assert go == 1 and gc <= small.cap_topics and gb <= small.cap_bytes
            full = host[r * small.slot_bytes + small.off_offsets:][:4 * (small.cap_topics + 1)].view(np.uint32)
            assert full[0] == 0 and np.all(np.diff(full[:gc + 1].astype(np.int64)) >= 0) and full[gc] == gb
            assert np.all(full[gc:] == gb)
            pairs = {int(gt[k]): bytes(gdata[int(goff[k]):int(goff[k + 1])]) for k in range(gc)}
            assert len(pairs) == gc and all(pairs[k] == tl[k] for k in pairs)
            base = send.data_ptr() + r * small.slot_bytes
            row = torch.full((small.cap_topics + 1,), -1, dtype=torch.int64, device=dev)
            ids = torch.zeros(4096, dtype=torch.int32, device=dev)
            gm.match_device_counted(base + small.off_bytes, small.cap_bytes, base + small.off_offsets,
                                    small.cap_topics, base, L.EGM_MODE_ROUTES, 0, row.data_ptr(), ids.data_ptr(),
                                    ids.numel())
            torch.cuda.synchronize()
            st = gm.last_stats()
            assert st["overflow"] == 0 and st["errors"] == 0 and st["n_ids"] == 0
            assert int(row.abs().sum().item()) == 0     # every row empty: an overflowed slot is not walked


def _prefix_logical(f, t, world, mode=L.EGM_MODE_ROUTES):
    """`world` ranks emulated on one GPU: each holds its partition (replicated
    filters + its keys, global ids) in a context of its own and routes its own
    slice of the batch; the all_to_all is a device copy of slot r of every
    sender into rank r's receive buffer; each rank matches its received slots
    with egm_match_device_counted (count read on the device).  Returns, per
    topic of the batch, its ids (as a CSR in batch order) and the partition
    sizes."""
    import torch
    from emqx_amd.dist import PrefixSlots, topic_slice
    dev = torch.device("cuda:0")
    vr, fr = _prefix_setup(f, world)
    fl = f.to_list()
    parts = [t.subset(np.arange(*topic_slice(t.n, r, world))) for r in range(world)]
    ps = PrefixSlots.for_batch(world, max(p.n for p in parts), max(len(p.blob) for p in parts))
    dvr = torch.from_numpy(vr).to(dev)
    stream = torch.cuda.current_stream().cuda_stream
    sends, sizes, ctxs = [], [], []
    for r in range(world):
        idx = np.nonzero((fr == r) | (fr == L.EGM_PREFIX_ALL))[0]
        sizes.append(len(idx))
        g = GpuMatcher(0, max_batch=ps.cap_topics)
        blob, off = pack_strings([fl[i] for i in idx])
        g.build(blob, off, idx.astype(np.uint32))
        ctxs.append(g)
        p = parts[r]
        b = torch.from_numpy(p.blob.copy()).to(dev)
        o = torch.from_numpy(p.off.view(np.int32).copy()).to(dev)
        send = torch.zeros(world * ps.slot_bytes, dtype=torch.uint8, device=dev)
        g.prefix_route(b.data_ptr(), o.data_ptr(), p.n, dvr.data_ptr(), len(vr), world, ps.cap_topics,
                       ps.cap_bytes, stream, send.data_ptr())
        sends.append(send)
    rows_by_topic = [None] * t.n
    for q in range(world):
        recv = torch.cat([sends[r][q * ps.slot_bytes:(q + 1) * ps.slot_bytes] for r in range(world)])
        for r in range(world):
            base = recv.data_ptr() + r * ps.slot_bytes
            row = torch.zeros(ps.cap_topics + 1, dtype=torch.int64, device=dev)
            ids = torch.zeros(ps.cap_topics * 64 + 4096, dtype=torch.int32, device=dev)
            ctxs[q].match_device_counted(base + ps.off_bytes, ps.cap_bytes, base + ps.off_offsets, ps.cap_topics, base,
                                         mode, stream, row.data_ptr(), ids.data_ptr(), ids.numel())
            torch.cuda.synchronize()
            st = ctxs[q].last_stats()
            assert st["overflow"] == 0 and st["errors"] == 0
            cnt, nb, ovf, tids, offs, data = ps.parse(recv.cpu().numpy(), r)
            assert ovf == 0
            rown = row.cpu().numpy()
            idn = ids.cpu().numpy().view(np.uint32)
            assert np.all(rown[cnt:] == rown[cnt])   # padding topics: empty rows
            lo = topic_slice(t.n, r, world)[0]
            for k in range(cnt):
                i = lo + int(tids[k])
                assert rows_by_topic[i] is None      # matched on exactly one rank
                rows_by_topic[i] = idn[rown[k]:rown[k + 1]]
    for g in ctxs:
        g.close()
    row = np.zeros(t.n + 1, np.uint64)
    row[1:] = np.cumsum([len(x) for x in rows_by_topic])
    ids = np.concatenate(rows_by_topic) if t.n else np.zeros(0, np.uint32)
    return row, ids.astype(np.uint32), sizes


@pytest.mark.parametrize("world", [1, 2, 4])
def test_prefix_partitions_equal_whole_table(gm, world):
    """The prefix layout's rows, over every rank, equal the whole table's
    (ROUTES mode, C2 shape at 300K filters); no rank holds the whole table."""
    f, t = synth.config("c2", n_filters=300_000, n_topics=150_000)
    row, ids, sizes = _prefix_logical(f, t, world)
    gm.build(f.blob, f.off)
    want = gm.match(t.blob, t.off, L.EGM_MODE_ROUTES)
    assert np.array_equal(row, want.row_ptr)
    assert np.array_equal(canonical(row, ids), canonical(want.row_ptr, want.ids))
    if world > 1:
        assert max(sizes) < f.n


# ---- PrefixExchange.run on logical ranks (threads, one context each) --------
class _ThreadComm:
    """all_to_all / all_max between `world` threads of one process on one GPU
    (the collectives PrefixExchange takes from torch.distributed), so the
    exchange's own code — including its rerun — runs at world 2 and 4 on the
    single GPU of a test box.  Barriers time out instead of hanging."""

    def __init__(self, world):
        import threading
        self.world = world
        self.bar = threading.Barrier(world, timeout=180)
        self.box = [None] * world

    def rank(self, r):
        hub = self

        class _C:
            def all_to_all(self, recv, send):
                import torch
                torch.cuda.synchronize()
                hub.box[r] = send
                hub.bar.wait()
                S = recv.numel() // hub.world
                for q in range(hub.world):
                    recv[q * S:(q + 1) * S].copy_(hub.box[q][r * S:(r + 1) * S])
                torch.cuda.synchronize()
                hub.bar.wait()

            def all_max(self, t):
                import torch
                torch.cuda.synchronize()
                hub.box[r] = t.clone()
                hub.bar.wait()
                out = torch.stack(hub.box).max(0).values
                hub.bar.wait()
                return out

        return _C()


def _skew_topics(f, t):
    """Every topic's first two words replaced by the most common literal
    two-word prefix of the filters: the whole batch routes to one rank."""
    from collections import Counter
    heads = [x.split(b"/")[:2] for x in f.to_list() if x.count(b"/") >= 2]
    pre = Counter(tuple(h) for h in heads if b"+" not in h and b"#" not in h)
    (w0, w1), _ = pre.most_common(1)[0]
    blob, off = pack_strings([b"/".join([w0, w1] + x.split(b"/")[2:]) for x in t.to_list()])
    return synth.StringSet(blob, off)


@pytest.mark.parametrize("case,world,ordered", [("skew", 2, False), ("skew", 4, False), ("bytes", 2, False),
                                                ("plain", 2, False), ("skew", 2, True)])
def test_prefix_exchange_run_logical_ranks(gm, case, world, ordered):
    """dist.PrefixExchange.run on `world` logical ranks (threads, a context
    and a table partition each, _ThreadComm for the collectives):
    * skew — every topic shares one a/b prefix, so one slot per sender
      overflows at the layout's default slack; run() redoes the step with
      grown slots on every rank;
    * bytes — the first layout has room for every topic but too few bytes,
      so the first step's slots overflow by bytes (matched as empty, no
      fault) and the rerun completes;
    * plain — no overflow, no rerun;
    * ordered — the slots' rows in the walk's order (the bench's form).
    Every topic is matched on exactly one rank and the rows equal the whole
    table's (ROUTES mode)."""
    import threading
    import torch
    from emqx_amd.dist import PrefixExchange, PrefixSlots, gpu_prefix_stages, topic_slice
    dev = torch.device("cuda:0")
    f, t = synth.config("c2", n_filters=200_000, n_topics=100_000)
    if case == "skew":
        t = _skew_topics(f, t)
    vr, fr = _prefix_setup(f, world)
    fl = f.to_list()
    parts = [t.subset(np.arange(*topic_slice(t.n, r, world))) for r in range(world)]
    mt, mb = max(p.n for p in parts), max(len(p.blob) for p in parts)
    if case == "bytes":
        ps0 = PrefixSlots(world, mt, mb // (4 * world))
    else:
        ps0 = PrefixSlots(world, int(mt * 1.25 / world) + 16, int(mb * 1.25 / world) + 1024)
    hub = _ThreadComm(world)
    results, errors = [None] * world, []

    def rank_main(r):
        try:
            idx = np.nonzero((fr == r) | (fr == L.EGM_PREFIX_ALL))[0]
            g = GpuMatcher(0, max_batch=mt)
            try:
                blob, off = pack_strings([fl[i] for i in idx])
                g.build(blob, off, idx.astype(np.uint32))
                dvr = torch.from_numpy(vr).to(dev)
                p = parts[r]
                b = torch.from_numpy(p.blob.copy()).to(dev)
                o = torch.from_numpy(p.off.view(np.int32).copy()).to(dev)
                ex = PrefixExchange(r, world, dev, ps0, gpu_prefix_stages(g, dvr, L.EGM_MODE_ROUTES, 0, 128, ordered),
                                    comm=hub.rank(r))
                out = ex.run(b, o, p.n, len(p.blob))
                torch.cuda.synchronize()
                assert not ex.overflowed()
                st = g.last_stats()
                assert st["errors"] == 0
                got = []
                for src, (row, ids, tids) in enumerate(out):
                    rown = row.cpu().numpy()
                    got.append((src, rown, ids.cpu().numpy().view(np.uint32), tids.cpu().numpy().view(np.uint32)))
                recv = (ex.recv if world > 1 else ex.route.send).cpu().numpy()
                counts = [ex.ps.parse(recv, src)[0] for src in range(world)]
                results[r] = (ex.reruns, got, counts, len(idx))
            finally:
                g.close()
        except BaseException as e:   # noqa: BLE001 - reported below, barrier released
            errors.append((r, repr(e)))
            hub.bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=600)
    assert not errors, errors
    rows_by_topic = [None] * t.n
    owners = set()
    for r in range(world):
        reruns, got, counts, nf = results[r]
        assert reruns == (0 if case == "plain" else 1), (r, reruns)
        if world > 1:
            assert nf < f.n
        for (src, rown, idn, tids), cnt in zip(got, counts):
            assert np.all(rown[cnt:] == rown[cnt])      # padding topics: empty rows
            lo = topic_slice(t.n, src, world)[0]
            for k in range(cnt):
                i = lo + int(tids[k])
                assert rows_by_topic[i] is None         # matched on exactly one rank
                rows_by_topic[i] = idn[rown[k]:rown[k + 1]]
                owners.add(r)
    assert all(x is not None for x in rows_by_topic)
    if case == "skew":
        assert len(owners) == 1
    row = np.zeros(t.n + 1, np.uint64)
    row[1:] = np.cumsum([len(x) for x in rows_by_topic])
    ids = np.concatenate(rows_by_topic)
    gm.build(f.blob, f.off)
    want = gm.match(t.blob, t.off, L.EGM_MODE_ROUTES)
    assert int(want.row_ptr[-1]) > t.n                # matches exist
    assert np.array_equal(row, want.row_ptr)
    assert np.array_equal(canonical(row, ids), canonical(want.row_ptr, want.ids))
