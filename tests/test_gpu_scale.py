"""GPU parity at the benchmarked sizes (C2, C4 and dense C3 were
benchmarked but never checked; VERDICT r5 item 1: every full-size row is
compared with the oracle as a SET, not by its count alone).

A row is compared through its count and an order-independent checksum of its
ids (tests/rowsum.py), the oracle computing the same checksum per row
(oracle/trie_oracle.cpp ot_match_sums); sampled rows are also compared id by
id.

* C2 at full size — 10M wildcard filters x 10M topics, the bench's own
  workload: every row (count + checksum) against the C++ oracle (in four
  parts, so no single test is silent for minutes), 200K sampled rows
  id-exact, determinism, the prefix-partition layout at 8 logical ranks and
  the walk-order row form — both against the oracle's rows.
* C4 at its full size: 100M filters with the subscriber table and the bench's
  10M-topic batch, match + fan-out; the oracle is built as 4 disjoint filter
  shards of 25M whose per-row checksums add up: the first 1M
  rows of the batch against it, 20K rows id-exact, every delivery row
  pointer of the 10M topics, sampled delivery rows element-for-element in
  emqx_broker:dispatch/2 order (apps/emqx/src/emqx_broker.erl:283-308).
* C3 at its full size: 10M depth-16 filters ('+' p=.35, '#' p=.7) and the
  bench's 10M-topic batch, both match modes, in the walk's depth-first regime
  (pops cut by the stack-room bound, counted by the kernel); the batch's first
  100K rows against the oracle, 5K id-exact, all 10M rows equal across the
  two modes, V_t.
* C3's $share-group fan-out at 1M filters.

The oracle is the pinned C++ restatement of emqx_trie compact mode
(oracle/trie_oracle.cpp; apps/emqx/src/emqx_trie.erl:251-266).
"""
import numpy as np
import pytest

from emqx_amd import _lib as L
from emqx_amd import synth
from emqx_amd.engine import GpuMatcher
from emqx_amd.hostinfo import usable_cpus
from oracle.cpp import OracleTrie, canonical
from tests.rowsum import row_checksums

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

THREADS = max(4, usable_cpus())


def sampled_rows(res_row, res_ids, idx):
    r = np.zeros(len(idx) + 1, np.uint64)
    r[1:] = np.cumsum(np.diff(res_row)[idx])
    parts = [res_ids[int(res_row[i]):int(res_row[i + 1])] for i in idx]
    ids = np.concatenate(parts) if parts else np.zeros(0, np.uint32)
    return r, ids


def assert_rows(got_cnt, got_sum, want_cnt, want_sum, base=0, what=""):
    """Every row equal as a set: count and order-independent checksum."""
    bad = np.nonzero((np.asarray(got_cnt, np.int64) != np.asarray(want_cnt, np.int64)) | (got_sum != want_sum))[0]
    assert len(bad) == 0, (what, len(bad), [(int(base + i), int(got_cnt[i]), int(want_cnt[i])) for i in bad[:5]])


# ------------------------------------------------------------------ C2 -------
@pytest.fixture(scope="class")
def c2():
    f, t = synth.config("c2")
    gm = GpuMatcher(0, max_batch=t.n)
    gm.build(f.blob, f.off)
    res = gm.match(t.blob, t.off, L.EGM_MODE_ROUTES)
    assert res.n_error == 0
    o = OracleTrie(True, L.EGM_MODE_ROUTES)
    o.add(f.blob, f.off)
    yield {"f": f, "t": t, "gm": gm, "res": res, "o": o, "want": {}}
    gm.close()


C2_PARTS = 4


def c2_part(c2, part):
    """The oracle's rows (count, checksum) for part `part` of the batch,
    computed once per class."""
    t, o = c2["t"], c2["o"]
    if part not in c2["want"]:
        lo, hi = t.n * part // C2_PARTS, t.n * (part + 1) // C2_PARTS
        c2["want"][part] = o.match_sums(t.blob, t.off[lo:hi + 1], threads=THREADS)   # absolute offsets into one blob
    return c2["want"][part]


def c2_oracle(c2):
    """The oracle's rows for the whole batch: (counts u32[n], checksums u64[n])."""
    parts = [c2_part(c2, k) for k in range(C2_PARTS)]
    return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])


def c2_gpu_sums(c2):
    if "gsum" not in c2:
        c2["gsum"] = row_checksums(c2["res"].row_ptr, c2["res"].ids)
    return c2["gsum"]


class TestC2Full:
    """C2 at full size; the class scope frees its 10M-filter table and oracle
    before the C4/C3 tests build theirs."""

    @pytest.mark.parametrize("part", range(C2_PARTS))
    def test_c2_full_rows(self, c2, part):
        """Every row of the 10M-topic batch against the oracle: count and
        order-independent checksum of its ids (emqx_router:match_routes/1,
        apps/emqx/src/emqx_router.erl:129-134)."""
        t, res = c2["t"], c2["res"]
        lo, hi = t.n * part // C2_PARTS, t.n * (part + 1) // C2_PARTS
        want, wsum = c2_part(c2, part)
        got = np.diff(res.row_ptr[lo:hi + 1]).astype(np.uint32)
        assert_rows(got, c2_gpu_sums(c2)[lo:hi], want, wsum, lo, "C2 part")

    def test_c2_full_sampled_rows_exact(self, c2):
        t, res, o = c2["t"], c2["res"], c2["o"]
        idx = np.sort(np.random.default_rng(2).choice(t.n, 200_000, replace=False))
        sub = t.subset(idx)
        row, ids = o.match(sub.blob, sub.off, threads=THREADS)
        grow, gids = sampled_rows(res.row_ptr, res.ids, idx)
        assert np.array_equal(grow, row)
        assert np.array_equal(canonical(grow, gids), canonical(row, ids))
        assert int(res.row_ptr[-1]) > 40 * t.n   # ~50 matches per C2 topic
        # the bench line's V_t (32 B per state of its 22.4 GB model): the sample's
        # kernel count equals the oracle's independent count
        vt, _ = o.visited_counts(sub.blob, sub.off, threads=THREADS)
        assert c2["gm"].match(sub.blob, sub.off, L.EGM_MODE_ROUTES).visited == vt

    def test_c2_full_eight_prefix_partitions(self, c2):
        """The prefix-partition layout of BASELINE C2 at 8 ranks on one GPU
        (VERDICT r3 item 5): the 10M filters partitioned by their first two
        words (egm_prefix_assign: 28 % replicated, the rest on one rank each),
        the 10M-topic batch split into 8 per-rank batches, each routed by
        egm_prefix_route, the all_to_all emulated by device copies of the
        slots, every received slot matched in place by
        egm_match_device_counted (count read on the device) against its
        rank's partition — every topic matched on exactly one rank, with the
        oracle's row (every row as a set: its count and a per-row
        order-independent checksum)."""
        import torch
        from emqx_amd.dist import PrefixSlots, prefix_assign, topic_slice
        f, t, res = c2["f"], c2["t"], c2["res"]
        dev = torch.device("cuda:0")
        s = torch.cuda.current_stream().cuda_stream
        G = 8
        vr, fr = prefix_assign(f, G)
        parts = [topic_slice(t.n, r, G) for r in range(G)]
        ps = PrefixSlots.for_batch(G, max(hi - lo for lo, hi in parts),
                                   max(int(t.off[hi]) - int(t.off[lo]) for lo, hi in parts))
        dvr = torch.from_numpy(vr).to(dev)
        d_blob = torch.from_numpy(t.blob).to(dev)
        sends = []
        m = GpuMatcher(0, max_batch=ps.cap_topics)
        for lo, hi in parts:   # each rank's batch: a slice of the blob, offsets rebased to 0
            sub_off = torch.from_numpy((t.off[lo:hi + 1] - t.off[lo]).astype(np.uint32).view(np.int32)).to(dev)
            send = torch.zeros(G * ps.slot_bytes, dtype=torch.uint8, device=dev)
            m.prefix_route(d_blob.data_ptr() + int(t.off[lo]), sub_off.data_ptr(), hi - lo, dvr.data_ptr(), len(vr), G,
                           ps.cap_topics, ps.cap_bytes, s, send.data_ptr())
            sends.append(send)
        torch.cuda.synchronize()
        # the slots as routed: any later change to a send buffer is a device-memory corruption
        snap = [x.cpu().numpy() for x in sends]
        got_tot = np.full(t.n, -1, np.int64)
        got_sum = np.zeros(t.n, np.uint64)
        sizes = []
        try:
            for q in range(G):
                idx = np.nonzero((fr == q) | (fr == L.EGM_PREFIX_ALL))[0].astype(np.uint32)
                sizes.append(len(idx))
                part = f.subset(idx)
                m.build(part.blob, part.off, idx)
                del part
                recv = torch.cat([sends[r][q * ps.slot_bytes:(q + 1) * ps.slot_bytes] for r in range(G)])
                host = recv.cpu().numpy()
                for r in range(G):
                    a = snap[r][q * ps.slot_bytes:(q + 1) * ps.slot_bytes]
                    b = host[r * ps.slot_bytes:(r + 1) * ps.slot_bytes]
                    if not np.array_equal(a, b):
                        d = np.nonzero(a != b)[0]
                        raise AssertionError(("send buffer changed after routing", q, r, len(d), d[:8].tolist(),
                                              a[d[:8]].tolist(), b[d[:8]].tolist()))
                row = torch.zeros(ps.cap_topics + 1, dtype=torch.int64, device=dev)
                ids = torch.zeros(ps.cap_topics * 96 + 4096, dtype=torch.int32, device=dev)
                for r in range(G):
                    base = recv.data_ptr() + r * ps.slot_bytes
                    m.match_device_counted(base + ps.off_bytes, ps.cap_bytes, base + ps.off_offsets, ps.cap_topics,
                                           base, L.EGM_MODE_ROUTES, s, row.data_ptr(), ids.data_ptr(), ids.numel())
                    torch.cuda.synchronize()
                    st = m.last_stats()
                    assert st["overflow"] == 0 and st["errors"] == 0, (q, r, st)
                    cnt, nb, ovf, tids, offs, data = ps.parse(host, r)
                    assert ovf == 0
                    rown = row.cpu().numpy().view(np.uint64)
                    assert np.all(rown[cnt:] == rown[cnt])   # padding: empty rows
                    gidx = parts[r][0] + tids.astype(np.int64)
                    seen = np.nonzero(got_tot[gidx] >= 0)[0]
                    assert len(seen) == 0, ("topic matched on two ranks", q, r, cnt, nb, len(tids), len(seen),
                                            seen[:5].tolist(), tids[seen[:5]].tolist(),
                                            int(tids.min()) if len(tids) else None,
                                            int(tids.max()) if len(tids) else None,
                                            parts[r], int(len(np.unique(tids))))   # matched on exactly one rank
                    got_tot[gidx] = np.diff(rown[:cnt + 1]).astype(np.int64)
                    got_sum[gidx] = row_checksums(rown[:cnt + 1], ids[:int(rown[cnt])].cpu().numpy().view(np.uint32))
        finally:
            m.close()
        assert np.all(got_tot >= 0)
        want, wsum = c2_oracle(c2)   # the oracle's rows, not the GPU's own input-order result
        assert_rows(got_tot, got_sum, want, wsum, 0, "8 prefix partitions")
        assert max(sizes) < 0.45 * f.n, sizes   # a partition, not a replica (37 % at 8 ranks)

    def test_c2_full_ordered_rows(self, c2):
        """The bench's result form at full size: egm_match_device_ordered (rows
        in walk order + the row -> topic map).  The map is a permutation and
        every topic's row equals the oracle's row for that topic (count and an
        order-independent checksum)."""
        import torch
        t, res, gm = c2["t"], c2["res"], c2["gm"]
        dev = torch.device("cuda:0")
        n, cap = t.n, int(res.row_ptr[-1]) + 4096
        d_blob = torch.from_numpy(t.blob).to(dev)
        d_off = torch.from_numpy(t.off.view(np.int32)).to(dev)
        d_row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        d_top = torch.full((n,), -1, dtype=torch.int32, device=dev)
        d_ids = torch.zeros(cap, dtype=torch.int32, device=dev)
        gm.match_device_ordered(d_blob.data_ptr(), int(t.off[-1]), d_off.data_ptr(), n, L.EGM_MODE_ROUTES, 0,
                                d_row.data_ptr(), d_top.data_ptr(), d_ids.data_ptr(), cap)
        st = gm.last_stats()
        assert st["overflow"] == 0 and st["errors"] == 0 and st["n_ids"] == int(res.row_ptr[-1])
        row_w = d_row.cpu().numpy().view(np.uint64)
        topic = d_top.cpu().numpy().view(np.uint32).astype(np.int64)
        ids_w = d_ids[:st["n_ids"]].cpu().numpy().view(np.uint32)
        del d_ids, d_row, d_top, d_blob, d_off
        assert np.array_equal(np.sort(topic), np.arange(n))
        assert np.count_nonzero(topic != np.arange(n)) > n // 2   # the walk's order, not the input's
        want, wsum = c2_oracle(c2)
        assert_rows(np.diff(row_w).astype(np.int64), row_checksums(row_w, ids_w), want[topic], wsum[topic], 0,
                    "walk-order rows")

    def test_c2_full_determinism(self, c2):
        t, res, gm = c2["t"], c2["res"], c2["gm"]
        again = gm.match(t.blob, t.off, L.EGM_MODE_ROUTES)
        assert np.array_equal(again.row_ptr, res.row_ptr)
        assert np.array_equal(row_checksums(again.row_ptr, again.ids), c2_gpu_sums(c2))
        st = gm.walk_counters()
        assert st["popped"] > 0


# ------------------------------------------------------------------ C4 -------
def _expected_deliveries(mids, srow, subs):
    mids = mids.astype(np.int64)
    cnt = (srow[mids + 1] - srow[mids]).astype(np.int64)
    fid = np.repeat(mids, cnt)
    starts = np.repeat(srow[mids].astype(np.int64) - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt)
    sub = subs[starts + np.arange(int(cnt.sum()))]
    return fid.astype(np.uint32), sub.astype(np.uint32)


def _oracle_shards(f, n_shards, mode, par=5):
    """The oracle over f as n_shards disjoint filter ranges (global ids =
    index), built `par` at a time: a string-keyed oracle of all 100M filters
    would not fit, and the match set over F is the disjoint union of the sets
    over its parts."""
    import threading
    bounds = [f.n * k // n_shards for k in range(n_shards + 1)]
    shards = [None] * n_shards

    def build(k):
        o = OracleTrie(True, mode)
        lo, hi = bounds[k], bounds[k + 1]
        o.add(f.blob, f.off[lo:hi + 1], np.arange(lo, hi, dtype=np.uint32))
        shards[k] = o

    for k0 in range(0, n_shards, par):
        th = [threading.Thread(target=build, args=(k,)) for k in range(k0, min(n_shards, k0 + par))]
        for x in th:
            x.start()
        for x in th:
            x.join()
    return shards


def test_c4_full_size_match_and_fanout():
    """BASELINE C4 at its full size (r5 weak 2: at the
    bench's batch size): 100M filters (20 % wildcard, depth 4-8) with the
    subscriber table (1+Poisson(1) subscribers, 0.1 % of filters with 2 000,
    10 % $share groups), the 10M-topic batch the bench times, ROUTES mode
    (emqx_router:match_routes/1) + fan-out (emqx_broker:dispatch/2,
    apps/emqx/src/emqx_broker.erl:283-324).  Checked against the pinned C++
    oracle (emqx_trie.erl:251-266) built as 4 disjoint filter shards of 25M:
    the batch's first 1M rows as sets (count + checksum, summed over the
    shards), 20K of them id-exact, every delivery row pointer of the 10M
    topics, and 3K delivery rows element for element."""
    import threading
    import time
    import torch
    t0 = time.time()
    f, t = synth.config("c4")
    assert f.n == 100_000_000 and t.n == 10_000_000
    print(f"[c4] generated in {time.time() - t0:.0f}s", flush=True)
    srow, subs = synth.subscribers(f.n, lam=1.0, p_big=0.001, n_big=2000, p_share=0.1,
                                   seed=synth.SEED_BASE + synth.CONFIG_INDEX["c4"])
    n_chk = 1_000_000
    # the oracle shards build on the host while the GPU works (ctypes drops the GIL)
    shards = [None]
    ob = threading.Thread(target=lambda: shards.__setitem__(0, _oracle_shards(f, 4, L.EGM_MODE_ROUTES, par=4)))
    gm = GpuMatcher(0, max_batch=t.n)
    try:
        t0 = time.time()
        gm.build(f.blob, f.off)
        gm.subs_build(srow, subs)
        print(f"[c4] table + subscribers built in {time.time() - t0:.0f}s: {gm.stats()}", flush=True)
        ob.start()
        dev = torch.device("cuda:0")
        s = torch.cuda.current_stream().cuda_stream
        d_blob = torch.from_numpy(t.blob).to(dev)
        d_off = torch.from_numpy(t.off.view(np.int32)).to(dev)
        n, cap = t.n, 64 * t.n
        d_row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        d_ids = torch.zeros(cap, dtype=torch.int32, device=dev)
        gm.match_device(d_blob.data_ptr(), int(t.off[-1]), d_off.data_ptr(), n, L.EGM_MODE_ROUTES, s,
                        d_row.data_ptr(), d_ids.data_ptr(), cap)
        torch.cuda.synchronize()
        st = gm.last_stats()
        assert st["overflow"] == 0 and st["errors"] == 0, st
        mrow = d_row.cpu().numpy().view(np.uint64)
        mids = d_ids[: int(mrow[-1])].cpu().numpy().view(np.uint32)
        # fan-out on the device, checked below
        cnt = (srow[mids.astype(np.int64) + 1] - srow[mids.astype(np.int64)]).astype(np.uint64)
        dpos = np.zeros(len(mids) + 1, np.uint64)
        np.cumsum(cnt, out=dpos[1:])
        del cnt
        tot = int(dpos[-1])
        assert tot > 100 * n   # the 2 000-subscriber filters dominate
        d_drow = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        d_fid = torch.zeros(tot + 8, dtype=torch.int32, device=dev)
        d_sub = torch.zeros(tot + 8, dtype=torch.int32, device=dev)
        gm.fanout_device(d_row.data_ptr(), d_ids.data_ptr(), cap, n, s, d_drow.data_ptr(), d_fid.data_ptr(),
                         d_sub.data_ptr(), tot + 8)
        torch.cuda.synchronize()
        drow = d_drow.cpu().numpy().view(np.uint64)
        assert np.array_equal(drow, dpos[mrow.astype(np.int64)])   # every delivery row of the 10M topics
        del dpos
        # rows checked id-exact against the oracle below, and 3K of them whose
        # delivery lists are also checked against the oracle's ids
        idx = np.sort(np.random.default_rng(4).choice(n_chk, 20_000, replace=False))
        dsel = np.sort(np.random.default_rng(5).choice(idx, 3_000, replace=False))
        got_dl = {}
        for i in dsel:
            a, b = int(mrow[i]), int(mrow[i + 1])
            wf, ws = _expected_deliveries(mids[a:b], srow, subs)   # dispatch order of the GPU's match row
            lo, hi = int(drow[i]), int(drow[i + 1])
            assert hi - lo == len(wf)
            gf = d_fid[lo:hi].cpu().numpy().view(np.uint32).copy()
            gs = d_sub[lo:hi].cpu().numpy().view(np.uint32).copy()
            assert np.array_equal(gf, wf) and np.array_equal(gs, ws), i
            got_dl[int(i)] = (gf, gs)
        grp = d_sub[: min(tot, 50_000_000)].cpu().numpy().view(np.uint32)
        assert np.count_nonzero(grp & np.uint32(L.GROUP_BIT)) > 0   # (filter, group) entries, never members
        del d_fid, d_sub, d_ids, grp, d_blob, d_off, d_row, d_drow
        torch.cuda.empty_cache()
        gm.close()
        gm = None
        c_row = mrow[:n_chk + 1]
        gsum = row_checksums(c_row, mids)
        t0 = time.time()
        ob.join()
        print(f"[c4] oracle shards ready {time.time() - t0:.0f}s after the GPU checks", flush=True)
        want = np.zeros(n_chk, np.uint64)
        wsum = np.zeros(n_chk, np.uint64)
        sub = t.subset(idx)
        chk = t.subset(np.arange(n_chk))
        parts = []
        for o in shards[0]:
            c, sm = o.match_sums(chk.blob, chk.off, threads=THREADS)
            want += c
            wsum += sm    # the shards are disjoint: the row's checksum is their sum (mod 2^64)
            parts.append(o.match(sub.blob, sub.off, threads=THREADS))
        print(f"[c4] oracle matched in {time.time() - t0:.0f}s", flush=True)
        assert_rows(np.diff(c_row), gsum, want, wsum, 0, "C4 first 1M rows")
        from tests.shard_ref import merge_shard_results
        orow, oids = merge_shard_results(parts)
        grow, gids = sampled_rows(mrow, mids, idx)
        assert np.array_equal(grow, orow)
        assert np.array_equal(canonical(grow, gids), canonical(orow, oids))
        # delivery multisets from the ORACLE's match ids (emqx_broker.erl:283-308)
        pos = {int(i): k for k, i in enumerate(idx)}
        for i, (gf, gs) in got_dl.items():
            k = pos[i]
            of = oids[int(orow[k]):int(orow[k + 1])]
            wf, ws = _expected_deliveries(of, srow, subs)
            want_pairs = np.sort(wf.astype(np.uint64) << np.uint64(32) | ws.astype(np.uint64))
            got_pairs = np.sort(gf.astype(np.uint64) << np.uint64(32) | gs.astype(np.uint64))
            assert np.array_equal(got_pairs, want_pairs), i
    finally:
        if gm is not None:
            gm.close()
        if ob.is_alive():
            ob.join()


# ------------------------------------------------------------------ C3 -------
def test_c3_full_size_dfs_regime_both_modes():
    """BASELINE C3 at its full size (r5 item 1 and weak 2:
    every checked row as a set, at the bench's batch size): 10M depth-16
    filters ('+' p=.35, '#' p=.7; 116.7M trie nodes) and the 10M-topic batch
    the bench times, both match modes.  The walk's deep pass must keep its
    pops full (lane occupancy > 0.6); the batch's first 100K rows (count +
    checksum) against the C++ oracle and 5K of them id-exact, in both modes;
    all 10M rows equal across the two modes."""
    import threading
    import time
    t0 = time.time()
    f = synth.config_filters("c3")
    assert f.n == 10_000_000
    n_chk = 100_000
    oracle = {}
    topics_ready = threading.Event()

    def run_oracle():   # on the host beside the topic generation and the GPU (ctypes drops the GIL)
        o = OracleTrie(True, L.EGM_MODE_ROUTES)
        o.add(f.blob, f.off)
        topics_ready.wait()
        oracle["rows"] = o.match_sums(oracle["chk"].blob, oracle["chk"].off, threads=THREADS)
        oracle["ids"] = o.match(oracle["sub"].blob, oracle["sub"].off, threads=THREADS)

    ot = threading.Thread(target=run_oracle)
    ot.start()
    try:
        t = synth.config_topics("c3", f)
    finally:
        if "t" not in locals():
            topics_ready.set()
    assert t.n == 10_000_000
    # Every C3 filter is a wildcard filter and no topic has a '+' or '#' byte,
    # so no topic equals a filter: emqx_router:match_routes/1's exact lookup
    # (emqx_router.erl:133) adds nothing and the two modes' expected rows are
    # the same — one oracle pass serves both.
    idx = np.sort(np.random.default_rng(3).choice(n_chk, 5_000, replace=False))
    oracle["chk"] = t.subset(np.arange(n_chk))
    oracle["sub"] = sub = t.subset(idx)
    topics_ready.set()
    assert not np.any((t.blob == ord("+")) | (t.blob == ord("#")))
    gm = GpuMatcher(0, max_batch=t.n)
    try:
        gm.build(f.blob, f.off)
        print(f"[c3] generated + built in {time.time() - t0:.0f}s: {gm.stats()}", flush=True)
        res = {}
        for m in (L.EGM_MODE_TRIE, L.EGM_MODE_ROUTES):
            r = gm.match(t.blob, t.off, m)
            assert r.n_error == 0, m
            st = gm.last_stats()
            assert st["overflow"] == 0 and st["errors"] == 0, (m, st)
            res[m] = (r.row_ptr, row_checksums(r.row_ptr, r.ids), r.visited, sampled_rows(r.row_ptr, r.ids, idx),
                      r.row_ptr[:n_chk + 1].copy())
            if m == L.EGM_MODE_TRIE:
                wc = gm.walk_counters()
                # the walk's deep pass keeps the pops of C3's wide frontiers
                # full (round 2, one 320-item pass: occupancy 0.39)
                assert wc["lane_occupancy"] > 0.6, wc
            del r
    finally:
        gm.close()
    rt, rr = res[L.EGM_MODE_TRIE], res[L.EGM_MODE_ROUTES]
    assert np.array_equal(rt[0], rr[0]) and np.array_equal(rt[1], rr[1])   # all 10M rows, both modes
    assert rt[2] == rr[2] > 0   # V_t (pinned against the oracle's count at the C3 shape in test_gpu_parity.py)
    t0 = time.time()
    ot.join()
    print(f"[c3] oracle ready {time.time() - t0:.0f}s after the GPU walks", flush=True)
    want, wsum = oracle["rows"]
    row, ids = oracle["ids"]
    for m in (L.EGM_MODE_TRIE, L.EGM_MODE_ROUTES):
        rp, gsum, _, (grow, gids), crow = res[m]
        assert_rows(np.diff(crow), gsum[:n_chk], want, wsum, 0, ("C3 first rows", m))
        assert np.array_equal(grow, row)
        assert np.array_equal(canonical(grow, gids), canonical(row, ids))


def test_c3_share_group_fanout():
    """bench --config c3's fan-out (1+Poisson(1) subscribers, 10 % of the
    filters through $share groups g0..g63 of 2-16 members) at 1M filters:
    every delivery row and 3K rows element for element
    (apps/emqx/src/emqx_broker.erl:283-308, emqx_shared_sub.erl:120-135)."""
    f, t = synth.config("c3", n_filters=1_000_000, n_topics=200_000)
    gm = GpuMatcher(0, max_batch=t.n)
    try:
        gm.build(f.blob, f.off)
        res = gm.match(t.blob, t.off, L.EGM_MODE_ROUTES)
        srow, subs = synth.subscribers(f.n, lam=1.0, p_big=0.001, n_big=2000, p_share=0.1, groups=64,
                                       seed=synth.SEED_BASE + synth.CONFIG_INDEX["c3"])
        gm.subs_build(srow, subs)
        drow, dfid, dsub = gm.fanout(res)
        mids = res.ids.astype(np.int64)
        cnt = (srow[mids + 1] - srow[mids]).astype(np.uint64)
        dpos = np.zeros(len(mids) + 1, np.uint64)
        np.cumsum(cnt, out=dpos[1:])
        assert np.array_equal(drow, dpos[res.row_ptr.astype(np.int64)])
        for i in np.random.default_rng(6).choice(t.n, 3_000, replace=False):
            a, b = int(res.row_ptr[i]), int(res.row_ptr[i + 1])
            wf, ws = _expected_deliveries(res.ids[a:b], srow, subs)
            lo, hi = int(drow[i]), int(drow[i + 1])
            assert np.array_equal(dfid[lo:hi], wf) and np.array_equal(dsub[lo:hi], ws), i
        assert np.count_nonzero(dsub & np.uint32(L.GROUP_BIT)) > 0
    finally:
        gm.close()
