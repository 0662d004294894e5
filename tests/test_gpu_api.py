"""The reference-shaped host API (emqx_amd.trie / router / broker) on the GPU,
checked with the reference suites' own cases and against the oracle."""
import random

import pytest

from emqx_amd.broker import Broker
from emqx_amd.router import Route, Router
from emqx_amd.trie import Trie
from oracle import trie_ref as R
from tests.kat import b, load
from tests.test_capi_cpu import rand_filter, rand_topic

pytestmark = pytest.mark.gpu
K = load()


@pytest.mark.parametrize("case", K["trie_cases"], ids=lambda c: c["name"])
def test_trie_suite_cases(case):
    t = Trie()
    with t.transaction():
        pass
    for op in case["ops"]:
        if op[0] == "insert":
            assert t.insert(b(op[1])) == "ok"
        elif op[0] == "delete":
            assert t.delete(b(op[1])) == "ok"
        elif op[0] == "assert_empty":
            assert t.empty() is op[1]
    for q, exp in case["queries"]:
        assert sorted(t.match(b(q))) == sorted(b(x) for x in exp)
    with pytest.raises(TypeError):
        t.match("not-a-binary")


def test_router_match_routes_suite():
    case = K["router_match_routes"]
    r = Router()
    for topic, d in case["routes"]:
        r.add_route(b(topic), d)
    got = sorted(r.match_routes(b(case["query"])))
    assert got == sorted(Route(b(t), d) for t, d in case["expected"])
    for topic, d in case["routes"]:
        r.delete_route(b(topic), d)
    assert r.match_routes(b(case["query"])) == []


def test_router_random_vs_oracle():
    rng = random.Random(3)
    r = Router()
    o = R.Router()
    fl = list(dict.fromkeys(rand_filter(rng) for _ in range(200)))
    for f in fl:
        for d in ("local", "n2") if rng.random() < 0.2 else ("local",):
            r.do_add_route(f, d)
            o.do_add_route(f, d)
    for f in fl[::5]:
        r.do_delete_route(f, "local")
        o.do_delete_route(f, "local")
    topics = [rand_topic(rng) for _ in range(500)]
    got = r.match_routes_batch(topics)
    for t, g in zip(topics, got):
        assert sorted(g) == sorted(Route(x, d) for x, d in o.match_routes(t)), t


def test_broker_suite_cases():
    for case in K["broker_delivery"]["cases"]:
        br = Broker(shared_strategy="round_robin")
        for flt, sub, group in case["subs"]:
            topic = b(flt) if group is None else b"$share/" + b(group) + b"/" + b(flt)
            br.subscribe(topic, sub)
        got = br.publish(b(case["publish"]))
        want = set((k, b(f), b(x) if isinstance(x, str) else x) for k, f, x in case["expected"])
        assert set(d[:3] for d in got) == want, case["name"]
        for d in got:
            if d[0] == "group":
                assert d[3] in br.shared[(d[2], d[1])]     # exactly one member of the group


def test_broker_random_deliveries_vs_oracle():
    rng = random.Random(9)
    br = Broker(shared_strategy="hash_topic")
    o = R.Router()
    subs = {}
    fl = list(dict.fromkeys(rand_filter(rng) for _ in range(150)))
    sid = 0
    for f in fl:
        for _ in range(rng.randint(1, 3)):
            br.subscribe(f, sid)
            subs.setdefault(f, []).append(sid)
            sid += 1
        o.do_add_route(f, ("node", "local"))
        if rng.random() < 0.2:
            g = b"g%d" % rng.randint(0, 3)
            br.subscribe(b"$share/" + g + b"/" + f, sid)
            sid += 1
            o.do_add_route(f, ("group", g))
    # a filter crossing the 1024-subscriber shard threshold
    for k in range(1100):
        br.subscribe(fl[0], 100000 + k)
        subs[fl[0]].append(100000 + k)
    topics = [rand_topic(rng) for _ in range(300)]
    got = br.publish_batch(topics)
    for t, g in zip(topics, got):
        want = R.deliveries(o, subs, t)
        assert set(d[:3] for d in g) == want, t


def test_publish_result_nosub_and_sub_pub():
    """emqx_broker_SUITE t_nosub_pub / t_sub_pub (test/emqx_broker_SUITE.erl:121-138)
    as publish/1 results and the dropped counters (emqx_broker.erl:232-235, 283-295)."""
    br = Broker()
    assert br.metrics["messages.dropped"] == 0
    assert br.publish_result(b"topic") == []
    assert br.metrics["messages.dropped"] == 1 and br.metrics["messages.dropped.no_subscribers"] == 1
    br.subscribe(b"topic", 1)
    assert br.publish_result(b"topic") == [("local", b"topic", ("ok", 1))]
    assert br.metrics["messages.dropped"] == 1
    br.subscribe(b"+", 2)
    br.subscribe(b"#", 3)
    br.subscribe(b"#", 4)
    got = br.publish_result(b"topic")
    assert sorted(got) == [("local", b"#", ("ok", 2)), ("local", b"+", ("ok", 1)), ("local", b"topic", ("ok", 1))]
    # a subscriber whose process is gone is not counted; no one left -> dropped
    br.kill(1)
    got = br.publish_result(b"topic")
    assert ("local", b"topic", ("error", "no_subscribers")) in got
    assert br.metrics["messages.dropped"] == 2
    # system messages are never counted as dropped (emqx_broker.erl:311-316)
    assert br.publish_result(b"$SYS/brokers") == []
    assert br.publish_result(b"a/b", sys=True) == [("local", b"#", ("ok", 2))]
    assert br.publish_result(b"$SYS/x/y", sys=False) == []
    assert br.metrics["messages.dropped"] == 2


def test_publish_result_share_and_forward():
    br = Broker(shared_strategy="round_robin")
    br.subscribe(b"$share/g/s/+", 10)
    br.subscribe(b"$share/g/s/+", 11)
    br.subscribe(b"$share/h/s/+", 12)
    br.router.do_add_route(b"s/#", "n2")
    got = br.publish_result(b"s/1")
    assert sorted(got, key=repr) == sorted([("share", b"s/+", ("ok", 1)), ("share", b"s/+", ("ok", 1)),
                                            ("n2", b"s/#", "forward")], key=repr)
    assert br.metrics["messages.forward"] == 1
    br.kill(12)
    got = br.publish_result(b"s/1")
    assert ("share", b"s/+", ("error", "no_subscribers")) in got and ("share", b"s/+", ("ok", 1)) in got
    assert br.metrics["messages.dropped"] == 0   # a shared group's miss is not a drop


def test_shared_dispatch_redispatches_on_nack_and_down():
    """emqx_shared_sub:dispatch/4 through the broker mirror (Broker.dispatch_shared):
    a (filter, group) entry from the GPU fan-out, a member that nacks or whose
    process is down (not yet cleaned up) skipped for a QoS 1 delivery with
    shared_dispatch_ack_enabled, {ok, 1} while the group has members."""
    br = Broker(shared_strategy="round_robin")
    for m in (20, 21, 22):
        br.subscribe(b"$share/g/q/+", m)
    got = br.publish_result(b"q/1")
    assert got == [("share", b"q/+", ("ok", 1))]
    br.kill(21)
    for _ in range(6):
        res, m, failed = br.dispatch_shared(b"g", b"q/+", b"q/1", qos=1, ack_enabled=True,
                                            respond=lambda x: "nack" if x == 22 else "ack")
        assert res == ("ok", 1) and m == 20 and set(failed) <= {21, 22}
    res, m, failed = br.dispatch_shared(b"g", b"q/+", b"q/1", qos=0)
    assert res == ("ok", 1) and m in (20, 21, 22) and failed == []   # QoS 0: a plain send, even to 21
    assert br.dispatch_shared(b"none", b"q/+", b"q/1") == (("error", "no_subscribers"), None, [])


def test_publish_result_random_vs_oracle():
    rng = random.Random(17)
    br = Broker(shared_strategy="random")
    o = R.Router()
    subs, groups = {}, {}
    fl = list(dict.fromkeys(rand_filter(rng) for _ in range(120)))
    sid = 0
    for f in fl:
        if rng.random() < 0.8:
            for _ in range(rng.randint(1, 3)):
                br.subscribe(f, sid)
                subs.setdefault(f, []).append(sid)
                sid += 1
            o.do_add_route(f, "local")
        if rng.random() < 0.2:
            g = b"g%d" % rng.randint(0, 2)
            br.subscribe(b"$share/" + g + b"/" + f, sid)
            groups.setdefault(f, set()).add(g)
            sid += 1
            o.do_add_route(f, ("group", g))
    dead = set(rng.sample(range(sid), sid // 4))
    for x in dead:
        br.kill(x)
    topics = [rand_topic(rng) for _ in range(300)]
    got = br.publish_result_batch(topics)
    dropped = 0
    for t, g in zip(topics, got):
        want = []
        for x, d in o.match_routes(t):
            if d == "local":
                n = sum(1 for s in subs.get(x, []) if s not in dead)
                want.append(("local", x, ("ok", n) if n else ("error", "no_subscribers")))
                dropped += 0 if n or t.startswith(b"$SYS/") else 1
            else:
                live = [m for m in br.shared[(d[1], x)] if m not in dead]
                want.append(("share", x, ("ok", 1) if live else ("error", "no_subscribers")))
        dropped += 0 if want or t.startswith(b"$SYS/") else 1
        assert sorted(g, key=repr) == sorted(want, key=repr), t
    assert br.metrics["messages.dropped"] == dropped


def test_broker_subscriber_churn_vs_oracle():
    """the fan-out's subscriber table follows
    subscribe/3, unsubscribe/1 and subscriber_down/1 between publishes
    (emqx_broker.erl:144-197, 331-345; emqx_broker_helper.erl:133-163) by
    deltas (egm_subs_apply_delta + egm_subs_commit), not rebuilds: eight
    rounds of random churn — new and repeated subscriptions, unsubscribes,
    dead subscribers purged, $share members joining and leaving, a filter
    crossing the 1024-subscriber shard threshold — each followed by a batch
    of publishes whose delivery sets equal the oracle broker's
    (oracle/trie_ref.py deliveries over the reference's match_routes)."""
    rng = random.Random(23)
    br = Broker(shared_strategy="hash_topic")
    o = R.Router()
    subs, shared = {}, {}          # oracle: filter -> [sub]; (group, filter) -> [member]
    fl = list(dict.fromkeys(rand_filter(rng) for _ in range(200)))
    nxt = [0]

    def sub(f, s=None):
        s = nxt[0] if s is None else s
        nxt[0] = max(nxt[0], s + 1)
        br.subscribe(f, s)
        lst = subs.setdefault(f, [])
        if s not in lst:
            lst.append(s)
        o.do_add_route(f, ("node", "local"))
        return s

    def unsub(f, s):
        br.unsubscribe(f, s)
        if s in subs.get(f, []):
            subs[f].remove(s)
            if not subs[f]:
                del subs[f]
                o.do_delete_route(f, ("node", "local"))

    def share(g, f, s):
        br.subscribe(b"$share/" + g + b"/" + f, s)
        mem = shared.setdefault((g, f), [])
        if s not in mem:
            mem.append(s)
        o.do_add_route(f, ("group", g))

    def unshare(g, f, s):
        br.unsubscribe(b"$share/" + g + b"/" + f, s)
        mem = shared.get((g, f), [])
        if s in mem:
            mem.remove(s)
            if not mem:
                del shared[(g, f)]
                o.do_delete_route(f, ("group", g))

    for f in fl[:150]:
        for _ in range(rng.randint(1, 3)):
            sub(f)
    rounds_checked = 0
    stats = []
    for rnd in range(8):
        if rnd:
            for _ in range(rng.randint(20, 80)):
                op = rng.random()
                if op < 0.35:       # subscribe (a new or an existing filter; sometimes a repeat)
                    f = rng.choice(fl)
                    if rng.random() < 0.2 and subs.get(f):
                        sub(f, rng.choice(subs[f]))
                    else:
                        sub(f)
                elif op < 0.6 and subs:      # unsubscribe
                    f = rng.choice(sorted(subs))
                    unsub(f, rng.choice(subs[f]))
                elif op < 0.7 and subs:      # subscriber_down: every subscription of one subscriber
                    f = rng.choice(sorted(subs))
                    s = rng.choice(subs[f])
                    br.subscriber_down(s)
                    for g, ff in [k for k in shared if s in shared[k]]:
                        mem = shared[(g, ff)]
                        mem.remove(s)
                        if not mem:
                            del shared[(g, ff)]
                            o.do_delete_route(ff, ("group", g))
                    for ff in [k for k in subs if s in subs[k]]:
                        subs[ff].remove(s)
                        if not subs[ff]:
                            del subs[ff]
                            o.do_delete_route(ff, ("node", "local"))
                elif op < 0.85:              # a $share member joins
                    share(b"g%d" % rng.randint(0, 3), rng.choice(fl), 500000 + rng.randint(0, 40))
                elif shared:                 # ... or leaves
                    g, f = rng.choice(sorted(shared))
                    unshare(g, f, rng.choice(shared[(g, f)]))
            if rnd == 4:   # one filter past the 1024-subscriber shard threshold
                for k in range(1100):
                    sub(fl[0], 200000 + k)
        topics = [rand_topic(rng) for _ in range(200)] + [f.replace(b"+", b"x").replace(b"#", b"y") for f in fl[:100]]
        got = br.publish_batch(topics)
        if rnd:
            stats.append(br.router.m.subs_last_commit())
        for t, g in zip(topics, got):
            want = R.deliveries(o, subs, t)
            assert set(d[:3] for d in g) == want, (rnd, t)
            for d in g:
                if d[0] == "group":
                    assert d[3] in shared[(d[2], d[1])]   # exactly one live member of that group
        rounds_checked += 1
    assert rounds_checked == 8
    assert any(not s["rebuilt"] and s["patched"] > 0 for s in stats), stats   # deltas, not rebuilds


def test_subs_delta_contract_and_bounded_rebuilds():
    """(1) full builds forced by superseded entries are sized from
    the largest live filter id, so repeated rebuilds under churn do not grow
    the slot table; (2) an added filter id far past the table is refused
    (EGM_E_INVAL) before it can size a rebuild; (3) a (filter, subscriber)
    pair in both lists of one delta is refused and nothing is applied.  The
    deliveries stay exact throughout (emqx_broker:dispatch/2,
    apps/emqx/src/emqx_broker.erl:283-308)."""
    import numpy as np
    from emqx_amd import _lib as L
    from emqx_amd.engine import GpuMatcher, pack_strings
    nf = 1000
    gm = GpuMatcher(0)
    try:
        fb, fo = pack_strings([b"a/%d" % i for i in range(nf)])
        gm.build(fb, fo)
        lists = {f: [f * 10 + k for k in range(1 + f % 3)] for f in range(nf)}
        row = np.zeros(nf + 1, np.uint64)
        row[1:] = np.cumsum([len(lists[f]) for f in range(nf)])
        gm.subs_build(row, np.concatenate([np.array(lists[f], np.uint32) for f in range(nf)]))
        slots0 = gm.subs_slots()
        assert slots0 >= nf
        tb, to = pack_strings([b"a/5", b"a/7", b"a/999", b"b/1"])

        def check():
            res = gm.match(tb, to, L.EGM_MODE_ROUTES)
            drow, dfid, dsub = gm.fanout(res)
            for i, f in enumerate((5, 7, 999, None)):
                got = sorted(dsub[int(drow[i]):int(drow[i + 1])].tolist())
                assert got == (sorted(lists[f]) if f is not None else []), (i, f)

        # a big row re-committed again and again: superseded entries force full builds
        big = [(5, 100000 + k) for k in range(70000)]
        gm.subs_apply_delta(add=big)
        lists[5] += [s for _, s in big]
        gm.subs_commit()
        rebuilt = 0
        for k in range(24):
            gm.subs_apply_delta(add=[(5, 900000 + k)])
            lists[5].append(900000 + k)
            gm.subs_commit()
            rebuilt += gm.subs_last_commit()["rebuilt"]
            assert gm.subs_slots() <= slots0, (k, gm.subs_slots(), slots0)
        assert rebuilt >= 5, rebuilt
        check()
        # a garbage filter id: refused, the table unchanged
        with pytest.raises(L.EgmError) as ei:
            gm.subs_apply_delta(add=[(7, 1), (0xFFFFFF00, 2)])
        assert ei.value.code == L.EGM_E_INVAL
        # the same pair added and removed in one delta: refused, nothing applied
        with pytest.raises(L.EgmError) as ei:
            gm.subs_apply_delta(add=[(7, 4242), (999, 1)], delete=[(7, 4242)])
        assert ei.value.code == L.EGM_E_INVAL
        gm.subs_commit()
        check()
        # a legitimate new filter id just past the slots: a full build that grows the table
        gm.subs_apply_delta(add=[(slots0 + 10, 77)], delete=[(7, lists[7][0])])
        lists[7].pop(0)
        gm.subs_commit()
        assert gm.subs_last_commit()["rebuilt"] and gm.subs_slots() > slots0 + 10
        check()
    finally:
        gm.close()
