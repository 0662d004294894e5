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
