"""Cross-check the two trie walks of the oracle against the brute-force
``emqx_topic:match/2`` restatement (SURVEY.md §0 "Semantics finding").

Random filter/topic sets over a tiny alphabet so collisions, empty words ('')
and '$' words are frequent.
"""
import random

import pytest

from oracle import trie_ref as R

ALPHA = [b"a", b"b", b"", b"$x", b"c", b"$", b"ab"]


def rand_filter(rng):
    d = rng.randint(1, 5)
    ws = []
    for i in range(d):
        p = rng.random()
        if p < 0.25:
            ws.append(b"+")
        elif p < 0.33 and i == d - 1:
            ws.append(b"#")
        else:
            ws.append(rng.choice(ALPHA))
    return b"/".join(ws)


def rand_topic(rng):
    d = rng.randint(1, 6)
    ws = [rng.choice(ALPHA) for _ in range(d)]
    if rng.random() < 0.03:
        ws[rng.randrange(d)] = rng.choice([b"+", b"#"])
    return b"/".join(ws)


@pytest.mark.parametrize("seed", range(6))
def test_walks_equal_brute_force(seed):
    rng = random.Random(seed)
    filters = list({rand_filter(rng) for _ in range(120)})
    # a handful of non-wildcard filters straight into the trie (t_insert style)
    filters = list(dict.fromkeys(filters + [b"$x", b"a/b", b"$"]))
    tc, tn = R.Trie(True), R.Trie(False)
    for f in filters:
        tc.insert(f)
        tn.insert(f)
    for _ in range(400):
        t = rand_topic(rng)
        want = sorted(R.trie_semantics(t, filters))
        gc = tc.match(t)
        gn = tn.match(t)
        assert len(gc) == len(set(gc)) and len(gn) == len(set(gn))
        assert sorted(gc) == want, t
        assert sorted(gn) == want, t


@pytest.mark.parametrize("seed", range(3))
def test_delete_restores(seed):
    rng = random.Random(100 + seed)
    filters = list({rand_filter(rng) for _ in range(80)})
    for compact in (True, False):
        t = R.Trie(compact)
        for f in filters:
            t.insert(f)
            t.insert(f)  # idempotent
        keep = filters[::2]
        for f in filters[1::2]:
            t.delete(f)
            t.delete(f)
        for _ in range(200):
            tp = rand_topic(rng)
            assert sorted(t.match(tp)) == sorted(R.trie_semantics(tp, keep))
        for f in keep:
            t.delete(f)
        assert t.empty()


def test_router_semantics():
    rng = random.Random(7)
    r = R.Router()
    fl = list({rand_filter(rng) for _ in range(60)} | {b"a/b", b"a", b"$x/a"})
    for f in fl:
        r.do_add_route(f, ("node", "local"))
    for _ in range(300):
        t = rand_topic(rng)
        got = sorted(f for f, _ in r.match_routes(t))
        assert got == sorted(R.routes_semantics(t, fl)), t
