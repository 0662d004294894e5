"""Retained reverse match on the GPU against the
reference's own retainer suite (KATs) and the oracle restatement of
emqx_retainer_mnesia (oracle/retainer_ref.py)."""
import random

import numpy as np
import pytest

from emqx_amd import _lib as L
from emqx_amd import synth
from emqx_amd.retainer import RetainedStore
from oracle import retainer_ref as RR
from tests.test_oracle_retainer import load_kats, run_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def store():
    s = RetainedStore(0)
    yield s
    s.close()


@pytest.mark.parametrize("case", load_kats(), ids=lambda c: c["name"])
def test_retainer_suite_kats(store, case):
    def fresh():
        store.clean()
        return store
    for flt, got, exp in run_case(case, fresh):
        assert got == exp, (case["name"], flt)


WORDS = [b"a", b"b", b"", b"$SYS", b"c", b"$x", b"dd", b"w" * 17, b"w" * 18]


def _topic(rng):
    return b"/".join(rng.choice(WORDS) for _ in range(rng.randint(1, 6)))


def _filter(rng, topics):
    if rng.random() < 0.3:   # from a stored topic, some words replaced
        ws = rng.choice(topics).split(b"/")
        ws = [b"+" if rng.random() < 0.3 else w for w in ws]
        if rng.random() < 0.4:
            ws = ws[: rng.randint(1, len(ws))] + [b"#"]
        return b"/".join(ws)
    d = rng.randint(1, 5)
    ws = [b"+" if rng.random() < 0.3 else rng.choice(WORDS + [b"zz"]) for _ in range(d)]
    if rng.random() < 0.4:
        ws[-1] = b"#"
    return b"/".join(ws)


@pytest.mark.parametrize("seed", range(3))
def test_random_vs_oracle(store, seed):
    rng = random.Random(seed)
    store.clean()
    ref = RR.RetainedTable()
    topics = list(dict.fromkeys(_topic(rng) for _ in range(3000)))
    for t in topics:
        e = rng.choice([0, 0, 0, 500, 1000, 1500])
        store.store_retained(t, t, e)
        ref.store_retained(t, t, e)
    # churn: overwrite some, delete some (plain and wildcard)
    for t in rng.sample(topics, 200):
        store.store_retained(t, t, 0)
        ref.store_retained(t, t, 0)
    for t in rng.sample(topics, 200):
        store.delete_message(t)
        ref.delete_message(t)
    for f in (b"a/+/#", b"+/b"):
        store.delete_message(f)
        ref.delete_message(f)
    assert store.size() == ref.size()
    filters = [_filter(rng, topics) for _ in range(600)] + [b"#", b"+", b"+/+", b"", b"/", b"$SYS/#", b"a"]
    for now in (0, 1000, 1200):
        got = store.dispatch_batch(filters, now)
        for f, g in zip(filters, got):
            assert sorted(g) == sorted(ref.dispatch(f, now)), (f, now)
        ids = store.match_ids(filters, now, L.EGM_RMODE_MATCH)
        for f, row in zip(filters, ids):
            assert len(set(row.tolist())) == len(row)
            assert sorted(store._msgs[int(i)][1] for i in row) == sorted(ref.match_messages(f, now)), (f, now)


def test_large_store_properties(store):
    """200K synthetic topics (C0-shaped): '#' returns every alive record, a
    filter set partitioned by its first word covers the store exactly once,
    and an exact filter per topic returns that topic alone."""
    f, t = synth.config("c0", n_topics=200_000)
    tl = list(dict.fromkeys(t.to_list()))
    tl = [x for x in tl if b"+" not in x.split(b"/") and b"#" not in x.split(b"/")]
    store.clean()
    rng = random.Random(3)
    exp = {}
    for x in tl:
        e = 0 if rng.random() < 0.8 else rng.choice([100, 300])
        store.store_retained(x, x, e)
        exp[x] = e
    now = 200
    alive = sorted(x for x in tl if exp[x] == 0 or exp[x] > now)
    r = store.match_ids([b"#"], now, L.EGM_RMODE_MATCH)[0]
    assert len(r) == len(alive) and len(set(r.tolist())) == len(r)
    assert sorted(store._msgs[int(i)][0] for i in r) == alive
    firsts = sorted(set(x.split(b"/")[0] for x in tl))
    rows = store.match_ids([w + b"/#" for w in firsts], now, L.EGM_RMODE_MATCH)
    cover = np.concatenate(rows)
    assert len(cover) == len(alive) and len(np.unique(cover)) == len(cover)
    sample = rng.sample(tl, 5000)
    rows = store.match_ids(sample, 0, L.EGM_RMODE_DISPATCH)
    for x, row in zip(sample, rows):
        assert [store._msgs[int(i)][0] for i in row] == [x]
