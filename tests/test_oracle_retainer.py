"""The retained reverse-match oracle against the reference's own suite (KATs)
and an independent word-by-word matcher."""
import json
import os
import random

import pytest

from oracle import retainer_ref as RR
from oracle import trie_ref as R

HERE = os.path.dirname(os.path.abspath(__file__))


def load_kats():
    with open(os.path.join(HERE, "golden", "kat_retainer.json")) as f:
        return json.load(f)["cases"]


def run_case(case, store_factory):
    """Drive a KAT case against a store with the oracle's interface; returns
    (query, got, expected) triples."""
    st = store_factory()
    out = []
    for op in case["ops"]:
        if op[0] == "put":
            st.store_retained(op[1].encode(), op[1].encode(), op[2])
        elif op[0] == "delete":
            st.delete_message(op[1].encode())
        elif op[0] == "clean":
            st.clean()
        elif op[0] == "query":
            _, flt, now, mode, exp = op
            got = st.dispatch(flt.encode(), now) if mode == "dispatch" else st.match_messages(flt.encode(), now)
            out.append((flt, sorted(got), sorted(x.encode() for x in exp)))
    return out


@pytest.mark.parametrize("case", load_kats(), ids=lambda c: c["name"])
def test_retainer_kats(case):
    for flt, got, exp in run_case(case, RR.RetainedTable):
        assert got == exp, (case["name"], flt)


def condition_examples():
    # condition/1 on the shapes the module handles (:215-220)
    assert RR.condition(R.words(b"a/+/c")) == [b"a", RR.ANY, b"c"]
    t = RR.condition(R.words(b"a/+/#"))
    assert isinstance(t, RR.Tail) and t.head == [b"a", RR.ANY]
    assert isinstance(RR.condition(R.words(b"#")), RR.Tail) and RR.condition(R.words(b"#")).head == []


def test_condition_shapes():
    condition_examples()


def _independent(topic: bytes, flt: bytes) -> bool:
    """Word-by-word: '+' any word, a last '#' any (possibly empty) rest, no '$' rule."""
    tw, fw = topic.split(b"/"), flt.split(b"/")
    for i, f in enumerate(fw):
        if f == b"#" and i == len(fw) - 1:
            return True
        if i >= len(tw):
            return False
        if f != b"+" and f != tw[i]:
            return False
    return len(tw) == len(fw)


WORDS = [b"a", b"b", b"", b"$SYS", b"c", b"$x", b"dd"]


def _topic(rng):
    return b"/".join(rng.choice(WORDS) for _ in range(rng.randint(1, 5)))


def _filter(rng):
    d = rng.randint(1, 5)
    ws = [b"+" if rng.random() < 0.3 else rng.choice(WORDS) for _ in range(d)]
    if rng.random() < 0.4:
        ws[-1] = b"#"
    return b"/".join(ws)


@pytest.mark.parametrize("seed", range(3))
def test_match_messages_vs_independent(seed):
    rng = random.Random(seed)
    st = RR.RetainedTable()
    topics = list(dict.fromkeys(_topic(rng) for _ in range(300)))
    exp = {}
    for t in topics:
        e = rng.choice([0, 0, 500, 1500])
        st.store_retained(t, t, e)
        exp[t] = e
    for _ in range(300):
        f = _filter(rng)
        now = rng.choice([0, 1000, 2000])
        got = sorted(st.match_messages(f, now))
        want = sorted(t for t in topics if _independent(t, f) and (exp[t] == 0 or exp[t] > now))
        assert got == want, f
        if not R.wildcard(f):
            want_r = [f] if f in exp and (exp[f] == 0 or exp[f] >= now) else []
            assert st.dispatch(f, now) == want_r
    # wildcard delete removes exactly what the pattern matches (expired or not)
    f = b"a/#"
    st.delete_message(f)
    assert not any(_independent(t, f) for t in (b"/".join(k_ if isinstance(k_, bytes) else b"" for k_ in k)
                                                 for k in st.recs))


@pytest.mark.parametrize("seed", range(2))
def test_cpp_scan_vs_python_oracle(seed):
    """oracle/retainer_scan.cpp (the CPU baseline) agrees with the restatement."""
    import numpy as np

    from emqx_amd.engine import pack_strings
    from oracle.cpp import OracleRetained
    rng = random.Random(10 + seed)
    st = RR.RetainedTable()
    cs = OracleRetained()
    topics = list(dict.fromkeys(_topic(rng) for _ in range(400)))
    exp = [rng.choice([0, 0, 500, 1500]) for _ in topics]
    for t, e in zip(topics, exp):
        st.store_retained(t, t, e)
    blob, off = pack_strings(topics)
    cs.put(blob, off, np.arange(len(topics), dtype=np.uint32), np.array(exp, dtype=np.uint64))
    filters = [_filter(rng) for _ in range(300)] + [t for t in topics[:50]]
    fb, fo = pack_strings(filters)
    for now in (0, 500, 1000):
        for mode in (0, 1):
            tot, counts = cs.match_counts(fb, fo, now, mode, threads=2)
            want = [len(st.dispatch(f, now) if mode else st.match_messages(f, now)) for f in filters]
            assert counts.tolist() == want and tot == sum(want)
