"""Pin the CPU oracle (oracle/trie_ref.py) to the reference's own known answers.

Every vector here is data from the reference's test suites (see the ``src`` of
each entry in tests/golden/kat_reference.json).  Parity of the GPU path is only
as good as this oracle, so it must pass every case in both trie modes.
"""
import pytest

from oracle import trie_ref as R
from tests.kat import b, dec_word, load

K = load()


@pytest.mark.parametrize("compact", [True, False], ids=["compact", "not_compact"])
@pytest.mark.parametrize("case", K["trie_cases"], ids=lambda c: c["name"])
def test_trie_suite(case, compact):
    t = R.Trie(compact)
    for op in case["ops"]:
        if op[0] == "insert":
            t.insert(b(op[1]))
        elif op[0] == "delete":
            t.delete(b(op[1]))
        elif op[0] == "assert_empty":
            assert t.empty() is op[1]
        elif op[0] == "assert_lookup_topic":
            assert t.lookup_topic(b(op[1])) == [b(x) for x in op[2]]
    for topic, expected in case["queries"]:
        got = t.match(b(topic))
        assert len(got) == len(set(got)), "duplicates"
        assert sorted(got) == sorted(b(x) for x in expected)
        # closed form over the live filter set agrees too
        live = [k[0] for k in t.tab if k[1] == 1]
        assert sorted(R.trie_semantics(b(topic), live)) == sorted(got)


@pytest.mark.parametrize("compact", [True, False], ids=["compact", "no_compact"])
def test_make_keys(compact):
    t = R.Trie(compact)
    for topic, tkey, pkeys in K["make_keys"]["compact" if compact else "no_compact"]:
        assert t.make_keys(b(topic)) == ((b(tkey), 1), [(b(p), 0) for p in pkeys])


@pytest.mark.parametrize("compact", [True, False], ids=["compact", "no_compact"])
def test_make_prefixes(compact):
    t = R.Trie(compact)
    for topic, pre in K["make_prefixes"]["compact" if compact else "no_compact"]:
        assert t.make_prefixes(R.words(b(topic))) == [b(p) for p in pre]


def test_do_compact():
    for topic, segs in K["do_compact"]["cases"]:
        assert R.do_compact(R.words(b(topic))) == [b(s) for s in segs]


def test_topic_match():
    for name, flt, exp in K["topic_match"]["cases"]:
        assert R.match(b(name), b(flt)) is exp, (name, flt)


def test_wildcard_words_tokens_levels_join():
    for t, exp in K["wildcard"]["cases"]:
        assert R.wildcard(b(t)) is exp
    for t, ws in K["words"]["cases"]:
        got = R.words(b(t))
        want = [dec_word(w) for w in ws]
        assert len(got) == len(want)
        for g, w in zip(got, want):
            assert (g is w) if isinstance(w, R._Atom) else (g == w)
    for t, toks in K["tokens"]["cases"]:
        assert R.tokens(b(t)) == [b(x) for x in toks]
    for t, n in K["levels"]["cases"]:
        assert len(R.tokens(b(t))) == n
    for ws, exp in K["join"]["cases"]:
        if isinstance(ws, str):
            ws = R.words(b(ws[len("words:"):]))
        else:
            ws = [dec_word(w) for w in ws]
        assert R.join(ws) == b(exp)


def test_validate_parse():
    for kind, t in K["validate"]["ok"]:
        assert R.validate(kind, b(t))
    for kind, t, reason in K["validate"]["error"]:
        with pytest.raises(ValueError) as ei:
            R.validate(kind, b(t))
        assert ei.value.args[0] == reason
    for t, flt, share in K["parse"]["ok"]:
        got_f, opts = R.parse(b(t))
        assert got_f == b(flt)
        assert opts.get("share") == (b(share) if share else None)
    for t, share in K["parse"]["error"]:
        with pytest.raises(ValueError):
            R.parse(b(t), {"share": b(share)} if share else None)


@pytest.mark.parametrize("compact", [True, False])
def test_router_match_routes(compact):
    case = K["router_match_routes"]
    r = R.Router(compact)
    for t, d in case["routes"]:
        r.do_add_route(b(t), d)
    got = sorted((t, d) for t, d in r.match_routes(b(case["query"])))
    assert got == sorted((b(t), d) for t, d in case["expected"])
    for t, d in case["routes"]:
        r.do_delete_route(b(t), d)
    assert r.match_routes(b(case["query"])) == []
    assert r.trie.empty()


def test_broker_delivery():
    for case in K["broker_delivery"]["cases"]:
        r = R.Router()
        subs = {}
        for flt, sub, group in case["subs"]:
            if group is None:
                r.do_add_route(b(flt), ("node", "local"))
                subs.setdefault(b(flt), []).append(sub)
            else:
                r.do_add_route(b(flt), ("group", b(group)))
        got = R.deliveries(r, subs, b(case["publish"]))
        want = set()
        for kind, flt, x in case["expected"]:
            want.add((kind, b(flt), b(x) if isinstance(x, str) else x))
        assert got == want, case["name"]
