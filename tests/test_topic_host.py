"""emqx_amd.topic (host mirror of emqx_topic) against the reference's KATs."""
import pytest

from emqx_amd import topic as T
from tests.kat import b, load

K = load()


def _w(s):
    return {"''": T.EMPTY, "'+'": T.PLUS, "'#'": T.HASH}.get(s, s.encode())


def test_match_cases():
    for name, flt, exp in K["topic_match"]["cases"]:
        assert T.match(b(name), b(flt)) is exp, (name, flt)


def test_words_tokens_levels_wildcard_join():
    for t, exp in K["wildcard"]["cases"]:
        assert T.wildcard(b(t)) is exp
    for t, ws in K["words"]["cases"]:
        got = T.words(b(t))
        want = [_w(x) for x in ws]
        assert len(got) == len(want)
        for g, w in zip(got, want):
            assert (g is w) if isinstance(w, T._Atom) else (g == w and not isinstance(g, T._Atom))
    for t, toks in K["tokens"]["cases"]:
        assert T.tokens(b(t)) == [b(x) for x in toks]
    for t, n in K["levels"]["cases"]:
        assert T.levels(b(t)) == n
    for ws, exp in K["join"]["cases"]:
        ws = T.words(b(ws[len("words:"):])) if isinstance(ws, str) else [_w(x) for x in ws]
        assert T.join(ws) == b(exp)


def test_validate_and_parse():
    for kind, t in K["validate"]["ok"]:
        assert T.validate(b(t), kind)
    for kind, t, reason in K["validate"]["error"]:
        with pytest.raises(T.TopicError) as ei:
            T.validate((kind, b(t)))
        assert ei.value.reason == reason
    with pytest.raises(T.TopicError) as ei:
        T.validate(("name", b"/".join([b"x"] * 40000)))
    assert ei.value.reason == "topic_too_long"
    for t, flt, share in K["parse"]["ok"]:
        f, o = T.parse(b(t))
        assert f == b(flt) and o.get("share") == (b(share) if share else None)
    for t, share in K["parse"]["error"]:
        with pytest.raises(T.TopicError):
            T.parse(b(t), {"share": b(share)} if share else None)


def test_prepend_feed_var_systop():
    # emqx_topic_SUITE.erl:145-152 and :177-183
    assert T.prepend(None, b"ab") == b"ab"
    assert T.prepend(b"", b"a/b") == b"a/b"
    assert T.prepend(b"x/", b"a/b") == b"x/a/b"
    assert T.prepend(b"x/y", b"a/b") == b"x/y/a/b"
    assert T.prepend(T.PLUS, b"a/b") == b"+/a/b"
    assert T.feed_var(b"$c", b"clientId", b"$queue/client/$c") == b"$queue/client/clientId"
    assert T.feed_var(b"%u", b"test", b"username/%u/client/x") == b"username/test/client/x"
    assert T.systop(b"xyz", "n@h") == b"$SYS/brokers/n@h/xyz"
