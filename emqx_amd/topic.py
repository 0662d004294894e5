"""Host mirror of ``emqx_topic`` (apps/emqx/src/emqx_topic.erl).

Topic algebra used around the lookup path: splitting, wildcard test, the
single-filter match (used e.g. by authz / rewrite, not by publish routing),
validation and ``$share``/``$queue`` parsing.  Words are ``bytes`` except the
three atoms, which are the module constants ``EMPTY`` (''), ``PLUS`` ('+')
and ``HASH`` ('#').  Errors raise :class:`TopicError` with the reference's
error term as its reason.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple, Union

MAX_TOPIC_LEN = 65535          # emqx_topic.erl:45


class _Atom(str):
    """A word atom ('' '+' '#'); distinct from the equal-looking binary."""

    def __repr__(self) -> str:
        return f"'{str.__str__(self)}'"


EMPTY = _Atom("")
PLUS = _Atom("+")
HASH = _Atom("#")

Word = Union[bytes, _Atom]


class TopicError(ValueError):
    def __init__(self, reason):
        super().__init__(reason)
        self.reason = reason


def _is_atom(w) -> bool:
    return isinstance(w, _Atom)


def tokens(topic: bytes) -> List[bytes]:
    """``tokens/1`` (emqx_topic.erl:153-154): split on every '/'."""
    return topic.split(b"/")


def _word(b: bytes) -> Word:
    if b == b"":
        return EMPTY
    if b == b"+":
        return PLUS
    if b == b"#":
        return HASH
    return b


def words(topic: bytes) -> List[Word]:
    """``words/1`` (emqx_topic.erl:158-164)."""
    return [_word(t) for t in tokens(topic)]


def levels(topic: bytes) -> int:
    """``levels/1`` (emqx_topic.erl:147-148)."""
    return len(tokens(topic))


def wildcard(t: Union[bytes, Sequence[Word]]) -> bool:
    """``wildcard/1`` (emqx_topic.erl:53-62)."""
    ws = words(t) if isinstance(t, (bytes, bytearray)) else t
    return any(w is PLUS or w is HASH for w in ws)


def _bin(w) -> bytes:
    if w is EMPTY:
        return b""
    if w is PLUS:
        return b"+"
    if w is HASH:
        return b"#"
    if isinstance(w, str):
        return w.encode()
    return bytes(w)


def join(ws: Sequence) -> bytes:
    """``join/1`` (emqx_topic.erl:184-195)."""
    if not ws:
        return b""
    return b"/".join(_bin(w) for w in ws)


def _eq(a, b) -> bool:
    if _is_atom(a) or _is_atom(b):
        return a is b
    return a == b


def match(name, flt) -> bool:
    """``match/2`` (emqx_topic.erl:68-87): one topic name against one filter."""
    if isinstance(name, (bytes, bytearray)) and isinstance(flt, (bytes, bytearray)):
        if name[:1] == b"$" and flt[:1] in (b"+", b"#"):
            return False
        n, f = words(name), words(flt)
    else:
        n, f = list(name), list(flt)
    i = 0
    while True:
        if i == len(n) and i == len(f):
            return True
        if i < len(n) and i < len(f) and (_eq(n[i], f[i]) or f[i] is PLUS):
            i += 1
            continue
        return len(f) - i == 1 and f[i] is HASH


def validate(topic, kind: str = "filter") -> bool:
    """``validate/1,2`` (emqx_topic.erl:90-127)."""
    if isinstance(topic, tuple):
        kind, topic = topic
    if kind not in ("name", "filter"):
        raise TopicError("function_clause")
    if topic == b"":
        raise TopicError("empty_topic")
    if len(topic) > MAX_TOPIC_LEN:
        raise TopicError("topic_too_long")
    ws = words(topic)
    for i, w in enumerate(ws):
        if w is HASH:
            if i != len(ws) - 1:
                raise TopicError("topic_invalid_#")
            break
        if _is_atom(w):
            continue
        for ch in w.decode("utf-8"):
            if ch in ("#", "+", "\x00"):
                raise TopicError("topic_invalid_char")
    if kind == "name" and wildcard(ws):
        raise TopicError("topic_name_error")
    return True


def prepend(parent, w) -> bytes:
    """``prepend/2`` (emqx_topic.erl:131-138)."""
    if parent is None or parent == b"" or parent == "":
        return _bin(w)
    p = _bin(parent)
    return p + _bin(w) if p.endswith(b"/") else p + b"/" + _bin(w)


def feed_var(var: bytes, val: bytes, topic: bytes) -> bytes:
    """``feed_var/3`` (emqx_topic.erl:173-181)."""
    return join([val if (not _is_atom(w) and w == var) else w for w in words(topic)])


def systop(name, node: str = "emqx@127.0.0.1") -> bytes:
    """``systop/1`` (emqx_topic.erl:167-171)."""
    return b"$SYS/brokers/" + node.encode() + b"/" + _bin(name)


def parse(topic_filter, options: Optional[dict] = None) -> Tuple[bytes, dict]:
    """``parse/1,2`` (emqx_topic.erl:197-220): ``$queue/`` and ``$share/G/``."""
    if isinstance(topic_filter, tuple):
        topic_filter, options = topic_filter
    opts = dict(options or {})
    if topic_filter.startswith(b"$queue/"):
        if "share" in opts:
            raise TopicError(("invalid_topic_filter", topic_filter))
        opts["share"] = b"$queue"
        return parse(topic_filter[len(b"$queue/"):], opts)
    if topic_filter.startswith(b"$share/"):
        if "share" in opts:
            raise TopicError(("invalid_topic_filter", topic_filter))
        rest = topic_filter[len(b"$share/"):]
        if b"/" not in rest:
            raise TopicError(("invalid_topic_filter", topic_filter))
        share, flt = rest.split(b"/", 1)
        if b"+" in share or b"#" in share:
            raise TopicError(("invalid_topic_filter", topic_filter))
        opts["share"] = share
        return parse(flt, opts)
    return topic_filter, opts
