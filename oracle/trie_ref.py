"""CPU oracle — literal restatement of the reference's route-lookup algorithm.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (``emqx_amd``, the C-ABI
library, the HIP kernels) may import, call or link this module.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
use it, and only as the checker.

Parity pinning: the reference is Erlang/OTP (EMQ X 5.0-alpha.3).  No ERTS exists
in this image (``erl``/``erlc``/``erl_nif.h`` absent — SURVEY.md §8c), so the
reference itself cannot be run.  This restatement is pinned instead by every
known-answer case the reference's own tests hold for this path
(``tests/golden/kat_*.json``, checked by ``tests/test_oracle_kat.py``) and by
cross-checking its two trie walks against the independent brute-force
``emqx_topic:match/2`` restatement on random inputs.

Erlang terms are mapped as follows:

* topic / filter binaries  -> ``bytes``
* the word atoms '' '+' '#' -> the singletons ``EMPTY``, ``PLUS``, ``HASH``
  (``emqx_topic.erl:161-164``); every other word stays ``bytes``
* the trie's virtual root ``empty`` -> ``ROOT`` (``emqx_trie.erl:154-158,201``)
* the mnesia ``emqx_trie`` ordered_set -> ``dict[(key_bytes, 0|1)] -> count``
  (``emqx_trie.erl:45-51``)
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple, Union


class _Atom:
    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = name

    def __repr__(self) -> str:  # pragma: no cover - debugging aid
        return f"'{self.name}'"


EMPTY = _Atom("")      # ''
PLUS = _Atom("+")      # '+'
HASH = _Atom("#")      # '#'
ROOT = _Atom("empty")  # emqx_trie's virtual root prefix

Word = Union[bytes, _Atom]


# ---------------------------------------------------------------------------
# emqx_topic  (apps/emqx/src/emqx_topic.erl)
# ---------------------------------------------------------------------------

def tokens(topic: bytes) -> List[bytes]:
    """``tokens/1`` — ``binary:split(Topic, <<"/">>, [global])`` (emqx_topic.erl:153-154).

    ``binary:split`` with ``global`` on ``<<>>`` yields ``[<<>>]``; every '/'
    produces a split, so N separators give N+1 tokens.
    """
    return topic.split(b"/")


def word(w: bytes) -> Word:
    """``word/1`` (emqx_topic.erl:161-164)."""
    if w == b"":
        return EMPTY
    if w == b"+":
        return PLUS
    if w == b"#":
        return HASH
    return w


def words(topic: bytes) -> List[Word]:
    """``words/1`` (emqx_topic.erl:158-159)."""
    return [word(t) for t in tokens(topic)]


def wildcard(t: Union[bytes, Sequence[Word]]) -> bool:
    """``wildcard/1`` (emqx_topic.erl:53-62): true iff a *word* is '+' or '#'."""
    ws = words(t) if isinstance(t, bytes) else t
    return any(w is PLUS or w is HASH for w in ws)


def bin_(w) -> bytes:
    """``bin/1`` (emqx_topic.erl:140-144)."""
    if w is EMPTY:
        return b""
    if w is PLUS:
        return b"+"
    if w is HASH:
        return b"#"
    if isinstance(w, (bytes, bytearray)):
        return bytes(w)
    raise TypeError(w)


def join(ws: Sequence) -> bytes:
    """``join/1`` (emqx_topic.erl:184-195)."""
    if len(ws) == 0:
        return b""
    if len(ws) == 1:
        return bin_(ws[0])
    return b"/".join(bin_(w) for w in ws)


def match(name, flt) -> bool:
    """``match/2`` (emqx_topic.erl:68-87) — the executable spec the trie must equal.

    The '$' rule is character level: a name starting with '$' never matches a
    filter whose first *character* is '+' or '#'.
    """
    if isinstance(name, bytes) and isinstance(flt, bytes):
        if name[:1] == b"$" and flt[:1] in (b"+", b"#"):
            return False
        return _match_words(words(name), words(flt))
    return _match_words(list(name), list(flt))


def _word_eq(a: Word, b: Word) -> bool:
    if isinstance(a, _Atom) or isinstance(b, _Atom):
        return a is b
    return a == b


def _match_words(n: List[Word], f: List[Word]) -> bool:
    i = 0
    while True:
        if i == len(n) and i == len(f):          # match([], []) -> true
            return True
        if i < len(n) and i < len(f) and _word_eq(n[i], f[i]):
            i += 1                                # match([H|T1], [H|T2])
            continue
        if i < len(n) and i < len(f) and f[i] is PLUS:
            i += 1                                # match([_H|T1], ['+'|T2])
            continue
        if len(f) - i == 1 and f[i] is HASH:      # match(_, ['#']) -> true
            return True
        return False                              # the three false clauses


def validate(kind: str, topic: bytes) -> bool:
    """``validate/2`` (emqx_topic.erl:96-127). Raises ValueError(reason)."""
    if topic == b"":
        raise ValueError("empty_topic")
    if len(topic) > 65535:
        raise ValueError("topic_too_long")
    ws = words(topic)
    _validate2(ws)
    if kind == "name" and wildcard(ws):
        raise ValueError("topic_name_error")
    return True


def _validate2(ws: List[Word]) -> None:
    for i, w in enumerate(ws):
        if w is HASH:
            if i != len(ws) - 1:
                raise ValueError("topic_invalid_#")
            return
        if w is EMPTY or w is PLUS:
            continue
        s = w.decode("utf-8")  # validate3 walks utf8 code points
        for ch in s:
            if ch in ("#", "+", "\x00"):
                raise ValueError("topic_invalid_char")


def parse(topic_filter: bytes, options: Optional[dict] = None) -> Tuple[bytes, dict]:
    """``parse/2`` (emqx_topic.erl:203-220): strips ``$queue/`` and ``$share/G/``."""
    options = dict(options or {})
    if topic_filter.startswith(b"$queue/"):
        if "share" in options:
            raise ValueError(("invalid_topic_filter", topic_filter))
        options["share"] = b"$queue"
        return parse(topic_filter[len(b"$queue/"):], options)
    if topic_filter.startswith(b"$share/"):
        if "share" in options:
            raise ValueError(("invalid_topic_filter", topic_filter))
        rest = topic_filter[len(b"$share/"):]
        if b"/" not in rest:
            raise ValueError(("invalid_topic_filter", topic_filter))
        share, flt = rest.split(b"/", 1)
        if b"+" in share or b"#" in share:
            raise ValueError(("invalid_topic_filter", topic_filter))
        options["share"] = share
        return parse(flt, options)
    return topic_filter, options


# ---------------------------------------------------------------------------
# emqx_trie  (apps/emqx/src/emqx_trie.erl)
# ---------------------------------------------------------------------------

def trie_join(prefix, w) -> bytes:
    """``join/2`` (emqx_trie.erl:154-158)."""
    if prefix is ROOT:
        if w is PLUS:
            return b"+"
        if w is HASH:
            return b"#"
        if w is EMPTY:
            return b""
        return w
    return join([prefix, w])


def do_compact(ws: Sequence[Word]) -> List[bytes]:
    """``do_compact/1,3`` (emqx_trie.erl:144-152)."""
    seg = ROOT
    acc: List[bytes] = []
    for w in ws:
        if w is PLUS or w is HASH:
            acc.append(trie_join(seg, w))
            seg = ROOT
        else:
            seg = trie_join(seg, w)
    if seg is not ROOT:
        acc.append(seg)
    return acc


class Trie:
    """The ``emqx_trie`` table plus its insert/delete/match (emqx_trie.erl:82-273)."""

    def __init__(self, compact: bool = True):
        self.compact = compact          # broker.perf.trie_compaction (emqx_trie.erl:272-276)
        self.tab: Dict[Tuple[bytes, int], int] = {}
        self.lookups = 0                # ETS probes issued (for instrumentation only)

    # -- key construction ---------------------------------------------------
    def _compact(self, ws):
        return do_compact(ws) if self.compact else list(ws)   # :132-136

    def make_prefixes(self, ws) -> List[bytes]:
        """``make_prefixes/1,3`` (emqx_trie.erl:160-169): longest prefix first."""
        segs = self._compact(ws)
        if len(segs) == 0:
            raise ValueError("function_clause")   # make_prefixes([], _, _) has no clause
        out = [join(segs[:k]) for k in range(1, len(segs))]
        out.reverse()
        return out

    def make_keys(self, topic: bytes):
        """``make_keys/1`` (emqx_trie.erl:128-130)."""
        ws = words(topic)
        return (topic, 1), [(p, 0) for p in self.make_prefixes(ws)]

    # -- table ops ------------------------------------------------------------
    def insert(self, topic: bytes) -> None:
        """``insert/1`` (emqx_trie.erl:82-87): idempotent per filter, prefixes ref-counted."""
        tkey, pkeys = self.make_keys(topic)
        if tkey in self.tab:
            return
        for k in [tkey] + pkeys:
            self.tab[k] = self.tab.get(k, 0) + 1          # insert_key :171-178

    def delete(self, topic: bytes) -> None:
        """``delete/1`` (emqx_trie.erl:91-96)."""
        tkey, pkeys = self.make_keys(topic)
        if tkey not in self.tab:
            return
        for k in [tkey] + pkeys:                           # delete_key :180-188
            c = self.tab.get(k)
            if c is None:
                continue
            if c > 1:
                self.tab[k] = c - 1
            else:
                del self.tab[k]

    def empty(self) -> bool:
        """``empty/0`` (emqx_trie.erl:118)."""
        return len(self.tab) == 0

    # -- probes -------------------------------------------------------------
    def lookup_topic(self, topic: bytes, is_wildcard: Optional[bool] = None) -> List[bytes]:
        """``lookup_topic/1,2`` (emqx_trie.erl:192-199)."""
        if is_wildcard is False:
            return []
        self.lookups += 1
        c = self.tab.get((topic, 1))
        return [topic] if c is not None and c > 0 else []

    def has_prefix(self, prefix) -> bool:
        """``has_prefix/1`` (emqx_trie.erl:201-206)."""
        if prefix is ROOT:
            return True
        self.lookups += 1
        c = self.tab.get((prefix, 0))
        return c is not None and c > 0

    def match_hash(self, prefix) -> List[bytes]:
        """``'match_#'/1`` (emqx_trie.erl:268-270)."""
        return self.lookup_topic(trie_join(prefix, HASH))

    # -- match ----------------------------------------------------------------
    def match(self, topic: bytes) -> List[bytes]:
        """``match/1`` (emqx_trie.erl:100-114)."""
        ws = words(topic)
        if wildcard(ws):
            return []
        return self._do_match(ws)

    def _do_match(self, ws: List[Word]) -> List[bytes]:
        """``do_match/1`` (emqx_trie.erl:208-217): the '$' rule."""
        first = ws[0]
        if isinstance(first, bytes) and first[:1] == b"$":
            rest = ws[1:]
            head = self.lookup_topic(first) if len(rest) == 0 else []
            return head + self._do_match2(rest, first)
        return self._do_match2(ws, ROOT)

    def _do_match2(self, ws, prefix):
        """``do_match/2`` (emqx_trie.erl:219-223)."""
        if self.compact:
            return self._match_compact(ws, 0, prefix, False, [])
        return self._match_no_compact(ws, 0, prefix, False, [])

    def _match_no_compact(self, ws, i, prefix, is_wc, acc):
        """``match_no_compact/4`` (emqx_trie.erl:225-249)."""
        if i == len(ws):
            return self.match_hash(prefix) + self.lookup_topic(prefix, is_wc) + acc
        if self.has_prefix(prefix):
            acc1 = self.match_hash(prefix) + acc
            acc2 = self._match_no_compact(ws, i + 1, trie_join(prefix, PLUS), True, acc1)
            return self._match_no_compact(ws, i + 1, trie_join(prefix, ws[i]), is_wc, acc2)
        return acc

    def _match_compact(self, ws, i, prefix, is_wc, acc0):
        """``match_compact/4`` (emqx_trie.erl:251-266)."""
        if i == len(ws):
            return self.match_hash(prefix) + self.lookup_topic(prefix, is_wc) + acc0
        acc1 = self.match_hash(prefix) + acc0
        acc = self._match_compact(ws, i + 1, trie_join(prefix, ws[i]), is_wc, acc1)
        wprefix = trie_join(prefix, PLUS)
        if i + 1 == len(ws) or self.has_prefix(wprefix):
            return self._match_compact(ws, i + 1, wprefix, True, acc)
        return acc


def trie_semantics(topic: bytes, filters: Iterable[bytes]) -> List[bytes]:
    """Closed form of ``emqx_trie:match/1`` over a trie holding ``filters``.

    Derived from emqx_trie.erl:190-270 and verified against both walks by
    ``tests/test_oracle_props.py``: a wildcard topic matches nothing
    (:102-111); a wildcard filter is returned iff ``emqx_topic:match/2`` holds
    (:68-87); a non-wildcard filter is returned only through the single-word
    '$' probe ``lookup_topic(Prefix)`` of ``do_match/1`` (:208-215), because
    ``lookup_topic(_, false)`` short-circuits (:192).
    """
    ws = words(topic)
    if wildcard(ws):
        return []
    out = []
    for f in filters:
        if wildcard(f):
            if match(topic, f):
                out.append(f)
        elif f == topic and len(ws) == 1 and isinstance(ws[0], bytes) and ws[0][:1] == b"$":
            out.append(f)
    return out


# ---------------------------------------------------------------------------
# emqx_router  (apps/emqx/src/emqx_router.erl)
# ---------------------------------------------------------------------------

class Router:
    """Route table (bag of {Topic, Dest}) + trie (emqx_router.erl:114-170,227-248)."""

    def __init__(self, compact: bool = True):
        self.trie = Trie(compact)
        self.routes: Dict[bytes, List[object]] = {}

    def lookup_routes(self, topic: bytes) -> List[Tuple[bytes, object]]:
        """``lookup_routes/1`` (emqx_router.erl:144-145)."""
        return [(topic, d) for d in self.routes.get(topic, [])]

    def do_add_route(self, topic: bytes, dest) -> None:
        """``do_add_route/2`` (emqx_router.erl:114-125, :230-235)."""
        if dest in self.routes.get(topic, []):
            return
        if wildcard(topic):
            if not self.routes.get(topic):
                self.trie.insert(topic)
        self.routes.setdefault(topic, []).append(dest)

    def do_delete_route(self, topic: bytes, dest) -> None:
        """``do_delete_route/2`` (emqx_router.erl:164-170, :240-248)."""
        cur = self.routes.get(topic, [])
        if wildcard(topic):
            if cur == [dest]:
                del self.routes[topic]
                self.trie.delete(topic)
                return
        if dest in cur:
            cur.remove(dest)
            if not cur:
                del self.routes[topic]

    def match_routes(self, topic: bytes) -> List[Tuple[bytes, object]]:
        """``match_routes/1`` + ``match_trie/1`` (emqx_router.erl:129-141)."""
        matched = [] if self.trie.empty() else self.trie.match(topic)
        if not matched:
            return self.lookup_routes(topic)
        out: List[Tuple[bytes, object]] = []
        for to in [topic] + matched:
            out.extend(self.lookup_routes(to))
        return out


def visited_states(topic: bytes, filters: Iterable[bytes]) -> int:
    """SURVEY §8d V_t of one topic: the NFA states a walk over ``filters``
    creates — the root plus every filter prefix (word prefixes up to a
    ``'#'``) of length l = 1..D that matches the topic's first l words
    (``'+'`` any word; never a root ``'+'`` under a ``'$'`` first word,
    emqx_trie.erl:208-215).  0 for a topic with a wildcard word (match/1
    returns [] at once, :102-111).  The roofline's byte model charges 32 B per
    state; this count is independent of the GPU table's layout."""
    ws = words(topic)
    if wildcard(ws):
        return 0
    prefixes = set()
    for f in filters:
        fw = words(f)
        for k in range(1, len(fw) + 1):
            if fw[k - 1] is HASH:
                break
            prefixes.add(tuple(bin_(w) for w in fw[:k]))
    dollar = isinstance(ws[0], bytes) and ws[0][:1] == b"$"
    v, cur = 1, [()]
    for l, w in enumerate(ws):
        nxt = []
        for p in cur:
            for x in (bin_(w), b"+"):
                if x == b"+" and l == 0 and dollar:
                    continue
                q = p + (x,)
                if q in prefixes:
                    v += 1
                    nxt.append(q)
        cur = nxt
    return v


def routes_semantics(topic: bytes, filters: Iterable[bytes]) -> List[bytes]:
    """Filter set whose routes ``match_routes/1`` returns (closed form).

    = {F == Topic} ∪ {wildcard F : emqx_topic:match(Topic, F)} when Topic is
    not a wildcard; = {F == Topic} when it is (emqx_router.erl:129-134: the
    trie yields [] and ``lookup_routes(Topic)`` still runs).
    """
    fs = list(filters)
    out = [f for f in fs if f == topic]
    if not wildcard(topic):
        out += [f for f in fs if wildcard(f) and match(topic, f)]
    return out


# ---------------------------------------------------------------------------
# emqx_broker fan-out  (apps/emqx/src/emqx_broker.erl:232-324)
# ---------------------------------------------------------------------------

def aggre(routes: List[Tuple[bytes, object]]) -> List[Tuple[bytes, object]]:
    """``aggre/1`` (emqx_broker.erl:249-260): node dests pass, shared dests usorted.

    A dest is ``('node', N)`` or ``('group', G)``; ``{Group, Node}`` collapses
    to the group.  Only the *set* is pinned (order is fold-dependent).
    """
    out = []
    seen = set()
    for to, dest in routes:
        if dest[0] == "node":
            out.append((to, dest))
        else:
            k = (to, ("group", dest[1]))
            if k not in seen:
                seen.add(k)
                out.append(k)
    return out


def deliveries(router: Router, subscribers: Dict[bytes, List[int]], topic: bytes,
               local_node="local") -> set:
    """Delivery set of ``publish/1`` for the local node (emqx_broker.erl:200-209,283-308).

    Returns {('sub', filter, sub_id)} for every local subscriber of every matched
    filter (shard entries ``{shard, Topic, I}`` flatten into the same set,
    emqx_broker.erl:297-308), {('group', filter, group)} for every shared group
    (one member is picked later, emqx_shared_sub.erl:120-135 — unpinned), and
    {('node', filter, node)} for remote node routes (forwarded, :242-245).
    """
    out = set()
    for to, dest in aggre(router.match_routes(topic)):
        if dest[0] == "node":
            if dest[1] == local_node:
                for s in subscribers.get(to, []):
                    out.add(("sub", to, s))
            else:
                out.add(("node", to, dest[1]))
        else:
            out.add(("group", to, dest[1]))
    return out
