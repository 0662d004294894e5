"""CPU oracle for the retained-message reverse match.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (``emqx_amd``, the C-ABI
library, the HIP kernels) may import, call or link this module.  Only
``tests/`` and ``bench_retained``'s CPU-baseline leg use it, as the checker.

Literal restatement of ``apps/emqx_retainer/src/emqx_retainer_mnesia.erl``:

* the table: an mnesia ``set`` keyed by ``topic2tokens(Topic)`` =
  ``emqx_topic:words/1`` (``:164-165``); ``store_retained`` overwrites the
  record of the same topic (``:73-101``), ``delete_message`` of a plain topic
  deletes it (``:114-129``), of a wildcard filter deletes every record the
  filter's pattern matches (``match_delete_messages``, ``:206-212``),
  ``clean`` empties the table (``:148-150``);
* ``condition/1`` (``:215-220``): every ``'+'`` becomes the match-spec
  wildcard ``'_'``; if the last word is ``'#'``, the FIRST ``'#'`` is removed
  (``--``) and the list gets the improper tail ``'_'``, which matches any
  remaining list, including ``[]``.  There is no ``$``-topic rule here (unlike
  ``emqx_topic:match/2``);
* ``make_match_spec/1`` (``:222-228``): a record matches when its key matches
  the pattern and ``expiry_time =:= 0`` or ``expiry_time > Now``;
* ``read_messages/1`` (``:187-198``): the exact key, alive when
  ``Et =:= 0 orelse Et >= Now`` (note ``>=``, not ``>``);
* ``emqx_retainer:dispatch/4`` (``apps/emqx_retainer/src/emqx_retainer.erl:107-117``):
  a wildcard filter goes to ``match_messages``, a plain topic to
  ``read_message``.

Pinned by the cases of ``apps/emqx_retainer/test/emqx_retainer_SUITE.erl``
transcribed as data into ``tests/golden/kat_retainer.json``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

from . import trie_ref as R

ANY = object()        # the match-spec wildcard '_'


class Tail:
    """An improper list ``[W1, ..., Wk | '_']`` (``condition/1``, :219)."""

    def __init__(self, head):
        self.head = list(head)


def condition(ws: Sequence) -> object:
    """``emqx_retainer_mnesia:condition/1`` (:215-220)."""
    ws1 = [ANY if w is R.PLUS else w for w in ws]
    if not ws1 or ws1[-1] is not R.HASH:
        return ws1
    rest = list(ws1)
    rest.remove(R.HASH)               # Ws1 -- ['#'] removes the first occurrence
    return Tail(rest)


def _eq(p, w) -> bool:
    if p is ANY:
        return True
    if isinstance(p, R._Atom) or isinstance(w, R._Atom):
        return p is w
    return p == w


def pattern_match(pat, key: List) -> bool:
    """ETS match of a key pattern (list, or improper list with a '_' tail)."""
    if isinstance(pat, Tail):
        if len(key) < len(pat.head):
            return False
        return all(_eq(p, w) for p, w in zip(pat.head, key))
    if len(key) != len(pat):
        return False
    return all(_eq(p, w) for p, w in zip(pat, key))


class RetainedTable:
    """The ``emqx_retained`` mnesia table: tokens -> (msg, expiry_time)."""

    def __init__(self):
        self.recs: Dict[Tuple, Tuple[object, int]] = {}

    @staticmethod
    def key(topic: bytes) -> Tuple:
        return tuple(R.words(topic))

    def store_retained(self, topic: bytes, msg, expiry_time: int = 0):   # :73-101 (no size limit)
        self.recs[self.key(topic)] = (msg, expiry_time)

    def delete_message(self, topic: bytes):                            # :114-129
        if R.wildcard(topic):
            pat = condition(R.words(topic))
            for k in [k for k in self.recs if pattern_match(pat, list(k))]:
                del self.recs[k]
        else:
            self.recs.pop(self.key(topic), None)

    def clean(self):                                                   # :148-150
        self.recs.clear()

    def read_messages(self, topic: bytes, now: int) -> List:          # :187-198
        r = self.recs.get(self.key(topic))
        if r is None:
            return []
        msg, et = r
        return [msg] if et == 0 or et >= now else []

    def match_messages(self, flt: bytes, now: int) -> List:           # :200-204, :222-228
        pat = condition(R.words(flt))
        return [m for k, (m, et) in self.recs.items()
                if pattern_match(pat, list(k)) and (et == 0 or et > now)]

    def dispatch(self, flt: bytes, now: int) -> List:                 # emqx_retainer.erl:107-117
        return self.match_messages(flt, now) if R.wildcard(flt) else self.read_messages(flt, now)

    def clear_expired(self, now: int):                                 # :103-112
        for k in [k for k, (_, et) in self.recs.items() if et != 0 and et < now]:
            del self.recs[k]

    def size(self) -> int:
        return len(self.recs)
