"""Host mirror of the retained-message store's match path on the GPU
(``apps/emqx_retainer/src/emqx_retainer_mnesia.erl``).

The store keeps one record per topic (``store_retained/2`` :73-101); a
subscription looks up the records its filter matches (``match_messages/1``
:200-204 with ``condition/1`` :215-220 and ``make_match_spec/1`` :222-228),
or, for a plain topic, the record of that topic (``read_messages/1``
:187-198), as ``emqx_retainer:dispatch/4`` does
(``apps/emqx_retainer/src/emqx_retainer.erl:107-117``).  The matching runs in
the C-ABI library (``egm_rstore_*``): a word trie of the stored topics in HBM,
walked level by level for a whole batch of filters at once.  Messages stay on
the host; the device holds topic -> message-id records.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .engine import pack_strings
from .topic import wildcard


class RetainedStore:
    """``emqx_retainer_mnesia`` backend semantics over one GPU."""

    def __init__(self, device: int = 0):
        self.lib = L.load()
        h = C.c_void_p()
        rc = self.lib.egm_rstore_open(device, C.byref(h))
        if rc != 0:
            raise L.EgmError(rc, f"egm_rstore_open(device={device}) failed — no usable HIP device?")
        self.h = h
        self._msgs: Dict[int, Tuple[bytes, object, int]] = {}   # id -> (topic, msg, timestamp)
        self._by_topic: Dict[bytes, int] = {}
        self._next = 0

    def close(self):
        if self.h:
            self.lib.egm_rstore_close(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.egm_rstore_last_error(self.h)
            raise L.EgmError(rc, f"{what}: {msg.decode() if msg else ''}")

    # -- records ---------------------------------------------------------------
    def store_retained(self, topic: bytes, msg=None, expiry_time: int = 0, timestamp: int = 0):
        """``store_retained/2`` (:73-101): the topic's record is replaced."""
        old = self._by_topic.get(topic)
        if old is not None:
            del self._msgs[old]
        mid = self._next
        self._next += 1
        self._check(self.lib.egm_rstore_put(self.h, topic, len(topic), mid, expiry_time), "egm_rstore_put")
        self._msgs[mid] = (topic, topic if msg is None else msg, timestamp)
        self._by_topic[topic] = mid

    def delete_message(self, topic: bytes):
        """``delete_message/2`` (:114-129): a wildcard filter deletes every
        record its pattern matches, expired or not (``match_delete_messages``
        :206-212)."""
        if wildcard(topic):
            for mid in self.match_ids([topic], now=0, mode=L.EGM_RMODE_MATCH)[0]:
                self._drop(self._msgs[int(mid)][0])
        else:
            self._drop(topic)

    def _drop(self, topic: bytes):
        mid = self._by_topic.pop(topic, None)
        if mid is not None:
            del self._msgs[mid]
        self._check(self.lib.egm_rstore_delete(self.h, topic, len(topic)), "egm_rstore_delete")

    def clean(self):
        """``clean/1`` (:148-150)."""
        self._check(self.lib.egm_rstore_clean(self.h), "egm_rstore_clean")
        self._msgs.clear()
        self._by_topic.clear()

    def size(self) -> int:
        n = C.c_uint64()
        self._check(self.lib.egm_rstore_size(self.h, C.byref(n)), "egm_rstore_size")
        return n.value

    def commit(self):
        self._check(self.lib.egm_rstore_commit(self.h), "egm_rstore_commit")

    # -- lookups ----------------------------------------------------------------
    def match_ids(self, filters: Sequence[bytes], now: int, mode: int = L.EGM_RMODE_DISPATCH) -> List[np.ndarray]:
        """Message ids per filter, one batched device call."""
        blob, off = pack_strings(list(filters))
        n = len(filters)
        res = C.POINTER(L.egm_result)()
        self._check(self.lib.egm_rstore_match(self.h, C.c_void_p(blob.ctypes.data), C.c_void_p(off.ctypes.data),
                                              n, now, mode, C.byref(res)), "egm_rstore_match")
        try:
            r = res.contents
            row = np.ctypeslib.as_array(r.row_ptr, shape=(n + 1,)).copy()
            nid = int(r.n_ids)
            ids = np.ctypeslib.as_array(r.ids, shape=(nid,)).copy() if nid else np.zeros(0, np.uint32)
        finally:
            self.lib.egm_result_free(res)
        return [ids[row[i]: row[i + 1]] for i in range(n)]

    def _messages(self, ids) -> List:
        recs = [self._msgs[int(i)] for i in ids]
        recs.sort(key=lambda x: x[2])          # sort_retained/1 (:154-159): by timestamp
        return [m for _, m, _ in recs]

    def match_messages(self, flt: bytes, now: int) -> List:
        """``match_messages/1`` (:200-204)."""
        return self._messages(self.match_ids([flt], now, L.EGM_RMODE_MATCH)[0])

    def read_messages(self, topic: bytes, now: int) -> List:
        """``read_messages/1`` (:187-198): the exact topic, alive when Et >= Now."""
        return self._messages(self.match_ids([topic], now, L.EGM_RMODE_DISPATCH)[0])

    def dispatch(self, flt: bytes, now: int) -> List:
        """``emqx_retainer:dispatch/4`` (emqx_retainer.erl:107-117)."""
        return self.match_messages(flt, now) if wildcard(flt) else self.read_messages(flt, now)

    def dispatch_batch(self, filters: Sequence[bytes], now: int) -> List[List]:
        """Many subscriptions at once (the GPU's reason to exist)."""
        return [self._messages(ids) for ids in self.match_ids(filters, now, L.EGM_RMODE_DISPATCH)]
