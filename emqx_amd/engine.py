"""GpuMatcher — Python handle on one libemqx_gpu_match context (one HIP device).

Thin: argument packing, error translation and result copies.  The table is
built and matched by the native library; nothing here computes a match.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib as L


def pack_strings(items: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    """bytes list -> (blob u8 padded to 4 B, offsets u32[n+1])."""
    n = len(items)
    lens = np.fromiter((len(s) for s in items), dtype=np.uint64, count=n)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    if off[-1] >= 2 ** 32:
        raise ValueError("batch larger than 4 GiB: split it (u32 offsets)")
    raw = b"".join(items)
    blob = np.zeros(len(raw) + 8, dtype=np.uint8)
    if raw:
        blob[: len(raw)] = np.frombuffer(raw, dtype=np.uint8)
    return blob, off.astype(np.uint32)


def unpack_strings(blob: np.ndarray, off: np.ndarray):
    b = blob.tobytes()
    return [b[int(off[i]): int(off[i + 1])] for i in range(len(off) - 1)]


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else C.c_void_p(a.ctypes.data)


@dataclass
class MatchResult:
    row_ptr: np.ndarray   # u64[n+1]
    ids: np.ndarray       # u32[n_ids]
    flags: np.ndarray     # u8[n]
    epoch: int
    visited: int
    n_heavy: int
    n_error: int
    id_bytes: int = 4     # 3: the batch crossed PCIe in the packed form (EGM_RESULT_PACKED)

    def row(self, i: int) -> np.ndarray:
        return self.ids[self.row_ptr[i]: self.row_ptr[i + 1]]

    @property
    def counts(self) -> np.ndarray:
        return np.diff(self.row_ptr).astype(np.uint32)


def _result_of(r) -> "MatchResult":
    """Copy an egm_result out of the library's memory, either form: plain
    (u64 row_ptr, u32 ids) or packed (u32 row32, 3-byte ids24; EGM_RESULT_PACKED)."""
    n, nid = int(r.n_topics), int(r.n_ids)
    if int(r.id_bytes) == 3:
        row = np.ctypeslib.as_array(r.row32, shape=(n + 1,)).astype(np.uint64)
        b = np.ctypeslib.as_array(r.ids24, shape=(3 * nid,)) if nid else np.zeros(0, np.uint8)
        b = b.reshape(nid, 3).astype(np.uint32)
        ids = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
    else:
        row = np.ctypeslib.as_array(r.row_ptr, shape=(n + 1,)).copy()
        ids = np.ctypeslib.as_array(r.ids, shape=(nid,)).copy() if nid else np.zeros(0, np.uint32)
    fl = np.ctypeslib.as_array(r.flags, shape=(n,)).copy() if n else np.zeros(0, np.uint8)
    return MatchResult(row, ids.astype(np.uint32), fl, int(r.epoch), int(r.visited), int(r.n_heavy), int(r.n_error),
                       int(r.id_bytes))


class GpuMatcher:
    """One ``egm_ctx``.  ``mode``: ``L.EGM_MODE_TRIE`` or ``L.EGM_MODE_ROUTES``."""

    def __init__(self, device: int = 0, max_batch: int = 0, compact: bool = True):
        self.lib = L.load()
        cfg = L.egm_config(device, 1 if compact else 0, max_batch, 0)
        ctx = C.c_void_p()
        rc = self.lib.egm_open(C.byref(cfg), C.byref(ctx))
        if rc != 0:
            raise L.EgmError(rc, f"egm_open(device={device}) failed — no usable HIP device?")
        self.ctx = ctx
        self.device = device

    # -- lifecycle ------------------------------------------------------------
    def close(self):
        if self.ctx:
            self.lib.egm_close(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self.lib.egm_last_error(self.ctx)
            raise L.EgmError(rc, f"{what}: {msg.decode() if msg else ''}")

    # -- table ----------------------------------------------------------------
    def build(self, blob: np.ndarray, off: np.ndarray, ids: Optional[np.ndarray] = None):
        off = np.ascontiguousarray(off, dtype=np.uint32)
        ids = None if ids is None else np.ascontiguousarray(ids, dtype=np.uint32)
        self._check(self.lib.egm_table_build(self.ctx, _ptr(blob), _ptr(off), len(off) - 1, _ptr(ids)),
                    "egm_table_build")

    def build_strings(self, filters: Sequence[bytes], ids: Optional[Sequence[int]] = None):
        blob, off = pack_strings(filters)
        self.build(blob, off, None if ids is None else np.asarray(ids, dtype=np.uint32))

    def apply(self, inserts: Optional[Sequence[bytes]] = None, deletes: Optional[Sequence[bytes]] = None,
              insert_ids: Optional[Sequence[int]] = None):
        keep = []

        def mk(items, ids=None):
            if not items:
                return None
            blob, off = pack_strings(items)
            idarr = None if ids is None else np.asarray(ids, dtype=np.uint32)
            keep.extend([blob, off, idarr])
            return L.egm_delta(blob.ctypes.data, off.ctypes.data, len(items),
                               None if idarr is None else idarr.ctypes.data)

        di, dd = mk(inserts, insert_ids), mk(deletes)
        self._check(self.lib.egm_table_apply_delta(self.ctx, C.byref(di) if di else None,
                                                   C.byref(dd) if dd else None), "egm_table_apply_delta")

    def commit(self) -> int:
        ep = C.c_uint64()
        self._check(self.lib.egm_table_commit(self.ctx, C.byref(ep)), "egm_table_commit")
        return ep.value

    def commit_stats(self) -> dict:
        """What the last commit moved (incremental patch vs whole copy)."""
        h, d, p = C.c_uint64(), C.c_uint64(), C.c_uint64()
        ms = C.c_double()
        self._check(self.lib.egm_last_commit_stats(self.ctx, C.byref(h), C.byref(d), C.byref(p), C.byref(ms)),
                    "egm_last_commit_stats")
        return {"h2d_bytes": h.value, "d2d_bytes": d.value, "patched": p.value, "ms": ms.value}

    def empty(self) -> bool:
        return self.lib.egm_table_empty(self.ctx) == 1

    def epoch(self) -> int:
        """The current (last published) table epoch (egm_table_epoch)."""
        ep = C.c_uint64()
        self._check(self.lib.egm_table_epoch(self.ctx, C.byref(ep)), "egm_table_epoch")
        return ep.value

    def stats(self) -> dict:
        v = [C.c_uint64() for _ in range(5)]
        self._check(self.lib.egm_table_stats(self.ctx, *[C.byref(x) for x in v]), "egm_table_stats")
        return dict(zip(("filters", "nodes", "edges", "words", "device_bytes"), (x.value for x in v)))

    def filter_id(self, f: bytes) -> Optional[int]:
        out = C.c_uint32()
        rc = self.lib.egm_filter_id(self.ctx, f, len(f), C.byref(out))
        if rc == L.EGM_E_NOTFOUND:
            return None
        self._check(rc, "egm_filter_id")
        return out.value

    def filter_bytes(self, fid: int) -> Optional[bytes]:
        p = C.POINTER(C.c_uint8)()
        n = C.c_uint32()
        rc = self.lib.egm_filter_bytes(self.ctx, fid, C.byref(p), C.byref(n))
        if rc == L.EGM_E_NOTFOUND:
            return None
        self._check(rc, "egm_filter_bytes")
        return C.string_at(p, n.value)

    # -- matching -------------------------------------------------------------
    def match(self, blob: np.ndarray, off: np.ndarray, mode: int = L.EGM_MODE_TRIE,
              allow_error: bool = False) -> MatchResult:
        off = np.ascontiguousarray(off, dtype=np.uint32)
        n = len(off) - 1
        res = C.POINTER(L.egm_result)()
        rc = self.lib.egm_match_batch(self.ctx, _ptr(blob), _ptr(off), n, mode, C.byref(res))
        if rc != 0 and not (rc == L.EGM_E_OVERFLOW and allow_error and res):
            if res:   # the library may hand back a result with an error: release it
                self.lib.egm_result_free(res)
            self._check(rc, "egm_match_batch")
        try:
            return _result_of(res.contents)
        finally:
            self.lib.egm_result_free(res)

    def submit(self, blob: np.ndarray, off: np.ndarray, mode: int = L.EGM_MODE_TRIE) -> int:
        """Queue a host batch on the pipeline (staged in pinned memory at once).
        mode may carry L.EGM_RESULT_PACKED (the packed result form)."""
        off = np.ascontiguousarray(off, dtype=np.uint32)
        t = C.c_uint64()
        self._check(self.lib.egm_match_submit(self.ctx, _ptr(blob), _ptr(off), len(off) - 1, mode, C.byref(t)),
                    "egm_match_submit")
        return t.value

    def wait(self, ticket: int, copy: bool = True) -> Optional[MatchResult]:
        """Result of a submitted batch (copied out, pinned memory released);
        copy=False releases it unread (throughput measurement)."""
        res = C.POINTER(L.egm_result)()
        rc = self.lib.egm_match_wait(self.ctx, ticket, C.byref(res))
        if rc != 0:
            if res:
                self.lib.egm_result_free(res)
            self._check(rc, "egm_match_wait")
        try:
            if not copy:
                return None
            return _result_of(res.contents)
        finally:
            self.lib.egm_result_free(res)

    def match_strings(self, topics: Sequence[bytes], mode: int = L.EGM_MODE_TRIE) -> MatchResult:
        blob, off = pack_strings(topics)
        return self.match(blob, off, mode)

    def match_device(self, d_blob: int, blob_bytes: int, d_off: int, n: int, mode: int, stream: int, d_row: int,
                     d_ids: int, ids_cap: int, d_flags: int = 0):
        """Enqueue a batch whose inputs already live in HBM (raw device pointers)."""
        self._check(self.lib.egm_match_device(self.ctx, d_blob, blob_bytes, d_off, n, mode, stream or None, d_row,
                                              d_ids, ids_cap, d_flags or None), "egm_match_device")

    def match_device_ordered(self, d_blob: int, blob_bytes: int, d_off: int, n: int, mode: int, stream: int,
                             d_row: int, d_topic: int, d_ids: int, ids_cap: int):
        """egm_match_device with rows in the walk's order: row k is input topic d_topic[k]."""
        self._check(self.lib.egm_match_device_ordered(self.ctx, d_blob, blob_bytes, d_off, n, mode, stream or None,
                                                      d_row, d_topic or None, d_ids, ids_cap),
                    "egm_match_device_ordered")

    def match_device_counted(self, d_blob: int, blob_bytes: int, d_off: int, n_max: int, d_n: int, mode: int,
                             stream: int, d_row: int, d_ids: int, ids_cap: int):
        """egm_match_device over a received prefix slot: d_n points to the
        slot's 16-B device header {count, bytes, overflow, 0} (the layout
        egm_prefix_route writes, include/emqx_gpu_match.h), not a bare u32
        count — the kernels read its count (<= n_max) and match the slot as
        empty when its overflow word is set."""
        self._check(self.lib.egm_match_device_counted(self.ctx, d_blob, blob_bytes, d_off, n_max, d_n, mode,
                                                      stream or None, d_row, d_ids, ids_cap),
                    "egm_match_device_counted")

    def match_device_counted_ordered(self, d_blob: int, blob_bytes: int, d_off: int, n_max: int, d_n: int,
                                     mode: int, stream: int, d_row: int, d_topic: int, d_ids: int, ids_cap: int):
        """match_device_counted with rows in the walk's order: row k is slot topic d_topic[k]."""
        self._check(self.lib.egm_match_device_counted_ordered(self.ctx, d_blob, blob_bytes, d_off, n_max, d_n, mode,
                                                              stream or None, d_row, d_topic, d_ids, ids_cap),
                    "egm_match_device_counted_ordered")

    def prefix_route(self, d_blob: int, d_off: int, n: int, d_vpart_rank: int, n_vparts: int, n_ranks: int,
                     cap_topics: int, cap_bytes: int, stream: int, d_send: int):
        """egm_prefix_route: a device topic batch -> n_ranks slots (egm_prefix_slot_bytes each) at d_send."""
        self._check(self.lib.egm_prefix_route(self.ctx, d_blob, d_off, n, d_vpart_rank, n_vparts, n_ranks,
                                              cap_topics, cap_bytes, stream or None, d_send), "egm_prefix_route")

    def cancel(self, ticket: int):
        """Give a submitted ticket up without its result (egm_match_cancel)."""
        self._check(self.lib.egm_match_cancel(self.ctx, ticket), "egm_match_cancel")

    def last_stats(self) -> dict:
        """Counters of the last batch.  `overflow` is capacity only (rerun with
        a bigger id buffer); a walk guard trip — a kernel invariant failed —
        raises EgmError(EGM_E_DEVICE) instead (see last_guard)."""
        a, b = C.c_uint64(), C.c_uint64()
        c, d, e = C.c_uint32(), C.c_uint32(), C.c_uint32()
        self._check(self.lib.egm_last_stats(self.ctx, C.byref(a), C.byref(b), C.byref(c), C.byref(d),
                                            C.byref(e)), "egm_last_stats")
        return {"n_ids": a.value, "visited": b.value, "deferred_chunks": c.value, "overflow": d.value,
                "errors": e.value}

    def last_guard(self) -> int:
        """Walk guard bits of the last batch (0 = none; EGM_GUARD_STACK / EGM_GUARD_LOOP)."""
        g = C.c_uint32()
        self._check(self.lib.egm_last_guard(self.ctx, C.byref(g)), "egm_last_guard")
        return g.value

    def walk_counters(self) -> dict:
        a, b, c, d, e = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._check(self.lib.egm_last_walk_counters(self.ctx, C.byref(a), C.byref(b), C.byref(c), C.byref(d),
                                                    C.byref(e)), "egm_last_walk_counters")
        occ = b.value / max(1, a.value * 64)
        sl, si = C.c_uint64(), C.c_uint64()
        self._check(self.lib.egm_last_walk_probes(self.ctx, C.byref(sl), C.byref(si)), "egm_last_walk_probes")
        return {"iters": a.value, "popped": b.value, "bounded": c.value, "lane_occupancy": occ,
                "lit_probes": d.value, "plus_reads": e.value, "slow_probes": sl.value, "slow_iters": si.value}

    def set_debug(self, flags: int):
        self._check(self.lib.egm_set_debug(self.ctx, flags), "egm_set_debug")

    def set_timing(self, on: bool):
        self._check(self.lib.egm_set_timing(self.ctx, 1 if on else 0), "egm_set_timing")

    def get_timing(self) -> dict:
        wm, fm = C.c_double(), C.c_double()
        wn, fn = C.c_uint64(), C.c_uint64()
        self._check(self.lib.egm_get_timing(self.ctx, C.byref(wm), C.byref(wn), C.byref(fm), C.byref(fn)),
                    "egm_get_timing")
        return {"walk_ms": wm.value, "walk_launches": wn.value, "fanout_ms": fm.value,
                "fanout_launches": fn.value}

    # -- fan-out --------------------------------------------------------------
    def subs_build(self, row: np.ndarray, subs: np.ndarray):
        row = np.ascontiguousarray(row, dtype=np.uint64)
        subs = np.ascontiguousarray(subs, dtype=np.uint32)
        self._check(self.lib.egm_subs_build(self.ctx, _ptr(row), len(row) - 1, _ptr(subs)), "egm_subs_build")

    def subs_apply_delta(self, add=(), delete=()):
        """egm_subs_apply_delta: (filter id, subscriber) pairs to add / remove."""
        a = np.ascontiguousarray(np.asarray(add, dtype=np.uint32).reshape(-1, 2))
        d = np.ascontiguousarray(np.asarray(delete, dtype=np.uint32).reshape(-1, 2))
        self._check(self.lib.egm_subs_apply_delta(self.ctx, _ptr(a) if len(a) else None, len(a),
                                                  _ptr(d) if len(d) else None, len(d)), "egm_subs_apply_delta")

    def subs_commit(self) -> int:
        """egm_subs_commit: publish the staged subscriber changes; returns the epoch."""
        ep = C.c_uint64()
        self._check(self.lib.egm_subs_commit(self.ctx, C.byref(ep)), "egm_subs_commit")
        return ep.value

    def debug_walk_sort(self, d_keys: int, d_vals: int, n: int, kbits: int, d_out: int):
        """egm_debug_walk_sort: the walk-order radix sort alone (test hook)."""
        self._check(self.lib.egm_debug_walk_sort(self.ctx, d_keys, d_vals, n, kbits, d_out), "egm_debug_walk_sort")

    def subs_slots(self) -> int:
        """egm_subs_slots: filter-id slots of the device subscriber records."""
        n = C.c_uint32()
        self._check(self.lib.egm_subs_slots(self.ctx, C.byref(n)), "egm_subs_slots")
        return n.value

    def subs_last_commit(self) -> dict:
        a, p, e = C.c_uint64(), C.c_uint64(), C.c_uint64()
        r = C.c_int()
        self._check(self.lib.egm_subs_last_commit(self.ctx, C.byref(a), C.byref(p), C.byref(r), C.byref(e)),
                    "egm_subs_last_commit")
        return {"appended": a.value, "patched": p.value, "rebuilt": bool(r.value), "entries": e.value}

    def fanout(self, m: MatchResult) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        n = len(m.row_ptr) - 1
        counts = np.diff(m.row_ptr).astype(np.uint32)
        r = L.egm_result(n, len(m.ids), counts.ctypes.data_as(L._u32p),
                         m.row_ptr.ctypes.data_as(L._u64p), m.ids.ctypes.data_as(L._u32p),
                         m.flags.ctypes.data_as(L._u8p), m.epoch, m.visited, m.n_heavy, m.n_error)
        out = C.POINTER(L.egm_delivery)()
        self._check(self.lib.egm_fanout_batch(self.ctx, C.byref(r), C.byref(out)), "egm_fanout_batch")
        try:
            d = out.contents
            tot = int(d.n_deliveries)
            row = np.ctypeslib.as_array(d.row_ptr, shape=(n + 1,)).copy()
            fid = np.ctypeslib.as_array(d.fid, shape=(tot,)).copy() if tot else np.zeros(0, np.uint32)
            sub = np.ctypeslib.as_array(d.sub, shape=(tot,)).copy() if tot else np.zeros(0, np.uint32)
            return row, fid, sub
        finally:
            self.lib.egm_result_free(out)

    def fanout_device(self, d_mrow: int, d_mids: int, mids_len: int, n: int, stream: int, d_drow: int, d_fid: int,
                      d_sub: int, cap: int):
        self._check(self.lib.egm_fanout_device(self.ctx, d_mrow, d_mids, mids_len, n, stream or None, d_drow,
                                               d_fid, d_sub, cap), "egm_fanout_device")

    def fanout_device_compact(self, d_mrow: int, d_mids: int, mids_len: int, n: int, stream: int, d_drow: int,
                              d_entry_pos: int, d_sub: int, cap: int):
        """egm_fanout_device_compact: subscriber ids only + each match entry's first delivery."""
        self._check(self.lib.egm_fanout_device_compact(self.ctx, d_mrow, d_mids, mids_len, n, stream or None, d_drow,
                                                       d_entry_pos, d_sub, cap), "egm_fanout_device_compact")

    def last_fanout(self) -> dict:
        """Delivery total of the last fan-out and whether its buffers were too small."""
        tot, ovf = C.c_uint64(), C.c_uint32()
        self._check(self.lib.egm_last_fanout(self.ctx, C.byref(tot), C.byref(ovf)), "egm_last_fanout")
        return {"deliveries": tot.value, "overflow": ovf.value}


    # -- multi-GPU filter shards --------------------------------------------------
    def shard_merge(self, n_shards: int, n: int, d_counts: int, d_shard_ids: Sequence[int], total: int,
                    stream: int, d_row: int, d_ids: int, ids_cap: int):
        """egm_shard_merge: G gathered shard CSRs (device) -> one CSR (device)."""
        arr = (C.c_void_p * n_shards)(*d_shard_ids)
        self._check(self.lib.egm_shard_merge(self.ctx, n_shards, n, d_counts, arr, total, stream or None, d_row,
                                             d_ids, ids_cap), "egm_shard_merge")


class TableImage:
    """Host-only build of the HBM image (no device): for layout tests on CPU."""

    def __init__(self):
        self.lib = L.load()
        self.h = self.lib.egm_image_new()

    def __del__(self):  # pragma: no cover
        if getattr(self, "h", None):
            self.lib.egm_image_free(self.h)
            self.h = None

    def insert(self, f: bytes, fid: int = L.NONE_ID) -> int:
        return self.lib.egm_image_insert(self.h, f, len(f), fid)

    def remove(self, f: bytes) -> int:
        return self.lib.egm_image_remove(self.h, f, len(f))

    def relayout(self):
        self.lib.egm_image_relayout(self.h)

    def bulk_build(self, blob: np.ndarray, off: np.ndarray, ids: Optional[np.ndarray] = None, threads: int = 0):
        """egm_image_build: the whole image at once (parallel, level by level)."""
        off = np.ascontiguousarray(off, dtype=np.uint32)
        ids = None if ids is None else np.ascontiguousarray(ids, dtype=np.uint32)
        rc = self.lib.egm_image_build(self.h, _ptr(blob), _ptr(off), len(off) - 1, _ptr(ids), threads)
        if rc != 0:
            raise L.EgmError(rc, "egm_image_build")

    def arrays(self) -> dict:
        v = L.egm_image_view()
        assert self.lib.egm_image_get_view(self.h, C.byref(v)) == 0

        def arr(p, n, dt):
            if n == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                         shape=(n,)).copy()

        nodes = arr(v.nodes, v.n_nodes * 4, np.uint32).reshape(-1, 4)
        edges = arr(v.edges, v.n_edge_slots * 8, np.uint32).reshape(-1, 8)
        dict_ = arr(v.dict, v.n_dict_slots * 8, np.uint32).reshape(-1, 8)
        return {
            "nodes": nodes, "hash_child": arr(v.hash_child, v.n_nodes, np.uint32), "edges": edges,
            "edge_mask": v.edge_mask, "dict": dict_, "dict_mask": v.dict_mask,
            "dict_off": arr(v.dict_off, v.n_words + 1, np.uint64),
            "dict_blob": arr(v.dict_blob, int(arr(v.dict_off, v.n_words + 1, np.uint64)[-1]), np.uint8),
            "n_filters": v.n_filters, "n_live_nodes": v.n_live_nodes, "n_edges": v.n_edges,
        }

    def take_dirty(self) -> dict:
        """Records changed since the previous call (what a commit patches)."""
        v = L.egm_dirty_view()
        assert self.lib.egm_image_take_dirty(self.h, C.byref(v)) == 0

        def arr(p, n):
            return np.ctypeslib.as_array(p, shape=(n,)).copy() if n else np.zeros(0, np.uint32)

        return {"nodes": arr(v.nodes, v.n_nodes), "edges": arr(v.edges, v.n_edges), "dict": arr(v.dict, v.n_dict),
                "nodes_full": bool(v.nodes_full), "edges_full": bool(v.edges_full),
                "dict_full": bool(v.dict_full), "words_full": bool(v.words_full)}

    def word_hash(self, w: bytes) -> int:
        return self.lib.egm_word_hash(w, len(w))

    def edge_bucket(self, parent: int, word: int, mask: int) -> int:
        return self.lib.egm_edge_bucket(parent, word, mask)
