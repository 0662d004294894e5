"""ctypes handle on oracle/liboracle_trie.so (the C++ restatement in trie_oracle.cpp).

TEST INFRASTRUCTURE ONLY — used by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(_HERE, "liboracle_trie.so")
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(PATH):
            raise ImportError(f"{PATH} not built — run `python -m emqx_amd.build`")
        lib = C.CDLL(PATH)
        P = C.c_void_p
        lib.ot_new.restype = P
        lib.ot_new.argtypes = [C.c_int, C.c_int]
        lib.ot_free.argtypes = [P]
        lib.ot_set_mode.restype = C.c_int
        lib.ot_set_mode.argtypes = [P, C.c_int]
        lib.ot_add.argtypes = [P, P, P, C.c_uint32, P]
        lib.ot_remove.argtypes = [P, P, P, C.c_uint32]
        lib.ot_match.restype = C.c_uint64
        lib.ot_match.argtypes = [P, P, P, C.c_uint32, C.c_int, P, C.POINTER(C.POINTER(C.c_uint32))]
        lib.ot_match_count.restype = C.c_uint64
        lib.ot_match_count.argtypes = [P, P, P, C.c_uint32, C.c_int]
        lib.ot_match_counts.restype = C.c_uint64
        lib.ot_match_counts.argtypes = [P, P, P, C.c_uint32, C.c_int, P]
        lib.ot_match_sums.restype = C.c_uint64
        lib.ot_match_sums.argtypes = [P, P, P, C.c_uint32, C.c_int, P, P]
        lib.ot_visited_counts.restype = C.c_uint64
        lib.ot_visited_counts.argtypes = [P, P, P, C.c_uint32, C.c_int, P]
        lib.ot_n_keys.restype = C.c_uint64
        lib.ot_n_keys.argtypes = [P]
        lib.ot_free_ptr.argtypes = [P]
        lib.rs_new.restype = P
        lib.rs_free.argtypes = [P]
        lib.rs_put.argtypes = [P, P, P, C.c_uint32, P, P]
        lib.rs_match_count.restype = C.c_uint64
        lib.rs_match_count.argtypes = [P, P, P, C.c_uint32, C.c_uint64, C.c_int, C.c_int, P]
        _lib = lib
    return _lib


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


class OracleTrie:
    """mode 0: emqx_trie:match/1; mode 1: emqx_router:match_routes/1 filter set."""

    def __init__(self, compact: bool = True, mode: int = 0):
        self.lib = _load()
        self.h = self.lib.ot_new(1 if compact else 0, mode)

    def __del__(self):  # pragma: no cover
        if getattr(self, "h", None):
            self.lib.ot_free(self.h)
            self.h = None

    def set_mode(self, mode: int):
        """Switch match mode (all-wildcard filter sets only: same trie in both)."""
        if self.lib.ot_set_mode(self.h, mode) != 0:
            raise ValueError("ot_set_mode: the filter set has exact filters; build one oracle per mode")

    def add(self, blob, off, ids=None):
        off = np.ascontiguousarray(off, dtype=np.uint32)
        ids = None if ids is None else np.ascontiguousarray(ids, dtype=np.uint32)
        self.lib.ot_add(self.h, _p(blob), _p(off), len(off) - 1, _p(ids))

    def remove(self, blob, off):
        off = np.ascontiguousarray(off, dtype=np.uint32)
        self.lib.ot_remove(self.h, _p(blob), _p(off), len(off) - 1)

    def match(self, blob, off, threads: int = 1):
        """-> (row_ptr u64[n+1], ids u32) in the walk's natural order."""
        off = np.ascontiguousarray(off, dtype=np.uint32)
        n = len(off) - 1
        row = np.zeros(n + 1, dtype=np.uint64)
        ip = C.POINTER(C.c_uint32)()
        tot = self.lib.ot_match(self.h, _p(blob), _p(off), n, threads, _p(row), C.byref(ip))
        ids = np.ctypeslib.as_array(ip, shape=(int(tot),)).copy() if tot else np.zeros(0, np.uint32)
        self.lib.ot_free_ptr(C.cast(ip, C.c_void_p))
        return row, ids

    def match_count(self, blob, off, threads: int = 1) -> int:
        off = np.ascontiguousarray(off, dtype=np.uint32)
        return int(self.lib.ot_match_count(self.h, _p(blob), _p(off), len(off) - 1, threads))

    def match_counts(self, blob, off, threads: int = 1) -> np.ndarray:
        """Per-topic match counts (u32[n]), no ids."""
        off = np.ascontiguousarray(off, dtype=np.uint32)
        n = len(off) - 1
        counts = np.zeros(n, dtype=np.uint32)
        self.lib.ot_match_counts(self.h, _p(blob), _p(off), n, threads, _p(counts))
        return counts

    def match_sums(self, blob, off, threads: int = 1):
        """Per-topic match counts (u32[n]) and per-row checksums (u64[n]): the
        sum of a 64-bit mix of each matched id, the mix of
        tests/test_gpu_scale.py::row_checksums — every row compared as a SET
        at full size; additive over disjoint filter shards."""
        off = np.ascontiguousarray(off, dtype=np.uint32)
        n = len(off) - 1
        counts = np.zeros(n, dtype=np.uint32)
        sums = np.zeros(n, dtype=np.uint64)
        self.lib.ot_match_sums(self.h, _p(blob), _p(off), n, threads, _p(counts), _p(sums))
        return counts, sums

    def visited_counts(self, blob, off, threads: int = 1):
        """SURVEY §8d V_t per topic (u64[n]) and its sum: the root plus every
        prefix of a filter (up to a '#') that the NFA over the topic reaches —
        counted from string prefixes, independently of the GPU table."""
        off = np.ascontiguousarray(off, dtype=np.uint32)
        n = len(off) - 1
        counts = np.zeros(n, dtype=np.uint64)
        tot = self.lib.ot_visited_counts(self.h, _p(blob), _p(off), n, threads, _p(counts))
        return int(tot), counts

    def n_keys(self) -> int:
        return int(self.lib.ot_n_keys(self.h))


def canonical(row, ids):
    """Sort ids within every row (sets are the parity unit)."""
    out = ids.copy()
    n = len(row) - 1
    # sort by (row, id) in one shot
    rid = np.repeat(np.arange(n, dtype=np.int64), np.diff(row).astype(np.int64))
    order = np.lexsort((out, rid))
    return out[order]


class OracleRetained:
    """retainer_scan.cpp: the reference's retained lookup as a full-table scan
    per filter (mnesia dirty_select with a partially bound key)."""

    def __init__(self):
        self.lib = _load()
        self.h = self.lib.rs_new()

    def __del__(self):  # pragma: no cover
        if getattr(self, "h", None):
            self.lib.rs_free(self.h)
            self.h = None

    def put(self, blob, off, ids, expiry):
        off = np.ascontiguousarray(off, dtype=np.uint32)
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        expiry = np.ascontiguousarray(expiry, dtype=np.uint64)
        self.lib.rs_put(self.h, _p(blob), _p(off), len(off) - 1, _p(ids), _p(expiry))

    def match_counts(self, blob, off, now: int, mode: int, threads: int = 1):
        off = np.ascontiguousarray(off, dtype=np.uint32)
        n = len(off) - 1
        counts = np.zeros(n, dtype=np.uint32)
        tot = self.lib.rs_match_count(self.h, _p(blob), _p(off), n, now, mode, threads, _p(counts))
        return int(tot), counts
