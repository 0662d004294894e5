"""Synthetic workloads for BASELINE.json's configs.

Wraps ``libegm_synth.so``.  Deterministic: seed = 0xE3C00000 + config index.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
SYNTH_PATH = os.path.join(_HERE, "libegm_synth.so")
SEED_BASE = 0xE3C00000


class egs_strings(C.Structure):
    _fields_ = [("blob", C.POINTER(C.c_uint8)), ("bytes", C.c_uint64), ("off", C.POINTER(C.c_uint32)),
                ("n", C.c_uint32)]


_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(SYNTH_PATH):
            raise ImportError(f"{SYNTH_PATH} not built — run `python -m emqx_amd.build`")
        lib = C.CDLL(SYNTH_PATH)
        lib.egs_filters.restype = C.c_int
        lib.egs_filters.argtypes = [C.c_uint64, C.c_uint32, C.c_int, C.c_int, C.c_double, C.c_double,
                                    C.c_double, C.c_double, C.c_double, C.c_uint32, C.POINTER(egs_strings)]
        lib.egs_topics.restype = C.c_int
        lib.egs_topics.argtypes = [C.c_uint64, C.POINTER(egs_strings), C.c_uint32, C.c_int, C.c_int,
                                   C.c_double, C.c_double, C.c_double, C.c_double, C.c_uint32,
                                   C.POINTER(egs_strings)]
        lib.egs_subscribers.restype = C.c_int
        lib.egs_subscribers.argtypes = [C.c_uint64, C.c_uint32, C.c_double, C.c_double, C.c_uint32,
                                        C.c_double, C.c_uint32, C.POINTER(C.POINTER(C.c_uint64)),
                                        C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.c_uint64)]
        lib.egs_subset.restype = C.c_int
        lib.egs_subset.argtypes = [C.POINTER(egs_strings), C.c_void_p, C.c_uint32, C.POINTER(egs_strings)]
        lib.egs_free.argtypes = [C.POINTER(egs_strings)]
        lib.egs_free_ptr.argtypes = [C.c_void_p]
        _lib = lib
    return _lib


@dataclass
class StringSet:
    blob: np.ndarray   # u8, padded to a multiple of 4 (+8 bytes)
    off: np.ndarray    # u32[n+1]

    @property
    def n(self) -> int:
        return len(self.off) - 1

    def __getitem__(self, i: int) -> bytes:
        return self.blob[self.off[i]: self.off[i + 1]].tobytes()

    def to_list(self):
        b = self.blob.tobytes()
        o = self.off
        return [b[int(o[i]): int(o[i + 1])] for i in range(self.n)]

    def subset(self, idx) -> "StringSet":
        """The strings at idx, in that order (native gather)."""
        idx = np.ascontiguousarray(idx, dtype=np.uint32)
        s = egs_strings()
        rc = _load().egs_subset(C.byref(self.as_struct()), C.c_void_p(idx.ctypes.data), len(idx), C.byref(s))
        if rc != 0:
            raise ValueError(f"egs_subset rc={rc}")
        return _take(s)

    def as_struct(self) -> egs_strings:
        s = egs_strings()
        s.blob = self.blob.ctypes.data_as(C.POINTER(C.c_uint8))
        s.bytes = int(self.off[-1])
        s.off = self.off.ctypes.data_as(C.POINTER(C.c_uint32))
        s.n = self.n
        return s


def _take(s: egs_strings) -> StringSet:
    n = s.n
    nbytes = int(s.bytes)
    pad = (nbytes + 8 + 3) & ~3
    blob = np.zeros(pad, dtype=np.uint8)
    if nbytes:
        blob[:nbytes] = np.ctypeslib.as_array(s.blob, shape=(nbytes,))
    off = np.ctypeslib.as_array(s.off, shape=(n + 1,)).copy()
    _load().egs_free(C.byref(s))
    return StringSet(blob, off)


# SURVEY §8d config knobs: depth range, wildcard fraction, p('+'), p('#' last)
CONFIGS = {
    "c0": dict(n_filters=10_000, n_topics=100_000, dmin=4, dmax=8, wc=1.0, p_plus=0.15, p_hash=0.5),
    "c1": dict(n_filters=1_000_000, n_topics=10_000_000, dmin=4, dmax=8, wc=0.2, p_plus=0.15, p_hash=0.5),
    "c2": dict(n_filters=10_000_000, n_topics=10_000_000, dmin=4, dmax=8, wc=1.0, p_plus=0.15, p_hash=0.5),
    "c3": dict(n_filters=10_000_000, n_topics=10_000_000, dmin=16, dmax=16, wc=1.0, p_plus=0.35, p_hash=0.7),
    "c4": dict(n_filters=100_000_000, n_topics=10_000_000, dmin=4, dmax=8, wc=0.2, p_plus=0.15, p_hash=0.5),
}
CONFIG_INDEX = {"c0": 0, "c1": 1, "c2": 2, "c3": 3, "c4": 4}


def filters(n: int, dmin=4, dmax=8, wc=1.0, p_plus=0.15, p_hash=0.5, p_empty=0.05, zipf_s=1.1,
            vmax=100_000, seed=SEED_BASE) -> StringSet:
    s = egs_strings()
    rc = _load().egs_filters(seed, n, dmin, dmax, wc, p_plus, p_hash, p_empty, zipf_s, vmax, C.byref(s))
    if rc != 0:
        raise ValueError(f"egs_filters rc={rc}")
    return _take(s)


def topics(n: int, flt: StringSet, dmin=4, dmax=8, p_from_filter=0.5, p_sys=0.01, p_empty=0.05, zipf_s=1.1,
           vmax=100_000, seed=SEED_BASE) -> StringSet:
    s = egs_strings()
    fs = flt.as_struct() if flt is not None and flt.n else None
    rc = _load().egs_topics(seed, C.byref(fs) if fs is not None else None, n, dmin, dmax, p_from_filter, p_sys,
                            p_empty, zipf_s, vmax, C.byref(s))
    if rc != 0:
        raise ValueError(f"egs_topics rc={rc}")
    return _take(s)


def subscribers(n_filters: int, lam=1.0, p_big=0.001, n_big=2000, p_share=0.1, groups=64,
                seed=SEED_BASE):
    """filter id -> subscriber CSR (row u64[n+1], ids u32; bit 31 = $share group id)."""
    lib = _load()
    rp = C.POINTER(C.c_uint64)()
    ip = C.POINTER(C.c_uint32)()
    tot = C.c_uint64()
    rc = lib.egs_subscribers(seed, n_filters, lam, p_big, n_big, p_share, groups, C.byref(rp), C.byref(ip),
                             C.byref(tot))
    if rc != 0:
        raise ValueError(f"egs_subscribers rc={rc}")
    row = np.ctypeslib.as_array(rp, shape=(n_filters + 1,)).copy()
    ids = np.ctypeslib.as_array(ip, shape=(int(tot.value),)).copy() if tot.value else np.zeros(0, np.uint32)
    lib.egs_free_ptr(C.cast(rp, C.c_void_p))
    lib.egs_free_ptr(C.cast(ip, C.c_void_p))
    return row, ids


def config_filters(name: str, scale: float = 1.0, n_filters=None) -> StringSet:
    """The filter set of a BASELINE config (config()'s first half)."""
    c = CONFIGS[name]
    seed = SEED_BASE + CONFIG_INDEX[name]
    nf = n_filters if n_filters is not None else max(1, int(c["n_filters"] * scale))
    return filters(nf, c["dmin"], c["dmax"], c["wc"], c["p_plus"], c["p_hash"], seed=seed)


def config_topics(name: str, f: StringSet, scale: float = 1.0, n_topics=None) -> StringSet:
    """The topic batch of a BASELINE config over its filters (config()'s second half)."""
    c = CONFIGS[name]
    seed = SEED_BASE + CONFIG_INDEX[name]
    nt = n_topics if n_topics is not None else max(1, int(c["n_topics"] * scale))
    return topics(nt, f, c["dmin"], c["dmax"], seed=seed)


def config(name: str, scale: float = 1.0, n_filters=None, n_topics=None):
    """(filters, topics) for a BASELINE config, optionally scaled down."""
    f = config_filters(name, scale, n_filters)
    return f, config_topics(name, f, scale, n_topics)
