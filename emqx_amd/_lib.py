"""ctypes binding of libemqx_gpu_match.so (include/emqx_gpu_match.h).

There is no fallback: if the shared library is missing or fails to load, this
module raises ImportError.  Build it with ``python -m emqx_amd.build``.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EGM_LIB") or os.path.join(_HERE, "libemqx_gpu_match.so")  # EGM_LIB: A/B tuning

EGM_OK = 0
EGM_PREFIX_ALL = 0xFFFFFFFF
EGM_E_INVAL = -1
EGM_E_NOMEM = -2
EGM_E_DEVICE = -3
EGM_E_OVERFLOW = -4
EGM_E_STATE = -5
EGM_E_NOTFOUND = -6

EGM_MODE_TRIE = 0
EGM_MODE_ROUTES = 1
EGM_RESULT_PACKED = 0x100   # mode flag: the packed host result (u32 rows, 3-byte ids)
EGM_RMODE_MATCH = 0
EGM_RMODE_DISPATCH = 1

EGM_TF_WILDCARD = 1
EGM_TF_DOLLAR = 2
EGM_TF_HEAVY = 4
EGM_TF_ERROR = 8

EGM_DEBUG_FORCE_HEAVY = 1
EGM_DEBUG_FAIL_COMMIT = 2
EGM_DEBUG_INPUT_ORDER = 4
EGM_DEBUG_FORCE_GUARD = 8
EGM_GUARD_STACK = 4
EGM_GUARD_LOOP = 8

NONE_ID = 0xFFFFFFFF
GROUP_BIT = 0x80000000

_u8p = C.POINTER(C.c_uint8)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)


class egm_config(C.Structure):
    _fields_ = [("device", C.c_int32), ("compact_mode", C.c_int32),
                ("max_batch", C.c_uint32), ("linger_us", C.c_uint32)]


class egm_delta(C.Structure):
    _fields_ = [("blob", C.c_void_p), ("offsets", C.c_void_p), ("n", C.c_uint32), ("ids", C.c_void_p)]


class egm_result(C.Structure):
    _fields_ = [("n_topics", C.c_uint32), ("n_ids", C.c_uint64), ("counts", _u32p), ("row_ptr", _u64p),
                ("ids", _u32p), ("flags", _u8p), ("epoch", C.c_uint64), ("visited", C.c_uint64),
                ("n_heavy", C.c_uint32), ("n_error", C.c_uint32),
                ("id_bytes", C.c_uint32), ("row32", _u32p), ("ids24", _u8p)]


class egm_delivery(C.Structure):
    _fields_ = [("n_topics", C.c_uint32), ("n_deliveries", C.c_uint64), ("row_ptr", _u64p),
                ("fid", _u32p), ("sub", _u32p)]


class egm_image_view(C.Structure):
    _fields_ = [("nodes", C.c_void_p), ("n_nodes", C.c_uint64), ("hash_child", _u32p),
                ("edges", C.c_void_p), ("n_edge_slots", C.c_uint64), ("edge_mask", C.c_uint32),
                ("dict", C.c_void_p), ("n_dict_slots", C.c_uint64), ("dict_mask", C.c_uint32),
                ("dict_blob", _u8p), ("dict_off", _u64p), ("n_words", C.c_uint64),
                ("n_filters", C.c_uint64), ("n_live_nodes", C.c_uint64), ("n_edges", C.c_uint64)]


class egm_dirty_view(C.Structure):
    _fields_ = [("nodes", _u32p), ("n_nodes", C.c_uint64), ("edges", _u32p), ("n_edges", C.c_uint64),
                ("dict", _u32p), ("n_dict", C.c_uint64), ("nodes_full", C.c_uint32),
                ("edges_full", C.c_uint32), ("dict_full", C.c_uint32), ("words_full", C.c_uint32)]


_P = C.c_void_p
# name: (restype, argtypes) — every symbol the public header declares
SIGNATURES = {
    "egm_open": (C.c_int, [C.POINTER(egm_config), C.POINTER(_P)]),
    "egm_close": (None, [_P]),
    "egm_last_error": (C.c_char_p, [_P]),
    "egm_version": (C.c_char_p, []),
    "egm_table_build": (C.c_int, [_P, _P, _P, C.c_uint32, _P]),
    "egm_table_apply_delta": (C.c_int, [_P, C.POINTER(egm_delta), C.POINTER(egm_delta)]),
    "egm_table_commit": (C.c_int, [_P, _u64p]),
    "egm_last_commit_stats": (C.c_int, [_P, _u64p, _u64p, _u64p, C.POINTER(C.c_double)]),
    "egm_table_empty": (C.c_int, [_P]),
    "egm_table_epoch": (C.c_int, [_P, _u64p]),
    "egm_table_stats": (C.c_int, [_P, _u64p, _u64p, _u64p, _u64p, _u64p]),
    "egm_filter_id": (C.c_int, [_P, _P, C.c_uint32, _u32p]),
    "egm_filter_bytes": (C.c_int, [_P, C.c_uint32, C.POINTER(_u8p), _u32p]),
    "egm_match_batch": (C.c_int, [_P, _P, _P, C.c_uint32, C.c_int, C.POINTER(C.POINTER(egm_result))]),
    "egm_match_submit": (C.c_int, [_P, _P, _P, C.c_uint32, C.c_int, _u64p]),
    "egm_match_wait": (C.c_int, [_P, C.c_uint64, C.POINTER(C.POINTER(egm_result))]),
    "egm_match_cancel": (C.c_int, [_P, C.c_uint64]),
    "egm_match_device": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint32, C.c_int, _P, _P, _P, C.c_uint64, _P]),
    "egm_match_device_ordered": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint32, C.c_int, _P, _P, _P, _P, C.c_uint64]),
    "egm_match_device_counted": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint32, _P, C.c_int, _P, _P, _P,
                                           C.c_uint64]),
    "egm_match_device_counted_ordered": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint32, _P, C.c_int, _P, _P, _P, _P,
                                                   C.c_uint64]),
    "egm_last_stats": (C.c_int, [_P, _u64p, _u64p, _u32p, _u32p, _u32p]),
    "egm_last_guard": (C.c_int, [_P, _u32p]),
    "egm_last_walk_counters": (C.c_int, [_P, _u64p, _u64p, _u64p, _u64p, _u64p]),
    "egm_last_walk_probes": (C.c_int, [_P, _u64p, _u64p]),
    "egm_set_timing": (C.c_int, [_P, C.c_int]),
    "egm_set_debug": (C.c_int, [_P, C.c_uint32]),
    "egm_get_timing": (C.c_int, [_P, C.POINTER(C.c_double), _u64p, C.POINTER(C.c_double), _u64p]),
    "egm_subs_build": (C.c_int, [_P, _P, C.c_uint32, _P]),
    "egm_subs_apply_delta": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint64]),
    "egm_subs_commit": (C.c_int, [_P, _P]),
    "egm_subs_last_commit": (C.c_int, [_P, _P, _P, _P, _P]),
    "egm_subs_slots": (C.c_int, [_P, _P]),
    "egm_debug_walk_sort": (C.c_int, [_P, _P, _P, C.c_uint32, C.c_uint32, _P]),
    "egm_fanout_batch": (C.c_int, [_P, C.POINTER(egm_result), C.POINTER(C.POINTER(egm_delivery))]),
    "egm_fanout_device": (C.c_int, [_P, _P, _P, C.c_uint64, C.c_uint32, _P, _P, _P, _P, C.c_uint64]),
    "egm_fanout_device_compact": (C.c_int, [_P, _P, _P, C.c_uint64, C.c_uint32, _P, _P, _P, _P, C.c_uint64]),
    "egm_last_fanout": (C.c_int, [_P, _u64p, _u32p]),
    "egm_shard_merge": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, C.POINTER(_P), C.c_uint64, _P, _P, _P,
                                  C.c_uint64]),
    "egm_prefix_assign": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P]),
    "egm_prefix_slot_bytes": (C.c_uint64, [C.c_uint32, C.c_uint32, C.c_uint64]),
    "egm_prefix_route": (C.c_int, [_P, _P, _P, C.c_uint32, _P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, _P,
                                   _P]),
    "egm_result_free": (None, [_P]),
    "egm_rstore_open": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "egm_rstore_close": (None, [_P]),
    "egm_rstore_last_error": (C.c_char_p, [_P]),
    "egm_rstore_put": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, C.c_uint64]),
    "egm_rstore_delete": (C.c_int, [_P, _P, C.c_uint32]),
    "egm_rstore_clean": (C.c_int, [_P]),
    "egm_rstore_size": (C.c_int, [_P, _u64p]),
    "egm_rstore_commit": (C.c_int, [_P]),
    "egm_rstore_match": (C.c_int, [_P, _P, _P, C.c_uint32, C.c_uint64, C.c_int,
                                   C.POINTER(C.POINTER(egm_result))]),
    "egm_image_new": (_P, []),
    "egm_image_free": (None, [_P]),
    "egm_image_insert": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32]),
    "egm_image_remove": (C.c_int, [_P, _P, C.c_uint32]),
    "egm_image_relayout": (None, [_P]),
    "egm_image_build": (C.c_int, [_P, _P, _P, C.c_uint32, _P, C.c_uint32]),
    "egm_image_get_view": (C.c_int, [_P, C.POINTER(egm_image_view)]),
    "egm_image_take_dirty": (C.c_int, [_P, C.POINTER(egm_dirty_view)]),
    "egm_shard_assign": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, _P]),
    "egm_word_hash": (C.c_uint64, [_P, C.c_uint32]),
    "egm_edge_bucket": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32]),
}

_lib = None


def load() -> C.CDLL:
    """Load the native library (cached).  Raises ImportError if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built — run `python -m emqx_amd.build` "
                          "(the HIP path has no CPU fallback)")
    # PyTorch-ROCm bundles its own HIP/HSA runtime (torch/lib/libamdhip64.so,
    # SONAME libamdhip64.so.7).  Loading torch first lets this library's
    # NEEDED libamdhip64.so.7 bind to that runtime, so device pointers and
    # streams are shared with torch in one runtime.  Loaded the other way
    # round, torch would map a second HIP/HSA runtime into the process.
    # Standalone users (the Erlang NIF) resolve /opt/rocm/lib via RUNPATH.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        if os.environ.get("EGM_LIB") and not hasattr(lib, name):
            continue   # an A/B build of an older source (tools/build_variant.py): its missing entry points stay unset
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class EgmError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"egm error {code}: {msg}")
        self.code = code
