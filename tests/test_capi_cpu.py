"""CPU-only checks of the native boundary: the C-ABI library loads, exports
every symbol include/emqx_gpu_match.h declares, and the host table builder
produces an HBM image that encodes the filter set (checked by walking the image
with tests/walk_emul.py against the pinned oracle).  No GPU compute here.
"""
import os
import random
import re

import numpy as np
import pytest

from emqx_amd import _lib as L
from emqx_amd.engine import TableImage
from oracle import trie_ref as R
from tests.kat import b, load
from tests.walk_emul import Emul

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    """The library's entry points the header declares (its static inline
    helpers, egm_result_row/egm_result_id, are header-only)."""
    src = open(os.path.join(ROOT, "include", "emqx_gpu_match.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    inline = set(re.findall(r"static\s+inline\s+[\w\s\*]+?\b(egm_[a-z_0-9]+)\s*\(", src))
    return sorted(set(re.findall(r"\b(egm_[a-z_0-9]+)\s*\(", src)) - inline)


def test_packed_result_helpers_decode_both_forms(tmp_path):
    """egm_result_row / egm_result_id (include/emqx_gpu_match.h) read the plain
    and the packed (EGM_RESULT_PACKED: u32 rows, 3-byte ids) result forms alike."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc missing")
    c = tmp_path / "t.c"
    c.write_text(r"""
#include <stdio.h>
#include "emqx_gpu_match.h"
int main(void) {
  uint64_t row[3] = {0, 2, 3};
  uint32_t ids[3] = {7, 0xFFFFFE, 65536};
  uint32_t row32[3] = {0, 2, 3};
  uint8_t pk[9] = {7, 0, 0, 0xFE, 0xFF, 0xFF, 0, 0, 1};
  egm_result a = {0}, b = {0};
  a.n_topics = b.n_topics = 2; a.n_ids = b.n_ids = 3;
  a.row_ptr = row; a.ids = ids; a.id_bytes = 4;
  b.row32 = row32; b.ids24 = pk; b.id_bytes = 3;
  for (uint32_t i = 0; i <= 2; ++i) if (egm_result_row(&a, i) != egm_result_row(&b, i)) return 1;
  for (uint64_t k = 0; k < 3; ++k) if (egm_result_id(&a, k) != egm_result_id(&b, k)) return 2;
  return 0;
}
""")
    exe = tmp_path / "t"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", f"-I{os.path.join(ROOT, 'include')}", str(c), "-o", str(exe)],
                   check=True)
    assert subprocess.run([str(exe)]).returncode == 0


def test_library_exports_every_header_symbol():
    lib = L.load()
    names = header_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n
        assert n in L.SIGNATURES, f"{n} missing from the ctypes binding"
    assert lib.egm_version().startswith(b"emqx_gpu_match")


def test_open_without_device_fails_cleanly():
    import ctypes as C
    lib = L.load()
    ctx = C.c_void_p()
    cfg = L.egm_config(999, 1, 0, 0)
    assert lib.egm_open(C.byref(cfg), C.byref(ctx)) != 0
    assert not ctx.value


def image_of(filters, relayout=True):
    im = TableImage()
    ids = {}
    for i, f in enumerate(filters):
        r = im.insert(f, i)
        assert r in (0, 1)
        if r == 0:
            ids[i] = f
    if relayout:
        im.relayout()
    return im, ids


@pytest.mark.parametrize("mode", [0, 1])
def test_image_reference_kats(mode):
    K = load()
    for case in K["trie_cases"]:
        im = TableImage()
        live = {}
        nxt = 0
        for op in case["ops"]:
            if op[0] == "insert":
                f = b(op[1])
                if f not in live.values():
                    assert im.insert(f, nxt) == 0
                    live[nxt] = f
                    nxt += 1
                else:
                    assert im.insert(f, 999) == 1
            elif op[0] == "delete":
                f = b(op[1])
                r = im.remove(f)
                hit = [k for k, v in live.items() if v == f]
                assert r == (0 if hit else 1)
                for k in hit:
                    del live[k]
        em = Emul(im, im.arrays())
        for topic, expected in case["queries"]:
            got = sorted(live[i] for i in em.match(b(topic), mode))
            if mode == 0:
                assert got == sorted(b(x) for x in expected), (case["name"], topic)
            else:
                assert got == sorted(R.routes_semantics(b(topic), live.values()))


ALPHA = [b"a", b"b", b"", b"$x", b"c", b"$", b"ab", b"w" * 20, b"w" * 21]


def rand_filter(rng):
    d = rng.randint(1, 5)
    ws = []
    for i in range(d):
        p = rng.random()
        if p < 0.25:
            ws.append(b"+")
        elif p < 0.33 and i == d - 1:
            ws.append(b"#")
        elif p < 0.35:
            ws.append(b"#")       # mid-filter '#' (invalid but insertable)
        else:
            ws.append(rng.choice(ALPHA))
    return b"/".join(ws)


def rand_topic(rng):
    d = rng.randint(1, 6)
    ws = [rng.choice(ALPHA + [b"zz"]) for _ in range(d)]
    if rng.random() < 0.05:
        ws[rng.randrange(d)] = rng.choice([b"+", b"#"])
    return b"/".join(ws)


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("relayout", [True, False])
def test_image_random_vs_oracle(seed, relayout):
    rng = random.Random(seed)
    filters = list(dict.fromkeys([rand_filter(rng) for _ in range(150)] + [b"$x", b"a/b", b"$", b""]))
    im, live = image_of(filters, relayout)
    # delete a third, re-add some
    for f in filters[::3]:
        assert im.remove(f) == 0
    for k in [k for k, v in live.items() if v in set(filters[::3])]:
        del live[k]
    for j, f in enumerate(filters[::6]):
        assert im.insert(f, 1000 + j) == 0
        live[1000 + j] = f
    if relayout:
        im.relayout()
    em = Emul(im, im.arrays())
    for _ in range(300):
        t = rand_topic(rng)
        for mode in (0, 1):
            got = em.match(t, mode)
            assert len(got) == len(set(got)), t
            want = R.trie_semantics(t, live.values()) if mode == 0 else R.routes_semantics(t, live.values())
            assert sorted(live[i] for i in got) == sorted(want), (t, mode)


def test_image_delete_all_frees_everything():
    rng = random.Random(11)
    filters = list(dict.fromkeys(rand_filter(rng) for _ in range(200)))
    im, _ = image_of(filters, relayout=False)
    for f in filters:
        assert im.remove(f) == 0
        assert im.remove(f) == 1
    a = im.arrays()
    assert a["n_filters"] == 0 and a["n_live_nodes"] == 1 and a["n_edges"] == 0
    root = a["nodes"][0]
    assert list(root[:3]) == [L.NONE_ID] * 3 and int(root[3]) == 0


# ---- incremental commit: the dirty log must name every
# record a delta changes, so patching a copy of the previous image with it
# reproduces the new image exactly (what egm_table_commit does on the device).
def _apply_log(prev, cur, log):
    out = {}
    for key, idx_key, full_key in (("nodes", "nodes", "nodes_full"), ("hash_child", "nodes", "nodes_full"),
                                   ("edges", "edges", "edges_full"), ("dict", "dict", "dict_full")):
        if log[full_key] or prev is None:
            out[key] = cur[key].copy()
            continue
        a = prev[key]
        if len(cur[key]) > len(a):   # appended records are in the log; the copy grows first
            a = np.concatenate([a, np.zeros((len(cur[key]) - len(a),) + a.shape[1:], a.dtype)])
        else:
            a = a.copy()
        idx = log[idx_key]
        a[idx] = cur[key][idx]
        out[key] = a
    for key in ("dict_blob", "dict_off"):   # append-only: copy + tail
        if log["words_full"] or prev is None:
            out[key] = cur[key].copy()
        else:
            n0 = len(prev[key])
            out[key] = np.concatenate([prev[key], cur[key][n0:]])
    return out


def _same_image(a, b):
    for key in ("nodes", "hash_child", "edges", "dict", "dict_blob", "dict_off"):
        assert a[key].shape == b[key].shape, key
        assert np.array_equal(a[key], b[key]), key


@pytest.mark.parametrize("seed", range(3))
def test_dirty_log_patches_reproduce_image(seed):
    rng = random.Random(100 + seed)
    im = TableImage()
    live = []
    for f in dict.fromkeys(rand_filter(rng) for _ in range(60)):
        assert im.insert(f) == 0
        live.append(f)
    im.relayout()
    log = im.take_dirty()
    assert log["nodes_full"] and log["edges_full"]        # a rebuild copies whole
    dev = im.arrays()
    saw_patch = saw_growth = False
    for rnd in range(25):
        # a delta: inserts (some new words -> dictionary/edge growth), deletes
        for _ in range(rng.randint(1, 40 if rnd % 5 else 400)):
            if live and rng.random() < 0.4:
                f = live.pop(rng.randrange(len(live)))
                assert im.remove(f) == 0
            else:
                f = rand_filter(rng) + b"/n%d" % rng.randrange(10 ** 6)
                if im.insert(f) == 0:
                    live.append(f)
        cur = im.arrays()
        log = im.take_dirty()
        saw_patch |= not log["edges_full"] and len(log["edges"]) > 0
        saw_growth |= log["edges_full"] or log["dict_full"]
        assert np.all(np.diff(log["nodes"].astype(np.int64)) > 0)   # sorted, unique
        dev = _apply_log(dev, cur, log)
        _same_image(dev, cur)
    assert saw_patch and saw_growth
    # an empty delta logs nothing
    assert not any(len(v) if isinstance(v, np.ndarray) else v for v in im.take_dirty().values())


def test_dirty_log_two_slot_protocol():
    """The device keeps two copies and writes the one not in use; a copy that
    skipped commits must get the union of their logs (egm_capi.cpp
    commit_locked: slot.pending ∪ this commit's log)."""
    rng = random.Random(7)
    im = TableImage()
    live = []
    for f in dict.fromkeys(rand_filter(rng) for _ in range(50)):
        im.insert(f)
        live.append(f)
    im.relayout()
    slots = [None, None]
    pending = [None, None]
    cur = -1
    for rnd in range(20):
        for _ in range(rng.randint(1, 30)):
            if live and rng.random() < 0.5:
                im.remove(live.pop(rng.randrange(len(live))))
            else:
                f = rand_filter(rng) + b"/s%d" % rng.randrange(1000)
                if im.insert(f) == 0:
                    live.append(f)
        img = im.arrays()
        d = im.take_dirty()
        x = 0 if cur < 0 else 1 - cur
        if slots[x] is None or pending[x] is None:
            slots[x] = _apply_log(None, img, d)
        else:
            need = {k: (np.union1d(pending[x][k], d[k]).astype(np.uint32) if isinstance(d[k], np.ndarray)
                        else pending[x][k] or d[k]) for k in d}
            slots[x] = _apply_log(slots[x], img, need)
        _same_image(slots[x], img)
        pending[x] = {k: (np.zeros(0, np.uint32) if isinstance(v, np.ndarray) else False) for k, v in d.items()}
        if cur >= 0:
            pending[cur] = {k: (np.union1d(pending[cur][k], d[k]).astype(np.uint32) if isinstance(d[k], np.ndarray)
                                else pending[cur][k] or d[k]) for k in d}
        cur = x
