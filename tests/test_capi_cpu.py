"""CPU-only checks of the native boundary: the C-ABI library loads, exports
every symbol include/emqx_gpu_match.h declares, and the host table builder
produces an HBM image that encodes the filter set (checked by walking the image
with tests/walk_emul.py against the pinned oracle).  No GPU compute here.
"""
import os
import random
import re

import pytest

from emqx_amd import _lib as L
from emqx_amd.engine import TableImage
from oracle import trie_ref as R
from tests.kat import b, load
from tests.walk_emul import Emul

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "emqx_gpu_match.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(egm_[a-z_]+)\s*\(", src)))


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
