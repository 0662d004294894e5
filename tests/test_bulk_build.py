"""egm_image_build / the bulk path of egm_table_build (egm_bulk.cpp): the
whole table built level by level on several threads must be the image the
one-by-one insert loop + relayout builds (emqx_trie:insert/1 per filter,
apps/emqx/src/emqx_trie.erl:82-87, first occurrence of a repeat wins).

Node records, '#' children and the edge slots are compared array for array
(with fewer than 65 536 edges the edge table is filled by one thread, in the
same child order as relayout); the dictionary by content (its slots depend on
the rehash history); filter ids through lookups; matching through the walk
emulator against the pinned oracle; and deltas applied after a bulk build must
behave as after a sequential one.  No GPU."""
import random

import numpy as np
import pytest

from emqx_amd import synth
from emqx_amd.engine import TableImage, pack_strings
from oracle import trie_ref as R
from tests.test_capi_cpu import rand_filter, rand_topic
from tests.walk_emul import Emul


def seq_image(filters, ids=None):
    im = TableImage()
    for i, f in enumerate(filters):
        im.insert(f, i if ids is None else ids[i])
    im.relayout()
    return im


def dict_content(a):
    d = a["dict"]
    return sorted(tuple(r) for r in d[d[:, 2] != 0xFFFFFFFF].tolist())


@pytest.mark.parametrize("seed", range(5))
@pytest.mark.parametrize("threads", [1, 4])
def test_bulk_equals_insert_loop_plus_relayout(seed, threads):
    rng = random.Random(seed)
    filters = [rand_filter(rng) for _ in range(400)] + [b"$x", b"a/b", b"$", b"", b"a/b", b"+/+", b"#"]
    rng.shuffle(filters)
    ids = None if seed % 2 else [5000 + 3 * i for i in range(len(filters))]
    a = seq_image(filters, ids).arrays()
    bi = TableImage()
    blob, off = pack_strings(filters)
    bi.bulk_build(blob, off, None if ids is None else np.asarray(ids, np.uint32), threads)
    b = bi.arrays()
    assert np.array_equal(a["nodes"], b["nodes"])
    assert np.array_equal(a["hash_child"], b["hash_child"])
    assert np.array_equal(a["edges"], b["edges"]) and a["edge_mask"] == b["edge_mask"]
    assert a["dict_mask"] == b["dict_mask"] and dict_content(a) == dict_content(b)
    assert np.array_equal(a["dict_off"], b["dict_off"]) and np.array_equal(a["dict_blob"], b["dict_blob"])
    assert (a["n_filters"], a["n_live_nodes"], a["n_edges"]) == (b["n_filters"], b["n_live_nodes"], b["n_edges"])


def test_bulk_large_multithreaded_matches_oracle_and_takes_deltas():
    """Past 65 536 edges the edge table is filled by bucket ranges in parallel
    (slot positions may then differ near range ends): compare node arrays and
    the edge SET, match through the emulator against the C++ oracle, then
    apply the same deltas to both images."""
    from emqx_amd import _lib as L
    from oracle.cpp import OracleTrie
    f, t = synth.config("c0", n_filters=60_000, n_topics=150)
    fl = f.to_list()
    seq = seq_image(fl)
    bulk = TableImage()
    bulk.bulk_build(f.blob, f.off, None, 8)
    a, b = seq.arrays(), bulk.arrays()
    assert np.array_equal(a["nodes"], b["nodes"]) and np.array_equal(a["hash_child"], b["hash_child"])

    def live(e):
        return sorted(map(tuple, e[(e[:, 0] != 0xFFFFFFFF) & (e[:, 0] != 0xFFFFFFFE)].tolist()))

    assert a["n_edges"] > 65536 and live(a["edges"]) == live(b["edges"])
    rng = random.Random(3)
    topics = t.to_list() + [rand_topic(rng) for _ in range(50)]
    em = Emul(bulk, b)
    o = OracleTrie(True, L.EGM_MODE_TRIE)
    o.add(f.blob, f.off)
    tb, to = pack_strings(topics)
    orow, oids = o.match(tb, to)
    for k, tp in enumerate(topics):
        assert sorted(em.match(tp, 0)) == sorted(oids[int(orow[k]):int(orow[k + 1])].tolist()), tp
    # the same deltas on both images: delete a third, add new filters
    dels = fl[::3]
    adds = list(dict.fromkeys(rand_filter(rng) for _ in range(300)))
    for im in (seq, bulk):
        for x in dels:
            im.remove(x)
        for j, x in enumerate(adds):
            im.insert(x, 100_000 + j)
    es, eb = Emul(seq, seq.arrays()), Emul(bulk, bulk.arrays())
    for tp in topics:
        for mode in (0, 1):
            assert sorted(es.match(tp, mode)) == sorted(eb.match(tp, mode)), (tp, mode)


def test_bulk_rejects_bad_ids():
    blob, off = pack_strings([b"a/+", b"b/#"])
    im = TableImage()
    with pytest.raises(Exception):
        im.bulk_build(blob, off, np.asarray([7, 7], np.uint32))      # duplicate id
    with pytest.raises(Exception):
        im.bulk_build(blob, off, np.asarray([1, 0xFFFFFFFF], np.uint32))   # NONE: assign-id path only


def _check_plus_flags(a):
    """Every live edge slot carries the flags of its child's '+' child (0: none)."""
    nodes, e = a["nodes"], a["edges"]
    live = e[(e[:, 0] != 0xFFFFFFFF) & (e[:, 0] != 0xFFFFFFFE)]
    pc = nodes[live[:, 2].astype(np.int64), 0]
    want = np.where(pc != 0xFFFFFFFF, nodes[np.where(pc != 0xFFFFFFFF, pc, 0).astype(np.int64), 3], 0)
    assert len(live) > 0 and np.array_equal(live[:, 7], want.astype(live.dtype))
    return int(np.count_nonzero(want))


def test_edge_slots_carry_plus_child_flags():
    """The slot field the walk uses to skip a '+' transition that would do
    nothing (egm_common.h EdgeSlot::child_pflags) stays equal to the '+'
    child's flags through inserts and removes without a relayout, after a
    relayout and after a bulk build."""
    rng = random.Random(11)
    words = [b"a", b"b", b"c", b"+", b"d"]

    def filt():
        ws = [rng.choice(words) for _ in range(rng.randint(1, 6))]
        if rng.random() < 0.3:
            ws.append(b"#")
        return b"/".join(ws)

    fl = list(dict.fromkeys(filt() for _ in range(600)))
    im = TableImage()
    for i, f in enumerate(fl):
        im.insert(f, i)
    assert _check_plus_flags(im.arrays()) > 0
    for f in fl[::2]:
        im.remove(f)
    more = [x for x in dict.fromkeys(filt() for _ in range(300)) if x not in set(fl[1::2])]
    for j, f in enumerate(more):
        im.insert(f, 10_000 + j)
    _check_plus_flags(im.arrays())
    im.relayout()
    _check_plus_flags(im.arrays())
    bi = TableImage()
    blob, off = pack_strings(fl)
    bi.bulk_build(blob, off, None, 4)
    _check_plus_flags(bi.arrays())
