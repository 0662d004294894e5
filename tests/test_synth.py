"""Synthetic generator: deterministic, distributions as SURVEY §8d states."""
import numpy as np

from emqx_amd import synth
from oracle import trie_ref as R


def test_deterministic_and_unique():
    a = synth.filters(5000, seed=synth.SEED_BASE + 1, wc=0.2)
    b = synth.filters(5000, seed=synth.SEED_BASE + 1, wc=0.2)
    assert np.array_equal(a.off, b.off) and np.array_equal(a.blob, b.blob)
    fl = a.to_list()
    assert len(set(fl)) == len(fl) == 5000
    wc = sum(R.wildcard(f) for f in fl) / len(fl)
    assert 0.15 < wc < 0.25
    for f in fl[:500]:
        d = len(f.split(b"/"))
        assert 4 <= d <= 8


def test_all_wildcard_and_topics():
    f = synth.filters(3000, wc=1.0)
    fl = f.to_list()
    assert all(R.wildcard(x) for x in fl)
    t = synth.topics(4000, f, p_sys=0.05)
    tl = t.to_list()
    assert not any(R.wildcard(x) for x in tl)
    sys = sum(x.startswith(b"$SYS") for x in tl) / len(tl)
    assert 0.02 < sys < 0.09
    # about half the topics are instantiated from a filter and so match it
    hit = sum(1 for x in tl[:400] if R.trie_semantics(x, fl))
    assert hit > 150


def test_subscribers_csr():
    row, ids = synth.subscribers(20000, p_big=0.001, n_big=2000, p_share=0.1)
    assert row[0] == 0 and row[-1] == len(ids) and np.all(np.diff(row.astype(np.int64)) >= 1)
    big = np.sum(np.diff(row) == 2000)
    assert 5 <= big <= 40
    grp = np.sum(ids >= 0x80000000)
    assert grp > 1000
