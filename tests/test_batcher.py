"""Linger/size batcher (emqx_batch policy) — host logic, no GPU."""
import threading
import time

import pytest

from emqx_amd.batcher import Batcher


def test_size_and_linger_flush():
    seen = []

    def commit(items):
        seen.append(len(items))
        return [x * 2 for x in items]

    b = Batcher(commit, batch_size=8, linger_ms=20)
    futs = [b.push(i) for i in range(8)]
    assert [f.result(timeout=2) for f in futs] == [i * 2 for i in range(8)]
    t0 = time.monotonic()
    f = b.push(100)
    assert f.result(timeout=2) == 200
    assert time.monotonic() - t0 >= 0.015          # waited for the linger
    b.close()
    assert seen[0] == 8 and seen[-1] == 1


def test_concurrent_publishers_and_errors():
    def commit(items):
        if any(x < 0 for x in items):
            raise ValueError("bad")
        return items

    b = Batcher(commit, batch_size=64, linger_ms=2)
    out = {}

    def worker(k):
        out[k] = [b.push(k * 1000 + i).result(timeout=5) for i in range(200)]

    th = [threading.Thread(target=worker, args=(k,)) for k in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for k in range(6):
        assert out[k] == [k * 1000 + i for i in range(200)]
    with pytest.raises(ValueError):
        b.push(-1).result(timeout=2)
    b.close()
    assert b.batches >= 600 // 64
