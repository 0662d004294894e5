"""Retained reverse-match benchmark.

Store: M retained topics (the C2 topic generator, wildcard-free); queries: a
batch of N subscription filters (the C2 filter generator, all wildcard:
'+' p=.15, last-level '#' p=.5).  A step = egm_rstore_match on the whole batch
through the host API (filters uploaded, rows of message ids returned), i.e.
emqx_retainer_mnesia:match_messages/1 for N subscriptions at once.

CPU baseline: oracle/retainer_scan.cpp — the reference's dirty_select, a scan
of every record per filter — on `--cpu-threads` threads over a bounded sample
of the filters; its counts are checked against the GPU rows.

    python tools/bench_retained.py [--topics 1000000] [--filters 100000]
One JSON line on stdout.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--topics", type=int, default=1_000_000)
    ap.add_argument("--filters", type=int, default=100_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    a = ap.parse_args()
    from emqx_amd import _lib as L
    from emqx_amd import synth
    from emqx_amd.engine import pack_strings
    from emqx_amd.retainer import RetainedStore
    from oracle.cpp import OracleRetained

    c = synth.CONFIGS["c2"]
    seed = synth.SEED_BASE + synth.CONFIG_INDEX["c2"]
    t0 = time.time()
    flt = synth.filters(a.filters, c["dmin"], c["dmax"], c["wc"], c["p_plus"], c["p_hash"], seed=seed)
    tp = synth.topics(int(a.topics * 1.05), flt, c["dmin"], c["dmax"], seed=seed + 17)
    topics = [x for x in dict.fromkeys(tp.to_list()) if b"+" not in x.split(b"/") and b"#" not in x.split(b"/")]
    topics = topics[: a.topics]
    print(f"generated {len(topics)} topics, {flt.n} filters in {time.time() - t0:.1f}s", file=sys.stderr,
          flush=True)

    rs = RetainedStore(0)
    lib, h = rs.lib, rs.h
    t0 = time.time()
    for i, t in enumerate(topics):
        lib.egm_rstore_put(h, t, len(t), i, 0)
    rs.commit()
    build_s = time.time() - t0
    print(f"store built in {build_s:.1f}s", file=sys.stderr, flush=True)

    import ctypes as C
    fb, fo = flt.blob, flt.off
    n = flt.n

    def step():
        res = C.POINTER(L.egm_result)()
        rc = lib.egm_rstore_match(h, C.c_void_p(fb.ctypes.data), C.c_void_p(fo.ctypes.data), n, 0,
                                  L.EGM_RMODE_MATCH, C.byref(res))
        assert rc == 0, rc
        r = res.contents
        tot = int(r.n_ids)
        counts = np.ctypeslib.as_array(r.counts, shape=(n,)).copy()
        lib.egm_result_free(res)
        return tot, counts

    step()
    ts = []
    for _ in range(a.steps):
        t1 = time.perf_counter()
        tot, counts = step()
        ts.append(time.perf_counter() - t1)
    ms = 1e3 * float(np.median(ts))

    # CPU: full-table scan per filter over a bounded sample
    o = OracleRetained()
    tb, to = pack_strings(topics)
    o.put(tb, to, np.arange(len(topics), dtype=np.uint32), np.zeros(len(topics), dtype=np.uint64))
    k = 16
    while True:
        sb, so = pack_strings([flt[i] for i in range(k)])
        t1 = time.perf_counter()
        ctot, ccounts = o.match_counts(sb, so, 0, 0, threads=a.cpu_threads)
        dt = time.perf_counter() - t1
        if dt > a.cpu_seconds / 4 or k >= n:
            break
        k = min(n, k * 4)
    assert np.array_equal(ccounts, counts[:k]), "CPU scan and GPU rows disagree"
    out = {
        "bench": "retained_match", "metric": "subscription filters matched/sec against the retained store",
        "value": n / (ms / 1e3), "unit": "filters/s", "ms_per_batch": ms, "ids_per_s": tot / (ms / 1e3),
        "config": {"workload": "c2-shaped", "stored_topics": len(topics), "filters_per_batch": n,
                   "matched_ids_per_batch": tot, "path": "host API: H2D filters, match, D2H rows"},
        "cpu_baseline": {"value": k / dt, "unit": "filters/s", "cores": a.cpu_threads, "kind": "port",
                         "sample": f"{k} filters, full-table scan each (oracle/retainer_scan.cpp)"},
        "store_build_s": build_s,
    }
    print(json.dumps(out))
    rs.close()


if __name__ == "__main__":
    main()
