"""Route-churn benchmark for the incremental epoch commit.

The reference applies every route add/delete as a mnesia transaction over the
trie (emqx_router.erl:114-125,164-170,252-303 -> emqx_trie:insert/delete,
emqx_trie.erl:82-96).  Here deltas are staged on the host table and published
by egm_table_commit, which patches only the changed records into the idle
device copy of the image.  This measures, on the C2 table (10M wildcard
filters), for deltas of D route changes (D/2 deletes of live filters + D/2
inserts of new ones):

  apply_ms   host staging of the delta (egm_table_apply_delta)
  commit_ms  publishing it (egm_table_commit), with the bytes it moved
  updates_per_s = D / (apply + commit)

and the full-upload commit of the initial build for comparison.  One JSON
line on stdout.

    python tools/bench_updates.py [--filters N] [--deltas 1000,10000,100000]
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filters", type=int, default=10_000_000)
    ap.add_argument("--deltas", default="1000,10000,100000")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--topics", type=int, default=1_000_000)
    a = ap.parse_args()
    from emqx_amd import _lib as L
    from emqx_amd import synth
    from emqx_amd.engine import GpuMatcher, pack_strings

    c = synth.CONFIGS["c2"]
    seed = synth.SEED_BASE + synth.CONFIG_INDEX["c2"]
    t0 = time.time()
    f = synth.filters(a.filters, c["dmin"], c["dmax"], c["wc"], c["p_plus"], c["p_hash"], seed=seed)
    deltas = [int(x) for x in a.deltas.split(",")]
    need = sum(deltas) * a.repeat // 2 + 1000
    pool = synth.filters(need * 2, c["dmin"], c["dmax"], c["wc"], c["p_plus"], c["p_hash"], seed=seed + 99991)
    t = synth.topics(a.topics, f, c["dmin"], c["dmax"], seed=seed)
    print(f"generated in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)

    gm = GpuMatcher(0, max_batch=a.topics)
    t0 = time.time()
    gm.build(f.blob, f.off)
    build_s = time.time() - t0
    full = gm.commit_stats()
    st = gm.stats()
    print(f"built in {build_s:.1f}s {st} full commit {full}", file=sys.stderr, flush=True)

    fl = f.to_list()
    live_idx = list(range(len(fl)))
    pl = [x for x in dict.fromkeys(pool.to_list())]
    pi = 0
    rng = random.Random(5)
    nid = len(fl) + 1

    # warm one match (and the first commit after the build, which copies the
    # other device slot)
    gm.apply(deletes=[fl[0]])
    gm.commit()
    first = gm.commit_stats()
    gm.match(t.blob, t.off, L.EGM_MODE_ROUTES)

    rows = []
    for d in deltas:
        for r in range(a.repeat):
            k = d // 2
            dels_i = [live_idx.pop(rng.randrange(len(live_idx))) for _ in range(k)]
            dels = [fl[i] for i in dels_i]
            ins = pl[pi: pi + (d - k)]
            pi += d - k
            ids = list(range(nid, nid + len(ins)))
            nid += len(ins)
            t0 = time.perf_counter()
            gm.apply(inserts=ins, deletes=dels, insert_ids=ids)
            t1 = time.perf_counter()
            gm.commit()
            t2 = time.perf_counter()
            cs = gm.commit_stats()
            t3 = time.perf_counter()
            res = gm.match(t.blob, t.off, L.EGM_MODE_ROUTES)
            t4 = time.perf_counter()
            rows.append({"delta": d, "apply_ms": (t1 - t0) * 1e3, "commit_ms": (t2 - t1) * 1e3,
                         "commit_native_ms": cs["ms"], "h2d_bytes": cs["h2d_bytes"],
                         "d2d_bytes": cs["d2d_bytes"], "patched": cs["patched"],
                         "updates_per_s": d / (t2 - t0), "match_1M_ms": (t4 - t3) * 1e3,
                         "matched_ids": int(len(res.ids))})
            print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    out = {"bench": "route_churn", "workload": "c2", "filters": a.filters, "table_bytes": st["device_bytes"],
           "build_s": build_s, "full_commit": full, "first_commit_after_build": first, "rows": rows,
           "note": "apply = host staging; commit = publish to the idle device slot (patch of changed records)"}
    print(json.dumps(out))
    gm.close()


if __name__ == "__main__":
    main()
