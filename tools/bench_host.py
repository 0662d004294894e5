"""Host-visible throughput of the drop-in path: topics/s
from a host topic blob to a host CSR result, through egm_match_submit /
egm_match_wait (pinned staging, H2D on a copy stream, match, D2H), with two
batches in flight — the PCIe-inclusive rate the NIF sees, never bench.py's
`value`.

    python tools/bench_host.py [--config c2] [--batch 1000000] [--batches 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--filters", type=int, default=None)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--packed", action="store_true", help="EGM_RESULT_PACKED: u32 rows + 3-byte ids (the NIF's form)")
    a = ap.parse_args()
    from emqx_amd import _lib as L
    from emqx_amd import synth
    from emqx_amd.engine import GpuMatcher
    import numpy as np
    c = synth.CONFIGS[a.config]
    seed = synth.SEED_BASE + synth.CONFIG_INDEX[a.config]
    f = synth.filters(a.filters or c["n_filters"], c["dmin"], c["dmax"], c["wc"], c["p_plus"], c["p_hash"],
                      seed=seed)
    t = synth.topics(a.batch * 2, f, c["dmin"], c["dmax"], seed=seed)
    halves = [t.subset(np.arange(0, a.batch)), t.subset(np.arange(a.batch, 2 * a.batch))]
    gm = GpuMatcher(0, max_batch=a.batch)
    gm.build(f.blob, f.off)
    mode = L.EGM_MODE_ROUTES | (L.EGM_RESULT_PACKED if a.packed else 0)
    # warm up: create and size the pipeline slots the deepest phase uses
    tk = [gm.submit(halves[k % 2].blob, halves[k % 2].off, mode) for k in range(4)]
    for x in tk:
        gm.wait(x, copy=False)
    out = {}
    for depth in (1, 2, 3, 4):
        ids = 0
        t_sub = t_wait = 0.0
        t0 = time.perf_counter()
        inflight = []
        for k in range(a.batches):
            ta = time.perf_counter()
            inflight.append(gm.submit(halves[k % 2].blob, halves[k % 2].off, mode))
            tb = time.perf_counter()
            t_sub += tb - ta
            if len(inflight) == depth:
                gm.wait(inflight.pop(0), copy=False)
                t_wait += time.perf_counter() - tb
                ids += gm.last_stats()["n_ids"]
        while inflight:
            tb = time.perf_counter()
            gm.wait(inflight.pop(0), copy=False)
            t_wait += time.perf_counter() - tb
            ids += gm.last_stats()["n_ids"]
        dt = time.perf_counter() - t0
        out[f"in_flight_{depth}"] = {"topics_per_s": a.batch * a.batches / dt, "ms_per_batch": dt / a.batches * 1e3,
                                     "ids_per_batch": ids / a.batches,
                                     "result_bytes_per_batch": (ids / a.batches * 3 + (a.batch + 1) * 4 + a.batch) if a.packed
                                     else (ids / a.batches * 4 + (a.batch + 1) * 8 + a.batch),
                                     "input_bytes_per_batch": int(halves[0].off[-1]) + 4 * (a.batch + 1),
                                     "submit_ms": t_sub / a.batches * 1e3, "wait_ms": t_wait / a.batches * 1e3}
    gm.close()
    line = {"what": "host_e2e: host topic blob -> host CSR (egm_match_submit/egm_match_wait, pinned staging)",
            "config": a.config, "filters": f.n, "batch": a.batch, "batches": a.batches, "packed": a.packed, **out}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
