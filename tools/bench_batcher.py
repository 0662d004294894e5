"""The batcher's operating points: saturated batches of
1K-64K C2 topics at 1-4 tickets in flight through egm_match_submit /
egm_match_wait — topics/s and per-batch submit -> wait-return latency
(p50/p99), from which erl/emqx_gpu_batch.erl's defaults are chosen
(INTEGRATION.md §2).

    python tools/bench_batcher.py [--config c2] [--seconds 0.3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--seconds", type=float, default=0.3)
    a = ap.parse_args()
    from bench import host_batcher_curve
    from emqx_amd import _lib as L
    from emqx_amd import synth
    from emqx_amd.engine import GpuMatcher
    f = synth.config_filters(a.config)
    t = synth.config_topics(a.config, f, n_topics=1 << 20)
    gm = GpuMatcher(0, max_batch=65536)
    gm.build(f.blob, f.off)
    sizes = (1024, 2048, 4096, 8192, 16384, 32768, 65536)
    for depth in (1, 2, 3, 4):
        r = host_batcher_curve(gm, t, L.EGM_MODE_ROUTES, sizes=sizes, depth=depth, seconds=a.seconds)
        print(json.dumps({"config": a.config, "filters": f.n, "depth": depth, "sweep": r["sweep"]}), flush=True)
    gm.close()


if __name__ == "__main__":
    main()
