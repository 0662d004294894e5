"""Where a small batch's time goes: B-topic C2 batches
through egm_match_submit / egm_match_wait one at a time (depth 1).  Run with
EGM_PIPE_TRACE=1 (host pipeline stamps on stderr) and/or under rocprofv3
--kernel-trace --memory-copy-trace (device timeline).

    python tools/batch_trace.py [batch] [batches] [filters]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402


def main():
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    nf = int(sys.argv[3]) if len(sys.argv) > 3 else 10_000_000
    from emqx_amd import _lib as L
    from emqx_amd import synth
    from emqx_amd.engine import GpuMatcher
    f = synth.config_filters("c2", n_filters=nf)
    t = synth.config_topics("c2", f, n_topics=16 * b)
    parts = [t.subset(np.arange(i * b, (i + 1) * b)) for i in range(16)]
    gm = GpuMatcher(0, max_batch=65536)
    gm.build(f.blob, f.off)
    for i in range(8):
        gm.wait(gm.submit(parts[i % 16].blob, parts[i % 16].off, L.EGM_MODE_ROUTES), copy=False)
    lat = []
    for i in range(nb):
        p = parts[i % 16]
        t0 = time.perf_counter()
        tk = gm.submit(p.blob, p.off, L.EGM_MODE_ROUTES)
        t1 = time.perf_counter()
        gm.wait(tk, copy=False)
        t2 = time.perf_counter()
        lat.append((t1 - t0, t2 - t1))
    a = np.array(lat) * 1e3
    print(f"batch {b}: submit p50 {np.median(a[:, 0]):.3f} ms, wait p50 {np.median(a[:, 1]):.3f} ms, "
          f"total p50 {np.median(a.sum(1)):.3f} ms", flush=True)
    gm.close()


if __name__ == "__main__":
    main()
