"""Summarise an A/B run: bench JSON lines and per-kernel average times.

    python tools/ab_summary.py gpurun_out cur occ16 pipe
"""
import csv
import json
import os
import sys

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for v in sys.argv[2:]:
    line = None
    for ln in open(os.path.join(out, f"ab_{v}.log")):
        if ln.startswith("{"):
            line = json.loads(ln)
    ks = {}
    p = os.path.join(out, "ab", v, "run_kernel_stats.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            ks[r["Name"].split("(")[0].replace("egm::", "")] = float(r["AverageNs"]) / 1e6
    if line:
        st = line["stats"]
        print(f"{v:8s} {line['value'] / 1e6:7.1f} M/s {line['ms_per_step']:6.2f} ms  walk {line['roofline']['kernel_ms']:.2f} "
              f"occ {st.get('walk_lane_occupancy', 0):.3f} def {st['deferred_chunks']} | "
              + " ".join(f"{k}={t:.2f}" for k, t in ks.items() if t > 0.05))
    else:
        print(v, "no result")
