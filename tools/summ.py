"""Summarise a tools/job.sh run: test tallies, bench lines and k_walk/k_compact
times per step.   python tools/summ.py TAG"""
import csv
import glob
import json
import os
import sys

tag = sys.argv[1]
out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
for log in sorted(glob.glob(os.path.join(out, f"{tag}_*.log"))):
    step = os.path.basename(log)[len(tag) + 1:-4]
    lines = open(log, errors="replace").read().splitlines()
    tally = [l for l in lines if " passed" in l or " failed" in l or "FAILED" in l or "Error" in l]
    js = [l for l in lines if l.startswith("{")]
    msg = ""
    if js:
        try:
            d = json.loads(js[-1])
            if "stats" in d:
                s = d["stats"]
                msg = "value %.1fM  walk %.2f ms  iters %s bounded %s occ %.3f" % (
                    d["value"] / 1e6, d["roofline"]["kernel_ms"], s.get("walk_iters"), s.get("walk_bounded_pops"),
                    s.get("walk_lane_occupancy") or 0)
            else:
                msg = js[-1][:300]
        except Exception as e:  # noqa: BLE001
            msg = f"bad json: {e}"
    print(f"{step:12s} {msg}")
    for t in tally[-3:]:
        print("    ", t[:200])
for d in sorted(glob.glob(os.path.join(out, f"{tag}_prof*"))):
    f = os.path.join(d, "run_kernel_stats.csv")
    if os.path.exists(f):
        ks = {r["Name"].split("(")[0].replace("egm::", ""): float(r["AverageNs"]) / 1e6 for r in csv.DictReader(open(f))}
        print(f"{os.path.basename(d):22s}", "  ".join(f"{k} {v:.3f}" for k, v in ks.items() if k.startswith("k_")))
