"""Per-kernel durations over the timed window of a bench.py run under
`rocprofv3 --kernel-trace --stats`: the last K dispatches of each kernel
(bench.py's K timed steps), next to the all-dispatch average of the stats CSV
(which includes the untimed sizing and warm-up launches, the first of them
cold).  This is the figure to compare with the line's roofline.kernel_ms.

    python tools/trace_window.py gpurun_out/TAG_prof --steps 20 [--out profiles/x.json]
"""
import argparse
import csv
import json
import os
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out")
    a = ap.parse_args()
    per = defaultdict(list)
    with open(os.path.join(a.prof_dir, "run_kernel_trace.csv")) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"].split("(")[0]
            per[name].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = {}
    for name, d in per.items():
        d.sort()
        dur = [(e - s) / 1e6 for s, e in d]
        last = dur[-a.steps:]
        out[name] = {"dispatches": len(dur), "all_avg_ms": statistics.mean(dur),
                     f"last{len(last)}_avg_ms": statistics.mean(last), "last_min_ms": min(last),
                     "last_max_ms": max(last)}
    top = sorted(out.items(), key=lambda kv: -kv[1]["all_avg_ms"] * kv[1]["dispatches"])[:12]
    for name, v in top:
        print(f"{name[:48]:48s} n={v['dispatches']:4d} all {v['all_avg_ms']:.3f}  "
              f"timed {list(v.values())[2]:.3f} ms")
    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"source": a.prof_dir, "steps": a.steps, "kernels": dict(top)}, fh, indent=1)


if __name__ == "__main__":
    main()
