"""Per-kernel average durations from a rocprofv3 kernel trace, split into
consecutive phases (e.g. a bench's timed steps and a later leg): prints the
kernel-name -> ms table for each run of calls between two launches of the
marker kernel.  Usage: python tools/ktrace_split.py TRACE.csv [marker]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_walk<false>"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    phases, cur = [], []
    for r in rows:
        if marker in r["Kernel_Name"] and cur and any(marker in x["Kernel_Name"] for x in cur):
            phases.append(cur)
            cur = []
        cur.append(r)
    phases.append(cur)
    # one "step" per marker: print per-step kernel times, grouped into runs of equal kernel sets
    for i, ph in enumerate(phases):
        d = defaultdict(float)
        for r in ph:
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
            d[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        span = (int(ph[-1]["End_Timestamp"]) - int(ph[0]["Start_Timestamp"])) / 1e6
        print(f"step {i:3d} span {span:7.3f} ms  " + "  ".join(f"{k}={v:.3f}" for k, v in sorted(d.items(), key=lambda x: -x[1])[:6]))


if __name__ == "__main__":
    main()
