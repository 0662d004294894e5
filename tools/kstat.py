"""Median per-kernel duration (ms) from a rocprofv3 kernel trace, over the
dispatches of the bench's timed steps only (the ones before the pipelined leg
overlap two streams): python tools/kstat.py gpurun_out/TAG_prof_V [...]"""
import collections
import csv
import statistics
import sys

KEYS = ("k_walk<true>", "k_walk", "k_tokenise", "k_compact_fix", "k_compact(", "k_scan", "onesweep", "k_heavy", "k_fan")

for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    walks = [i for i, r in enumerate(rows) if "k_walk" in r["Kernel_Name"] and "k_walk<true>" not in r["Kernel_Name"]]
    # the first 2/3 of the walk launches: sizing, warm-up and the timed steps, before the pipelined leg
    cut = rows[walks[int(len(walks) * 2 / 3)]]["Start_Timestamp"] if len(walks) > 6 else None
    per = collections.defaultdict(list)
    for r in rows:
        if cut and int(r["Start_Timestamp"]) >= int(cut):
            break
        name = r["Kernel_Name"]
        key = next((k for k in KEYS if k in name), None) or ("sort" if "rocprim" in name else None)
        if key:
            per[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print(d, {k: round(statistics.median(v), 3) for k, v in sorted(per.items())})
