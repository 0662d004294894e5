"""Per-kernel PMC counter averages from rocprofv3 counter_collection CSVs.

    python tools/pmc_summary.py gpurun_out/pmc_tcc gpurun_out/pmc_sq ...
"""
import collections
import csv
import os
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = r["Kernel_Name"].split("(")[0].replace("egm::", "")
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    for (k, c), v in sorted(agg.items()):
        if k.startswith("k_") or "rand" in k:
            print(f"{os.path.basename(d):10s} {k:14s} {c:22s} {v / n[(k, c)]:16.4g}  (x{n[(k, c)]})")
