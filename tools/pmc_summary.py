"""Per-kernel means of rocprofv3 --pmc passes: python tools/pmc_summary.py TAG > profiles/X.txt
(reads gpurun_out/TAG_pmc_*/run_counter_collection.csv)."""
import collections
import csv
import glob
import os
import sys

tag = sys.argv[1]
root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
for d in sorted(glob.glob(os.path.join(root, f"{tag}_pmc_*"))):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(lambda: [0.0, 0])
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"].split("(")[0].replace("egm::", "").replace("void ", ""), r["Counter_Name"])
            acc[k][0] += float(r["Counter_Value"])
            acc[k][1] += 1
        for (kn, cn), (v, c) in sorted(acc.items()):
            if kn.startswith("k_"):
                print(f"{os.path.basename(d)[len(tag) + 1:]:10s} {kn:14s} {cn:22s} {v / max(1, c):12.4g}  (mean of {c})")
