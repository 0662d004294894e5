"""Average / min duration (ms) of kernels matching the given names in
rocprofv3 --stats output dirs: python tools/kavg.py DIR [DIR ...] -k name1,name2"""
import csv
import sys

args = sys.argv[1:]
names = ["k_sort_pass", "k_sort_hist", "k_walk<false>", "k_rec_burst", "k_tokenise"]
if "-k" in args:
    i = args.index("-k")
    names = args[i + 1].split(",")
    args = args[:i] + args[i + 2:]
for d in args:
    try:
        rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
    except OSError as e:
        print(d, "missing", e)
        continue
    out = {}
    for r in rows:
        for k in names:
            if k in r["Name"]:
                out[k] = (int(r["Calls"]), round(float(r["AverageNs"]) / 1e6, 4), round(float(r["MinNs"]) / 1e6, 4))
    print(d, out)
