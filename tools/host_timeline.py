"""Summarise the host path's timeline (tools/job.sh host_trace: rocprofv3
--kernel-trace --memory-copy-trace over tools/bench_host.py): for the batches
of the last in-flight phase, each match kernel's median time alone and beside
a result D2H (copy-out kernel or DMA copy), and the batch period.

    python tools/host_timeline.py gpurun_out/TAG_host_trace [label] > profiles/rN_host_trace.json
"""
import csv
import json
import os
import statistics
import sys

d = sys.argv[1]
label = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(d)
K = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
mp = os.path.join(d, "run_memory_copy_trace.csv")
M = list(csv.DictReader(open(mp))) if os.path.exists(mp) else []


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("egm::", "")
    return "sort" if ("rocprim" in n or "cub" in n) else n


ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in K]
ms = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"]) for r in M]
# the result's D2H intervals: copy-out kernels, or device->host DMA copies of more than 1 MB' worth of time
d2h = [(a, b) for a, b, n in ks if n == "k_copy_out"]
d2h += [(a, b) for a, b, dr in ms if "DEVICE_TO_HOST" in dr and b - a > 100_000]
d2h.sort()


def overlaps(a, b):
    return any(x < b and a < y for x, y in d2h)


per = {}
for a, b, n in ks:
    if n == "k_copy_out":
        continue
    key = (n, overlaps(a, b))
    per.setdefault(key, []).append((b - a) / 1e6)
walk = sorted(a for a, b, n in ks if n == "k_walk<false>")
period = statistics.median([y - x for x, y in zip(walk[-8:], walk[-7:])]) / 1e6 if len(walk) > 8 else None
out = {"trace": label, "batch_period_ms_last_phase": period,
       "d2h_ms_median": statistics.median([(b - a) / 1e6 for a, b in d2h]) if d2h else None,
       "kernels": {f"{n} ({'beside D2H' if o else 'alone'})": {"median_ms": round(statistics.median(v), 4),
                                                                "launches": len(v)}
                   for (n, o), v in sorted(per.items()) if statistics.median(v) > 0.02}}
print(json.dumps(out, indent=1))
