"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes over bench.py into the
per-launch HBM traffic of the walk kernel, for bench.py's roofline.traffic.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write \
        --workload c2 --filters 10000000 --topics 10000000 --out profiles/r1_c2_walk_pmc.json

Units and corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB and count the L2's memory-side requests.  The guide's
x2 correction applies to reads of whole 128-B lines (a 128-B request is
tallied at 64 B).  The walk reads 64-B halves of its 128-B edge buckets and
16-B node records, and tools/granule.hip measured that shape on MI355X
(profiles/r3_granule.json): a random read of 16, 32 or 64 B costs one 64-B
fetch and FETCH_SIZE counts it at exactly 64 B (67.1M reads -> 4.26-4.29 GB
for each width), the memory system serves ~50 G such requests/s whatever the
width, and a whole 128-B line takes ~1.7x the time of a 64-B half but is
counted at 64 B.  So the granule is 64 B and no factor applies to the walk.
Each counter is the median over the k_walk dispatches of one run (every
dispatch matches the same batch).
"""
import argparse
import csv
import json
import os
import statistics


def per_dispatch(run_dir, counter):
    """Per walk launch: the first pass (k_walk<false>) plus the deep pass that
    follows it on the stream (k_walk<true>, the chunks of more than DEEP_MIN
    levels; empty at C2), paired in dispatch order."""
    first, deep = [], []
    rows = list(csv.DictReader(open(os.path.join(run_dir, "run_counter_collection.csv"))))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    acc = {}
    for r in rows:
        if "k_walk" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            k = (int(r["Dispatch_Id"]), "k_walk<true>" in r["Kernel_Name"])
            acc[k] = acc.get(k, 0.0) + float(r["Counter_Value"]) * 1024.0
    for (d, is_deep), v in sorted(acc.items()):
        (deep if is_deep else first).append(v)
    if deep and len(deep) == len(first):
        return [a + b for a, b in zip(first, deep)]
    return first


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--filters", type=int, required=True)
    ap.add_argument("--topics", type=int, required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    f = per_dispatch(a.fetch_dir, "FETCH_SIZE")
    w = per_dispatch(a.write_dir, "WRITE_SIZE")
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_src_sha
    rec = {
        "kernel": "k_walk", "workload": a.workload, "filters": a.filters, "topics": a.topics,
        "kernel_src_sha": kernel_src_sha(),
        "fetch_bytes_per_launch": statistics.median(f), "write_bytes_per_launch": statistics.median(w),
        "dispatches": [len(f), len(w)],
        "traffic_bytes_per_launch": statistics.median(f) + statistics.median(w),
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py "
                  "(KiB x 1024; no x2: random reads of <= 64 B are one 64-B fetch each, counted exactly, "
                  "tools/granule.hip, profiles/r3_granule.json)",
        "granule_bytes": 64,
    }
    with open(a.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
