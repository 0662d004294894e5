"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes over bench.py into the
per-launch HBM traffic of the walk kernel, for bench.py's roofline.traffic.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write \
        --workload c2 --filters 10000000 --topics 10000000 --out profiles/r1_c2_walk_pmc.json

Units and corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB and count the L2's memory-side requests.  The guide's
x2 correction applies to wide coalesced streaming reads; the walk reads random
16-B pieces of 64-B lines, and tools/membench.hip run under the same counter
(gpurun_out/cal_fetch) shows FETCH_SIZE = 64 B per L2 miss for that shape
(67.1M random 64-B reads of a 16 MB table at a 76 % miss rate -> 3.27 GB),
so no factor is applied here.  Each counter is averaged over the k_walk
dispatches of one run (every dispatch matches the same batch).
"""
import argparse
import csv
import json
import os
import statistics


def per_dispatch(run_dir, counter, kernel="k_walk"):
    vals = []
    for r in csv.DictReader(open(os.path.join(run_dir, "run_counter_collection.csv"))):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]) * 1024.0)
    return vals


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
                  "(KiB x 1024; 64 B per L2 miss calibrated with tools/membench.hip)",
    }
    with open(a.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
