"""Summarise an A/B job (tools/job.sh ab_V steps): the bench line and the
rocprof per-kernel median launch times of each variant, one JSON object per variant.

    python tools/ab_summary.py TAG V [V ...] [--flags V=-DX=1,...] > profiles/rN_walk_ab.jsonl

reads gpurun_out/TAG_ab_V.log and gpurun_out/TAG_prof_V/run_kernel_trace.csv.
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(ROOT, "gpurun_out")
args = sys.argv[1:]
flags = {}
if "--flags" in args:
    i = args.index("--flags")
    for kv in args[i + 1].split(";"):
        k, _, v = kv.partition("=")
        flags[k] = v
    args = args[:i] + args[i + 2:]
tag, variants = args[0], args[1:]
for v in variants:
    line = None
    log = os.path.join(out, f"{tag}_ab_{v}.log")
    if os.path.exists(log):
        for ln in open(log):
            if ln.startswith("{"):
                line = json.loads(ln)
    # per-kernel MEDIAN launch time from the trace: the bench's extra legs (two
    # batches in flight) stretch some launches, and the stats file averages them in
    runs = {}
    p = os.path.join(out, f"{tag}_prof_{v}", "run_kernel_trace.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("egm::", "")
            if "rocprim" in name or "cub" in name:
                name = "sort:" + r["Kernel_Name"]
            runs.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    ks = {k: round(statistics.median(x), 4) for k, x in runs.items() if not k.startswith("sort:")}
    nw = len(runs.get("k_walk<false>", [])) or 1   # the sort's passes: median x launches per walk
    srt = sum(statistics.median(x) * len(x) / nw for k, x in runs.items() if k.startswith("sort:"))
    if srt:
        ks["sort (all passes)"] = round(srt, 4)
    rec = {"tag": tag, "variant": v, "flags": flags.get(v, "")}
    if line:
        rec.update({"topics_per_s": line["value"], "ms_per_step": line["ms_per_step"],
                    "k_walk_ms_events": line["roofline"]["kernel_ms"], "kernel_src_sha": line["roofline"].get("kernel_src_sha")})
    else:
        rec["result"] = None
    rec["rocprof_median_ms"] = {k: t for k, t in ks.items() if t > 0.02}
    print(json.dumps(rec))
