"""Summarise a bench log (its JSON line) and the rocprof kernel stats beside it.
python tools/show.py gpurun_out/c2.log gpurun_out/prof_c2"""
import csv
import json
import sys

for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print(f"value {d['value'] / 1e6:.1f} M/s  ms/step {d['ms_per_step']:.3f}")
        print("roofline", {k: d["roofline"][k] for k in ("achieved", "frac", "kernel_ms", "traffic")})
        print("stats", d["stats"])
        if d.get("fanout"):
            print("fanout", d["fanout"])
        if d.get("cpu_baseline"):
            print("cpu", {k: d["cpu_baseline"][k] for k in ("value", "cores", "value_1thread")})
if len(sys.argv) > 2:
    for x in list(csv.DictReader(open(sys.argv[2] + "/run_kernel_stats.csv")))[:12]:
        print(f"  {x['Name'][:40]:40s} {x['Calls']:>4s} avg {float(x['AverageNs']) / 1e6:9.3f} "
              f"min {float(x['MinNs']) / 1e6:9.3f} ms {float(x['Percentage']):6.2f}%")
