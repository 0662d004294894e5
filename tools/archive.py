"""Copy a GPU job's bench line and rocprof kernel stats into profiles/.

    python tools/archive.py r2a_bench r2a_prof profiles/r2_c2_base
      -> profiles/r2_c2_base_bench.json, profiles/r2_c2_base_kernel_stats.csv
"""
import json
import os
import shutil
import sys

log, prof, dst = sys.argv[1:4]
line = None
for ln in open(os.path.join("gpurun_out", log + ".log")):
    if ln.startswith("{"):
        line = json.loads(ln)
if line is None:
    sys.exit(f"no JSON line in gpurun_out/{log}.log")
with open(dst + "_bench.json", "w") as fh:
    json.dump(line, fh, indent=1)
src = os.path.join("gpurun_out", prof, "run_kernel_stats.csv")
if os.path.exists(src):
    shutil.copy(src, dst + "_kernel_stats.csv")
print("archived", dst)
