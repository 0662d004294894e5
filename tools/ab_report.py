"""Summarise tools/ab.sh output: per variant, bench value and per-kernel avg time."""
import csv, glob, json, os, sys
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for d in sorted(glob.glob(os.path.join(root, "ab", "*"))):
    v = os.path.basename(d)
    line = None
    try:
        for l in open(os.path.join(root, f"ab_{v}.log")):
            if l.startswith("{"):
                line = json.loads(l)
    except OSError:
        pass
    ks = {}
    for f in glob.glob(os.path.join(d, "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Name"].split("(")[0].replace("egm::", "")
            ks[name] = float(r["AverageNs"]) / 1e3
    val = f"{line['value']/1e6:8.1f}M/s ms/step={line['ms_per_step']:.2f} defer={line['stats']['deferred_chunks']}" if line else "n/a"
    parts = " ".join(f"{k}={ks[k]:.0f}us" for k in ("k_walk", "k_tokenise", "k_compact", "k_heavy") if k in ks)
    print(f"{v:8s} {val} {parts}")
