# Retained-match bench (+ rocprof kernel stats) and the route-churn bench
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run retained 600 python tools/bench_retained.py
run retained_prof 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ret -o run --output-format csv -- python $R/tools/bench_retained.py --steps 3 --cpu-seconds 1
run updates 600 python tools/bench_updates.py
