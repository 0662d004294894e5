# Retained: tests, bench, rocprof stats after the segmented range count
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_retained.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ret.log 2>&1; rc=$?; echo "retained rc=$rc"; tail -5 gpurun_out/pytest_ret.log
[ $rc -eq 0 ] || exit $rc
run retained 600 python tools/bench_retained.py
run retained_prof 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ret -o run --output-format csv -- python $R/tools/bench_retained.py --steps 3 --cpu-seconds 1
