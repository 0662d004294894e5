# Hybrid fan-out fill: fan-out tests, C4 at 10M and at the full 100M filters under rocprof
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fanout" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_fan.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_fan.log
[ $rc -eq 0 ] || exit $rc
run c4_10m 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4s -o run --output-format csv -- python $R/bench.py --config c4 --filters 10000000 --steps 10 --warmup 2 --cpu-baseline off
run c4_full 1000 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4 -o run --output-format csv -- python $R/bench.py --config c4 --steps 10 --warmup 2
