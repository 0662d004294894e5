# Fan-out (wave-cooperative fill): GPU tests, C4-shape bench at 10M filters under rocprof, C3 bench
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fanout" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fan.log 2>&1; rc=$?; echo "pytest fan rc=$rc"; tail -5 gpurun_out/pytest_fan.log
[ $rc -eq 0 ] || exit $rc
run c4_10m 420 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4s -o run --output-format csv -- python $R/bench.py --config c4 --filters 10000000 --steps 10 --warmup 2
run c3 420 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3 -o run --output-format csv -- python $R/bench.py --config c3 --steps 10 --warmup 2 --cpu-seconds 8
