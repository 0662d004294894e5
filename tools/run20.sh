# Segmented tokenise + unrolled fan-out fill: GPU tests, C3 / C4(10M) / C2 under rocprof
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/ -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
run c3 420 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3 -o run --output-format csv -- python $R/bench.py --config c3 --steps 10 --warmup 2 --cpu-baseline off
run c4_10m 420 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4s -o run --output-format csv -- python $R/bench.py --config c4 --filters 10000000 --steps 10 --warmup 2 --cpu-baseline off
run c2 420 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2 -o run --output-format csv -- python $R/bench.py --steps 20 --warmup 3 --cpu-baseline off
