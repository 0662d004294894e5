source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 420 python -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m "gpu and not slow" -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
run bench_cur 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab/cur -o run --output-format csv -- python $R/bench.py --cpu-baseline off --steps 10 --warmup 2
