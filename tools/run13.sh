# Round-1 evidence run: parity, full bench (with CPU baseline) under rocprof
# stats, separate FETCH_SIZE / WRITE_SIZE passes for the walk's traffic.
source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 420 python -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m "gpu and not slow" -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_full 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_full -o run --output-format csv -- python $R/bench.py
B="python $R/bench.py --steps 2 --warmup 0 --cpu-baseline off"
run pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- $B
run pmc_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- $B
run pmc_tcc 600 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_tcc -o run --output-format csv -- $B
