source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
run pytest_gpu 420 python -m pytest tests/test_gpu_parity.py -m "gpu and not slow" -q
run bench_full 900 python bench.py
export TMPDIR=/tmp
run prof_full 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_full -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 1 --cpu-baseline off
run pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 0 --cpu-baseline off
run pmc_write 900 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_write -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 0 --cpu-baseline off
