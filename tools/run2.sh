source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
run pytest_gpu 420 python -m pytest tests/test_gpu_parity.py -m "gpu and not slow" -q
run bench_small 420 python bench.py --filters 1000000 --topics 2000000 --steps 10 --warmup 2 --cpu-baseline off
export TMPDIR=/tmp
run prof_small 420 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_small -o run --output-format csv -- python $R/bench.py --filters 1000000 --topics 2000000 --steps 5 --warmup 1 --cpu-baseline off
