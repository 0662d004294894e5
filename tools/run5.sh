source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
run bench_sorted 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sorted -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 1 --cpu-baseline off --x-presort
