source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python $R/bench.py --steps 2 --warmup 0 --cpu-baseline off"
run pmc_u 600 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_u -o run --output-format csv -- $B
run pmc_s 600 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_s -o run --output-format csv -- $B --x-presort
run bench_s 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bench_s -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 2 --cpu-baseline off --x-presort
