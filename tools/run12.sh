source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python $R/bench.py --steps 2 --warmup 0 --cpu-baseline off"
run pmc_tcc 600 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_tcc -o run --output-format csv -- $B
run pmc_sq 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU -d $R/gpurun_out/pmc_sq -o run --output-format csv -- $B
run pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- $B
run pmc_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- $B
run cal_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/cal_fetch -o run --output-format csv -- $R/tools/membench
run sorted 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab/sorted -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 2 --cpu-baseline off --x-presort
