source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
run listc 120 rocprofv3 -L
B="python $R/bench.py --steps 2 --warmup 0 --cpu-baseline off"
run pmc_sq 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU -d $R/gpurun_out/pmc_sq -o run --output-format csv -- $B
run pmc_tcc 600 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU -d $R/gpurun_out/pmc_tcc -o run --output-format csv -- $B
run pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- $B
