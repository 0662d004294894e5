source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python $R/bench.py --steps 2 --warmup 0 --cpu-baseline off"
run pmc_u 600 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_u -o run --output-format csv -- $B
run pmc_sq 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU -d $R/gpurun_out/pmc_sq -o run --output-format csv -- $B
for v in cur xcd; do
  if [ "$v" = cur ]; then lib=$R/emqx_amd/libemqx_gpu_match.so; else lib=$R/emqx_amd/libemqx_gpu_match_$v.so; fi
  EGM_LIB=$lib run sorted_$v 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab/s_$v -o run --output-format csv -- python $R/bench.py --cpu-baseline off --steps 10 --warmup 2 --x-presort
done
