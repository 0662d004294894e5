# A/B: compaction grid at C2, bigger walk stack at C3
source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in b32k b64k b32k16; do
  EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run ab_$v 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab/$v -o run --output-format csv -- python $R/bench.py --cpu-baseline off --steps 10 --warmup 2
done
for v in cur st640 st1024; do
  if [ "$v" = cur ]; then lib=$R/emqx_amd/libemqx_gpu_match.so; else lib=$R/emqx_amd/libemqx_gpu_match_$v.so; fi
  EGM_LIB=$lib run ab_c3_$v 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab/c3_$v -o run --output-format csv -- python $R/bench.py --cpu-baseline off --config c3 --steps 5 --warmup 1
done
