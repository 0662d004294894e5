# A/B: compaction grid 131072, tokenise 20 KB staging, against the current build (C2)
source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in cur b128k tokC; do
  if [ "$v" = cur ]; then lib=$R/emqx_amd/libemqx_gpu_match.so; else lib=$R/emqx_amd/libemqx_gpu_match_$v.so; fi
  EGM_LIB=$lib run ab_$v 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab/$v -o run --output-format csv -- python $R/bench.py --cpu-baseline off --steps 10 --warmup 2
done
