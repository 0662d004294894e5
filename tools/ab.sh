# A/B of library variants on one box: tools/ab.sh "name1 name2 ..." [bench args]
source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
variants=$1; shift
for v in $variants; do
  if [ "$v" = cur ]; then lib=$R/emqx_amd/libemqx_gpu_match.so; else lib=$R/emqx_amd/libemqx_gpu_match_$v.so; fi
  EGM_LIB=$lib run ab_$v 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab/$v -o run --output-format csv -- python $R/bench.py --cpu-baseline off "$@"
done
