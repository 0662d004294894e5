source tools/gpu_steps.sh
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 420 python -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m "gpu and not slow" -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-cur occ16n occ20 occ20n occ24n}; do
  if [ "$v" = cur ]; then lib=$R/emqx_amd/libemqx_gpu_match.so; else lib=$R/emqx_amd/libemqx_gpu_match_$v.so; fi
  EGM_LIB=$lib run ab_$v 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab/$v -o run --output-format csv -- python $R/bench.py --cpu-baseline off --steps 10 --warmup 2
done
