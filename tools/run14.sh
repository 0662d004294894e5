# Incremental commit: full GPU test suite, then the route-churn benchmark on C2.
source tools/gpu_steps.sh
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -45 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
run updates 600 python tools/bench_updates.py
