# Retained reverse match: GPU tests (new file first), then the full GPU suite.
source tools/gpu_steps.sh
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_retained.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_ret.log 2>&1; rc=$?; echo "retained rc=$rc"; tail -30 gpurun_out/pytest_ret.log
[ $rc -eq 0 ] || exit $rc
