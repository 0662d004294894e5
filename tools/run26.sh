# After the compaction-grid change: GPU parity tests, smoke, default bench (C2) under rocprof stats
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run c2_bench 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2b -o run --output-format csv -- python $R/bench.py
