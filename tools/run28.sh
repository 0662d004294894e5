# After the tokenise LDS change: GPU parity tests, smoke, C2 bench under rocprof, C3 bench
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run c2_bench 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2c -o run --output-format csv -- python $R/bench.py
run c3_bench 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3c -o run --output-format csv -- python $R/bench.py --config c3 --steps 5 --warmup 1
