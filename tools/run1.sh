source tools/gpu_steps.sh
run pytest_gpu 420 python -m pytest tests/test_gpu_parity.py -m "gpu and not slow" -q -x
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
run bench_small 420 python bench.py --filters 1000000 --topics 2000000 --steps 10 --warmup 2 --cpu-seconds 5
