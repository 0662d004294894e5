# C4 at full size: 100M filters, 10M-topic batch, match + subscriber fan-out, rocprof stats
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run c4_full 1100 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4 -o run --output-format csv -- python $R/bench.py --config c4 --steps 10 --warmup 2
