# C1 (1M filters, 20% wildcard) under rocprof stats; the filter-shard path (RCCL broadcast + gather) at N=1
source tools/gpu_steps.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run c1_bench 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c1 -o run --output-format csv -- python $R/bench.py --config c1
run c2_shard1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --mode shard --steps 10 --warmup 2 --cpu-baseline off
