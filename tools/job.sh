#!/bin/bash
# One parameterised GPU job for gpurun (replaces the per-lease run*.sh files).
#
#   gpurun --timeout 1200 -- 'bash tools/job.sh TAG step [step ...]'
#
# Steps (each under its own time limit, logs in gpurun_out/TAG_<step>.log):
#   tests      pytest -m gpu, fast tests only (not the full-size ones)
#   scale      pytest -m "gpu and slow": the full-size C1/C2/C3/C4 parity tests
#   bench      bench.py C2 under rocprofv3 --stats -> gpurun_out/TAG_prof (host leg off: the
#              rocprof averages are then over the 10M-topic launches only)
#   drv        the driver's command as is (python bench.py --gpus 1 --steps 20 --warmup 5)
#   bench_sK   the C2 bench with K streams (bench_s1: no overlap of consecutive batches)
#   bench_c1|bench_c3|bench_c4   the other configs under rocprofv3 --stats
#   shard1     bench.py --mode shard at world 1 via torch.distributed.run
#   prefix1    bench.py --mode prefix (root-word partitions, one all_to_all) at world 1
#   pmc        FETCH_SIZE and WRITE_SIZE passes over the C2 bench (one counter per pass)
#   sq         SQ wait/active counters + TCC hit/miss over the C2 bench
#   host       host-visible path (egm_match_batch, pinned staging) bench
#   host_trace the same under rocprofv3 --kernel-trace --memory-copy-trace (timeline)
#   s2         the C2 bench with two streams (consecutive batches overlap), then sorted / input order
#   orders     the C2 bench, then the walk-order A/B (sort key shapes) in the same process
#   smoke      __graft_entry__.smoke()
#   c4m, c4m_V C4's shape at 10M filters (match + fan-out), default library / variant V
#   ab_V       the C2 bench on variant V (emqx_amd/libemqx_gpu_match_V.so, tools/build_variant.py)
# An ordinary failure (exit 1..5) moves on; a fault, abort or timeout ends the job.
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python $R/bench.py"

run() {
  local name=$1 secs=$2; shift 2
  local log="gpurun_out/${TAG}_$name.log"
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -n 4 "$log"
  # a device fault surfaces as an ordinary Python exception (exit 1): stop there too
  if grep -q -E "illegal memory access|hipErrorIllegalAddress|Memory access fault|HSA_STATUS_ERROR" "$log"; then
    echo "FATAL: $name hit a GPU fault — stopping"; exit 99
  fi
  case $rc in
    0|1|2|3|4|5) return 0 ;;
    *) echo "FATAL: $name exited $rc — stopping"; exit $rc ;;
  esac
}

for step in "$@"; do
  case $step in
    tests) run tests 900 python -u -m pytest tests -m "gpu and not slow" -x -v --timeout 300 --timeout-method thread ;;
    prefixdiag) run prefixdiag 1150 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread -k "not slow or eight_prefix" ;;
    slowrest) run slowrest 900 python -u -m pytest tests -m "gpu and slow" -x -q --timeout 600 --timeout-method thread -k "not TestC2Full" ;;
    c2full) run c2full 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k TestC2Full ;;
    gpuall) run gpuall 1150 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread --durations=15 ;;   # the driver's whole GPU tier
    scale) run scale 1100 python -u -m pytest tests -m "gpu and slow" -x -v --timeout 600 --timeout-method thread ;;
    bench) run bench 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run --output-format csv -- $B --steps 20 --warmup 5 --host-e2e off --pipelined off ;;
    drv) run drv 600 python $R/bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench_presort[0-9])
      k=${step#bench_presort}
      run "$step" 900 python $R/bench.py --steps 10 --warmup 2 --streams 1 --x-presort "$k" --cpu-baseline off ;;
    bench_s[0-9])
      k=${step#bench_s}
      run "$step" 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof_s$k" -o run --output-format csv -- $B --steps 20 --warmup 5 --streams "$k" --cpu-baseline off --host-e2e off ;;
    bench_c1|bench_c3|bench_c4)
      cfg=${step#bench_}
      run "$step" 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof_$cfg" -o run --output-format csv -- $B --config "$cfg" --steps 10 --warmup 2 --host-e2e off --pipelined off ;;
    shardfan) run shardfan 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --config c4 --filters 2000000 --topics 1000000 --mode shard --steps 5 --warmup 1 --cpu-baseline off ;;
    shardleg) run shardleg 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29535 bench.py --sharded-leg on --steps 5 --warmup 1 --cpu-baseline off --host-e2e off --pipelined off ;;
    slowd) run slowd 1100 python -u -m pytest tests -m "gpu and slow" -x -v --timeout 900 --timeout-method thread --durations=0 ;;
    prefix1) run prefix1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29536 bench.py --mode prefix --steps 10 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off ;;
    shard1) run shard1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --mode shard --steps 10 --warmup 2 --cpu-baseline off ;;
    pmc)
      run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/${TAG}_pmc_fetch" -o run --output-format csv -- $B --steps 3 --warmup 0 --cpu-baseline off --host-e2e off --pipelined off
      run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/${TAG}_pmc_write" -o run --output-format csv -- $B --steps 3 --warmup 0 --cpu-baseline off --host-e2e off --pipelined off ;;
    pmc_c3)   # FETCH_SIZE / WRITE_SIZE passes over the C3 bench (depth 16, the deep pass)
      run pmc_c3_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/${TAG}_pmc_c3_fetch" -o run --output-format csv -- $B --config c3 --steps 2 --warmup 0 --cpu-baseline off --host-e2e off --pipelined off
      run pmc_c3_write 600 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/${TAG}_pmc_c3_write" -o run --output-format csv -- $B --config c3 --steps 2 --warmup 0 --cpu-baseline off --host-e2e off --pipelined off ;;
    pmc_c4)   # FETCH_SIZE / WRITE_SIZE passes over the C4 bench (100M filters, match + fan-out)
      run pmc_c4_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/${TAG}_pmc_c4_fetch" -o run --output-format csv -- $B --config c4 --steps 2 --warmup 0 --cpu-baseline off --host-e2e off --pipelined off
      run pmc_c4_write 600 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/${TAG}_pmc_c4_write" -o run --output-format csv -- $B --config c4 --steps 2 --warmup 0 --cpu-baseline off --host-e2e off --pipelined off ;;
    sq)
      run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU -d "$R/gpurun_out/${TAG}_pmc_sq" -o run --output-format csv -- $B --steps 3 --warmup 0 --cpu-baseline off --host-e2e off
      run pmc_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$R/gpurun_out/${TAG}_pmc_tcc" -o run --output-format csv -- $B --steps 3 --warmup 0 --cpu-baseline off --host-e2e off ;;
    sq_c3)   # SQ + TCC counter passes over the C3 bench (the deep pass)
      run pmc_c3_sq 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU -d "$R/gpurun_out/${TAG}_pmc_c3_sq" -o run --output-format csv -- $B --config c3 --steps 2 --warmup 0 --cpu-baseline off --host-e2e off --pipelined off
      run pmc_c3_tcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$R/gpurun_out/${TAG}_pmc_c3_tcc" -o run --output-format csv -- $B --config c3 --steps 2 --warmup 0 --cpu-baseline off --host-e2e off --pipelined off ;;
    sq_*)   # SQ + TCC counter passes over the C2 bench on variant V
      v=${step#sq_}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "pmc_sq_$v" 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU -d "$R/gpurun_out/${TAG}_pmc_sq_$v" -o run --output-format csv -- $B --steps 3 --warmup 0 --cpu-baseline off --host-e2e off --pipelined off
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "pmc_tcc_$v" 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$R/gpurun_out/${TAG}_pmc_tcc_$v" -o run --output-format csv -- $B --steps 3 --warmup 0 --cpu-baseline off --host-e2e off --pipelined off
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "pmc_sq2_$v" 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_SMEM -d "$R/gpurun_out/${TAG}_pmc_sq2_$v" -o run --output-format csv -- $B --steps 3 --warmup 0 --cpu-baseline off --host-e2e off --pipelined off ;;
    host) run host 600 python tools/bench_host.py ;;
    batcher) run batcher 600 python tools/bench_batcher.py ;;
    btrace)   # one small batch at a time: host pipeline stamps, then the device timeline
      EGM_PIPE_TRACE=1 run btrace 300 python tools/batch_trace.py 4096 200
      run btrace_k 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$R/gpurun_out/${TAG}_btrace_k" -o run --output-format csv -- python tools/batch_trace.py 4096 200 ;;
    host_ptrace) EGM_PIPE_TRACE=1 run host_ptrace 600 python tools/bench_host.py ;;   # pipeline events on stderr
    hostpk) run hostpk 600 python tools/bench_host.py --packed ;;   # the packed result form (EGM_RESULT_PACKED)
    hostpk_ptrace) EGM_PIPE_TRACE=1 run hostpk_ptrace 600 python tools/bench_host.py --packed --batches 12 ;;
    hostpk_*)  # the packed host path on variant V
      v=${step#hostpk_}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "$step" 600 python tools/bench_host.py --packed ;;
    host_hip) EGM_PIPE_COPY=hip run host_hip 600 python tools/bench_host.py ;;   # A/B: hipMemcpyAsync (blit kernel)
    host_k) EGM_PIPE_COPY=kernel run host_k 600 python tools/bench_host.py ;;   # A/B: the copy-out kernel
    host_trace)   # the host path's timeline: kernels and copies (no counters)
      run host_trace 600 rocprofv3 --kernel-trace --memory-copy-trace -d "$R/gpurun_out/${TAG}_host_trace" -o run --output-format csv -- python tools/bench_host.py --batches 10 ;;
    host_*)  # the host-visible path on variant V
      v=${step#host_}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "$step" 600 python tools/bench_host.py ;;
    s2) run s2 400 python $R/bench.py --steps 20 --warmup 3 --streams 2 --cpu-baseline off --host-e2e off --x-orders "a86,0" ;;
    orders4) run orders4 500 python $R/bench.py --steps 10 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off --x-orders "a86,68a8,8a86,a86,68a8,8a86,9a8" ;;
    orders5) run orders5 600 python $R/bench.py --steps 10 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off --x-orders "8a86,a886,88a6,8a95,6a88,7a87,8a86,7a96,8b75" ;;
    orders7) run orders7 600 python $R/bench.py --steps 10 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off --x-orders "7764,4444,5542,4453,3355,7764,6622" ;;   # 16-bit keys: 2 sort passes (round 6)
    orders8) run orders8 600 python $R/bench.py --steps 10 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off --x-orders "7764,8888,6a88,8a86,7764,9887,7864" ;;   # 32-bit keys: 4 sort passes (round 6)
    orders6) run orders6 600 python $R/bench.py --steps 10 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off --x-orders "8a86,a86,6864,8862,6666,7764,8a86" ;;   # 24-bit keys: 3 sort passes
    orders) run orders 400 python $R/bench.py --steps 10 --warmup 2 --cpu-baseline off --host-e2e off --x-orders "a86,0,a86/128,a86" ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    granule)   # random-read granule (tools/granule.hip): timing, then FETCH_SIZE per kernel
      run granule 120 "$R/tools/granule"
      run granule_pmc 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_granule_pmc" -o run --output-format csv -- "$R/tools/granule" ;;
    granule_tcc)   # L2 requests per read (lanes sharing a line: merged or not?)
      run granule 120 "$R/tools/granule"
      run granule_tcc 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$R/gpurun_out/${TAG}_granule_tcc" -o run --output-format csv -- "$R/tools/granule" ;;
    walkmix)   # what bounds the walk: its memory mix with 0-600 VALU per round at 8-32 waves per CU (tools/walkmix.hip)
      run walkmix 300 "$R/tools/walkmix" ;;
    walkmix2)  # the same with the walk's measured 68 L2 requests per iteration and its flush stores
      run walkmix2 300 "$R/tools/walkmix" 2 ;;
    d2h)   # device <-> pinned host copy rates (tools/d2hbench.hip)
      run d2h 120 "$R/tools/d2hbench" ;;
    bench_c4_in) EGM_FAN_ORDER=input run bench_c4_in 900 python $R/bench.py --config c4 --steps 10 --warmup 2 --host-e2e off --pipelined off --cpu-baseline off ;;   # A/B: fan-out count in input order
    c4m) run c4m 400 python $R/bench.py --config c4 --filters 10000000 --steps 5 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off ;;
    c4m_*)  # the same on variant V (tools/build_variant.py)
      v=${step#c4m_}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "$step" 400 python $R/bench.py --config c4 --filters 10000000 --steps 5 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off ;;
    c4_*)   # full C4 (100M filters, match + fan-out) on variant V
      v=${step#c4_}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "$step" 900 python $R/bench.py --config c4 --steps 10 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off ;;
    c3_*)   # C3 on variant V (tools/build_variant.py)
      v=${step#c3_}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "$step" 600 python $R/bench.py --config c3 --steps 5 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off ;;
    c3base) run c3base 600 python $R/bench.py --config c3 --steps 5 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off ;;
    tests_*)   # the fast GPU tests on variant V
      v=${step#tests_}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "$step" 900 python -u -m pytest tests -m "gpu and not slow" -x -v --timeout 300 --timeout-method thread ;;
    abnp_*)   # A/B variant, single-stream steps only (rocprof averages over the timed launches alone)
      v=${step#abnp_}; v=${v%%.*}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "$step" 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_profnp_${step#abnp_}" -o run --output-format csv -- $B --steps 20 --warmup 3 --cpu-baseline off --host-e2e off --pipelined off ;;
    c3np_*)   # C3 on variant V under rocprof stats (single-stream steps)
      v=${step#c3np_}; v=${v%%.*}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "$step" 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_profc3_${step#c3np_}" -o run --output-format csv -- $B --config c3 --steps 5 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off ;;
    abx_*)   # A/B variant, second sample (own log/prof names)
      v=${step#abx_}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "abx_$v" 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_profx_$v" -o run --output-format csv -- $B --steps 10 --warmup 2 --cpu-baseline off --host-e2e off ;;
    sort)   # the walk-order sort alone (tools/sort_bench.py) under rocprof stats
      run sort 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_sort" -o run --output-format csv -- python $R/tools/sort_bench.py ;;
    sort_*)   # the same on variant V
      v=${step#sort_}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "$step" 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_sort_$v" -o run --output-format csv -- python $R/tools/sort_bench.py ;;
    ab_*)   # A/B variant built by tools/build_variant.py: C2 bench under rocprof stats
      v=${step#ab_}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "$step" 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof_$v" -o run --output-format csv -- $B --steps 10 --warmup 2 --cpu-baseline off --host-e2e off ;;
    c3ab_*)   # the C3 bench line (no profiler) on variant V (c3ab_default: the default library)
      v=${step#c3ab_}
      lib=$R/emqx_amd/libemqx_gpu_match_$v.so; [ "$v" = default ] && lib=$R/emqx_amd/libemqx_gpu_match.so
      EGM_LIB=$lib run "$step" 900 $B --config c3 --steps 10 --warmup 2 --cpu-baseline off --host-e2e off --pipelined off ;;
    pmcw_*)   # WRITE_SIZE pass over the C2 bench on variant V
      v=${step#pmcw_}
      EGM_LIB=$R/emqx_amd/libemqx_gpu_match_$v.so run "$step" 300 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/${TAG}_pmc_write_$v" -o run --output-format csv -- $B --steps 3 --warmup 0 --cpu-baseline off --host-e2e off --pipelined off ;;
    chunkhist) run chunkhist 600 env PYTHONPATH=$R python $R/tools/chunk_hist.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$(date +%T)] job $TAG done"
