#!/bin/bash
# Run GPU steps one after another; each has its own time limit.  An ordinary
# failure (exit 1..5) moves on; a fault, abort or timeout ends the script.
mkdir -p gpurun_out
run() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -n 3 "gpurun_out/$name.log"
  case $rc in
    0|1|2|3|4|5) return 0 ;;
    *) echo "FATAL: $name exited $rc — stopping"; exit $rc ;;
  esac
}
