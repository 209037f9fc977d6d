#!/bin/bash
# Round 5 z4: the driver's bench command on the final tree once more (another box).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05z4}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 600 bench_$V.json python3 -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 2
echo done >> gpurun_out/progress_$V.txt
