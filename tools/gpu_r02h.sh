#!/bin/bash
# Round-2 v14 bench: the default bench.py (headline + extras incl. the GPU R1CS
# solver), then a rocprofv3 kernel-trace summary of the solver + prove pipeline.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-h}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 700 bench_$V.json python3 -u bench.py || exit 2
echo done >> gpurun_out/progress_$V.txt
