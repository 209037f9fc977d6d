#!/bin/bash
# Round 3 ac: PlonK parity after the solo switch, then the default bench line
# (Groth16 and PlonK split projections).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-ac}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 600 pytest_${V}.txt python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_plonk_prove.py || exit 2
step 900 bench_${V}.json python3 -u bench.py || exit 2
echo done >> gpurun_out/progress_$V.txt
