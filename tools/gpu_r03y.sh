#!/bin/bash
# Round 3 y: PlonK (parallel scan power tables) parity and timing; BLS12-381
# Groth16 incl. bucket stripes.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-y}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 900 pytest_${V}.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_plonk_poly.py tests/test_gpu_plonk_prove.py tests/test_gpu_bls_groth16.py ${PYTEST_ARGS} || exit 2
step 600 plonk_${V}.json python3 -u tools/bench_plonk.py 22 4 || exit 2
echo done >> gpurun_out/progress_$V.txt
