#!/bin/bash
# Round-2 validation: the GPU R1CS solver tests (gg_r1cs_*).
# Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-p}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 240 pytest_blsg16_$V.txt python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bls_groth16.py || exit 2
echo done >> gpurun_out/progress_$V.txt
