#!/bin/bash
# Quick GPU iteration: MSM / Groth16 parity tests, then the default bench
# (headline only, no CPU baseline).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${TAG:-chk}"
T="${TESTS:-tests/test_gpu_msm.py tests/test_gpu_groth16.py tests/test_gpu_groth16_size.py}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$TAG.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$TAG.txt
  return $rc
}
if [ -n "$T" ] && [ "$T" != none ]; then
  step 900 pytest_$TAG.txt python -u -m pytest $T -x -v -s --timeout 600 --timeout-method thread || exit 2
fi
if [ -n "$BENCH" ]; then
  step 600 bench_$TAG.json python3 -u bench.py $BENCH || exit 2
fi
if [ -n "$PROF" ]; then
  step 400 prof_$TAG.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py $PROF || exit 2
fi
echo done >> gpurun_out/progress_$TAG.txt
