#!/bin/bash
# Round 3 an: distributed computeH without c's coset transform (linearity):
# distributed-H / multi-GPU parity incl. the 2^24 8-shard proof, then the
# split projection.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-an}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 900 pytest_${V}.txt python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dist_h.py tests/test_gpu_groth16_multi.py tests/test_gpu_groth16_size.py || exit 2
step 600 bench_${V}.json python3 -u bench.py --steps 4 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 \
  --plonk-log-n 0 --no-cpu-baseline --solver 0 || exit 2
echo done >> gpurun_out/progress_$V.txt
