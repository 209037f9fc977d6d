#!/bin/bash
# Round-2: GPU R1CS solver tests (strand + level schedules), then the headline
# bench with the solver extra only.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-k}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 300 pytest_solver_$V.txt python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_solver.py || exit 2
step 300 bench_solver_$V.json python3 -u bench.py --steps 3 --warmup 1 --no-variants --msm-log-n 0 \
  --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline || exit 2
echo done >> gpurun_out/progress_$V.txt
