#!/bin/bash
# Round-2 v15: rocprofv3 kernel trace of the headline + the GPU solver extra
# (k_solve_level per level), then smoke and the whole -m gpu suite.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-i}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
HEAD="--steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline"
step 300 prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$V -o run -- python3 bench.py $HEAD || exit 2
step 300 smoke_$V.txt python -c "import __graft_entry__ as g; g.smoke()" || exit 2
step 600 pytest_gpu_$V.txt python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread || exit 2
echo done >> gpurun_out/progress_$V.txt
