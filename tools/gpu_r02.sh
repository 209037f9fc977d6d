#!/bin/bash
# Round-2 GPU session: default bench, rocprof kernel trace of the headline alone,
# HBM traffic of the headline (two separate --pmc passes).  Stops at the first
# failure (exit codes >= 124 = time limit / signal).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
HEAD="--steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress.txt
  return $rc
}
S="${STEPS:-bench,prof,pmc}"
if [[ "$S" == *bench* ]]; then step 600 bench.json python3 -u bench.py || exit 2; fi
if [[ "$S" == *prof* ]]; then
  step 300 prof.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py $HEAD || exit 2
fi
if [[ "$S" == *pmc* ]]; then
  step 300 pmc_f.txt rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run -- python3 bench.py $HEAD || exit 2
  step 300 pmc_w.txt rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run -- python3 bench.py $HEAD || exit 2
fi
echo done >> gpurun_out/progress.txt
