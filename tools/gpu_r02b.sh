#!/bin/bash
# Round-2 measurement session, part 1: every GPU test, then the default bench.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-v2}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-test,bench}"
if [[ "$S" == *test* ]]; then step 900 pytest_gpu_$V.txt python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread || exit 2; fi
if [[ "$S" == *smoke* ]]; then step 300 smoke_$V.txt python -c "import __graft_entry__ as g; g.smoke()" || exit 2; fi
if [[ "$S" == *bench* ]]; then step 900 bench_$V.json python3 -u bench.py || exit 2; fi
HEAD="--steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline"
if [[ "$S" == *prof* ]]; then
  step 400 prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$V -o run -- python3 bench.py $HEAD || exit 2
fi
if [[ "$S" == *pmc* ]]; then
  step 400 pmc_f_$V.txt rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_$V -o run -- python3 bench.py $HEAD || exit 2
  step 400 pmc_w_$V.txt rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_$V -o run -- python3 bench.py $HEAD || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
