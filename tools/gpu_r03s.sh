#!/bin/bash
# Round 3 checkpoint of the restored tree: smoke, every -m gpu test, the
# default bench line, and a kernel-trace summary of the headline prove.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-s}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-smoke,test,bench,prof}"
if [[ "$S" == *smoke* ]]; then step 300 smoke_$V.txt python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit 2; fi
if [[ "$S" == *test* ]]; then
  step 1000 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests ${PYTEST_ARGS} || exit 2
fi
if [[ "$S" == *bench* ]]; then step 600 bench_$V.json python3 -u bench.py || exit 2; fi
if [[ "$S" == *prof* ]]; then
  step 600 prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$V -o run -- \
    python3 -u bench.py --steps 5 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection '' || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
