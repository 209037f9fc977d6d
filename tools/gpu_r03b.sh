#!/bin/bash
# Round 3, call b: the whole GPU suite (PlonK templated over the curve, BN254
# PlonK, byte-exact PlonK vs the oracle prover), smoke, the default bench, and the
# profiles of the headline: rocprof kernel stats, FETCH / WRITE / SQ counter
# passes (one counter group per pass).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-b}"
HEAD="--steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-test,smoke,bench,prof,pmc}"
if [[ "$S" == *test* ]]; then
  step 900 pytest_$V.txt python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests ${PYTEST_ARGS} || exit 2
fi
if [[ "$S" == *smoke* ]]; then step 300 smoke_$V.txt python -u -c "import __graft_entry__ as g; g.smoke()" || exit 2; fi
if [[ "$S" == *bench* ]]; then step 600 bench_$V.json python3 -u bench.py || exit 2; fi
if [[ "$S" == *prof* ]]; then
  step 300 prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$V -o run -- python3 bench.py $HEAD || exit 2
fi
if [[ "$S" == *pmc* ]]; then
  step 300 pmc_f_$V.txt timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_$V -o run -- python3 bench.py $HEAD || exit 2
  step 300 pmc_w_$V.txt timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_$V -o run -- python3 bench.py $HEAD || exit 2
  step 300 pmc_sq_$V.txt timeout -s KILL 280 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -d gpurun_out/pmc_sq_$V -o run -- python3 bench.py $HEAD || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
