#!/bin/bash
# One GPU session: microbench, smoke, GPU parity tests, bench, rocprof summary.
# Stops at the first GPU fault / abort / timeout (exit codes >= 124 or signals).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
run() {  # run <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" | tee -a gpurun_out/progress.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" | tee -a gpurun_out/progress.txt
  return $rc
}
STEPS="${STEPS:-all}"
if [[ "$STEPS" == *mb* || "$STEPS" == all ]]; then run 120 mbench.txt ./tools/mbench_field || ok $? || exit 2; fi
if [[ "$STEPS" == *smoke* || "$STEPS" == all ]]; then run 300 smoke.txt python -c "import __graft_entry__ as g; g.smoke()" || ok $? || exit 2; fi
if [[ "$STEPS" == *test* || "$STEPS" == all ]]; then run 900 pytest_gpu.txt python -m pytest tests -m gpu -q -x ${PYTEST_ARGS} || ok $? || exit 2; fi
if [[ "$STEPS" == *bench* || "$STEPS" == all ]]; then run 600 bench.txt python bench.py || ok $? || exit 2; fi
if [[ "$STEPS" == *prof* || "$STEPS" == all ]]; then
  export TMPDIR=/tmp
  run 600 rocprof.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline || ok $? || exit 2
fi
echo done >> gpurun_out/progress.txt
