#!/bin/bash
# Round 4 d: the full -m gpu suite, smoke, the PlonK 8-part probe, and the
# default bench line of the current tree.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04d}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-test,smoke,probe,bench}"
if [[ "$S" == *test* ]]; then
  step 900 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ || exit 2
fi
if [[ "$S" == *smoke* ]]; then
  step 300 smoke_$V.txt python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit 2
fi
if [[ "$S" == *probe* ]]; then
  step 300 probe_$V.txt python3 -u tools/plonk_part_probe.py 22 8 3 || exit 2
fi
if [[ "$S" == *bench* ]]; then step 600 bench_$V.json python3 -u bench.py || exit 2; fi
echo done >> gpurun_out/progress_$V.txt
