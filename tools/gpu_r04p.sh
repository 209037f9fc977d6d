#!/bin/bash
# Round 4 p: the full -m gpu suite and smoke on the final tree.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04p}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 900 pytest_$V.txt python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ || exit 2
step 300 smoke_$V.txt python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit 2
echo done >> gpurun_out/progress_$V.txt
