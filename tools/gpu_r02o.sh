#!/bin/bash
# Round-2 final check: smoke and the whole -m gpu suite on the final tree.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-o}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 300 smoke_$V.txt python -c "import __graft_entry__ as g; g.smoke()" || exit 2
step 600 pytest_gpu_$V.txt python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread || exit 2
echo done >> gpurun_out/progress_$V.txt
