#!/bin/bash
# Round 3 x: kernel trace of the BLS12-381 PlonK 2^22 prove (configs[4]) --
# per-kernel time and the GPU's busy fraction (tools/busy.py).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-x}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 600 plonk_${V}.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${V}_plonk -o run -- \
  python3 -u tools/bench_plonk.py ${LOGN:-22} 3 || exit 2
echo done >> gpurun_out/progress_$V.txt
