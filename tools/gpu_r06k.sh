#!/bin/bash
# Round 6 k: kernel traces of one rehearsed PlonK part (2^22, 8 parts on GPU 0):
# part 2 (the slowest in r06h) and part 0, for the per-kernel fixed costs of the
# slice MSMs (tools/part_breakdown.py).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r06k}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 300 part2_$V.txt env PROBE_PARTS=2 rocprofv3 --kernel-trace --stats -d gpurun_out/part2_$V -o run -- python3 -u tools/plonk_part_probe.py 22 8 3 || exit 2
step 300 part0_$V.txt env PROBE_PARTS=0 rocprofv3 --kernel-trace --stats -d gpurun_out/part0_$V -o run -- python3 -u tools/plonk_part_probe.py 22 8 3 || exit 2
echo done >> gpurun_out/progress_$V.txt
