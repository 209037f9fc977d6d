#!/bin/bash
# Round 4 aa: where a rehearsed PlonK part spends its proof on the final tree --
# kernel traces of part 0 and peer 5 of the 2^22 x 8 key (the probe sleeps
# 30 ms between proofs so tools/part_breakdown.py can cut out the last one).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04aa}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 300 part0_$V.txt env PROBE_PARTS=0 rocprofv3 --kernel-trace --stats -d gpurun_out/part0_$V -o run -- python3 -u tools/plonk_part_probe.py 22 8 3 || exit 2
step 300 peer5_$V.txt env PROBE_PARTS=5 rocprofv3 --kernel-trace --stats -d gpurun_out/peer5_$V -o run -- python3 -u tools/plonk_part_probe.py 22 8 3 || exit 2
step 300 one_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/one_$V -o run -- python3 -u tools/plonk_part_probe.py 22 1 3 || exit 2
echo done >> gpurun_out/progress_$V.txt
