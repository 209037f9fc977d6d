#!/bin/bash
# Round 4 r: the bucket reduction's host tail (GG_RED_HOST_N: pieces of <= N
# elements finish on the host after one read-back) for PlonK's BLS12-381
# slices -- part 0 and part 5 of the 2^22 x 8 key rehearsed alone; environment
# only, same box, back to back.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04r}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
export PROBE_PARTS=0,5
step 300 h8_$V.txt python3 -u tools/plonk_part_probe.py 22 8 4 || exit 2
step 300 h4_$V.txt env GG_RED_HOST_N=4 python3 -u tools/plonk_part_probe.py 22 8 4 || exit 2
step 300 h2_$V.txt env GG_RED_HOST_N=2 python3 -u tools/plonk_part_probe.py 22 8 4 || exit 2
step 300 h16_$V.txt env GG_RED_HOST_N=16 python3 -u tools/plonk_part_probe.py 22 8 4 || exit 2
step 300 h8b_$V.txt python3 -u tools/plonk_part_probe.py 22 8 4 || exit 2
echo done >> gpurun_out/progress_$V.txt
