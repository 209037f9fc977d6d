#!/bin/bash
# Round 3 aj: the 2^20 G1 MSM (configs[1]) and 2^21 / 2^22 MSMs with the segment
# path from 2^16 / 2^15 buckets vs the default (2^17), alternating.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-aj}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
for k in 1 2; do
  for M in 17 16 15; do
    for L in 20 19; do
      step 300 msm_${V}_m${M}_L${L}_${k}.txt env GG_MSM_SEGSUM_MINLOG=$M python3 -u tools/bench_msm.py G1 $L 20 || exit 2
    done
  done
done
echo done >> gpurun_out/progress_$V.txt
