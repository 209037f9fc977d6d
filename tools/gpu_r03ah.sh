#!/bin/bash
# Round 3 ah: B1 / G2 window 22 (the A / K window) vs the default 20, alternating:
# what the accumulations and the larger bucket reduction cost before any sort
# sharing.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-ah}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
HEAD="--steps 8 --warmup 2 --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection ''"
for k in 1 2; do
  step 600 b20_${k}.json python3 -u bench.py $HEAD || exit 2
  step 600 b22_${k}.json env GG_G16_B_WINDOW=22 python3 -u bench.py $HEAD || exit 2
done
echo done >> gpurun_out/progress_$V.txt
