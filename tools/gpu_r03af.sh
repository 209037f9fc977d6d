#!/bin/bash
# Round 3 af: segment-path threshold 2^17 (new default) vs 2^18, alternating:
# the 8-way shard projection and the 2^20 G1 MSM (configs[1]).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-af}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
HEAD="--steps 6 --warmup 2 --no-variants --msm-log-n 20 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection 8"
for k in 1 2; do
  step 600 g16_${V}_m17_${k}.json python3 -u bench.py $HEAD || exit 2
  step 600 g16_${V}_m18_${k}.json env GG_MSM_SEGSUM_MINLOG=18 python3 -u bench.py $HEAD || exit 2
done
echo done >> gpurun_out/progress_$V.txt
