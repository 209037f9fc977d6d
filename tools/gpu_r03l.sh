#!/bin/bash
# Round 3: is the G1 accumulation bound by the gather's TLB reach?  The same
# proof from a key with precompute groups G = 2 (half the table, the same
# gathers, twice the buckets) and G = 1, alternating.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-l}"
HEAD="--steps 6 --warmup 2 --no-variants --ntt-log-n 0 --plonk-log-n 0 --msm-log-n 0 --no-cpu-baseline --solver 0"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
for r in 1 2; do
  for g in ${G_LIST:-1 2 4}; do
    step 300 bench_${V}_g$g$r.json env GG_MSM_GROUPS=$g python3 -u bench.py $HEAD || exit 2
  done
done
echo done >> gpurun_out/progress_$V.txt
