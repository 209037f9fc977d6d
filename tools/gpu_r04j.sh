#!/bin/bash
# Round 4 j: window width of the 8-way Groth16 shard's 2^21-point MSMs
# (choose_c picks 19): the shard proved alone (split_projection) with every
# base at c = 17 / 18 / 19 (GG_MSM_WINDOW; the one-GPU headline in these runs
# is not comparable -- only shard_ms).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04j}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
B="--steps 1 --warmup 0 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection 8"
step 300 shard_def_$V.json python3 -u bench.py $B || exit 2
step 300 shard_c17_$V.json env GG_MSM_WINDOW=17 python3 -u bench.py $B || exit 2
step 300 shard_c18_$V.json env GG_MSM_WINDOW=18 python3 -u bench.py $B || exit 2
step 300 shard_def2_$V.json python3 -u bench.py $B || exit 2
echo done >> gpurun_out/progress_$V.txt
