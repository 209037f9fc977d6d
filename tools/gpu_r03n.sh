#!/bin/bash
# Round 3: the one-process multi-GPU path (gg_groth16_mpk_*) rehearsed with
# 8 and 4 key shards on this one GPU (bench.py --devices), beside the
# single-key headline: the total work of the split and its per-shard share.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-n}"
HEAD="--steps 4 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 400 bench_${V}_single.json python3 -u bench.py $HEAD || exit 2
step 500 bench_${V}_shards8.json python3 -u bench.py $HEAD --gpus 8 --devices 0,0,0,0,0,0,0,0 || exit 2
step 500 bench_${V}_shards4.json python3 -u bench.py $HEAD --gpus 4 --devices 0,0,0,0 || exit 2
step 400 bench_${V}_serial.json env GG_G16_SERIAL=1 python3 -u bench.py $HEAD || exit 2
echo done >> gpurun_out/progress_$V.txt
