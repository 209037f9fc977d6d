#!/bin/bash
# Round 3: window width (GG_MSM_WINDOW forces every MSM's c) in the 8-shard
# rehearsal of the one-process multi-GPU prove, against the chosen widths.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-o}"
HEAD="--steps 4 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
for c in ${C_LIST:-17 19 20 22}; do
  step 500 bench_${V}_shards8_c$c.json env GG_MSM_WINDOW=$c python3 -u bench.py $HEAD --gpus 8 --devices 0,0,0,0,0,0,0,0 || exit 2
done
step 500 bench_${V}_shards8_def.json python3 -u bench.py $HEAD --gpus 8 --devices 0,0,0,0,0,0,0,0 || exit 2
echo done >> gpurun_out/progress_$V.txt
