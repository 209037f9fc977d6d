#!/bin/bash
# Round 4 i: where one shard of the 8-way Groth16 split spends its 17.9 ms
# (split_projection: shard 0 of an 8-shard key proved alone) -- kernel trace.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04i}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 500 shard8_prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/shard8_prof_$V -o run -- \
  python3 -u bench.py --steps 2 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection 8 || exit 2
echo done >> gpurun_out/progress_$V.txt
