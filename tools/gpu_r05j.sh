#!/bin/bash
# Round 5 j: outlier hunt for the dedicated task queues -- 40 one-GPU 2^24
# proves per run (new, old, new), then the driver's bench command.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05j}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 300 g16_new1_$V.txt python3 -u tools/g16_time.py 24 40 3 || exit 2
step 300 g16_old1_$V.txt env GG_TASK_QUEUES=0 python3 -u tools/g16_time.py 24 40 3 || exit 2
step 300 g16_new2_$V.txt python3 -u tools/g16_time.py 24 40 3 || exit 2
step 300 g16_q1_$V.txt env GG_TASK_QUEUES=1 python3 -u tools/g16_time.py 24 40 3 || exit 2
step 900 bench_$V.json python3 -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 2
echo done >> gpurun_out/progress_$V.txt
