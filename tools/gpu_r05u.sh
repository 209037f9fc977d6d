#!/bin/bash
# Round 5 u: the driver's bench command on the final tree once more (another
# box); the quad-cooperative bucket reduction everywhere (GG_MSM_SEGSUM=0)
# against the default on the one-GPU prove, alternating.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05u}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 600 bench_$V.json python3 -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 2
step 150 g_def1_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_quad_$V.txt env GG_MSM_SEGSUM=0 python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_def2_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
echo done >> gpurun_out/progress_$V.txt
