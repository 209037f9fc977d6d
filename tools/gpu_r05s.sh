#!/bin/bash
# Round 5 s: the driver's bench command once more on the final tree (another
# box: the spread between boxes, r05z_clock_by_box), with the G1 clock from a
# short GRBM pass beside it.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05s}"
HEAD="--steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection="
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 600 bench_$V.json python3 -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 2
step 300 clk_$V.txt timeout -s KILL 280 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/clk_$V -o run -- python3 bench.py $HEAD || exit 2
echo done >> gpurun_out/progress_$V.txt
