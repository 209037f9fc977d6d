#!/bin/bash
# Round 6 z: queue knobs on the final tree (kept worker threads): PlonK device
# parts on dedicated CU-masked queues (GG_PLONK_PART_QUEUES=1) and the Groth16
# tasks on HIP's shared queues (GG_TASK_QUEUES=0), against the defaults.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V="${V:-r06z}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
G16="--steps 10 --warmup 2 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection=8"
for i in 1 2; do
  step 240 plonk_def_${i}_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 240 plonk_pq_${i}_$V.json env GG_PLONK_PART_QUEUES=1 GG_WAIT_TIMEOUT_S=60 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 300 g16_def_${i}_$V.json python3 -u bench.py $G16 || exit 2
  step 300 g16_tq0_${i}_$V.json env GG_TASK_QUEUES=0 python3 -u bench.py $G16 || exit 2
done
echo done >> gpurun_out/progress_$V.txt
