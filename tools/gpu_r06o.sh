#!/bin/bash
# Round 6 o: host tasks on kept worker threads (common.h run_task, GG_TASK_POOL)
# -- the thread-launch probe, the full -m gpu suite on the pool, then A/B
# alternating: the PlonK 2^22 prove + 8-part projection and the Groth16 2^24
# prove + 8-way shard projection, GG_TASK_POOL=1 (default) vs 0.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V="${V:-r06o}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
G16="--steps 10 --warmup 2 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection=8"
step 60 thread_launch_$V.txt ./tools/probe/thread_launch || exit 2
step 900 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ || exit 2
for i in 1 2; do
  step 240 plonk_p1_${i}_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 240 plonk_p0_${i}_$V.json env GG_TASK_POOL=0 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 300 g16_p1_${i}_$V.json python3 -u bench.py $G16 || exit 2
  step 300 g16_p0_${i}_$V.json env GG_TASK_POOL=0 python3 -u bench.py $G16 || exit 2
done
echo done >> gpurun_out/progress_$V.txt
