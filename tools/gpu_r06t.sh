#!/bin/bash
# Round 6 t: kept workers that poll 200 us before sleeping (GG_TASK_SPIN_US,
# default) against sleeping at once (=0): PlonK 2^22 + 8-part projection and the
# Groth16 2^24 prove + 8-way shard, alternating.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V="${V:-r06t}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
G16="--steps 10 --warmup 2 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection=8"
step 300 pytest_$V.txt python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_plonk_group.py tests/test_gpu_groth16_multi.py || exit 2
for i in 1 2 3; do
  step 240 plonk_w200_${i}_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 240 plonk_w0_${i}_$V.json env GG_TASK_SPIN_US=0 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
done
for i in 1 2; do
  step 300 g16_w200_${i}_$V.json python3 -u bench.py $G16 || exit 2
  step 300 g16_w0_${i}_$V.json env GG_TASK_SPIN_US=0 python3 -u bench.py $G16 || exit 2
done
echo done >> gpurun_out/progress_$V.txt
