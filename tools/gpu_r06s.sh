#!/bin/bash
# Round 6 s: runsum segments per bucket group (GG_MSM_SEGS_LOG 17 = default,
# 18, 19: L = 16 / 8 / 4 buckets per lane at 2^21 buckets per group), isolated
# MSMs and the 2^24 Groth16 prove, alternating.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V="${V:-r06s}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" >> "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
G16="--steps 10 --warmup 2 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection=8"
step 300 pytest_$V.txt env GG_MSM_SEGS_LOG=19 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_groups.py || exit 2
for i in 1 2; do
  for s in 17 18 19; do
    step 120 msm_$V.txt env TAG=s$s GG_MSM_SEGS_LOG=$s python3 -u tools/bench_msm.py G1 24 5 || exit 2
    step 120 msm_$V.txt env TAG=s$s GG_MSM_SEGS_LOG=$s python3 -u tools/bench_msm.py G2 23 5 || exit 2
  done
done
for i in 1 2; do
  step 300 g16_s17_${i}_$V.json env GG_MSM_SEGS_LOG=17 python3 -u bench.py $G16 || exit 2
  step 300 g16_s18_${i}_$V.json env GG_MSM_SEGS_LOG=18 python3 -u bench.py $G16 || exit 2
done
echo done >> gpurun_out/progress_$V.txt
