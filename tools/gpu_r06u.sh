#!/bin/bash
# Round 6 u: the quad-path level 2 with the partials converted inside the
# combine (k_bucket_combine_r, GG_MSM_COMBINE_FUSED=1, default) against three
# conversion launches first (=0): parity, then configs[1]'s 2^20 MSM, the PlonK
# 2^22 8-part projection and the Groth16 prove + 8-way shard, alternating.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V="${V:-r06u}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" >> "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
G16="--steps 10 --warmup 2 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection=8"
step 900 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_batch.py tests/test_gpu_msm_groups.py tests/test_gpu_msm_stripe.py tests/test_gpu_bls.py tests/test_gpu_plonk_prove.py tests/test_gpu_plonk_group.py tests/test_gpu_groth16.py tests/test_gpu_groth16_multi.py || exit 2
for i in 1 2 3; do
  step 120 msm_$V.txt env TAG=fused1 python3 -u tools/bench_msm.py G1 20 20 || exit 2
  step 120 msm_$V.txt env TAG=fused0 GG_MSM_COMBINE_FUSED=0 python3 -u tools/bench_msm.py G1 20 20 || exit 2
done
for i in 1 2; do
  step 240 plonk_f1_${i}_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 240 plonk_f0_${i}_$V.json env GG_MSM_COMBINE_FUSED=0 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 300 g16_f1_${i}_$V.json python3 -u bench.py $G16 || exit 2
  step 300 g16_f0_${i}_$V.json env GG_MSM_COMBINE_FUSED=0 python3 -u bench.py $G16 || exit 2
done
echo done >> gpurun_out/progress_$V.txt
