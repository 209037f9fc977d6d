#!/bin/bash
# Round 6 r: the split level 2 (k_bucket_pass_r + k_bucket_add_r, GG_MSM_SUM_SPLIT=1,
# default) against the one-launch k_bucket_sum_r (=0): MSM parity on the split,
# isolated MSM phases and the 2^24 Groth16 prove alternating, one kernel trace.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r06r}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" >> "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
G16="--steps 10 --warmup 2 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection=8"
step 600 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_batch.py tests/test_gpu_msm_groups.py tests/test_gpu_msm_stripe.py tests/test_gpu_bls.py tests/test_gpu_groth16.py || exit 2
for i in 1 2; do
  step 120 msm_$V.txt env TAG=split1 python3 -u tools/bench_msm.py G2 23 5 || exit 2
  step 120 msm_$V.txt env TAG=split0 GG_MSM_SUM_SPLIT=0 python3 -u tools/bench_msm.py G2 23 5 || exit 2
  step 120 msm_$V.txt env TAG=split1 python3 -u tools/bench_msm.py G1 24 5 || exit 2
  step 120 msm_$V.txt env TAG=split0 GG_MSM_SUM_SPLIT=0 python3 -u tools/bench_msm.py G1 24 5 || exit 2
done
step 200 tr_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$V -o run -- python3 -u tools/bench_msm.py G2 23 3 || exit 2
for i in 1 2; do
  step 300 g16_s1_${i}_$V.json python3 -u bench.py $G16 || exit 2
  step 300 g16_s0_${i}_$V.json env GG_MSM_SUM_SPLIT=0 python3 -u bench.py $G16 || exit 2
done
echo done >> gpurun_out/progress_$V.txt
