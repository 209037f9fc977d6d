#!/bin/bash
# Round 3: the BN254 G2 bucket reduction in the radix form (k_bucket_sum_r /
# k_bucket_runsum over Xyzz2_29).  MSM / Groth16 GPU tests, then the headline
# with this tree's library and the previous one (lib_prev), alternating.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-p}"
HEAD="--steps 6 --warmup 2 --no-variants --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-test,ab}"
if [[ "$S" == *test* ]]; then
  step 700 pytest_$V.txt python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_msm.py tests/test_gpu_msm_groups.py tests/test_gpu_msm_device_base.py \
    tests/test_gpu_groth16.py tests/test_gpu_groth16_size.py tests/test_gpu_groth16_multi.py ${PYTEST_ARGS} || exit 2
fi
if [[ "$S" == *ab* ]]; then
  step 400 bench_${V}_new1.json python3 -u bench.py $HEAD || exit 2
  step 400 bench_${V}_prev1.json env GNARK_AMD_LIB=gnark-fork_amd/lib_prev/libgnark_amd.so python3 -u bench.py $HEAD || exit 2
  step 400 bench_${V}_new2.json python3 -u bench.py $HEAD || exit 2
  step 400 bench_${V}_prev2.json env GNARK_AMD_LIB=gnark-fork_amd/lib_prev/libgnark_amd.so python3 -u bench.py $HEAD || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
