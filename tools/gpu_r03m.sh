#!/bin/bash
# Round 3: range-head buckets from a kernel of their own (no binary search at
# the head of every accumulation lane).  MSM / Groth16 / PlonK GPU tests, then the
# headline + 2^20 MSM + PlonK 2^22 with this tree's library and with the
# previous one (lib_prev, GNARK_AMD_LIB), alternating, one process each.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-m}"
HEAD="--steps 6 --warmup 2 --no-variants --ntt-log-n 0 --no-cpu-baseline --solver 0"
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
    tests/test_gpu_msm.py tests/test_gpu_msm_groups.py tests/test_gpu_msm_device_base.py tests/test_gpu_bls.py \
    tests/test_gpu_bls_groth16.py tests/test_gpu_groth16.py tests/test_gpu_groth16_size.py tests/test_gpu_plonk_prove.py \
    ${PYTEST_ARGS} || exit 2
fi
if [[ "$S" == *ab* ]]; then
  step 400 bench_${V}_new1.json python3 -u bench.py $HEAD || exit 2
  step 400 bench_${V}_prev1.json env GNARK_AMD_LIB=gnark-fork_amd/lib_prev/libgnark_amd.so python3 -u bench.py $HEAD || exit 2
  step 400 bench_${V}_new2.json python3 -u bench.py $HEAD || exit 2
  step 400 bench_${V}_prev2.json env GNARK_AMD_LIB=gnark-fork_amd/lib_prev/libgnark_amd.so python3 -u bench.py $HEAD || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
