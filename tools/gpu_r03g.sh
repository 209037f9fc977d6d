#!/bin/bash
# Round 3, the fused level-2 + weighted-sum pass (k_bucket_segsum): MSM / Groth16
# / PlonK GPU tests, then the headline with and without it (GG_MSM_SEGSUM=0),
# and the 2^20 MSM / PlonK extras of the default bench.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-g}"
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
    tests/test_gpu_groth16.py tests/test_gpu_groth16_size.py tests/test_gpu_plonk_prove.py ${PYTEST_ARGS} || exit 2
fi
if [[ "$S" == *ab* ]]; then
  for seg in ${SEG_LIST:-1 0}; do
    step 400 bench_${V}_seg$seg.json env GG_MSM_SEGSUM=$seg python3 -u bench.py $HEAD || exit 2
  done
fi
echo done >> gpurun_out/progress_$V.txt
