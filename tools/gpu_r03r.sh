#!/bin/bash
# Round 3: batched bucket-reduction tail (every group's and list's tree sums in
# the same launches, one read-back per MSM) and the fixed-point terms of the
# combination started before a sharded prove.  MSM / Groth16 / multi-GPU GPU
# tests, then the prove at 2^21 (the per-GPU work of an 8-GPU split) and 2^24
# with this tree's library and the previous one (lib_prev), alternating.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r}"
HEAD="--steps 8 --warmup 2 --no-variants --msm-log-n 20 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0"
PREV_ENV="GG_RED_SPLIT=1"
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
  step 900 pytest_$V.txt python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_msm.py tests/test_gpu_msm_groups.py tests/test_gpu_msm_device_base.py tests/test_gpu_bls.py \
    tests/test_gpu_groth16.py tests/test_gpu_groth16_multi.py tests/test_gpu_dist_h.py tests/test_gpu_bls_groth16.py \
    tests/test_gpu_groth16_size.py ${PYTEST_ARGS} || exit 2
fi
if [[ "$S" == *ab* ]]; then
  for L in ${SIZES:-21 24}; do
    step 400 bench_${V}_${L}_new1.json python3 -u bench.py $HEAD --log-n $L || exit 2
    step 400 bench_${V}_${L}_prev1.json env $PREV_ENV python3 -u bench.py $HEAD --log-n $L || exit 2
    step 400 bench_${V}_${L}_new2.json python3 -u bench.py $HEAD --log-n $L || exit 2
    step 400 bench_${V}_${L}_prev2.json env $PREV_ENV python3 -u bench.py $HEAD --log-n $L || exit 2
  done
fi
echo done >> gpurun_out/progress_$V.txt
