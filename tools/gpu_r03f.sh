#!/bin/bash
# Round 3, A/B of the sort placement: the MSM / Groth16 GPU tests (16-bit sort
# keys), then the headline prove with the sorts on every CU (default) and on
# CU-masked streams (GG_SORT_CUS = 64, 128), one short bench each.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-f}"
HEAD="--steps 6 --warmup 2 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0"
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
  step 600 pytest_$V.txt python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_msm.py tests/test_gpu_msm_groups.py tests/test_gpu_bls.py tests/test_gpu_groth16.py \
    tests/test_gpu_groth16_size.py ${PYTEST_ARGS} || exit 2
fi
if [[ "$S" == *ab* ]]; then
  for cus in ${CUS_LIST:-0 64 128}; do
    step 300 bench_${V}_cus$cus.json env GG_SORT_CUS=$cus python3 -u bench.py $HEAD || exit 2
  done
fi
echo done >> gpurun_out/progress_$V.txt
