#!/bin/bash
# Round 3, call a: FETCH_SIZE width calibration, the multi-shard Groth16 parity
# tests (2^24 with 8 shards on this GPU, BLS12-381 mpk), and the one-process
# N-GPU bench path rehearsed with 8 shards on device 0.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-a}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-calib,test,bench}"
if [[ "$S" == *calib* ]]; then
  step 60 calib_stdout_$V.txt tools/mbench_gather_calib || exit 2
  step 60 calib_pmc_$V.txt rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib_$V -o run -- tools/mbench_gather_calib || exit 2
fi
if [[ "$S" == *test* ]]; then
  step 600 pytest_$V.txt python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_groth16_multi.py tests/test_gpu_bls_groth16.py tests/test_gpu_plonk_prove.py tests/test_gpu_groth16_size.py ${PYTEST_ARGS} || exit 2
fi
if [[ "$S" == *bench* ]]; then
  step 400 bench_mpk8_$V.json python -u bench.py --gpus 8 --devices 0,0,0,0,0,0,0,0 --steps 5 --warmup 1 \
    --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
