#!/bin/bash
# Round 3: bucket-stripe multi-GPU split.  MSM stripe parity, the multi-GPU
# Groth16 tests (both splits), then the 2^24 prove with 8 / 4 / 2 shards on
# this GPU (total work of the N-GPU split) for stripes vs wire slices, and the
# one-GPU headline for reference.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-t}"
HEAD="--steps 4 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0"
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
  step 900 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_msm_stripe.py tests/test_gpu_groth16_multi.py tests/test_gpu_dist_h.py \
    tests/test_gpu_groth16_size.py tests/test_gpu_msm.py ${PYTEST_ARGS} || exit 2
fi
if [[ "$S" == *ab* ]]; then
  for D in ${DEVS:-0,0,0,0,0,0,0,0 0,0,0,0}; do
    N=$(echo $D | tr ',' '\n' | wc -l)
    step 600 bench_${V}_stripes_${N}.json python3 -u bench.py $HEAD --gpus $N --devices $D || exit 2
    step 600 bench_${V}_wires_${N}.json env GG_MPK_SPLIT=wires python3 -u bench.py $HEAD --gpus $N --devices $D || exit 2
  done
  step 600 bench_${V}_single.json python3 -u bench.py $HEAD || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
