#!/bin/bash
# Round 3 v: size-N DFT steps of the distributed computeH in registers
# (radix 2).  Distributed-H / multi-GPU parity, the per-GPU work of the N-GPU
# split (GG_MPK_SOLO), then the full checkpoint (smoke, every -m gpu test,
# default bench line, kernel trace of the headline).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-v}"
HEAD="--steps 6 --warmup 2 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 600 pytest_${V}_dist.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dist_h.py tests/test_gpu_groth16_multi.py || exit 2
for D in 0,0,0,0,0,0,0,0 0,0,0,0 0,0; do
  N=$(echo $D | tr ',' '\n' | wc -l)
  step 600 bench_${V}_wires_${N}_solo0.json env GG_MPK_SOLO=0 python3 -u bench.py $HEAD --gpus $N --devices $D || exit 2
done
V=$V STEPS=smoke,test,bench,prof bash tools/gpu_r03s.sh || exit 2
echo done >> gpurun_out/progress_$V.txt
