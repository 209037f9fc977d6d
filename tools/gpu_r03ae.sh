#!/bin/bash
# Round 3 ae: small-MSM bucket reduction path (segment sums from 2^k buckets,
# GG_MSM_SEGSUM_MINLOG) A/B on the split projections (Groth16 N = 8 shard,
# PlonK N = 8 primary part), alternating; then MSM parity with the switch on.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-ae}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
HEAD="--steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection 8"
for k in 1 2; do
  for M in 18 16; do
    step 600 g16_${V}_m${M}_${k}.json env GG_MSM_SEGSUM_MINLOG=$M python3 -u bench.py $HEAD || exit 2
    step 600 plonk_${V}_m${M}_${k}.json env GG_MSM_SEGSUM_MINLOG=$M python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  done
done
step 600 pytest_${V}.txt env GG_MSM_SEGSUM_MINLOG=14 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  -m gpu tests/test_gpu_msm.py tests/test_gpu_bls.py tests/test_gpu_msm_stripe.py || exit 2
echo done >> gpurun_out/progress_$V.txt
