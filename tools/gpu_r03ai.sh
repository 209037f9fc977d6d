#!/bin/bash
# Round 3 ai: B1 / G2 sorted entries derived from the A / K sort (one sort fewer
# per proof).  Groth16 parity (single key, shards, stripes, distributed H,
# BLS12-381, BSB22, sizes to 2^24), then A/B against GG_G16_B_DERIVE=0,
# alternating, with the 8-way shard projection.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-ai}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 900 pytest_${V}.txt env GG_G16_B_DERIVE=1 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_groth16.py tests/test_gpu_groth16_multi.py tests/test_gpu_dist_h.py tests/test_gpu_groth16_size.py \
  tests/test_gpu_bls_groth16.py tests/test_gpu_groth16_bsb22.py tests/test_gpu_msm_groups.py tests/test_gpu_solver.py || exit 2
HEAD="--steps 8 --warmup 2 --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection 8"
for k in 1 2; do
  step 600 derive_${V}_${k}.json env GG_G16_B_DERIVE=1 python3 -u bench.py $HEAD || exit 2
  step 600 own_${V}_${k}.json python3 -u bench.py $HEAD || exit 2
done
echo done >> gpurun_out/progress_$V.txt
