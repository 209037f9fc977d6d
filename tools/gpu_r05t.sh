#!/bin/bash
# Round 5 t: batched same-base MSMs (gg_msm_batch) -- their parity tests, the
# MSM and PlonK parity tests on the changed sort, then PlonK 2^22 one-GPU and
# 8-part rehearsal with the batched LRO / H commitments against three MSMs
# (GG_PLONK_BATCH=0), alternating; the Groth16 headline as a check of the
# single-vector path.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05t}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 400 pytest_batch_$V.txt python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm_batch.py || exit 2
step 600 pytest_msm_plonk_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_groups.py tests/test_gpu_bls.py tests/test_gpu_plonk_prove.py tests/test_gpu_plonk_group.py || exit 2
step 150 plonk_b1_$V.json python3 -u tools/bench_plonk.py 22 6 8 || exit 2
step 150 plonk_s1_$V.json env GG_PLONK_BATCH=0 python3 -u tools/bench_plonk.py 22 6 8 || exit 2
step 150 plonk_b2_$V.json python3 -u tools/bench_plonk.py 22 6 8 || exit 2
step 150 plonk_s2_$V.json env GG_PLONK_BATCH=0 python3 -u tools/bench_plonk.py 22 6 8 || exit 2
step 150 g16_$V.txt python3 -u tools/g16_time.py 24 12 3 || exit 2
echo done >> gpurun_out/progress_$V.txt
