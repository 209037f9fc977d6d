#!/bin/bash
# Round 6 q: the stage hand-over's host tail -- a batch's reduction results
# finished side by side on kept workers, the stage's commitments made affine
# with one inversion (GG_HOST_TAIL=1, default) against the variant build
# GG_HOST_TAIL=0 (lib/var/libgnark_amd_tail0.so), alternating; parity first.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V="${V:-r06q}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
T0=gnark-fork_amd/lib/var/libgnark_amd_tail0.so
step 600 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_batch.py tests/test_gpu_plonk_prove.py tests/test_gpu_plonk_group.py tests/test_gpu_bls.py || exit 2
for i in 1 2 3; do
  step 240 plonk_t1_${i}_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 240 plonk_t0_${i}_$V.json env GNARK_AMD_LIB=$T0 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
done
echo done >> gpurun_out/progress_$V.txt
