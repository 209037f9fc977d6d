#!/bin/bash
# Round 4 x: bin-scatter tile width A/B (GG_BIN_BS 256 / 512 / 1024 threads over
# the same 512-scalar tile): MSM parity for 512 and 1024, then isolated 2^24 G1
# and 2^22 G2 MSM phase times (tools/bench_msm.py), two alternating rounds.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04x}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" >> "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
for bs in 512 1024; do
  export GG_BIN_BS=$bs TAG=bs$bs
  step 300 pytest_bs${bs}_$V.txt python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_stripe.py || exit 2
done
for round in 1 2; do
  for bs in 256 512 1024; do
    export GG_BIN_BS=$bs TAG=bs$bs
    step 200 msm_$V.txt python3 -u tools/bench_msm.py G1 24 10 || exit 2
    step 200 msm_$V.txt python3 -u tools/bench_msm.py G2 22 10 || exit 2
  done
done
echo done >> gpurun_out/progress_$V.txt
