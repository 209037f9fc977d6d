#!/bin/bash
# Round 4 y: bin bits (GG_SORT_H 8 / 6 / 5: 256 / 64 / 32 bins, the rest in
# segmented passes of <= 8 bits) x bin-scatter tile width (GG_BIN_BS 256 / 1024),
# isolated 2^24 G1 and 2^22 G2 MSM phase times, two rounds; MSM parity for H=6
# and H=5.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04y}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" >> "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
for h in 6 5; do
  export GG_SORT_H=$h GG_BIN_BS=1024
  step 300 pytest_h${h}_$V.txt python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py || exit 2
done
for round in 1 2; do
  for h in 8 6 5; do for bs in 256 1024; do
    export GG_SORT_H=$h GG_BIN_BS=$bs TAG=h${h}_bs$bs
    step 200 msm_$V.txt python3 -u tools/bench_msm.py G1 24 10 || exit 2
    step 200 msm_$V.txt python3 -u tools/bench_msm.py G2 22 10 || exit 2
  done; done
done
echo done >> gpurun_out/progress_$V.txt
