#!/bin/bash
# Round 6 j: the bin-scatter tile (GG_SORT_SPB 1024 = 12288-entry tiles at W = 12,
# 4 scalars per thread in the digit pass) against the default 512, alternating;
# parity of the sort under the knob; the stream-deadline test.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V="${V:-r06j}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" >> "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 200 pytest_$V.txt python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_wait_timeout.py || exit 2
step 300 pytest_$V.txt env GG_SORT_SPB=1024 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_batch.py || exit 2
for i in 1 2; do
  step 120 msm_$V.txt env TAG=spb512 python3 -u tools/bench_msm.py G1 24 5 || exit 2
  step 120 msm_$V.txt env TAG=spb1024 GG_SORT_SPB=1024 python3 -u tools/bench_msm.py G1 24 5 || exit 2
done
step 120 msm_$V.txt env TAG=h7 GG_SORT_H=7 python3 -u tools/bench_msm.py G1 24 5 || exit 2
step 120 msm_$V.txt env TAG=h6 GG_SORT_H=6 python3 -u tools/bench_msm.py G1 24 5 || exit 2
step 120 msm_$V.txt env TAG=spb1024h7 GG_SORT_SPB=1024 GG_SORT_H=7 python3 -u tools/bench_msm.py G1 24 5 || exit 2
step 120 msm_$V.txt env TAG=spb512 python3 -u tools/bench_msm.py G2 23 5 || exit 2
step 120 msm_$V.txt env TAG=spb1024 GG_SORT_SPB=1024 python3 -u tools/bench_msm.py G2 23 5 || exit 2
step 120 msm_$V.txt env TAG=spb512 python3 -u tools/bench_msm.py G1 20 10 || exit 2
step 120 msm_$V.txt env TAG=spb1024 GG_SORT_SPB=1024 python3 -u tools/bench_msm.py G1 20 10 || exit 2
echo done >> gpurun_out/progress_$V.txt
