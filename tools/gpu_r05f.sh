#!/bin/bash
# Round 5 f: PlonK 2^22 (one GPU and the 8-part rehearsal): the level-2 path of
# the parts' 2^19-point KZG slices (2^15 buckets: quad path by default) vs the
# radix segment-sum path (GG_MSM_SEGSUM_MINLOG), alternating; then the byte-exact
# PlonK tests up to 2^14.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05f}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
for v in def m15 m14 def2 m152; do
  unset GG_MSM_SEGSUM_MINLOG
  case $v in m15*) export GG_MSM_SEGSUM_MINLOG=15 ;; m14) export GG_MSM_SEGSUM_MINLOG=14 ;; esac
  step 400 plonk_${v}_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
done
unset GG_MSM_SEGSUM_MINLOG
step 900 pytest_$V.txt python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_plonk_prove.py -k "match_oracle or distinct or same_device" || exit 2
echo done >> gpurun_out/progress_$V.txt
