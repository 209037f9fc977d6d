#!/bin/bash
# Round 6 w: knob sweep on the PlonK 2^22 8-part projection (final tree):
# radix segment level 2 for the parts' 2^15-bucket slices (GG_MSM_SEGSUM_MINLOG
# 15) and range lengths 48 / 96 (GG_MSM_K1) against the defaults, twice.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V="${V:-r06w}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
for i in 1 2; do
  step 240 plonk_def_${i}_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 240 plonk_seg15_${i}_$V.json env GG_MSM_SEGSUM_MINLOG=15 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 240 plonk_k48_${i}_$V.json env GG_MSM_K1=48 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 240 plonk_k96_${i}_$V.json env GG_MSM_K1=96 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
done
echo done >> gpurun_out/progress_$V.txt
