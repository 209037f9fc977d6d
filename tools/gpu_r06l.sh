#!/bin/bash
# Round 6 l: the bucket reduction's host tail (GG_RED_HOST_N: weighted sums of
# <= N elements finish on the host) on the PlonK 2^22 prove and its 8-part
# projection -- the parts wait ~0.5 ms for the host after each batched commitment
# (r06k trace) -- default 8 against 4 and 2, alternating.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V="${V:-r06l}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
for i in 1 2; do
  step 240 plonk_h8_${i}_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 240 plonk_h4_${i}_$V.json env GG_RED_HOST_N=4 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  step 240 plonk_h2_${i}_$V.json env GG_RED_HOST_N=2 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
done
echo done >> gpurun_out/progress_$V.txt
