#!/bin/bash
# Round 6 y: range length of the BN254 G2 accumulation (GG_MSM_K1 192 / 256 / 384
# against the occupancy-derived default): fewer, longer ranges mean fewer
# straddling buckets for the level 2 (k_bucket_sum_r<Fp2>, 2.6 ms per 2^24
# proof), at the accumulation's expense.  Isolated 2^24 G2 MSM, alternating.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V="${V:-r06y}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" >> "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
for i in 1 2; do
  step 200 msm_$V.txt env TAG=kdef python3 -u tools/bench_msm.py G2 24 5 || exit 2
  step 200 msm_$V.txt env TAG=k192 GG_MSM_K1=192 python3 -u tools/bench_msm.py G2 24 5 || exit 2
  step 200 msm_$V.txt env TAG=k256 GG_MSM_K1=256 python3 -u tools/bench_msm.py G2 24 5 || exit 2
  step 200 msm_$V.txt env TAG=k384 GG_MSM_K1=384 python3 -u tools/bench_msm.py G2 24 5 || exit 2
done
echo done >> gpurun_out/progress_$V.txt
