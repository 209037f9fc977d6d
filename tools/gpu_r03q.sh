#!/bin/bash
# Round 3: strong-scaling proxy.  A 2^24 proof split over N GPUs gives each GPU
# the MSMs of a 2^(24 - log N) key shard plus a 1/N share of the four-step
# computeH: the one-GPU prove at 2^21 / 2^22 / 2^23 is the per-GPU work of the
# 8 / 4 / 2-GPU split (less the exchanges).  Headline sizes 21..24 on one GPU,
# then a kernel trace of the 2^21 prove (what a shard's proof is made of).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-q}"
HEAD="--steps 8 --warmup 2 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
for L in ${SIZES:-21 22 23 24}; do
  step 400 bench_${V}_2p${L}.json python3 -u bench.py $HEAD --log-n $L || exit 2
done
if [[ "${TRACE:-1}" == 1 ]]; then
  step 400 prof_${V}_2p21.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${V}_2p21 -o run -- \
    python3 -u bench.py $HEAD --log-n 21 --steps 3 || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
