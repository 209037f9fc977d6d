#!/bin/bash
# Round 3: per-GPU work of the N-GPU split, timed one shard at a time
# (GG_MPK_SOLO=r: the shard runs alone on this GPU, exchanges skip the peers):
# bucket stripes vs wire slices at N = 8 / 4 / 2, and a kernel trace of one
# stripe shard and one wire shard of the 8-way split.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-u}"
HEAD="--steps 6 --warmup 2 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
for D in 0,0,0,0,0,0,0,0 0,0,0,0 0,0; do
  N=$(echo $D | tr ',' '\n' | wc -l)
  for SP in stripes wires; do
    step 600 bench_${V}_${SP}_${N}_solo0.json env GG_MPK_SPLIT=$SP GG_MPK_SOLO=0 python3 -u bench.py $HEAD --gpus $N --devices $D || exit 2
  done
done
step 600 bench_${V}_stripes_8_solo7.json env GG_MPK_SPLIT=stripes GG_MPK_SOLO=7 python3 -u bench.py $HEAD --gpus 8 --devices 0,0,0,0,0,0,0,0 || exit 2
if [[ "${TRACE:-1}" == 1 ]]; then
  for SP in stripes wires; do
    export GG_MPK_SPLIT=$SP GG_MPK_SOLO=0
    step 600 prof_${V}_${SP}.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${V}_${SP} -o run -- \
      python3 -u bench.py $HEAD --steps 3 --gpus 8 --devices 0,0,0,0,0,0,0,0 || exit 2
  done
fi
echo done >> gpurun_out/progress_$V.txt
