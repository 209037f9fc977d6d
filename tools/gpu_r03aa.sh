#!/bin/bash
# Round 3 aa: the driver's N = 2 launch (torch.distributed.run, bench.py --gpus 2)
# at the headline size, rehearsed on one GPU over gloo (two ranks share it; the
# exchanges go through host memory, so the time is not the N-GPU time): checks
# that the 2^24 sharded path runs end to end and both ranks agree on the proof.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-aa}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
export GG_DIST_BACKEND=gloo
step 900 torchrun_${V}_2p24.json python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --steps 3 --warmup 1 \
  --msm-log-n 20 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline || exit 2
echo done >> gpurun_out/progress_$V.txt
