#!/bin/bash
# Round 3 w: the driver's N > 1 launch shape (torch.distributed.run, one
# process per rank, bench.py --gpus N) rehearsed on one GPU over gloo (RCCL
# needs distinct GPUs): 2 and 4 ranks at 2^20 with the MSM and PlonK extras,
# wire slices and bucket stripes; then the one-process path at 2^20.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-w}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
EX="--steps 3 --warmup 1 --log-n 20 --msm-log-n 16 --ntt-log-n 0 --plonk-log-n 12 --no-cpu-baseline"
export GG_DIST_BACKEND=gloo
step 600 torchrun_${V}_2.json python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 $EX || exit 2
step 600 torchrun_${V}_4.json python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 4 $EX || exit 2
step 600 torchrun_${V}_2_stripes.json env GG_MPK_SPLIT=stripes python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29563 bench.py --gpus 2 $EX || exit 2
unset GG_DIST_BACKEND
step 600 mpk_${V}_4.json python3 -u bench.py --gpus 4 --devices 0,0,0,0 $EX || exit 2
echo done >> gpurun_out/progress_$V.txt
