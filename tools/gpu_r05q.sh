#!/bin/bash
# Round 5 q: the driver's process-per-GPU launch shape on the final tree
# (torch.distributed.run, gloo, every rank on GPU 0) with the dedicated task
# queues: 2, 4 and 8 ranks; each rank's Groth16 shard holds up to 5 CU-masked
# streams on the shared card.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05q}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
EX="--steps 3 --warmup 1 --log-n 20 --msm-log-n 16 --ntt-log-n 0 --plonk-log-n 14 --no-cpu-baseline"
export GG_DIST_BACKEND=gloo
step 300 torchrun_${V}_2.json python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29591 bench.py --gpus 2 $EX || exit 2
step 300 torchrun_${V}_4.json python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29592 bench.py --gpus 4 $EX || exit 2
step 400 torchrun_${V}_8.json python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29593 bench.py --gpus 8 $EX || exit 2
echo done >> gpurun_out/progress_$V.txt
