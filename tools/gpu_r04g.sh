#!/bin/bash
# Round 4 g: the driver's N > 1 launch shape (torch.distributed.run, one process
# per rank, bench.py --gpus N, the scaling run's path) rehearsed on one GPU over
# gloo (RCCL needs distinct GPUs; ranks share device 0, so times are not N-GPU
# times): 2 / 4 / 8 ranks at 2^20 with the MSM and PlonK extras, 2 ranks at the
# 2^24 headline; plus the uneven-weight PlonK parity test.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04g}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 300 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_plonk_prove.py -k "part0_weight or rehearsal" || exit 2
EX="--steps 3 --warmup 1 --log-n 20 --msm-log-n 16 --ntt-log-n 0 --plonk-log-n 12 --no-cpu-baseline"
export GG_DIST_BACKEND=gloo
step 600 torchrun_${V}_2.json python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 2 $EX || exit 2
step 600 torchrun_${V}_4.json python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29582 bench.py --gpus 4 $EX || exit 2
step 600 torchrun_${V}_8.json python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29583 bench.py --gpus 8 $EX || exit 2
step 900 torchrun_${V}_2p24.json python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29584 bench.py --gpus 2 --steps 3 --warmup 1 \
  --msm-log-n 20 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline || exit 2
echo done >> gpurun_out/progress_$V.txt
