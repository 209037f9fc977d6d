#!/bin/bash
# Round-2 rehearsal of bench.py's N > 1 path on a one-GPU box: torch.distributed
# ranks share the GPU with GG_DIST_BACKEND=gloo (RCCL refuses two ranks on one
# device), reduced sizes; checks the JSON line, the strong-scaled sharded prove
# (proof identical on all ranks) and the MSM / PlonK extras at N = 2 and 4.
# Also runs the PlonK numerator parity tests after a kernel change.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-e}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 240 pytest_num_$V.txt python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bls.py -k "numerator or divide" || exit 2
SMALL="--log-n 20 --steps 3 --warmup 1 --msm-log-n 18 --ntt-log-n 0 --plonk-log-n 14 --no-cpu-baseline"
export GG_DIST_BACKEND=gloo
step 300 bench_w2_$V.txt python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 $SMALL || exit 2
step 300 bench_w4_$V.txt python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 4 $SMALL || exit 2
echo done >> gpurun_out/progress_$V.txt
