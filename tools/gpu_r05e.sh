#!/bin/bash
# Round 5 e: (1) the queue microbenchmark under a kernel + copy trace (the copy
# on a high-priority stream finishes while the MSM-shaped kernel runs; on a
# shared queue it waits), (2) nontemporal G1 gathers default vs GG_PT_NT=0,
# alternating, (3) the driver's N > 1 launch shape rehearsed over gloo (ranks
# share GPU 0): torchrun 2 / 4 ranks with the PlonK leader key, (4) GPU tests.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05e}"
HEAD="--steps 5 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection="
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-trace,ab,torch,test}"
if [[ "$S" == *trace* ]]; then
  step 200 xqtrace_$V.txt rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/xqtrace_$V -o run -- tools/mbench_xqueue2 8 176 12 400 || exit 2
fi
if [[ "$S" == *ab* ]]; then
  for lib in main nt0 main2 nt02; do
    case $lib in main*) export GNARK_AMD_LIB=$PWD/gnark-fork_amd/lib/libgnark_amd.so ;;
      *) export GNARK_AMD_LIB=$PWD/gnark-fork_amd/lib/var/libgnark_amd_nt0.so ;; esac
    step 300 bench_${lib}_$V.json python3 -u bench.py $HEAD || exit 2
  done
  unset GNARK_AMD_LIB
fi
if [[ "$S" == *torch* ]]; then
  EX="--steps 3 --warmup 1 --log-n 20 --msm-log-n 16 --ntt-log-n 0 --plonk-log-n 14 --no-cpu-baseline"
  export GG_DIST_BACKEND=gloo
  step 600 torchrun_${V}_2.json python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29591 bench.py --gpus 2 $EX || exit 2
  step 600 torchrun_${V}_4.json python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29592 bench.py --gpus 4 $EX || exit 2
  unset GG_DIST_BACKEND
fi
if [[ "$S" == *test* ]]; then
  step 900 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_msm.py tests/test_gpu_groth16.py tests/test_gpu_groth16_multi.py tests/test_gpu_plonk_prove.py \
    tests/test_gpu_plonk_group.py tests/test_c_caller.py || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
