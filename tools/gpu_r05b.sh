#!/bin/bash
# Round 5 b: the G1 accumulation's prefetch fixed (unconditional loads, no wait
# on the fresh gather) + high-priority copy streams: MSM / Groth16 / multi-GPU /
# PlonK parity, the queue microbenchmark v2 (host-timed), the headline kernel
# trace, the 8-shard rehearsal's push times.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05b}"
HEAD="--steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection="
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-test,xq,prof,reh}"
if [[ "$S" == *test* ]]; then
  step 600 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_msm.py tests/test_gpu_groth16.py tests/test_gpu_groth16_multi.py tests/test_gpu_msm_stripe.py \
    tests/test_gpu_msm_groups.py tests/test_c_caller.py tests/test_gpu_plonk_group.py || exit 2
fi
if [[ "$S" == *xq* ]]; then step 150 xq2_$V.txt tools/mbench_xqueue2 8 176 12 400 || exit 2; fi
if [[ "$S" == *prof* ]]; then
  step 400 prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$V -o run -- python3 -u bench.py $HEAD || exit 2
fi
if [[ "$S" == *reh* ]]; then
  step 500 reh8_$V.json python3 -u bench.py --gpus 1 --devices 0,0,0,0,0,0,0,0 --steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection= || exit 2
fi
if [[ "$S" == *size* ]]; then
  step 900 pytest_size_$V.txt python3 -u -m pytest -x -v --timeout 800 --timeout-method thread -m gpu tests/test_gpu_groth16_size.py || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
