#!/bin/bash
# Round 5 a: (1) does an exchange copy wait for a kernel on another stream
# (tools/mbench_xqueue), (2) the new C99 caller + Groth16 GPU tests, (3) the
# headline's kernel trace with the product library and with the traffic-probe
# build (points from L2: how much of the G1 accumulation is the gathers), (4)
# the 8-shard one-GPU rehearsal's exchange push times (baseline).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05a}"
HEAD="--steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection="
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-xq,test,prof,probe,reh}"
if [[ "$S" == *xq* ]]; then step 150 xq_$V.txt tools/mbench_xqueue 8 176 12 400 || exit 2; fi
if [[ "$S" == *test* ]]; then
  step 400 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_c_caller.py tests/test_gpu_groth16.py tests/test_gpu_groth16_multi.py || exit 2
fi
if [[ "$S" == *prof* ]]; then
  step 400 prof_base_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_base_$V -o run -- python3 -u bench.py $HEAD || exit 2
fi
if [[ "$S" == *probe* ]]; then
  export GNARK_AMD_LIB=$PWD/gnark-fork_amd/lib/var/libgnark_amd_probe.so GNARK_AMD_ALLOW_PROBE=1
  step 400 prof_probe_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_probe_$V -o run -- python3 -u bench.py $HEAD || exit 2
  unset GNARK_AMD_LIB GNARK_AMD_ALLOW_PROBE
fi
if [[ "$S" == *reh* ]]; then
  step 500 reh8_$V.json python3 -u bench.py --gpus 1 --devices 0,0,0,0,0,0,0,0 --steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection= || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
