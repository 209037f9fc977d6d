#!/bin/bash
# Round 5 o: the nontemporal hint per launch (tables >= GG_ACCUM_NT_GB, default
# 4 GB) -- shard 0 of the 8-way split (1.7-GB tables: hint off now) and the
# one-GPU 2^24 prove (12.9-GB tables: on), each against the other policy,
# alternating; the MSM and Groth16 parity tests.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05o}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
export PROBE_SLEEP=0
step 150 s_def1_$V.txt python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 s_nt_$V.txt env GG_ACCUM_NT_GB=0 python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 s_def2_$V.txt python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 g_def1_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_nont_$V.txt env GG_ACCUM_NT_GB=1000 python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_def2_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 900 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_groups.py tests/test_gpu_msm_stripe.py tests/test_gpu_groth16_size.py tests/test_gpu_groth16_multi.py || exit 2
echo done >> gpurun_out/progress_$V.txt
