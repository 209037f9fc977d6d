#!/bin/bash
# Round 5 y: the BN254 G1 LDS gathers with the nontemporal hint on 4-GB tables
# and up (variant -DGG_G1_LDS_NT=1) against the default policy, one-GPU 2^24
# prove, alternating; G1 MSM parity on the variant.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05y}"
VL=gnark-fork_amd/lib/var/libgnark_amd_g1ldsnt.so
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 300 pytest_nt_$V.txt env GNARK_AMD_LIB=$VL python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py || exit 2
step 150 g_def1_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_nt_1_$V.txt env GNARK_AMD_LIB=$VL python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_def2_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_nt_2_$V.txt env GNARK_AMD_LIB=$VL python3 -u tools/g16_time.py 24 20 3 || exit 2
echo done >> gpurun_out/progress_$V.txt
