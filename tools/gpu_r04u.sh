#!/bin/bash
# Round 4 u: isolated 2^24 G1 MSM phase times (tools/bench_msm.py, HIP-event
# profiler) per sort variant, two alternating rounds: default; GG_SEG_CH=2048
# and GG_SEG_HIST_V libraries (build_var/); GG_SORT_KEYPAD=1 (256-B aligned key
# rows); GG_SORT_SWZ=1 (XCD-aware digit-histogram tiles); all three of hv / kp /
# swz.  MSM parity tests for swz and for all.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04u}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" >> "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
setvar() {
  unset GG_SORT_KEYPAD GG_SORT_SWZ
  export GNARK_AMD_LIB=$PWD/gnark-fork_amd/lib/libgnark_amd.so
  case $1 in
    ch2048|hv) export GNARK_AMD_LIB=$PWD/build_var/libgnark_amd_$1.so ;;
    kp) export GG_SORT_KEYPAD=1 ;;
    swz) export GG_SORT_SWZ=1 ;;
    all) export GNARK_AMD_LIB=$PWD/build_var/libgnark_amd_hv.so GG_SORT_KEYPAD=1 GG_SORT_SWZ=1 ;;
  esac
  export TAG=$1
}
for var in swz all; do
  setvar $var
  step 300 pytest_${var}_$V.txt python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_stripe.py || exit 2
done
for round in 1 2; do
  for var in base ch2048 hv kp swz all; do
    setvar $var
    step 200 msm_$V.txt python3 -u tools/bench_msm.py G1 24 10 || exit 2
  done
done
echo done >> gpurun_out/progress_$V.txt
