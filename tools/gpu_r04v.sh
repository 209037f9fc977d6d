#!/bin/bash
# Round 4 v: with the 4-key-vector chunk histogram as the default, isolated
# 2^24 G1 MSM phase times (tools/bench_msm.py) per sort variant, two alternating
# rounds: default (GG_SEG_CH 4096, spb 512); GG_SEG_CH 2048 / 1024 libraries
# (build_var/); GG_SORT_SPB 256 / 128 (smaller bin-scatter tiles); 2048 + 256.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04v}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" >> "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
setvar() {
  unset GG_SORT_SPB
  export GNARK_AMD_LIB=$PWD/gnark-fork_amd/lib/libgnark_amd.so
  case $1 in
    ch2048|ch1024) export GNARK_AMD_LIB=$PWD/build_var/libgnark_amd_$1.so ;;
    spb256) export GG_SORT_SPB=256 ;;
    spb128) export GG_SORT_SPB=128 ;;
    ch2048spb256) export GNARK_AMD_LIB=$PWD/build_var/libgnark_amd_ch2048.so GG_SORT_SPB=256 ;;
  esac
  export TAG=$1
}
for var in base ch2048 ch1024 spb256 ch2048spb256; do
  setvar $var
  step 300 pytest_${var}_$V.txt python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_stripe.py || exit 2
done
for round in 1 2; do
  for var in base ch2048 ch1024 spb256 spb128 ch2048spb256; do
    setvar $var
    step 200 msm_$V.txt python3 -u tools/bench_msm.py G1 24 10 || exit 2
    step 200 msm_$V.txt python3 -u tools/bench_msm.py G2 22 10 || exit 2
  done
done
echo done >> gpurun_out/progress_$V.txt
