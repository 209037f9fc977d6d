#!/bin/bash
# Round 4 t: sort-pass A/B through GNARK_AMD_LIB variants built from the same
# tree (build_var/): segmented-pass chunk size GG_SEG_CH 2048 / 8192 against the
# default 4096, and the 4-key-vector chunk histogram (GG_SEG_HIST_V).  Each
# variant (kp: the default library with GG_SORT_KEYPAD=1, key rows on 256-B
# boundaries): the MSM parity tests, then a kernel trace of the 2^24 prove.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04t}"
HEAD="--steps 5 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection="
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
for var in base ch2048 ch8192 hv hv8192 kp base2; do
  unset GG_SORT_KEYPAD; [ $var = kp ] && export GG_SORT_KEYPAD=1
  case $var in base|base2|kp) lib=gnark-fork_amd/lib/libgnark_amd.so ;; *) lib=build_var/libgnark_amd_$var.so ;; esac
  export GNARK_AMD_LIB=$PWD/$lib
  if [ "$var" != base2 ]; then
    step 400 pytest_${var}_$V.txt python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_stripe.py || exit 2
  fi
  step 300 prof_${var}_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${var}_$V -o run -- python3 -u bench.py $HEAD || exit 2
done
echo done >> gpurun_out/progress_$V.txt
