#!/bin/bash
# Round 5 c: A/B of the accumulation loops on one box.  Libraries: main (G1
# software pipeline without same-step waits, G2 next point gathered into LDS),
# r4loop (round 4's loops, -DGG_ACCUM_R4LOOP=1), probe (main with the points
# pinned to 1024 cached ones).  Per library: the headline bench (HIP-event
# kernel times) and a GRBM_GUI_ACTIVE pass (effective clock per kernel).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05c}"
HEAD="--steps 5 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection="
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 600 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_msm.py tests/test_gpu_groth16.py tests/test_gpu_msm_groups.py tests/test_gpu_msm_stripe.py || exit 2
for lib in main r4loop probe main2; do
  case $lib in main|main2) export GNARK_AMD_LIB=$PWD/gnark-fork_amd/lib/libgnark_amd.so ;;
    *) export GNARK_AMD_LIB=$PWD/gnark-fork_amd/lib/var/libgnark_amd_$lib.so ;; esac
  [ $lib = probe ] && export GNARK_AMD_ALLOW_PROBE=1
  step 300 bench_${lib}_$V.json python3 -u bench.py $HEAD || exit 2
  step 300 clk_${lib}_$V.txt timeout -s KILL 280 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/clk_${lib}_$V -o run -- python3 -u bench.py $HEAD || exit 2
  unset GNARK_AMD_ALLOW_PROBE
done
echo done >> gpurun_out/progress_$V.txt
