#!/bin/bash
# Round 3: G1 accumulation occupancy / prefetch depth A/B (this tree: 2 waves per
# SIMD, points 2 deep; lib_w3: 3 waves, 1 deep; lib_pf1: 2 waves, 1 deep), with
# the MSM / Groth16 tests on each library first.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-k}"
HEAD="--steps 6 --warmup 2 --no-variants --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
T="tests/test_gpu_msm.py tests/test_gpu_groth16.py tests/test_gpu_msm_groups.py"
step 400 pytest_${V}_def.txt python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $T || exit 2
step 400 pytest_${V}_w3.txt env GNARK_AMD_LIB=gnark-fork_amd/lib_w3/libgnark_amd.so python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $T || exit 2
for r in 1 2; do
  step 300 bench_${V}_def$r.json python3 -u bench.py $HEAD || exit 2
  step 300 bench_${V}_w3$r.json env GNARK_AMD_LIB=gnark-fork_amd/lib_w3/libgnark_amd.so python3 -u bench.py $HEAD || exit 2
  step 300 bench_${V}_pf1$r.json env GNARK_AMD_LIB=gnark-fork_amd/lib_pf1/libgnark_amd.so python3 -u bench.py $HEAD || exit 2
done
echo done >> gpurun_out/progress_$V.txt
