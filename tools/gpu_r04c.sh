#!/bin/bash
# Round 4 c: PlonK canonical forms on the peer parts -- PlonK parity (one GPU and
# multi-part keys, every part on device 0), then the 8-part probe (real proof +
# rehearsals of part 0) plain and under the kernel trace.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04c}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-test,probe,sortab}"
if [[ "$S" == *test* ]]; then
  step 600 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_msm.py tests/test_gpu_bls.py tests/test_gpu_plonk_prove.py tests/test_gpu_plonk_poly.py || exit 2
fi
if [[ "$S" == *probe* ]]; then
  step 300 probe_$V.txt python3 -u tools/plonk_part_probe.py 22 8 3 || exit 2
  step 300 probe_prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/probe_prof_$V -o run -- \
    python3 -u tools/plonk_part_probe.py 22 8 2 || exit 2
fi
if [[ "$S" == *sortab* ]]; then  # bin scatter from the scalars (default) vs from a stored key array
  H="--steps 5 --warmup 1 --no-variants --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection ''"
  step 300 sort_new_$V.json python3 -u bench.py $H || exit 2
  step 300 sort_keys_$V.json env GG_SORT_KEYS=1 python3 -u bench.py $H || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
