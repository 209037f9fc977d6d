#!/bin/bash
# Round 4 e: PlonK parity after the early unit evaluations, the 8-part probe,
# and the one-GPU PlonK 2^22 proof's kernel trace + SQ counters (is the
# BLS12-381 accumulation at its issue ceiling?).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04e}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-test,probe,plonk1}"
if [[ "$S" == *test* ]]; then
  step 600 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_plonk_prove.py tests/test_gpu_scs_solver.py tests/test_gpu_solver.py || exit 2
fi
if [[ "$S" == *probe* ]]; then
  step 300 probe_$V.txt python3 -u tools/plonk_part_probe.py 22 8 3 || exit 2
  step 300 smoke_$V.txt python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit 2
fi
if [[ "$S" == *plonk1* ]]; then
  step 300 plonk1_prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/plonk1_prof_$V -o run -- \
    python3 -u tools/plonk_part_probe.py 22 1 2 || exit 2
  step 300 plonk1_sq_$V.txt timeout -s KILL 280 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
    -d gpurun_out/plonk1_sq_$V -o run -- python3 -u tools/plonk_part_probe.py 22 1 1 || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
