#!/bin/bash
# Round 5 l: why PlonK stalled on the dedicated queues (r05k: bench_plonk 22 8 8
# silent for 180 s, 13 s on the shared pool in r05f) -- small PlonK proofs per
# test, then the one-GPU 2^22 prove alone, each under a short limit; the shared
# pool for contrast.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05l}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 150 pytest_small_old_$V.txt env GG_TASK_QUEUES=0 python3 -u -m pytest -x -v --timeout 60 --timeout-method thread -m gpu tests/test_gpu_plonk_prove.py -k "match_oracle" || exit 2
step 120 plonk1_old_$V.json env GG_TASK_QUEUES=0 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
step 150 pytest_small_new_$V.txt python3 -u -m pytest -x -v --timeout 60 --timeout-method thread -m gpu tests/test_gpu_plonk_prove.py -k "match_oracle" || exit 2
step 120 plonk1_new_$V.json python3 -u tools/bench_plonk.py 22 3 || exit 2
echo done >> gpurun_out/progress_$V.txt
