#!/bin/bash
# Round 6 i: openZ's quotient and the linearized polynomial in one batched MSM
# (pk.Kzg): PlonK parity (byte-identical proofs vs the oracle prover and the
# one-GPU proof from multi-part keys), then 2^22 with its 8-part projection,
# alternating with GG_PLONK_BATCH_OPEN=0.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r06i}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 600 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_plonk_prove.py tests/test_gpu_plonk_group.py tests/test_gpu_task_queues.py || exit 2
step 200 plonk_b_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
step 200 plonk_nb_$V.json env GG_PLONK_BATCH_OPEN=0 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
step 200 plonk_b2_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
step 200 plonk_nb2_$V.json env GG_PLONK_BATCH_OPEN=0 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
echo done >> gpurun_out/progress_$V.txt
