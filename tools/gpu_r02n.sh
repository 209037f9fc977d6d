#!/bin/bash
# Round-2: rocprofv3 kernel trace of the BLS12-381 PlonK 2^22 prove (bench's
# configs[4] extra; the Groth16 headline shrunk to 2^16 so the trace is the
# PlonK prover's).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-n}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 400 prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$V -o run -- python3 bench.py --log-n 16 \
  --steps 1 --warmup 0 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 22 --no-cpu-baseline --solver 0 || exit 2
echo done >> gpurun_out/progress_$V.txt
