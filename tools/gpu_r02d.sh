#!/bin/bash
# Round-2 headline profile set: rocprofv3 kernel trace of the bench headline
# alone (2^24 Groth16 prove), FETCH_SIZE / WRITE_SIZE and SQ VALU counters in
# separate --pmc passes (MI355X_MICROARCH.md: one block budget per pass).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-v9}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
HEAD="--steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline"
step 300 prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$V -o run -- python3 bench.py $HEAD || exit 2
step 200 pmc_f_$V.txt timeout -s KILL 190 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_$V -o run -- python3 bench.py $HEAD || exit 2
step 200 pmc_w_$V.txt timeout -s KILL 190 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_$V -o run -- python3 bench.py $HEAD || exit 2
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY"
step 200 pmc_sq_$V.txt timeout -s KILL 190 rocprofv3 --pmc $SQ -d gpurun_out/pmc_sq_$V -o run -- python3 bench.py $HEAD || exit 2
echo done >> gpurun_out/progress_$V.txt
