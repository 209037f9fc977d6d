#!/bin/bash
# Round-2 profiling session: per-dispatch NTT pass durations and SQ VALU
# counters (separate --pmc passes) for the NTT and the G1 MSM accumulation.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-c}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-trace,pmc}"
NTT="${NTT_LOG:-24}"
if [[ "$S" == *trace* ]]; then
  step 300 ntt_trace_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/ntt_trace_$V -o run -- python3 tools/bench_ntt.py $NTT || exit 2
fi
if [[ "$S" == *pmc* ]]; then
  SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY"
  step 120 pmc_ntt_$V.txt timeout -s KILL 100 rocprofv3 --pmc $SQ -d gpurun_out/pmc_ntt_$V -o run -- python3 tools/bench_ntt.py $NTT || exit 2
  step 120 pmc_msm_$V.txt timeout -s KILL 100 rocprofv3 --pmc $SQ -d gpurun_out/pmc_msm_$V -o run -- python3 tools/bench_msm.py G1 20 3 || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
