#!/bin/bash
# Round 4 b: the roofline record of the current tree -- PMC passes of the 2^24
# prove (FETCH_SIZE, WRITE_SIZE, SQ; each its own rocprofv3 run), a FETCH_SIZE
# pass with the accumulation's point gathers pinned to 1024 cached points
# (GG_ACCUM_PROBE=1: what is NOT point bytes), the kernel-trace summary of the
# headline, then the default bench line.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04b}"
HEAD="--steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection ''"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-pmc,probe,prof,reh,bench}"
if [[ "$S" == *pmc* ]]; then
  step 300 pmc_f_$V.txt timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_$V -o run -- python3 bench.py $HEAD || exit 2
  step 300 pmc_w_$V.txt timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_$V -o run -- python3 bench.py $HEAD || exit 2
  step 300 pmc_sq_$V.txt timeout -s KILL 280 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -d gpurun_out/pmc_sq_$V -o run -- python3 bench.py $HEAD || exit 2
fi
if [[ "$S" == *probe* ]]; then
  export GG_ACCUM_PROBE=1
  step 300 pmc_fprobe_$V.txt timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fprobe_$V -o run -- python3 bench.py $HEAD || exit 2
  step 300 pmc_wprobe_$V.txt timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_wprobe_$V -o run -- python3 bench.py $HEAD || exit 2
  unset GG_ACCUM_PROBE
fi
if [[ "$S" == *prof* ]]; then
  step 400 prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$V -o run -- \
    python3 -u bench.py --steps 5 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection '' || exit 2
fi
if [[ "$S" == *reh* ]]; then
  step 400 reh8_$V.json python3 -u bench.py --gpus 1 --devices 0,0,0,0,0,0,0,0 --steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --no-cpu-baseline --solver 0 --projection '' || exit 2
fi
if [[ "$S" == *bench* ]]; then step 600 bench_$V.json python3 -u bench.py || exit 2; fi
echo done >> gpurun_out/progress_$V.txt
