#!/bin/bash
# Round 6 h: the final tree -- the roofline record's PMC passes of the 2^24
# headline (FETCH_SIZE, WRITE_SIZE, SQ + GRBM_GUI_ACTIVE, FETCH_SIZE of the
# traffic-probe build) and of configs[1]'s 2^20 G1 MSM (FETCH, WRITE, SQ + GRBM),
# the kernel-trace summary, the driver's bench command, the -m gpu suite, smoke.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r06h}"
HEAD="--steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection="
PROBE_LIB=gnark-fork_amd/lib/var/libgnark_amd_probe.so
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 300 pmc_f_$V.txt timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_$V -o run -- python3 bench.py $HEAD || exit 2
step 300 pmc_w_$V.txt timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_$V -o run -- python3 bench.py $HEAD || exit 2
step 300 pmc_sq_$V.txt timeout -s KILL 280 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq_$V -o run -- python3 bench.py $HEAD || exit 2
step 300 pmc_fprobe_$V.txt env GNARK_AMD_LIB=$PROBE_LIB GNARK_AMD_ALLOW_PROBE=1 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fprobe_$V -o run -- python3 bench.py $HEAD || exit 2
step 150 msm_f_$V.txt timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/msm_f_$V -o run -- python3 tools/bench_msm.py G1 20 5 || exit 2
step 150 msm_w_$V.txt timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/msm_w_$V -o run -- python3 tools/bench_msm.py G1 20 5 || exit 2
step 150 msm_sq_$V.txt timeout -s KILL 140 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/msm_sq_$V -o run -- python3 tools/bench_msm.py G1 20 5 || exit 2
step 400 prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$V -o run -- python3 -u bench.py --steps 5 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection= || exit 2
step 600 bench_$V.json python3 -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 2
step 900 pytest_$V.txt python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ || exit 2
step 300 smoke_$V.txt python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit 2
echo done >> gpurun_out/progress_$V.txt
