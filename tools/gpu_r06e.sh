#!/bin/bash
# Round 6 e: task slots keep their own streams and borrow dedicated queues
# (common.h TaskQueue; no stream created or destroyed in a rehearsal): the
# 4-shard rehearsal probe that stalled in r06c/r06d, the queue / multi-GPU /
# PlonK GPU tests, r05k's PlonK command on dedicated part queues, then the A/B
# of the 16-B entry chunks (GG_RING_CHUNKS=0 variant) and their FETCH / L2 counters.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r06e}"
VL=gnark-fork_amd/lib/var/libgnark_amd_rc0.so
HEAD="--steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection="
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 100 probe_$V.txt env GG_TRACE_STREAMS=1 GG_WAIT_TIMEOUT_S=30 python3 -u tools/mpk_rehearsal_probe.py 4 1 3 0 || exit 2
step 900 pytest_$V.txt env GG_WAIT_TIMEOUT_S=60 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_task_queues.py tests/test_gpu_groth16_multi.py tests/test_gpu_plonk_prove.py tests/test_gpu_plonk_group.py || exit 2
step 240 plonk_pq_$V.json env GG_PLONK_PART_QUEUES=1 GG_WAIT_TIMEOUT_S=40 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
step 150 g_new1_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_rc01_$V.txt env GNARK_AMD_LIB=$VL python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_new2_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_rc02_$V.txt env GNARK_AMD_LIB=$VL python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 s_new_$V.txt env PROBE_SLEEP=0 python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 s_rc0_$V.txt env PROBE_SLEEP=0 GNARK_AMD_LIB=$VL python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 300 pmc_f_new_$V.txt timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_new_$V -o run -- python3 bench.py $HEAD || exit 2
step 300 pmc_f_rc0_$V.txt env GNARK_AMD_LIB=$VL timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_rc0_$V -o run -- python3 bench.py $HEAD || exit 2
step 300 pmc_h_new_$V.txt timeout -s KILL 280 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_h_new_$V -o run -- python3 bench.py $HEAD || exit 2
step 300 pmc_h_rc0_$V.txt env GNARK_AMD_LIB=$VL timeout -s KILL 280 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_h_rc0_$V -o run -- python3 bench.py $HEAD || exit 2
echo done >> gpurun_out/progress_$V.txt
