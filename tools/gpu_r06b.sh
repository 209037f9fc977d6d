#!/bin/bash
# Round 6 b: (1) the VALU issue costs in counted cycles (k_mad_tp under
# SQ_INSTS_VALU / GRBM_GUI_ACTIVE) for roofline.valu; (2) configs[1]'s 2^20 G1
# MSM: FETCH, WRITE and SQ+GRBM passes of this tree; (3) the PlonK parts on
# dedicated hardware queues with rehearsal hand-overs (GG_PLONK_PART_QUEUES=1):
# the GPU test, the group tests, then r05k's command (bench_plonk 22 8 8) with
# every library wait bounded at 40 s -- a stall ends in GG_ERR_TIMEOUT naming the
# wait instead of a silent kill.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r06b}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 120 cap_$V.txt timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/cap_$V -o run -- tools/mbench_field || exit 2
step 150 msm_f_$V.txt timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/msm_f_$V -o run -- python3 tools/bench_msm.py G1 20 5 || exit 2
step 150 msm_w_$V.txt timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/msm_w_$V -o run -- python3 tools/bench_msm.py G1 20 5 || exit 2
step 150 msm_sq_$V.txt timeout -s KILL 140 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/msm_sq_$V -o run -- python3 tools/bench_msm.py G1 20 5 || exit 2
step 100 msm_t_$V.txt python3 tools/bench_msm.py G1 20 20 || exit 2
step 400 pytest_q_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_task_queues.py tests/test_gpu_plonk_group.py || exit 2
step 240 plonk_pq_$V.json env GG_PLONK_PART_QUEUES=1 GG_WAIT_TIMEOUT_S=40 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
echo done >> gpurun_out/progress_$V.txt
