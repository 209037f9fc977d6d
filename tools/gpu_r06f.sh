#!/bin/bash
# Round 6 f: counters.  (1) G1 accumulation FETCH_SIZE and L2 hits / misses with
# the 16-B entry chunks and without (GG_RING_CHUNKS=0 variant), GRBM clock;
# (2) the VALU issue costs in counted cycles (k_mad_tp); (3) configs[1]'s 2^20
# G1 MSM: FETCH, WRITE, SQ + GRBM passes of this tree; (4) the 8-way Groth16
# shard's kernels task by task (GG_G16_SERIAL=1) for the per-kernel sort and
# reduction times.  Every rocprofv3 pass in a run of its own.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r06f}"
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
step 300 pmc_f_new_$V.txt timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_new_$V -o run -- python3 bench.py $HEAD || exit 2
step 300 pmc_f_rc0_$V.txt env GNARK_AMD_LIB=$VL timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_rc0_$V -o run -- python3 bench.py $HEAD || exit 2
step 300 pmc_h_new_$V.txt timeout -s KILL 280 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_h_new_$V -o run -- python3 bench.py $HEAD || exit 2
step 300 pmc_h_rc0_$V.txt env GNARK_AMD_LIB=$VL timeout -s KILL 280 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_h_rc0_$V -o run -- python3 bench.py $HEAD || exit 2
step 120 cap_$V.txt timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/cap_$V -o run -- tools/mbench_field || exit 2
step 150 msm_f_$V.txt timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/msm_f_$V -o run -- python3 tools/bench_msm.py G1 20 5 || exit 2
step 150 msm_w_$V.txt timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/msm_w_$V -o run -- python3 tools/bench_msm.py G1 20 5 || exit 2
step 150 msm_sq_$V.txt timeout -s KILL 140 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/msm_sq_$V -o run -- python3 tools/bench_msm.py G1 20 5 || exit 2
step 100 msm_t_$V.txt python3 tools/bench_msm.py G1 20 20 || exit 2
step 200 shard_ser_$V.txt env GG_G16_SERIAL=1 PROBE_SLEEP=0.05 rocprofv3 --kernel-trace --stats -d gpurun_out/shard_ser_$V -o run -- python3 -u tools/g16_shard_probe.py 24 8 0 3 || exit 2
VG=gnark-fork_amd/lib/var/libgnark_amd_g2s2.so
step 150 g_new_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_g2s2_$V.txt env GNARK_AMD_LIB=$VG python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_new2_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_g2s22_$V.txt env GNARK_AMD_LIB=$VG python3 -u tools/g16_time.py 24 20 3 || exit 2
step 200 plonk_def_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
step 200 plonk_w16_$V.json env GG_MSM_WINDOW=16 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
step 200 plonk_w15_$V.json env GG_MSM_WINDOW=15 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
echo done >> gpurun_out/progress_$V.txt
