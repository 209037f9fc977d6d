#!/bin/bash
# Round 6 a: the LDS-ring accumulations read their sorted entries in 16-B chunks
# (EntryChunks, msm_impl.cuh) instead of one 4-B entry per step -- parity of the
# MSM groups and the 2^24 proof, then A/B against the round-5 loop (variant
# build -DGG_RING_CHUNKS=0): one-GPU 2^24 prove and the 8-way shard, alternating,
# and the G1 accumulation's FETCH_SIZE, L2 hits / misses and clock both ways.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r06a}"
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
step 900 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_batch.py tests/test_gpu_bls.py tests/test_gpu_groth16_size.py tests/test_gpu_groth16_multi.py tests/test_gpu_plonk_prove.py tests/test_gpu_task_queues.py || exit 2
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
