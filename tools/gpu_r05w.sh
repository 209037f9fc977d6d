#!/bin/bash
# Round 5 w: BN254 G1 accumulation gathering the next point straight into LDS
# (variant build -DGG_G1_LDS=1, the ring the G2 / BLS12-381 accumulations use)
# against the default register loop: G1 parity on the variant, then the one-GPU
# 2^24 prove and the 8-way shard, alternating.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05w}"
VL=gnark-fork_amd/lib/var/libgnark_amd_g1lds.so
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 600 pytest_lds_$V.txt env GNARK_AMD_LIB=$VL python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_msm_batch.py tests/test_gpu_groth16_size.py || exit 2
step 150 g_def1_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_lds1_$V.txt env GNARK_AMD_LIB=$VL python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_def2_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_lds2_$V.txt env GNARK_AMD_LIB=$VL python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 s_def_$V.txt env PROBE_SLEEP=0 python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 s_lds_$V.txt env PROBE_SLEEP=0 GNARK_AMD_LIB=$VL python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 300 clk_lds_$V.txt env GNARK_AMD_LIB=$VL timeout -s KILL 280 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/clk_lds_$V -o run -- python3 bench.py --steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection= || exit 2
echo done >> gpurun_out/progress_$V.txt
