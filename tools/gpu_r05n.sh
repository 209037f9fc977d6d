#!/bin/bash
# Round 5 n: the 8-way shard's accumulation runs 24 % above 1/8 of the one-GPU
# one (r05m serial trace) -- range length (GG_MSM_K1; 64 is picked below 2^26
# entries) and the B1 / G2 window (GG_G16_B_WINDOW) swept on shard 0.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05n}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
export PROBE_SLEEP=0
step 150 s_def_$V.txt python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 s_k128_$V.txt env GG_MSM_K1=128 python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 s_k96_$V.txt env GG_MSM_K1=96 python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 s_k48_$V.txt env GG_MSM_K1=48 python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 s_b16_$V.txt env GG_G16_B_WINDOW=16 python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 s_b18_$V.txt env GG_G16_B_WINDOW=18 python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 s_def2_$V.txt python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 s_nt0_$V.txt env GNARK_AMD_LIB=gnark-fork_amd/lib/var/libgnark_amd_nt0.so python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
echo done >> gpurun_out/progress_$V.txt
