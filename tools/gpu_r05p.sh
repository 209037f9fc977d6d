#!/bin/bash
# Round 5 p: scheduling / sort knobs on the 8-way shard and the one-GPU prove:
# computeH task at the greatest priority (GG_G16_H_PRIORITY=1), B1 / G2 entries
# derived from the A / K sort (GG_G16_B_DERIVE=1, one sort fewer), shorter
# accumulation ranges (GG_MSM_K1=48), alternating with the default.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05p}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
export PROBE_SLEEP=0
step 150 s_def1_$V.txt python3 -u tools/g16_shard_probe.py 24 8 0 10 || exit 2
step 150 s_hp_$V.txt env GG_G16_H_PRIORITY=1 python3 -u tools/g16_shard_probe.py 24 8 0 10 || exit 2
step 150 s_der_$V.txt env GG_G16_B_DERIVE=1 python3 -u tools/g16_shard_probe.py 24 8 0 10 || exit 2
step 150 s_k48_$V.txt env GG_MSM_K1=48 python3 -u tools/g16_shard_probe.py 24 8 0 10 || exit 2
step 150 s_def2_$V.txt python3 -u tools/g16_shard_probe.py 24 8 0 10 || exit 2
step 150 g_def1_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_hp_$V.txt env GG_G16_H_PRIORITY=1 python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_der_$V.txt env GG_G16_B_DERIVE=1 python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 g_def2_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
echo done >> gpurun_out/progress_$V.txt
