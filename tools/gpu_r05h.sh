#!/bin/bash
# Round 5 h: dedicated hardware queues for the Groth16 prove's five tasks
# (create_task_stream) -- A/B against the shared pool (GG_TASK_QUEUES=0) on the
# one-GPU headline and on shard 0 of the 8-way split; window widths for the
# shard; kernel trace of the shard with the new queues.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05h}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 200 g16_new1_$V.txt python3 -u tools/g16_time.py 24 12 3 || exit 2
step 200 g16_old1_$V.txt env GG_TASK_QUEUES=0 python3 -u tools/g16_time.py 24 12 3 || exit 2
step 200 g16_new2_$V.txt python3 -u tools/g16_time.py 24 12 3 || exit 2
step 200 g16_old2_$V.txt env GG_TASK_QUEUES=0 python3 -u tools/g16_time.py 24 12 3 || exit 2
step 200 shard_new_$V.txt python3 -u tools/g16_shard_probe.py 24 8 0 5 || exit 2
step 200 shard_old_$V.txt env GG_TASK_QUEUES=0 python3 -u tools/g16_shard_probe.py 24 8 0 5 || exit 2
step 200 shard_w17_$V.txt env GG_MSM_WINDOW=17 python3 -u tools/g16_shard_probe.py 24 8 0 5 || exit 2
step 200 shard_w18_$V.txt env GG_MSM_WINDOW=18 python3 -u tools/g16_shard_probe.py 24 8 0 5 || exit 2
step 300 shard0_tr_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/shard0_$V -o run -- python3 -u tools/g16_shard_probe.py 24 8 0 3 || exit 2
step 300 g16_tr_new_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/g16new_$V -o run -- python3 -u tools/g16_time.py 24 3 2 || exit 2
GG_TASK_QUEUES=0 step 300 g16_tr_old_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/g16old_$V -o run -- python3 -u tools/g16_time.py 24 3 2 || exit 2
echo done >> gpurun_out/progress_$V.txt
