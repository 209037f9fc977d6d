#!/bin/bash
# Round 5 i: the timing rehearsal's solo shard on dedicated hardware queues
# (g16_restream) -- shard 0 / 3 of the 8-way 2^24 split timed and traced; the
# Groth16 multi-GPU and size tests on the new streams.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05i}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 200 shard0_$V.txt python3 -u tools/g16_shard_probe.py 24 8 0 6 || exit 2
step 200 shard3_$V.txt python3 -u tools/g16_shard_probe.py 24 8 3 6 || exit 2
step 200 shard0w18_$V.txt env GG_MSM_WINDOW=18 python3 -u tools/g16_shard_probe.py 24 8 0 6 || exit 2
step 300 shard0_tr_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/shard0_$V -o run -- python3 -u tools/g16_shard_probe.py 24 8 0 3 || exit 2
step 600 pytest_g16_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_groth16_multi.py tests/test_gpu_groth16_size.py || exit 2
echo done >> gpurun_out/progress_$V.txt
