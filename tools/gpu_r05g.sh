#!/bin/bash
# Round 5 g: where one GPU's share goes -- kernel traces of (1) shard 0 of the
# 2^24 Groth16 key split 8 ways (tools/g16_shard_probe.py), (2) PlonK 2^22 x 8
# parts 1 and 3 (part 3 is the slowest part of the rehearsals, r05d/f).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05g}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 400 shard0_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/shard0_$V -o run -- python3 -u tools/g16_shard_probe.py 24 8 0 3 || exit 2
step 300 part1_$V.txt env PROBE_PARTS=1 rocprofv3 --kernel-trace --stats -d gpurun_out/part1_$V -o run -- python3 -u tools/plonk_part_probe.py 22 8 3 || exit 2
step 300 part3_$V.txt env PROBE_PARTS=3 rocprofv3 --kernel-trace --stats -d gpurun_out/part3_$V -o run -- python3 -u tools/plonk_part_probe.py 22 8 3 || exit 2
echo done >> gpurun_out/progress_$V.txt
