#!/bin/bash
# Round 6 p: one rehearsed PlonK part (2^22, 8 parts, part 2) on the kept-worker
# tree with the HIP API trace beside the kernel trace: what the host threads do
# in the part's idle gaps (the challenge hand-overs).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r06p}"
echo "=== $(date +%T) part2 hip trace" >> gpurun_out/progress_$V.txt
timeout -k 10 300 env PROBE_PARTS=2 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/part2h_$V -o run -- python3 -u tools/plonk_part_probe.py 22 8 3 > gpurun_out/part2h_$V.txt 2>&1 || exit 2
echo "=== rc=0 $(date +%T)" >> gpurun_out/progress_$V.txt
