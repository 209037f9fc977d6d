#!/bin/bash
# Round 3 ad: kernel trace of the primary part of an 8-part PlonK 2^22 key proved
# with its peers idle (GG_PLONK_SOLO) -- where the critical GPU's 36 ms go.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-ad}"
echo "=== $(date +%T)" >> gpurun_out/progress_$V.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${V} -o run -- \
  python3 -u tools/bench_plonk.py 22 3 8 > gpurun_out/plonk_${V}.txt 2>&1
echo "=== rc=$? $(date +%T)" >> gpurun_out/progress_$V.txt
