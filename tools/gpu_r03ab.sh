#!/bin/bash
# Round 3 ab: the default bench line (with the split projection extra).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-ab}"
echo "=== $(date +%T) bench" >> gpurun_out/progress_$V.txt
timeout -k 10 900 python3 -u bench.py > gpurun_out/bench_$V.json 2>&1
echo "=== rc=$? $(date +%T)" >> gpurun_out/progress_$V.txt
