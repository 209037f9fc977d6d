#!/bin/bash
# Round 4 l: the default bench line (driver's command) after the PlonK
# projection's round-robin rehearsals.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04l}"
echo "=== $(date +%T) bench" >> gpurun_out/progress_$V.txt
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$V.json 2>&1
rc=$?
echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
exit $rc
