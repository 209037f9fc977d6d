#!/bin/bash
# Round 6 x: the driver's bench command and smoke once more on the final tree
# (another box: the box-to-box spread of the headline)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V="${V:-r06x}"
echo "=== $(date +%T) bench" >> gpurun_out/progress_$V.txt
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$V.json 2>&1 || exit 2
echo "=== $(date +%T) smoke" >> gpurun_out/progress_$V.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$V.txt 2>&1 || exit 2
echo done >> gpurun_out/progress_$V.txt
