#!/bin/bash
# MSM sizes after the occupancy-based range length (round 2).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
rm -f gpurun_out/sweep.txt
LOGS="20 24" CONFIGS="none" bash tools/sweep_msm.sh || exit 1
GROUP=G2 LOGS="23" REPS=3 CONFIGS="none" bash tools/sweep_msm.sh || exit 1
