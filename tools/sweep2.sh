#!/bin/bash
# MSM sweep: G1 2^20 and 2^24 over window / range-length settings (round 2).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
rm -f gpurun_out/sweep.txt
LOGS=20 CONFIGS="none GG_MSM_K1=16 GG_MSM_K1=64 GG_MSM_WINDOW=19 GG_MSM_WINDOW=19,GG_MSM_K1=16" bash tools/sweep_msm.sh || exit 1
LOGS=24 REPS=4 CONFIGS="none GG_MSM_K1=128 GG_MSM_WINDOW=22 GG_MSM_WINDOW=22,GG_MSM_K1=32 GG_MSM_WINDOW=22,GG_MSM_K1=128" bash tools/sweep_msm.sh || exit 1
GROUP=G2 LOGS=23 REPS=3 CONFIGS="none GG_MSM_WINDOW=22" bash tools/sweep_msm.sh || exit 1
