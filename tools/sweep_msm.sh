# MSM tuning sweep with tools/bench_msm.py: CONFIGS = space-separated list of
# comma-joined env assignments ("none" = defaults), LOGS = log sizes.
mkdir -p gpurun_out
for L in ${LOGS:-20 24}; do for C in ${CONFIGS:-none}; do
  ( [ "$C" != none ] && export $(echo $C | tr ',' ' ');
    TAG="$C" timeout -k 10 120 python tools/bench_msm.py ${GROUP:-G1} $L ${REPS:-10} >> gpurun_out/sweep.txt 2>&1 ) || exit 1
done; done
