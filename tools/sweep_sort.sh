# MSM tuning sweep: MSM tests, then msm phase times per configuration.
# CONFIGS: space-separated list of comma-joined env assignments, e.g. "GG_SORT_H=6,GG_SORT_RMAX=8"
set -e
mkdir -p gpurun_out
[ -n "$NOTEST" ] || timeout -k 10 500 python -m pytest tests/test_gpu_msm.py -m gpu -q -x > gpurun_out/pt_msm.txt 2>&1
for L in ${LOGS:-20 24}; do for C in ${CONFIGS:-none}; do
  ( [ "$C" != none ] && export $(echo $C | tr ',' ' ');
    timeout -k 10 200 python bench.py --log-n $L --steps 5 --warmup 1 --no-cpu-baseline --groth16-log-n 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('L=$L $C ${TAG}', round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()})" >> gpurun_out/sweep.txt )
done; done
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --log-n ${PROF} --steps 3 --warmup 1 --no-cpu-baseline --groth16-log-n 0 > gpurun_out/prof.log 2>&1
fi
