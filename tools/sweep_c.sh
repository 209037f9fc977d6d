#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for c in ${CS:-16 17 18 19 20 21 22}; do
  GG_MSM_WINDOW=$c timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --groth16-log-n 0 --log-n ${LOGN:-20} > gpurun_out/sweep_c$c.txt 2>&1 || exit 2
  python -c "import json;d=json.loads(open('gpurun_out/sweep_c$c.txt').read().strip().splitlines()[-1]);print($c, round(d['ms_per_step'],3), {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()})" | tee -a gpurun_out/sweep.txt
done
