#!/bin/bash
# Sweep of the bucket-reduction variants on the headline 2^20 G1 MSM:
# GG_RED_BLOCK (1: one block-tree launch per round, 0: lockstep levels) x
# GG_RED_HOST_N (host-tail size).  Run on the GPU box.
set -o pipefail
mkdir -p gpurun_out
for blk in 1 0; do
  for hn in 16 8 4; do
    GG_RED_BLOCK=$blk GG_RED_HOST_N=$hn timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --groth16-log-n 0 --ntt-log-n 0 --plonk-log-n 0 > gpurun_out/sw_${blk}_${hn}.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/sw_${blk}_${hn}.json'));k=d['kernels'];print('block=$blk host_n=$hn', round(d['ms_per_step'],4), round(d['value'],1), {x:round(v['avg_ms'],4) for x,v in k.items()})"
  done
done
