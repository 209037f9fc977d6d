#!/bin/bash
# Round 5 k: dedicated hardware queues for PlonK's compute streams -- one-GPU
# 2^22 BLS12-381 prove and the 8-part rehearsal, new vs shared pool
# (GG_TASK_QUEUES=0), alternating; the 8-way Groth16 shard on the round-4
# accumulation loops (variant builds) against the default; the PlonK GPU tests.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05k}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 400 plonk_new1_$V.json python3 -u tools/bench_plonk.py 22 8 8 || exit 2
step 400 plonk_old1_$V.json env GG_TASK_QUEUES=0 python3 -u tools/bench_plonk.py 22 8 8 || exit 2
step 400 plonk_new2_$V.json python3 -u tools/bench_plonk.py 22 8 8 || exit 2
step 400 plonk_old2_$V.json env GG_TASK_QUEUES=0 python3 -u tools/bench_plonk.py 22 8 8 || exit 2
step 200 shard_def_$V.txt python3 -u tools/g16_shard_probe.py 24 8 0 6 || exit 2
step 200 shard_nt0_$V.txt env GNARK_AMD_LIB=gnark-fork_amd/lib/var/libgnark_amd_nt0.so python3 -u tools/g16_shard_probe.py 24 8 0 6 || exit 2
step 200 shard_r4_$V.txt env GNARK_AMD_LIB=gnark-fork_amd/lib/var/libgnark_amd_r4loop.so python3 -u tools/g16_shard_probe.py 24 8 0 6 || exit 2
step 900 pytest_plonk_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_plonk_prove.py tests/test_gpu_plonk_group.py || exit 2
echo done >> gpurun_out/progress_$V.txt
