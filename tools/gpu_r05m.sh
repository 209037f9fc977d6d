#!/bin/bash
# Round 5 m: PlonK with dedicated queues for one-device keys only (parts on the
# shared pool again) -- 2^22 one-GPU + 8-part rehearsal, alternating with the
# shared pool; the PlonK GPU tests; the 8-way Groth16 shard timed without idle
# gaps and traced task by task on the shared pool (GG_G16_SERIAL=1) for its
# per-kernel work.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05m}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 150 plonk_new1_$V.json python3 -u tools/bench_plonk.py 22 6 8 || exit 2
step 150 plonk_old1_$V.json env GG_TASK_QUEUES=0 python3 -u tools/bench_plonk.py 22 6 8 || exit 2
step 150 plonk_new2_$V.json python3 -u tools/bench_plonk.py 22 6 8 || exit 2
step 150 shard_def_$V.txt env PROBE_SLEEP=0 python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 shard_nt0_$V.txt env PROBE_SLEEP=0 GNARK_AMD_LIB=gnark-fork_amd/lib/var/libgnark_amd_nt0.so python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 150 shard_r4_$V.txt env PROBE_SLEEP=0 GNARK_AMD_LIB=gnark-fork_amd/lib/var/libgnark_amd_r4loop.so python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 200 shard_ser_tr_$V.txt env GG_TASK_QUEUES=0 GG_G16_SERIAL=1 rocprofv3 --kernel-trace --stats -d gpurun_out/shard_ser_$V -o run -- python3 -u tools/g16_shard_probe.py 24 8 0 3 || exit 2
step 900 pytest_plonk_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_plonk_prove.py tests/test_gpu_plonk_group.py || exit 2
echo done >> gpurun_out/progress_$V.txt
