#!/bin/bash
# Round 5 v: traces for round 6's plan -- (1) the host-input 2^24 prove with
# its copies (kernel + memory-copy trace: when W lands, when the sorts and the
# computeH chain start), (2) a one-GPU 2^22 PlonK proof with the batched
# commitments (kernel trace, tools/part_breakdown.py).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05v}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 400 host_tr_$V.txt rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/host_$V -o run -- python3 -u bench.py --host-inputs --steps 3 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection= || exit 2
step 300 plonk1_tr_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/plonk1_$V -o run -- python3 -u tools/plonk_part_probe.py 22 1 3 || exit 2
echo done >> gpurun_out/progress_$V.txt
