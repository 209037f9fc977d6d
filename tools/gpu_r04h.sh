#!/bin/bash
# Round 4 h: the per-MSM fixed cost of PlonK's 2^19-point BLS12-381 slices
# (2^22 key, 8 parts): part 0 and part 1 rehearsed alone under window / bucket
# reduction variants (environment knobs only, no rebuild).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04h}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
export PROBE_PARTS=0,1
step 300 probe_base_$V.txt python3 -u tools/plonk_part_probe.py 22 8 4 || exit 2
step 300 probe_seg16_$V.txt env GG_MSM_SEGSUM_MINLOG=16 python3 -u tools/plonk_part_probe.py 22 8 4 || exit 2
step 300 probe_c16_$V.txt env GG_MSM_WINDOW=16 python3 -u tools/plonk_part_probe.py 22 8 4 || exit 2
step 300 probe_c18_$V.txt env GG_MSM_WINDOW=18 python3 -u tools/plonk_part_probe.py 22 8 4 || exit 2
step 300 probe_c19_$V.txt env GG_MSM_WINDOW=19 python3 -u tools/plonk_part_probe.py 22 8 4 || exit 2
step 300 probe_base2_$V.txt python3 -u tools/plonk_part_probe.py 22 8 4 || exit 2
echo done >> gpurun_out/progress_$V.txt
