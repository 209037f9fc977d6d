#!/bin/bash
# Round 6 g: the sort with fewer launches (2-launch scans, chunk descriptors in
# the hist / scatter blocks, one-block chunk plan, no histogram zeroing): the
# whole -m gpu suite (parity of every MSM group, both provers, multi-GPU
# rehearsals), smoke, then timings -- one-GPU 2^24 prove, the 8-way shard, and
# PlonK 2^22 with its 8-part projection at the default part window and at 18 / 19.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r06g}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 1100 pytest_$V.txt env GG_WAIT_TIMEOUT_S=120 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ || exit 2
step 200 smoke_$V.txt python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit 2
step 150 g_$V.txt python3 -u tools/g16_time.py 24 20 3 || exit 2
step 150 s_$V.txt env PROBE_SLEEP=0 python3 -u tools/g16_shard_probe.py 24 8 0 8 || exit 2
step 200 plonk_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
step 200 plonk_pw18_$V.json env GG_PLONK_PART_WINDOW=18 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
step 200 plonk_pw19_$V.json env GG_PLONK_PART_WINDOW=19 python3 -u tools/bench_plonk.py 22 3 8 || exit 2
echo done >> gpurun_out/progress_$V.txt
