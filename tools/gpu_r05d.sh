#!/bin/bash
# Round 5 d: accumulation A/B on one box, second pass.  Libraries: main (BN254 G1
# round-4 loop, BN254 G2 + BLS12-381 G1 next point gathered into LDS), nt (main
# with nontemporal point gathers), r4loop (round 4's loops everywhere), probe
# (main with points from 1024 cached entries).  Per library: the headline
# bench and the 2^22 PlonK prove with its 8-part rehearsal (tools/bench_plonk.py).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05d}"
HEAD="--steps 5 --warmup 1 --no-variants --msm-log-n 0 --ntt-log-n 0 --plonk-log-n 0 --no-cpu-baseline --solver 0 --projection="
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
step 900 pytest_$V.txt python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_msm.py tests/test_gpu_bls.py tests/test_gpu_groth16.py tests/test_gpu_plonk_prove.py \
  tests/test_gpu_bls_groth16.py tests/test_gpu_plonk_group.py || exit 2
for lib in main nt r4loop probe main2; do
  case $lib in main|main2) export GNARK_AMD_LIB=$PWD/gnark-fork_amd/lib/libgnark_amd.so ;;
    *) export GNARK_AMD_LIB=$PWD/gnark-fork_amd/lib/var/libgnark_amd_$lib.so ;; esac
  [ $lib = probe ] && export GNARK_AMD_ALLOW_PROBE=1
  step 300 bench_${lib}_$V.json python3 -u bench.py $HEAD || exit 2
  if [ $lib != probe ]; then
    step 400 plonk_${lib}_$V.json python3 -u tools/bench_plonk.py 22 3 8 || exit 2
  fi
  unset GNARK_AMD_ALLOW_PROBE
done
echo done >> gpurun_out/progress_$V.txt
