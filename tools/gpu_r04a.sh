#!/bin/bash
# Round 4 a: FETCH_SIZE calibration over a 16-GiB gather table (the 2^24 G1
# tables are 12.9 GB), parity of the reworked multi-GPU paths (BLS12-381
# distributed computeH, rehearsal API, per-shard timings, the 2^24 proof
# through the default 8-way wire split), and a kernel trace of the primary
# part of an 8-part 2^22 PlonK proof.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r04a}"
step() {  # step <secs> <log> cmd...
  local secs=$1 logf=$2; shift 2
  echo "=== $(date +%T) $*" >> gpurun_out/progress_$V.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$logf" 2>&1
  local rc=$?
  echo "=== rc=$rc $(date +%T)" >> gpurun_out/progress_$V.txt
  return $rc
}
S="${STEPS:-test,probe}"
if [[ "$S" == *calib* ]]; then
  step 120 calib_stdout_$V.txt tools/mbench_gather_calib 16 || exit 2
  step 120 calib_pmc_$V.txt timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib_$V -o run -- tools/mbench_gather_calib 16 || exit 2
fi
if [[ "$S" == *r29* ]]; then  # the radix-2^29 BN254 fr passes (opt-in until measured)
  step 300 pytest_r29_$V.txt env GG_NTT_R29=1 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_ntt.py tests/test_gpu_dist_h.py -k "not bls" || exit 2
  step 200 ntt_r29_$V.txt env GG_NTT_R29=1 python3 -u tools/bench_ntt.py || exit 2
  step 200 ntt_r32_$V.txt python3 -u tools/bench_ntt.py || exit 2
fi
if [[ "$S" == *test* ]]; then
  step 900 pytest_$V.txt python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_ntt.py tests/test_gpu_msm.py tests/test_gpu_dist_h.py tests/test_gpu_groth16_multi.py tests/test_gpu_bls_groth16.py \
    tests/test_gpu_plonk_poly.py tests/test_gpu_plonk_prove.py tests/test_gpu_groth16_size.py ${PYTEST_ARGS} || exit 2
fi
if [[ "$S" == *probe* ]]; then
  step 300 probe_$V.txt python3 -u tools/plonk_part_probe.py 22 8 3 || exit 2
  step 300 probe_prof_$V.txt rocprofv3 --kernel-trace --stats -d gpurun_out/probe_prof_$V -o run -- \
    python3 -u tools/plonk_part_probe.py 22 8 2 || exit 2
fi
echo done >> gpurun_out/progress_$V.txt
