#!/bin/bash
# Round 5 r: the task-queue GPU tests (queue budgets, keys beyond the budget,
# rehearsal hand-over, PlonK one-device key on either placement).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${V:-r05r}"
echo "=== $(date +%T) pytest" >> gpurun_out/progress_$V.txt
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_task_queues.py > gpurun_out/pytest_tq_$V.txt 2>&1
echo "=== rc=$? $(date +%T)" >> gpurun_out/progress_$V.txt
