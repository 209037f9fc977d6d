#!/bin/bash
# Round 6 n: host cost of starting GPU work from a fresh thread vs a persistent
# worker (tools/probe/thread_launch.hip, built in-tree beforehand).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probe/thread_launch > gpurun_out/thread_launch_r06n.txt 2>&1 || exit 2
timeout -k 10 60 ./tools/probe/thread_launch >> gpurun_out/thread_launch_r06n.txt 2>&1 || exit 2
