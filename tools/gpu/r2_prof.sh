#!/bin/bash
# per-kernel time of the 1-GPU step and of the loopback P=8 exchange path
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/p1 -o p1 -- python3 bench.py --steps 100 --warmup 5 --prewarm 300 > gpurun_out/prof/p1.log 2>&1 || { echo P1 FAILED; tail -20 gpurun_out/prof/p1.log; exit 1; }
tail -1 gpurun_out/prof/p1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/lb8 -o lb8 -- python3 bench.py --steps 100 --warmup 5 --prewarm 300 --loopback 8 > gpurun_out/prof/lb8.log 2>&1 || { echo LB FAILED; tail -20 gpurun_out/prof/lb8.log; exit 1; }
tail -1 gpurun_out/prof/lb8.log
find gpurun_out/prof -name "*kernel_stats.csv" | head
