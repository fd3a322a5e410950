#!/bin/bash
# per-kernel time + one-step timeline of the 1-GPU steady-state DiFacto step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/p1 -o p1 -- python3 bench.py --steps 100 --warmup 5 --prewarm 1000 > gpurun_out/prof/p1.log 2>&1 || { echo P1 FAILED; tail -20 gpurun_out/prof/p1.log; exit 1; }
grep '^{' gpurun_out/prof/p1.log | cut -c1-300
