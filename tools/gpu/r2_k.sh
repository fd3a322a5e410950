#!/bin/bash
# kernel-trace summary of the 1-GPU DiFacto step (last 50 of 100 steps).
# Usage: bash tools/gpu/r2_k.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-k}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd csv -d gpurun_out/prof_$TAG/p1 -o p1 -- python3 bench.py --steps 100 --warmup 5 "$@" > gpurun_out/prof_$TAG/p1.log 2>&1 || exit $?
tail -1 gpurun_out/prof_$TAG/p1.log | cut -c1-200
python3 tools/prof_summary.py "$(find gpurun_out/prof_$TAG/p1 -name "*.db" -print -quit)" --last-steps 50 --step-kernel k_fm_fwd --top 30 > gpurun_out/$TAG.kernels.txt 2>&1
python3 tools/step_timeline.py gpurun_out/prof_$TAG/p1 k_fm_fwd 3 > gpurun_out/$TAG.timeline.txt 2>&1
rm -rf gpurun_out/prof_$TAG/p1
cat gpurun_out/$TAG.kernels.txt
