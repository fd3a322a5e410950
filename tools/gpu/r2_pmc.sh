#!/bin/bash
# PMC passes over the 1-GPU DiFacto step, summarised on the box (raw CSVs are
# deleted: they exceed what gpurun copies back). Usage: bash tools/gpu/r2_pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_pmc.sh $TAG --steps 20 --warmup 2 --prewarm 300 || exit $?
python3 tools/pmc_summary.py gpurun_out/$TAG 30 > gpurun_out/$TAG.txt 2>&1
rm -rf gpurun_out/$TAG
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/p1 -o p1 -- python3 bench.py --steps 100 --warmup 5 --prewarm 1000 > gpurun_out/prof_$TAG/p1.log 2>&1 || exit $?
python3 tools/prof_summary.py "$(find gpurun_out/prof_$TAG/p1 -name "*.db" -print -quit)" --last-steps 50 --top 28 > gpurun_out/$TAG.kernels.txt 2>&1
rm -rf gpurun_out/prof_$TAG/p1
cat gpurun_out/$TAG.txt | head -40
