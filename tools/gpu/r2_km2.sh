#!/bin/bash
# k-means bench (persistent split-precision assignment) + kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/km2
for i in 1 2; do
  timeout -k 10 200 python3 -u benchmarks/bench_kmeans.py --iters 20 > gpurun_out/km2/bench_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/km2/bench_$i.log | cut -c1-260
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/km2/prof -o km -- python3 benchmarks/bench_kmeans.py --iters 5 --warmup 1 > gpurun_out/km2/prof.log 2>&1 || exit 1
python3 tools/prof_summary.py "$(find gpurun_out/km2/prof -name "*.db" -print -quit)" --top 14 > gpurun_out/km2/kernels.txt 2>&1
rm -rf gpurun_out/km2/prof
cat gpurun_out/km2/kernels.txt
