#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py -k kmeans -m gpu > gpurun_out/km_tests.log 2>&1 || { echo TESTS FAILED; tail -60 gpurun_out/km_tests.log; exit 1; }
tail -1 gpurun_out/km_tests.log
for v in "WH_KMEANS_PREC=fp32" "WH_KMEANS_PREC=split"; do
  env $v timeout -k 10 300 python -u benchmarks/bench_kmeans.py --iters 10 > gpurun_out/km.tmp 2>&1 || { echo KM FAILED; tail -30 gpurun_out/km.tmp; exit 1; }
  grep '^{' gpurun_out/km.tmp
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/km -o km -- python3 benchmarks/bench_kmeans.py --iters 5 > gpurun_out/prof/km.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof/km.log; exit 1; }
