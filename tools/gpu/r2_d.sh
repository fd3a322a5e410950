#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_psx.py tests/test_deterministic_gpu.py -m gpu > gpurun_out/d_tests.log 2>&1 || { echo TESTS FAILED; tail -60 gpurun_out/d_tests.log; exit 1; }
tail -1 gpurun_out/d_tests.log
for v in "WH_LOCALIZE=hash" "WH_LOCALIZE=part" "WH_LOC_TIMING=1"; do
  env $v timeout -k 10 120 python -u benchmarks/bench_localize.py 2>&1 | grep '^{' || { echo FAILED $v; exit 1; }
done
for a in "--steps 100 --warmup 10" "--steps 100 --warmup 10 --loopback 8"; do
  timeout -k 10 300 python -u bench.py $a > gpurun_out/r2_bench.tmp 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/r2_bench.tmp; exit 1; }
  grep '^{' gpurun_out/r2_bench.tmp | cut -c1-250
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/p1 -o p1 -- python3 bench.py --steps 100 --warmup 5 > gpurun_out/prof/p1.log 2>&1 || { echo P1 FAILED; tail -20 gpurun_out/prof/p1.log; exit 1; }
