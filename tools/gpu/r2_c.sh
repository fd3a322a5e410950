#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_psx.py tests/test_store_guard.py tests/test_kernels_gpu.py tests/test_kv_exchange.py tests/test_checkpoint.py -m gpu > gpurun_out/r2c_tests.log 2>&1 || { echo TESTS FAILED; tail -50 gpurun_out/r2c_tests.log; exit 1; }
tail -2 gpurun_out/r2c_tests.log
for a in "--steps 100 --warmup 10" "--steps 100 --warmup 10 --loopback 8"; do
  timeout -k 10 300 python -u bench.py $a > gpurun_out/r2_bench.tmp 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/r2_bench.tmp; exit 1; }
  tail -1 gpurun_out/r2_bench.tmp | cut -c1-330
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/lb8 -o lb8 -- python3 bench.py --steps 100 --warmup 5 --prewarm 300 --loopback 8 > gpurun_out/prof/lb8.log 2>&1 || { echo LB FAILED; tail -20 gpurun_out/prof/lb8.log; exit 1; }
