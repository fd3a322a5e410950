#!/bin/bash
# round 2: multi-shard exchange path on one GPU (tests + loopback bench) and
# the steady-state headline bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_psx.py tests/test_kernels_gpu.py -m gpu > gpurun_out/r2_tests.log 2>&1 || { echo TESTS FAILED; tail -50 gpurun_out/r2_tests.log; exit 1; }
tail -3 gpurun_out/r2_tests.log
for a in "--steps 20 --warmup 5" "--steps 200 --warmup 20" "--steps 100 --warmup 10 --loopback 8" "--steps 100 --warmup 10 --loopback 8 --max-concurrency 1" "--steps 100 --warmup 10 --prewarm 0"; do
  echo "== bench $a"
  timeout -k 10 300 python -u bench.py $a > gpurun_out/r2_bench.tmp 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/r2_bench.tmp; exit 1; }
  tail -1 gpurun_out/r2_bench.tmp | tee -a gpurun_out/r2_bench.jsonl
done
