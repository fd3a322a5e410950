#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_psx.py tests/test_store_guard.py -m gpu > gpurun_out/r2b_tests.log 2>&1 || { echo TESTS FAILED; tail -50 gpurun_out/r2b_tests.log; exit 1; }
tail -3 gpurun_out/r2b_tests.log
for a in "--steps 100 --warmup 10" "--steps 100 --warmup 10 --loopback 8"; do
  echo "== bench $a"
  timeout -k 10 300 python -u bench.py $a > gpurun_out/r2_bench.tmp 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/r2_bench.tmp; exit 1; }
  tail -1 gpurun_out/r2_bench.tmp | tee -a gpurun_out/r2b_bench.jsonl
done
timeout -k 10 400 python -u benchmarks/bench_store_growth.py > gpurun_out/r2b_store.log 2>&1 || { echo STORE FAILED; tail -30 gpurun_out/r2b_store.log; exit 1; }
tail -1 gpurun_out/r2b_store.log
