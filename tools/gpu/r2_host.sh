#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for a in "--steps 100 --warmup 10 --prewarm 200" "--steps 100 --warmup 10 --prewarm 200 --loopback 8"; do
  echo "== bench $a"
  timeout -k 10 300 python -u bench.py $a > gpurun_out/r2_bench.tmp 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/r2_bench.tmp; exit 1; }
  tail -1 gpurun_out/r2_bench.tmp | cut -c1-400
  WH_HOST_PROFILE=gpurun_out/hostprof_$(echo $a | tr -d ' -') timeout -k 10 300 python -u bench.py $a > gpurun_out/r2_bench.tmp 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/r2_bench.tmp; exit 1; }
  tail -1 gpurun_out/r2_bench.tmp | cut -c1-300
done
