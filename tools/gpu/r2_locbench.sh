#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "localize or learner" -m gpu > gpurun_out/loc_tests.log 2>&1 || { echo TESTS FAILED; tail -60 gpurun_out/loc_tests.log; exit 1; }
tail -1 gpurun_out/loc_tests.log
for v in "WH_LOCALIZE=hash" "WH_LOCALIZE=part" "SKEW=0" "WH_LOC_TIMING=1" "WH_LOC_TIMING=1 SKEW=0"; do
  env $v timeout -k 10 120 python -u benchmarks/bench_localize.py 2>&1 | grep '^{' || { echo FAILED $v; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/loc -o loc -- python3 benchmarks/bench_localize.py > gpurun_out/prof/loc.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof/loc.log; exit 1; }
