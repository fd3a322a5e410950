#!/bin/bash
# GBDT A/B on one box: GPU tests, then bench_gbdt.py interleaved per variant
# Usage: TREES=100 bash tools/gpu/gbdt_ab.sh TAG "name|ENV=v ..." ...
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_apps_gpu.py tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k gbdt > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for round in 1 2; do
  for v in "$@"; do
    IFS='|' read -r n e <<< "$v"
    timeout -k 10 300 env $e python benchmarks/bench_gbdt.py --trees ${TREES:-100} > $O/$n.$round.log 2>&1 || { tail -20 $O/$n.$round.log; exit 1; }
    echo "$n $round [$e]: $(grep -o '"value": [0-9.]*' $O/$n.$round.log) $(grep -o '"ms_per_tree": [0-9.]*' $O/$n.$round.log)"
  done
done
