#!/bin/bash
# k-means assignment A/B on one box: kernel tests, then bench_kmeans.py interleaved per variant
# Usage: bash tools/gpu/km_ab.sh TAG "name|ENV=v ..." ...
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_apps_gpu.py -x -q --timeout 150 --timeout-method thread -k kmeans > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for round in 1 2; do
  for v in "$@"; do
    IFS='|' read -r n e <<< "$v"
    timeout -k 10 300 env $e python benchmarks/bench_kmeans.py --iters 10 --warmup 2 > $O/$n.$round.log 2>&1 || { tail -20 $O/$n.$round.log; exit 1; }
    echo "$n $round [$e]: $(grep -o '"value": [0-9.]*' $O/$n.$round.log) $(grep -o '"ms_per_iter": [0-9.]*' $O/$n.$round.log)"
  done
done
