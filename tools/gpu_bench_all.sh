#!/bin/bash
# All 1-GPU benchmarks at the BASELINE.json configs. Usage: bash tools/gpu_bench_all.sh <tag>
set -o pipefail
TAG=${1:-benchall}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/difacto.log 2>&1 || exit $?
tail -1 $OUT/difacto.log
timeout -k 10 300 python bench.py --model linear > $OUT/linear.log 2>&1 || exit $?
tail -1 $OUT/linear.log
timeout -k 10 600 python benchmarks/bench_kmeans.py --rows 10000000 --dim 128 --k 1000 > $OUT/kmeans.log 2>&1 || exit $?
tail -1 $OUT/kmeans.log
timeout -k 10 600 python benchmarks/bench_gbdt.py --rows 11000000 --features 28 --depth 8 --trees 20 > $OUT/gbdt.log 2>&1 || exit $?
tail -1 $OUT/gbdt.log
echo bench-all done
