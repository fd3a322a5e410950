#!/bin/bash
# The README's HEAD numbers in one GPU call (one box): DiFacto P = 1 / loopback 8,
# linear P = 1 / loopback 8 / RCCL loopback, GBDT 500 trees, k-means, L-BFGS.
# Usage: bash tools/gpu/headline_set.sh TAG
set -o pipefail
O=gpurun_out/${1:-headline}; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 400 "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 $O/$tag.log; exit 1; }; echo "$tag: $(grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"ms_per_tree": [0-9.]*\|"ms_per_iter": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; }
run dif_p1_a python bench.py
run dif_p1_b python bench.py
run dif_lb8 python bench.py --loopback 8
run dif_lb8r python bench.py --loopback 8 --loopback-rccl
run lin_p1 python bench.py --model linear --steps 1000 --warmup 50
run lin_lb8 python bench.py --model linear --loopback 8 --steps 1000 --warmup 50
run gbdt500 python benchmarks/bench_gbdt.py --trees 500
run kmeans python benchmarks/bench_kmeans.py
run lbfgs python benchmarks/bench_lbfgs.py
