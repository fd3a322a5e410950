#!/bin/bash
# RCCL transport of the multi-shard step on one GPU: GPU test + loopback-8
# bench with every exchange a real RCCL all-to-all (1-rank group).
set -o pipefail
OUT=gpurun_out/${1:-rccl}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_psx.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }
tail -3 $OUT/test.log
timeout -k 10 300 python bench.py --loopback 8 --steps 100 --warmup 10 > $OUT/lb8.log 2>&1 || { tail -20 $OUT/lb8.log; exit 1; }
tail -1 $OUT/lb8.log | cut -c1-260
timeout -k 10 300 python bench.py --loopback 8 --loopback-rccl --steps 100 --warmup 10 > $OUT/lb8_rccl.log 2>&1 || { tail -20 $OUT/lb8_rccl.log; exit 1; }
tail -1 $OUT/lb8_rccl.log | cut -c1-260
echo done
