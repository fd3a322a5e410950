#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-push}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_psx.py tests/test_kv_exchange.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
bash tools/gpu/env_ab.sh $(basename $OUT)_lb8 WH_PSX_PUSH_STREAM=0 --loopback 8 --steps 200 --warmup 20 || exit 1
timeout -k 10 300 python bench.py --loopback 8 --loopback-rccl --steps 100 --warmup 10 > $OUT/lb8_rccl.log 2>&1 || { tail -20 $OUT/lb8_rccl.log; exit 1; }
tail -1 $OUT/lb8_rccl.log | cut -c1-200
