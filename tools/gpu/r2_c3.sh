#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-c3}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_psx.py tests/test_kv_exchange.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
bash tools/gpu/env_ab.sh $(basename $OUT)_rccl WH_PSX_C3_LATE=0 --loopback 8 --loopback-rccl --steps 200 --warmup 20 || exit 1
bash tools/gpu/env_ab.sh $(basename $OUT)_lb8 WH_PSX_C3_LATE=0 --loopback 8 --steps 200 --warmup 20 || exit 1
