#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-auc2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu/env_ab.sh $(basename $OUT)_lb8 WH_AUC_LATE=0 --loopback 8 --steps 200 --warmup 20 || exit 1
