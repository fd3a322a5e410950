#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-plan}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu/env_ab.sh $(basename $OUT)_d WH_BWD_PLAN_STREAM=0 --steps 200 --warmup 20 || exit 1
