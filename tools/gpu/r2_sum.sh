#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-sum}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $OUT/d.$i.log 2>&1 || exit 1
  echo "d $i $(tail -1 $OUT/d.$i.log | cut -c1-150)"
  timeout -k 10 300 python bench.py --loopback 8 --steps 200 --warmup 20 > $OUT/lb.$i.log 2>&1 || exit 1
  echo "lb8 $i $(tail -1 $OUT/lb.$i.log | cut -c1-150)"
done
